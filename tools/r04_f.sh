#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04/pytest_gpu_spec.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r04/pytest_gpu_spec.log; exit 1; }
bash tools/ab_libs.sh r04/ab_spec 4 0 gpu-ray-tracer_amd/librt_dbl.so gpu-ray-tracer_amd/librt_spec.so > gpurun_out/r04/ab_spec.log 2>&1
cat gpurun_out/r04/ab_spec.log
