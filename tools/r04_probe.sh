#!/bin/bash
# Round-4 probe: bench at the driver's settings (with query occupancy), the new CLI /
# multi-device / config-5 tests, the CLI frames-in-flight timings, A/Bs of this round's changes.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04/bench0.log 2>&1 || exit 1
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_cli.py tests/test_gpu_multi.py tests/test_gpu_fullsize.py tests/test_gpu_pipeline.py -k "cli or multi or config5_full or pipeline or bench_frame" > gpurun_out/r04/pytest_cli_multi.log 2>&1 || exit 1
for a in "--gpus 1 --ranks 8 --in-flight 8" "--gpus 1 --ranks 8 --in-flight 4" "--gpus 1 --ranks 8 --in-flight 1" "--in-flight 8" "--in-flight 1"; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 ./gpu-ray-tracer_amd/rtracer -c scenes/world8_stress.json --width 1920 --height 1080 --spp 8 --frames 40 $a >> gpurun_out/r04/cli_inflight.log 2>&1 || exit 1
done
# A/B: heavy-first by work (RT_HEAVY_Q=6) vs off (0)
bash tools/ab_env.sh r04/ab_heavy RT_HEAVY_Q 0 6 3 > gpurun_out/r04/ab_heavy.log 2>&1 || exit 1
# A/B: scene view read in place at use sites (librt_amd.so) vs the by-value argument (librt_fs0.so), heavy-first off in both
RT_HEAVY_Q=0 bash tools/ab_libs.sh r04/ab_fresh 3 0 gpu-ray-tracer_amd/librt_fs0.so gpu-ray-tracer_amd/librt_amd.so > gpurun_out/r04/ab_fresh.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --scene world16 --width 3840 --height 2160 --spp 64 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04/bench_w16.log 2>&1
