#!/bin/bash
# Round 4, second probe: the whole GPU suite after the history-mode fix, bench (occupancy),
# per-rank slices with / without the work-based heavy list, and a kernel trace of the CLI's
# frames in flight.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04/pytest_gpu_b.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04/bench_b.log 2>&1 || exit 1
for i in 1 2; do
  for q in 0 6; do
    RT_HEAVY_Q=$q NS=1,2,4,8 DEPTHS=8 timeout -k 10 240 python3 -u tools/pipe_slices.py > gpurun_out/r04/slices_q${q}_$i.log 2>&1 || exit 1
  done
done
R=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r04/kt_cli" -o kt_cli -- "$R/gpu-ray-tracer_amd/rtracer" -c "$R/scenes/world8_stress.json" --width 1920 --height 1080 --spp 8 --frames 40 --in-flight 8 > "$R/gpurun_out/r04/kt_cli.log" 2>&1) || { echo "kt_cli failed"; exit 1; }
echo "r04_b done"
