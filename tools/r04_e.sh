#!/bin/bash
# grid policy of frames issued while another runs, at the driver's 20 steps and at 60
set -o pipefail
mkdir -p gpurun_out/r04
bash tools/ab_sweep.sh r04/sweep_grid RT_BENCH_GRID "half last-full full" 3 > gpurun_out/r04/sweep_grid.log 2>&1 || exit 1
for d in 4 6; do for k in 20 60; do timeout -k 10 200 python3 bench.py --steps $k --warmup 5 --no-cpu-baseline --frames-in-flight $d > gpurun_out/r04/depth${d}_$k.log 2>&1 || exit 1; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['frame_ms'])" gpurun_out/r04/depth${d}_$k.log; done; done >> gpurun_out/r04/sweep_grid.log
echo done
