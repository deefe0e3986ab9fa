#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04
bash tools/ab_sweep.sh r04/sweep_heavy RT_HEAVY_Q "0 4 5 6 8" 2 > gpurun_out/r04/sweep_heavy.log 2>&1 || exit 1
for a in "--gpus 1 --ranks 8 --in-flight 8" "--gpus 1 --ranks 8 --in-flight 4" "--gpus 1 --ranks 8 --in-flight 1" "--gpus 1 --ranks 2 --in-flight 8"; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 ./gpu-ray-tracer_amd/rtracer -c scenes/world8_stress.json --width 1920 --height 1080 --spp 8 --frames 100 $a 2>&1 | grep "ms/frame" >> gpurun_out/r04/cli_inflight_d.log
done
cat gpurun_out/r04/cli_inflight_d.log
echo "r04_d done"
