#!/bin/bash
# Round-4 profiles at HEAD: the headline (full PMC set), config 5 (world16 4K 64 spp), world8 and
# world1 brute force (quick sets); a kernel trace of the pipelined bench at the driver's 20 steps;
# the CLI's frames in flight with 16 hardware queues set in the environment.
set -o pipefail
mkdir -p gpurun_out/r04
bash tools/profile.sh r04/prof_w8s > gpurun_out/r04/prof_w8s.log 2>&1 || { echo "headline profile failed"; exit 1; }
QUICK=1 bash tools/profile.sh r04/prof_w16 --scene world16 --width 3840 --height 2160 --spp 64 > gpurun_out/r04/prof_w16.log 2>&1 || { echo "w16 profile failed"; exit 1; }
QUICK=1 bash tools/profile.sh r04/prof_w8 --scene world8 > gpurun_out/r04/prof_w8.log 2>&1 || { echo "w8 profile failed"; exit 1; }
QUICK=1 bash tools/profile.sh r04/prof_w1b --scene world1 --spp 1 --brute > gpurun_out/r04/prof_w1b.log 2>&1 || { echo "w1 profile failed"; exit 1; }
R=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r04/kt20" -o kt20 -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/r04/kt20.log" 2>&1) || { echo "kt20 failed"; exit 1; }
for a in "--gpus 1 --ranks 8 --in-flight 8" "--gpus 1 --ranks 8 --in-flight 1" "--in-flight 8" "--in-flight 1"; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 ./gpu-ray-tracer_amd/rtracer -c scenes/world8_stress.json --width 1920 --height 1080 --spp 8 --frames 40 $a >> gpurun_out/r04/cli_inflight_q16.log 2>&1 || exit 1
done
echo "r04_prof done"
