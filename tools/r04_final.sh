#!/bin/bash
# Round-4 closing evidence on one MI355X: the GPU suite, smoke(), bench.py at the driver's
# settings (twice) and at 60 steps, the CLI's frames in flight, the rocprofv3 kernel-trace
# summary of the driver's command and the PMC profile of world8_stress (tools/profile.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r04/final
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > $O/bench20_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench20_$i.log; exit 1; }
done
timeout -k 10 200 python3 -u bench.py --steps 60 --warmup 5 --no-cpu-baseline > $O/bench60.log 2>&1 || { echo "bench60 failed"; exit 1; }
for a in "--gpus 1 --ranks 8 --in-flight 8" "--gpus 1 --ranks 8 --in-flight 1" "--in-flight 8" "--in-flight 1"; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 ./gpu-ray-tracer_amd/rtracer -c scenes/world8_stress.json --width 1920 --height 1080 --spp 8 --frames 100 $a > $O/cli.tmp 2>&1 || { echo "cli $a failed"; cat $O/cli.tmp; exit 1; }
  echo "$a: $(grep 'ms/frame' $O/cli.tmp)" >> $O/cli_inflight.log
done
cat $O/cli_inflight.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt20" -o kt20 -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/kt20.log" 2>&1) || { echo "kt20 failed"; exit 1; }
timeout -k 10 900 bash tools/profile.sh r04/final/prof_w8s > $O/profile.log 2>&1 || { echo "profile failed"; tail $O/profile.log; exit 1; }
echo "final evidence done"
