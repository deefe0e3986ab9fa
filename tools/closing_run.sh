#!/bin/bash
# Closing evidence at HEAD on one MI355X: the GPU suite, smoke(), bench.py at the driver's
# settings (twice) and at 60 steps, the per-step PMC of the driver's command (tools/profile_step.sh,
# device-resident window), its kernel-trace summary, the PMC profile of the headline's lone frames
# (tools/profile.sh), config 5 / config 2 / config 3 lines and config 5's traffic, the CLI's -b
# (tools/cli_bench.sh) and the copy-engine fallback check under the profiler.
# Usage: FINAL=r06/final tools/closing_run.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
F=${FINAL:-r06/final}
O=gpurun_out/$F
mkdir -p $O
# PART=a: suite, smoke, benches, per-step PMC, kernel trace, headline PMC; PART=b: config 5 PMC,
# the other configs, CLI -b, the copy check (two gpurun calls of < 20 min each); default both
if [ "${PART:-ab}" != "b" ]; then
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench20_1.log 2>&1 || { echo "bench failed"; tail -20 $O/bench20_1.log; exit 1; }
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_2.log 2>&1 || { echo "bench 2 failed"; exit 1; }
timeout -k 10 200 python3 -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-camera-path > $O/bench60.log 2>&1 || { echo "bench60 failed"; exit 1; }
for f in bench20_1 bench20_2 bench60; do tail -1 $O/$f.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], d['value'], (d.get('device_resident') or {}).get('ms_per_step'), d.get('cold_frame_ms'), d.get('frame_latency_ms'), (d.get('camera_path') or {}).get('ms_per_step'))" $f; done
timeout -k 10 600 bash tools/profile_step.sh $F/step_w8s > $O/profile_step.log 2>&1 || { echo "profile_step failed"; tail $O/profile_step.log; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt20" -o kt20 -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path > "$R/$O/kt20.log" 2>&1) || { echo "kt20 failed"; exit 1; }
timeout -k 10 900 bash tools/profile.sh $F/prof_w8s > $O/profile.log 2>&1 || { echo "profile failed"; tail $O/profile.log; exit 1; }
fi
[ "${PART:-ab}" == "a" ] && { echo "part a done"; exit 0; }
QUICK=1 timeout -k 10 400 bash tools/profile.sh $F/prof_w16 --scene world16 --width 3840 --height 2160 --spp 64 > $O/prof_w16.log 2>&1 || { echo "profile w16 failed"; tail $O/prof_w16.log; exit 1; }
W16="--scene world16 --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2 --no-cpu-baseline --no-camera-path"
timeout -k 10 300 python3 -u bench.py $W16 > $O/cfg_world16.log 2>&1 || { echo "w16 failed"; exit 1; }
timeout -k 10 300 python3 -u bench.py $W16 --scene world16_tex --textures > $O/cfg_world16_tex.log 2>&1 || { echo "w16tex failed"; exit 1; }
timeout -k 10 200 python3 -u bench.py --scene world1 --spp 1 --brute --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path > $O/cfg_world1_brute.log 2>&1 || { echo "w1 failed"; exit 1; }
timeout -k 10 200 python3 -u bench.py --scene world8 --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path > $O/cfg_world8.log 2>&1 || { echo "w8 failed"; exit 1; }
for f in cfg_world16 cfg_world16_tex cfg_world1_brute cfg_world8; do tail -1 $O/$f.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], d['value'], d.get('trace_kernel_ms'))" $f; done
TAG=$F/cli_b timeout -k 10 200 bash tools/cli_bench.sh > $O/cli_b_run.log 2>&1 || { echo "cli -b failed"; exit 1; }
TAG=$F/copyprof timeout -k 10 300 bash tools/copy_profiler_check.sh > $O/copyprof_run.log 2>&1 || { echo "copy check failed"; exit 1; }
tail -3 $O/copyprof_run.log
echo "final evidence done"
