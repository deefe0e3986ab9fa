#!/bin/bash
# One build -> measure iteration on one MI355X: the GPU suite (or PYTEST_ARGS), bench.py at the
# driver's settings twice, and a kernel + memory-copy trace of the driver's bench command.
# Usage: TAG=r06/x tools/iter.sh [extra bench args]   (SKIP_TESTS=1: bench and trace only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
T=${TAG:-iter}
O=gpurun_out/$T
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${PYTEST_ARGS:-tests} > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/bench20_$i.log 2>&1 || { echo "bench failed"; tail -30 $O/bench20_$i.log; exit 1; }
  tail -1 $O/bench20_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], 'dev', d.get('device_resident'), 'cold', d.get('cold_frame_ms'), 'load', d.get('scene_load_ms'), 'lat', d.get('frame_latency_ms'), 'cam', (d.get('camera_path') or {}).get('ms_per_step'))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt20" -o kt20 -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path "$@" > "$R/$O/kt20.log" 2>&1) || { echo "kt20 failed"; tail "$R/$O/kt20.log"; exit 1; }
cut -c1-150 $O/kt20/kt20_kernel_stats.csv
echo "iter done"
