#!/bin/bash
# Heavy-group threshold (RT_HEAVY_Q, wave queries per group) swept on the headline at the
# driver's 20 steps, interleaved rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/heavyq; mkdir -p $O
run() { local tag=$1 q=$2; shift 2; RT_HEAVY_Q=$q timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-12s ms/frame %.4f  latency %.3f  trace %s  camera %s' % (sys.argv[1], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms'), (d.get('camera_path') or {}).get('ms_per_step')))" $tag; }
for i in 1 2 3; do
  for q in 4 5 6 8 10; do run q${q}_$i $q --steps 20 --warmup 5 || exit 1; done
done
echo "r05_heavyq done"
