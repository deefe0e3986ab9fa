#!/bin/bash
# bench.py at the driver's settings with 4 / 6 / 8 frames in flight, interleaved rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05/depth; mkdir -p $O
cd "$R" || exit 1
for i in 1 2 3 4; do
  for d in 4 6 8; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path --frames-in-flight $d > $O/w8s_d${d}_$i.log 2>&1 || { echo "d$d failed"; exit 1; }
    tail -1 $O/w8s_d${d}_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('depth %s round %s ms/frame %.4f' % (sys.argv[1], sys.argv[2], d['ms_per_step']))" $d $i
  done
done
