#!/bin/bash
# bench.py at the driver's settings under grid policies, interleaved rounds (same library).
# Usage: tools/r05_grid.sh TAG ROUNDS policy1 policy2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ROUNDS=$2; shift 2
O=$R/gpurun_out/$TAG; mkdir -p $O
cd "$R" || exit 1
for i in $(seq 1 "$ROUNDS"); do
  for g in "$@"; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path --grid $g > $O/w8s_${g}_$i.log 2>&1 || { echo "$g failed"; tail -5 $O/w8s_${g}_$i.log; exit 1; }
    tail -1 $O/w8s_${g}_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-18s round %s ms/frame %.4f' % (sys.argv[1], sys.argv[2], d['ms_per_step']))" $g $i
  done
done
