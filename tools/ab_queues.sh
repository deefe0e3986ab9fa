#!/bin/bash
# Same-box A/B of GPU_MAX_HW_QUEUES for bench.py (4 = HIP's and the pool's default, 8 = bench.py's
# setting), interleaved rounds; then the per-rank slice pipeline (tools/pipe_slices.py) at each.
# Usage: tools/ab_queues.sh TAG [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-abq}; ROUNDS=${2:-3}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for q in 8 4; do
    RT_BENCH_HW_QUEUES=$q timeout -k 10 240 python3 -u "$R/bench.py" --steps 60 --warmup 5 --no-cpu-baseline \
      > "$OUT/bench_q${q}_$i.log" 2>&1 || { echo "bench q=$q round $i failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('q=%s round %s frame_ms %.4f readback %.4f' % (sys.argv[2], sys.argv[3], d['frame_ms'], d['ms_per_step_with_readback']))" "$OUT/bench_q${q}_$i.log" $q $i
  done
done
for q in 8 4; do
  RT_BENCH_HW_QUEUES=$q NS=1,2,4,8 DEPTHS=1,4 timeout -k 10 240 python3 -u "$R/tools/pipe_slices.py" > "$OUT/slices_q$q.log" 2>&1 \
    || { echo "slices q=$q failed"; exit 1; }
  sed "s/^/q=$q /" "$OUT/slices_q$q.log" | grep ms_per_frame
done
