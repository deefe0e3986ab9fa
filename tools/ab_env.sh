#!/bin/bash
# Same-box A/B of a runtime switch of the library: bench.py (and optionally the per-rank slice
# pipeline) run alternately with VAR=A and VAR=B, ROUNDS interleaved rounds.
# Usage: tools/ab_env.sh TAG VAR A B [ROUNDS] [slices]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; VAR=$2; A=$3; B=$4; ROUNDS=${5:-3}; SLICES=${6:-}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for arm in A B; do
    if [ $arm = A ]; then v=$A; else v=$B; fi
    env "$VAR=$v" timeout -k 10 240 python3 -u "$R/bench.py" --steps 60 --warmup 5 --no-cpu-baseline \
      > "$OUT/bench_${arm}_$i.log" 2>&1 || { echo "bench $VAR=$v round $i failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%s round %s frame_ms %.4f trace %.4f readback %.4f' % (sys.argv[2], sys.argv[3], d['frame_ms'], d['trace_kernel_ms'], d['ms_per_step_with_readback']))" "$OUT/bench_${arm}_$i.log" "$VAR=$v" $i
  done
done
if [ -n "$SLICES" ]; then
  for i in 1 2; do
    for arm in A B; do
      if [ $arm = A ]; then v=$A; else v=$B; fi
      env "$VAR=$v" NS=1,2,4,8 DEPTHS=4 timeout -k 10 240 python3 -u "$R/tools/pipe_slices.py" > "$OUT/slices_${arm}_$i.log" 2>&1 \
        || { echo "slices $VAR=$v failed"; exit 1; }
      grep ms_per_frame "$OUT/slices_${arm}_$i.log" | sed "s|^|$VAR=$v |"
    done
  done
fi
