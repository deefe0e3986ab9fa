#!/bin/bash
# Same-box sweep of a runtime switch: bench.py at the driver's settings (--steps 20 --warmup 5)
# and at 60 steps, VAR set to each value in turn, ROUNDS interleaved rounds.
# Usage: tools/ab_sweep.sh TAG VAR "v1 v2 ..." [ROUNDS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; VAR=$2; VALS=$3; ROUNDS=${4:-3}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for v in $VALS; do
    for k in 20 60; do
      env "$VAR=$v" timeout -k 10 240 python3 -u "$R/bench.py" --steps $k --warmup 5 --no-cpu-baseline \
        > "$OUT/bench_${v}_${k}_$i.log" 2>&1 || { echo "bench $VAR=$v round $i failed"; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%s=%s steps %s round %s frame_ms %.4f trace %.4f latency %.4f' % (sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5], d['frame_ms'], d['trace_kernel_ms'], d['frame_latency_ms']))" "$OUT/bench_${v}_${k}_$i.log" "$VAR" "$v" $k $i
    done
  done
done
