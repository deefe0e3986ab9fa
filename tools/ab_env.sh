#!/bin/bash
# Same-box A/B of bench.py settings given as environment assignments (one arm per argument,
# e.g. RT_BENCH_GRID=half RT_BENCH_GRID=stream), ROUNDS interleaved rounds, STEPS timed steps.
# Usage: STEPS=20 tools/ab_env.sh TAG ROUNDS 'VAR=a' 'VAR=b' ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ROUNDS=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for arm in "$@"; do
    n=$(echo "$arm" | tr -c 'A-Za-z0-9_\n' '_')
    env $arm timeout -k 10 240 python3 -u "$R/bench.py" --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --no-camera-path \
      > "$OUT/bench_${n}_$i.log" 2>&1 || { echo "bench $arm round $i failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-24s round %s frame_ms %.4f device-resident %.4f trace %.4f latency %.4f cold %.4f' % (sys.argv[2], sys.argv[3], d['frame_ms'], (d.get('device_resident') or {}).get('ms_per_step', float('nan')), d['trace_kernel_ms'], d['frame_latency_ms'], d.get('cold_frame_ms', float('nan'))))" "$OUT/bench_${n}_$i.log" "$arm" $i
  done
done
