#!/bin/bash
# Same-box A/B/C... of library builds: bench.py (and optionally the per-rank slice pipeline)
# run with each library in turn (RTAMD_LIB), ROUNDS interleaved rounds.
# Usage: tools/ab_libs.sh TAG ROUNDS SLICES(0|1) lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ROUNDS=$2; SLICES=$3; shift 3
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    RTAMD_LIB=$lib timeout -k 10 240 python3 -u "$R/bench.py" --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline \
      > "$OUT/bench_${n}_$i.log" 2>&1 || { echo "bench $n round $i failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-12s round %s frame_ms %.4f trace %.4f latency %.4f readback %.4f' % (sys.argv[2], sys.argv[3], d['frame_ms'], d['trace_kernel_ms'], d['frame_latency_ms'], d['ms_per_step_with_readback']))" "$OUT/bench_${n}_$i.log" "$n" $i
    if [ "$SLICES" = 1 ]; then
      RTAMD_LIB=$lib NS=1,2,4,8 DEPTHS=${DEPTHS:-8} timeout -k 10 240 python3 -u "$R/tools/pipe_slices.py" > "$OUT/slices_${n}_$i.log" 2>&1 \
        || { echo "slices $n failed"; exit 1; }
      echo "$n round $i slices N=1/2/4/8: $(grep -o '"ms_per_frame": [0-9.]*' "$OUT/slices_${n}_$i.log" | awk '{print $2}' | tr '\n' ' ')"
    fi
  done
done
