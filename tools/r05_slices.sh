#!/bin/bash
# Per-rank slice pipelines (N = 1/2/4/8, eight in flight) for each library, interleaved rounds.
# Usage: tools/r05_slices.sh TAG ROUNDS lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ROUNDS=$2; shift 2
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    RTAMD_LIB=$R/$lib NS=1,2,4,8 DEPTHS=8 timeout -k 10 240 python3 -u "$R/tools/pipe_slices.py" > "$OUT/slices_${n}_$i.log" 2>&1 || { echo "slices $n failed"; tail -3 "$OUT/slices_${n}_$i.log"; exit 1; }
    echo "$n round $i N=1/2/4/8: $(grep -o '"ms_per_frame": [0-9.]*' "$OUT/slices_${n}_$i.log" | awk '{print $2}' | tr '\n' ' ')"
  done
done
