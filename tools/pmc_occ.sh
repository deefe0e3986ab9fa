#!/bin/bash
# Mean resident waves per CU of the headline's lone frames, per library (MeanOccupancyPerCU).
# Usage: tools/pmc_occ.sh TAG lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for lib in "$@"; do
  n=$(basename "$lib" .so)
  RTAMD_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc MeanOccupancyPerCU --output-format csv -d "$OUT/${n}_occ" -o o -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-overlap --no-camera-path > "$OUT/${n}_occ.log" 2>&1 || { echo "$n occ failed"; tail -3 "$OUT/${n}_occ.log"; exit 1; }
  echo "== $n"; python3 "$R/tools/pmc_summary.py" "$OUT/${n}_occ" "trace_kernel<0, true, 180>"
done
