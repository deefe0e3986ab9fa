#!/bin/bash
# One SQ pass (instructions + wave-time split) and one memory pass per library, lone headline
# frames.  Usage: tools/pmc_ab.sh TAG lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-overlap --no-camera-path"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  RTAMD_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/${n}_sq" -o s -- python3 "$R/bench.py" $ARGS > "$OUT/${n}_sq.log" 2>&1 || { echo "$n sq failed"; exit 1; }
  RTAMD_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_INSTS_LDS SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/${n}_mem" -o m -- python3 "$R/bench.py" $ARGS > "$OUT/${n}_mem.log" 2>&1 || { echo "$n mem failed"; exit 1; }
  RTAMD_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/${n}_fetch" -o f -- python3 "$R/bench.py" $ARGS > "$OUT/${n}_fetch.log" 2>&1 || { echo "$n fetch failed"; exit 1; }
done
for lib in "$@"; do n=$(basename "$lib" .so); echo "== $n"; python3 "$R/tools/pmc_summary.py" "$OUT/${n}_sq" "trace_kernel<0, true, 180>"; python3 "$R/tools/pmc_summary.py" "$OUT/${n}_mem" "trace_kernel<0, true, 180>" | tail -3; python3 "$R/tools/pmc_summary.py" "$OUT/${n}_fetch" "trace_kernel<0, true, 180>" | tail -1; done
