#!/bin/bash
# Profile bench.py with rocprofv3: kernel-trace stats, then PMC passes (each its own run,
# --kernel-trace only beside --pmc, per the pool rules).  Usage: tools/profile.sh TAG [bench args...]
# QUICK=1: only the kernel trace, FETCH_SIZE, WRITE_SIZE and the SQ instruction counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-prof}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-overlap $*"   # serial frames: one launch at a time, as bench.py times the kernel
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- python3 "$R/bench.py" $ARGS > "$OUT/$name.log" 2>&1; }
run kt --kernel-trace --stats || { echo "kernel-trace run failed"; exit 1; }
run fetch --kernel-trace --pmc FETCH_SIZE || { echo "pmc FETCH_SIZE failed"; exit 1; }
run write --kernel-trace --pmc WRITE_SIZE || { echo "pmc WRITE_SIZE failed"; exit 1; }
run sq1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS || { echo "pmc sq1 failed"; exit 1; }
[ -n "$QUICK" ] && { echo "profile done (quick: kernel trace, FETCH/WRITE, SQ instructions)"; exit 0; }
run sq2 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY || { echo "pmc sq2 failed"; exit 1; }
run ea --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum || echo "pmc ea failed (non-fatal)"
run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum || echo "pmc tcc failed (non-fatal)"
echo "profile done"
