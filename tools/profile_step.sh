#!/bin/bash
# Counters of bench.py's own timed window (frames in flight, the driver's step count): a
# kernel-trace pass and separate --pmc passes over the same command, each a run of its own
# (pool rules: --kernel-trace only beside --pmc), then tools/pmc_step.py sums the dispatches
# between bench.py's profile markers.  The CPU baseline and the moving-camera figure are
# skipped (no GPU work in the former; the latter runs after the window).
# Usage: tools/profile_step.sh TAG [bench args...]   (default: the headline at --steps 20 --warmup 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-step}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
STEPS=${STEPS:-20}
ARGS="--steps $STEPS --warmup 5 --no-cpu-baseline --no-camera-path --pmc-window device $*"
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- python3 "$R/bench.py" $ARGS > "$OUT/$name.log" 2>&1; }
run kt --kernel-trace --stats || { echo "kernel-trace run failed"; exit 1; }
run fetch --kernel-trace --pmc FETCH_SIZE || { echo "pmc FETCH_SIZE failed"; exit 1; }
run write --kernel-trace --pmc WRITE_SIZE || { echo "pmc WRITE_SIZE failed"; exit 1; }
run sq1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS || { echo "pmc sq1 failed"; exit 1; }
run sq2 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY || { echo "pmc sq2 failed"; exit 1; }
echo "profile_step done"
