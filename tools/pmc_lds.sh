#!/bin/bash
# LDS / scalar-unit / issue counters of the headline's lone frames (two --pmc passes, each its
# own run).  Usage: tools/pmc_lds.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-lds}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-overlap --no-camera-path $*"
run() { local name=$1; shift; timeout -k 10 200 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- python3 "$R/bench.py" $ARGS > "$OUT/$name.log" 2>&1; }
run lds1 --kernel-trace --pmc SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU || { echo "pmc lds1 failed"; exit 1; }
run lds2 --kernel-trace --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU2 SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU || { echo "pmc lds2 failed"; exit 1; }
run lds3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_VALU || { echo "pmc lds3 failed"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT" "trace_kernel<0, true, 180>"
