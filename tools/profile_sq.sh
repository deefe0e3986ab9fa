#!/bin/bash
# PMC passes (SQ/LDS/cache) on a given python command; usage: tools/profile_sq.sh TAG cmd...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp || exit 1
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o "$name" -- python3 $CMD > "$OUT/$name.log" 2>&1; }
CMD="$*"
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY || exit 1
run p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES || exit 1
run p3 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC || exit 1
run p4 SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_SENDMSG SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT || echo "p4 failed"
echo done
