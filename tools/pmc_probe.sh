#!/bin/bash
# PMC passes (one rocprofv3 run each, --kernel-trace beside --pmc only) over any command:
# tools/pmc_probe.sh TAG -- python3 tools/cam_probe.py ...   Summaries: tools/pmc_summary.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift; [ "$1" == "--" ] && shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { local name=$1; shift; local pmc="$*"; timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d "$OUT/$name" -o "$name" -- "${CMD[@]}" > "$OUT/$name.log" 2>&1; }
CMD=("$@")
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS || { echo "sq1 failed"; exit 1; }
run sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY || { echo "sq2 failed"; exit 1; }
run sq3 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH || echo "sq3 failed (non-fatal)"
echo "pmc probe done"
