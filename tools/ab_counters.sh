#!/bin/bash
# Per-step instruction counters of library variants (A/B of a kernel change): for each library,
# one --pmc pass over bench.py's device-resident window (tools/profile_step.sh's command, 20
# steps) with the issue counters, summarised per step by tools/pmc_step.py into
# gpurun_out/TAG/<lib>.json.  Usage: TAG=... tools/ab_counters.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-ab_counters}
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-camera-path --pmc-window device"
for L in "$@"; do
  n=$(basename "$L" .so)
  RTAMD_LIB=$R/$L timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$O/$n" -o sq -- python3 "$R/bench.py" $ARGS > "$O/$n.log" 2>&1 || { echo "pmc $n failed"; tail "$O/$n.log"; exit 1; }
  python3 "$R/tools/pmc_step.py" "$O/$n" "$n" 20 "$O/$n.json" > /dev/null || exit 1
  python3 - "$O/$n.json" "$n" <<'PY'
import json, sys
e = json.load(open(sys.argv[1]))[sys.argv[2]]["per_step"]
print("%-12s VALU %.4e  SALU %.4e  SMEM %.4e  LDS %.4e  WAIT_INST_ANY %.4e  WAVE_CYCLES %.4e" % (
    sys.argv[2], e.get("SQ_INSTS_VALU", 0), e.get("SQ_INSTS_SALU", 0), e.get("SQ_INSTS_SMEM", 0),
    e.get("SQ_INSTS_LDS", 0), e.get("SQ_WAIT_INST_ANY", 0), e.get("SQ_WAVE_CYCLES", 0)))
PY
done
