#!/bin/bash
# The cold-frame probe (tools/cold_probe.py) alone, then under a HIP-API + kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-cold}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 -u $R/tools/cold_probe.py > $O/probe.log 2>&1 || { tail $O/probe.log; exit 1; }
cat $O/probe.log
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o trace -- python3 -u $R/tools/cold_probe.py > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
echo done
