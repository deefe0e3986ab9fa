#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-rbprobe}
mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python3 -u $R/tools/readback_probe.py 0 > $O/dev_$i.log 2>&1 || { tail $O/dev_$i.log; exit 1; }
timeout -k 10 120 python3 -u $R/tools/readback_probe.py 1 > $O/rb_$i.log 2>&1 || { tail $O/rb_$i.log; exit 1; }
done
for f in $O/*.log; do tail -1 $f | cut -c1-900; done
