#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-rbprobe}
mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python3 -u $R/tools/readback_probe.py 0 > $O/dev_$i.log 2>&1 || { tail $O/dev_$i.log; exit 1; }
timeout -k 10 120 python3 -u $R/tools/readback_probe.py 1 > $O/rb_$i.log 2>&1 || { tail $O/rb_$i.log; exit 1; }
for L in ${DEFERS:-}; do timeout -k 10 120 python3 -u $R/tools/readback_probe.py 1 > $O/rbdefer${L}_$i.log 2>&1 || { tail $O/rbdefer${L}_$i.log; exit 1; }; done
done
for f in $O/*.log; do echo $f; tail -1 $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d[\"ms_per_frame\"], \"maxissue\", max(d[\"issue_ms\"]), \"waits\", round(sum(d[\"wait_ms\"]),2), \"lat\", d.get(\"render_done_to_copy_done_ms\", [])[:24])"; done
