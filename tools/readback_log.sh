#!/bin/bash
# The host-readable pipeline probe under the HIP runtime's log: what the host does in its
# multi-millisecond issue stalls (gaps between consecutive log lines, with context).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-rblog}
mkdir -p $O
AMD_LOG_LEVEL=4 timeout -k 10 120 python3 -u $R/tools/readback_probe.py 1 > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
python3 - $O/log.txt > $O/gaps.txt <<'PY'
import re, sys
lines = open(sys.argv[1], errors="replace").read().splitlines()
ts = []
for i, l in enumerate(lines):
    m = re.search(r": (\d+) us: ", l)
    if m:
        ts.append((int(m.group(1)), i))
for (a, i), (b, j) in zip(ts, ts[1:]):
    if b - a > 2000:
        print("=== gap %d us between lines %d and %d" % (b - a, i, j))
        for l in lines[max(0, i - 12): j + 3]:
            print(l[:260])
PY
wc -l $O/log.txt
head -150 $O/gaps.txt
echo "== API calls over 1 ms (after start-up) =="
grep -n "duration: [0-9]\{4,\} us" $O/log.txt | tail -30 | cut -c1-250
