#!/bin/bash
# Why host copies show as blit kernels under rocprofv3 in a torch process: the runtime's log of
# the readback probe with and without the profiler (its own "falling to Blit copy" line).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-copyprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
AMD_LOG_LEVEL=3 timeout -k 10 120 python3 -u $R/tools/readback_probe.py 1 > $O/plain.txt 2>&1 || { tail $O/plain.txt; exit 1; }
AMD_LOG_LEVEL=3 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o prof -- python3 -u $R/tools/readback_probe.py 1 > $O/profiled.txt 2>&1 || { tail $O/profiled.txt; exit 1; }
for f in plain profiled; do
  echo "$f: HSA copies (SDMA) $(grep -c 'HSA Copy copy_engine' $O/$f.txt), blit fallbacks $(grep -ci 'falling to Blit' $O/$f.txt), copy failures $(grep -ci 'HSA copy failed' $O/$f.txt)"
done
grep -i "falling to Blit\|HSA copy failed" $O/profiled.txt > $O/fallbacks.txt || true; sed -n 1,3p $O/fallbacks.txt | cut -c1-250
