#!/bin/bash
# tools/copy_probe2.py's variants under a kernel trace (blit kernels or not) and one under the
# runtime's log (why).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-copy2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for q in 16 4; do for v in "8 1" "1 1" "8 0"; do
  n=q${q}_$(echo $v | tr ' ' _)
  RT_BENCH_HW_QUEUES=$q timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/$n -o $n -- python3 -u $R/tools/copy_probe2.py $v > $O/$n.log 2>&1 || { tail $O/$n.log; exit 1; }
  echo "$n: $(grep streams $O/$n.log) blit kernels: $(grep -c copyBuffer $O/$n/${n}_kernel_trace.csv) sdma copies: $(($(wc -l < $O/$n/${n}_memory_copy_trace.csv) - 1))"
done; done
AMD_LOG_LEVEL=4 timeout -k 10 120 python3 -u $R/tools/copy_probe2.py 8 1 > $O/log4.txt 2>&1 || { tail $O/log4.txt; exit 1; }
grep -iE "copy|blit|sdma" $O/log4.txt | grep -v "^$" | head -60 > $O/log4_copy.txt
wc -l $O/log4.txt
head -40 $O/log4_copy.txt
