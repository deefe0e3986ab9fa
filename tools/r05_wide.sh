#!/bin/bash
# Wide RGBA stores for one-pixel groups (config 5): parity tests with the new library, same-box
# A/B of the lone trace and pipelined frame, WRITE_SIZE per launch of both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/wide; mkdir -p $O
RTAMD_LIB=$R/tools/_exp/lib_wide.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k config5 > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 bash tools/r05_w16ab.sh r05/wide 2 tools/_exp/lib_h0.so tools/_exp/lib_wide.so || exit 1
export TMPDIR=/tmp
for l in h0 wide; do
  (cd /tmp && RTAMD_LIB=$R/tools/_exp/lib_$l.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_$l -o w -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-overlap --no-camera-path --scene world16 --width 3840 --height 2160 --spp 64 > $R/$O/pmc_$l.log 2>&1) || { echo "pmc $l failed"; exit 1; }
  echo "== $l"; python3 tools/pmc_summary.py $O/pmc_$l "trace_kernel<0, true, 692>"
done
