#!/bin/bash
# Idle frame slots primed at the first frame of a layout (history reset + instance records,
# prime_idle_slots): frames-in-flight parity tests on the new library, same-box A/B of the
# headline at the driver's 20 steps (interleaved) and at 60, and the new library's window trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/prime; mkdir -p $O
RTAMD_LIB=$R/tools/_exp/lib_prime.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_bench_n2.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local tag=$1 l=$2; shift 2; RTAMD_LIB=$R/tools/_exp/lib_$l.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-camera-path "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-16s ms/frame %.4f  latency %.3f  trace %s' % (sys.argv[1], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $tag; }
for i in 1 2 3 4; do
  for l in head prime; do run s20_${l}_$i $l --steps 20 --warmup 5 || exit 1; done
done
for l in head prime; do run s60_${l} $l --steps 60 --warmup 5 || exit 1; done
export TMPDIR=/tmp
(cd /tmp && RTAMD_LIB=$R/tools/_exp/lib_prime.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_prime -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path > $R/$O/kt_prime.log 2>&1) || { echo "kt failed"; exit 1; }
echo "r05_prime done"
