#!/bin/bash
# Frames in flight with each slot's BVH build (RT_PRIO_PRE=1), or its build and sky pre-pass
# (=2), on a high-priority stream: the frames-in-flight parity tests under =2, then a same-box
# A/B of the headline at the driver's 20 steps and at 60, and a kernel trace of =2's window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/prio; mkdir -p $O
RT_PRIO_PRE=2 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_cli.py::test_cli_frames_in_flight tests/test_gpu_bench_n2.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local tag=$1 p=$2; shift 2; RT_PRIO_PRE=$p timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-camera-path "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-12s ms/frame %.4f  latency %.3f  trace %s' % (sys.argv[1], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $tag; }
for i in 1 2 3; do
  for p in 0 1 2; do run s20_p${p}_$i $p --steps 20 --warmup 5 || exit 1; done
done
for p in 0 2; do run s60_p${p} $p --steps 60 --warmup 5 || exit 1; done
export TMPDIR=/tmp
for p in 0 2; do
  (cd /tmp && RT_PRIO_PRE=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_p$p -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path > $R/$O/kt_p$p.log 2>&1) || { echo "kt $p failed"; exit 1; }
done
echo "r05_prio done"
