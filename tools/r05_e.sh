#!/bin/bash
# Round 5: next-node prefetch in the traversal (RT_PREFETCH 0/1), same-box A/B at the driver's
# settings (static camera and the moving-camera figure), 4 interleaved rounds; then the
# heavy-first history off (RT_HEAVY_Q=0) against on, static and moving camera.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/${TAG:-e}; mkdir -p $O
run() { local tag=$1 lib=$2; shift 2; RTAMD_LIB=$R/$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-18s ms/frame %.4f  latency %.3f  trace %s  camera_path %s' % (sys.argv[1], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms'), (d.get('camera_path') or {}).get('ms_per_step')))" $tag; }
for i in 1 2 3 4; do
  for l in ${LIBS:-pf0 pf1}; do run w8s_${l}_$i tools/_exp/lib_$l.so --steps 20 --warmup 5; done
done
if [ -n "$HEAVY" ]; then
for i in 1 2; do
  for q in 0 6; do RT_HEAVY_Q=$q run w8s_q${q}_$i tools/_exp/lib_$HEAVY.so --steps 20 --warmup 5; done
done
fi
echo "done"
