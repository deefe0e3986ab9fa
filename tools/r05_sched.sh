#!/bin/bash
# AMDGPU machine-scheduler variants of the whole library (Makefile EXTRA): same-box interleaved
# A/B of the headline at the driver's 20 steps; parity of the fastest variant follows separately.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/sched; mkdir -p $O
run() { local tag=$1 l=$2; shift 2; RTAMD_LIB=$R/tools/_exp/lib_$l.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-camera-path "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-16s ms/frame %.4f  latency %.3f  trace %s' % (sys.argv[1], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $tag; }
for i in 1 2 3; do
  for l in head trk itilp bias0; do run s20_${l}_$i $l --steps 20 --warmup 5 || exit 1; done
done
for l in head trk itilp; do run w16_$l $l --scene world16 --width 3840 --height 2160 --spp 64 --steps 4 --warmup 1 || exit 1; done
echo "r05_sched done"
