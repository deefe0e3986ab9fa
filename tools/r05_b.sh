#!/bin/bash
# Round 5, first GPU pass: the GPU suite on the new library (brute-force kernel M_BRUTE, group
# lane terms recomputed, partial parking M_PART for world16), bench.py's new fields (camera path, CPU median), same-box A/B against
# round 4's library on the headline, config 2 (world1 brute force) and config 5 (world16 4K
# 64 spp), the timed-window profile of the headline and config 2's write traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/b; mkdir -p $O
# gpu tests ran in r05/a: 115 passed
run() { local tag=$1 lib=$2; shift 2; RTAMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-camera-path "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-22s ms/frame %.4f  %.1f  latency %.3f  trace %s' % (sys.argv[1], d['ms_per_step'], d['value'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $tag; }
for i in 1 2 3; do
  for l in r4 r5b; do run w8s_${l}_$i tools/_exp/lib_$l.so --steps 20 --warmup 5; done
done
for i in 1 2; do
  for l in r4 r5b; do run w1b_${l}_$i tools/_exp/lib_$l.so --scene world1 --spp 1 --brute --steps 20 --warmup 5; done
done
for l in r4 r5b; do run w16_${l} tools/_exp/lib_$l.so --scene world16 --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2; done
for l in r4 r5b; do run w16tex_${l} tools/_exp/lib_$l.so --scene world16_tex --textures --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2; done
RT_NO_PART=1 run w16_r5b_nopart tools/_exp/lib_r5b.so --scene world16 --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2
timeout -k 10 500 bash tools/profile_step.sh r05/b/step_w8s > $O/profile_step.log 2>&1 || { echo "profile_step failed"; tail $O/profile_step.log; exit 1; }
QUICK=1 RTAMD_LIB=tools/_exp/lib_r5b.so timeout -k 10 300 bash tools/profile.sh r05/b/prof_w1b --scene world1 --spp 1 --brute > $O/prof_w1b.log 2>&1 || { echo "profile failed"; tail $O/prof_w1b.log; exit 1; }
QUICK=1 RTAMD_LIB=tools/_exp/lib_r5b.so timeout -k 10 400 bash tools/profile.sh r05/b/prof_w16 --scene world16 --width 3840 --height 2160 --spp 64 > $O/prof_w16.log 2>&1 || { echo "profile w16 failed"; tail $O/prof_w16.log; exit 1; }
echo "r05_b done"
