#!/bin/bash
# Round 5: run-preserving ticket scramble (RT_RUN_LOG 0 = round 4's full scramble, 3, 5):
# same-box A/B on the headline (driver settings, 3 interleaved rounds) and config 5, then the
# trace stage's WRITE_SIZE per launch for 0 and 5 (lone serial frames).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/d; mkdir -p $O
run() { local tag=$1 lib=$2; shift 2; RTAMD_LIB=$R/$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-18s ms/frame %.4f  latency %.3f  trace %s  camera_path %s' % (sys.argv[1], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms'), (d.get('camera_path') or {}).get('ms_per_step')))" $tag; }
for i in 1 2 3; do
  for l in run0 run3 run5; do run w8s_${l}_$i tools/_exp/lib_$l.so --steps 20 --warmup 5; done
done
for l in run0 run5; do run w16_${l} tools/_exp/lib_$l.so --no-camera-path --scene world16 --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2; done
export TMPDIR=/tmp
for l in run0 run5; do
  for cfg in "w8s:" "w16:--scene world16 --width 3840 --height 2160 --spp 64"; do
    t=${cfg%%:*}; a=${cfg#*:}
    (cd /tmp && RTAMD_LIB=$R/tools/_exp/lib_$l.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_${t}_$l -o w -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-overlap --no-camera-path $a > $R/$O/pmc_${t}_$l.log 2>&1) || { echo "pmc $t $l failed"; exit 1; }
    python3 tools/pmc_summary.py $O/pmc_${t}_$l "" | grep -A1 "trace_kernel<0\|sky" | grep -v "^--"
  done
done
echo "r05_d done"
