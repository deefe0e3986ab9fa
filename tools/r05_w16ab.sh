#!/bin/bash
# Same-box A/B of libraries on config 5 (world16 4K 64 spp; world16_tex), interleaved rounds.
# Usage: tools/r05_w16ab.sh TAG ROUNDS lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ROUNDS=$2; shift 2
O=$R/gpurun_out/$TAG; mkdir -p $O
cd "$R" || exit 1
W16="--scene world16 --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2 --no-cpu-baseline --no-camera-path"
for i in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    RTAMD_LIB=$R/$lib timeout -k 10 300 python3 -u bench.py $W16 > $O/w16_${n}_$i.log 2>&1 || { echo "$n failed"; tail -5 $O/w16_${n}_$i.log; exit 1; }
    tail -1 $O/w16_${n}_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-14s round %s ms/frame %.3f  latency %.3f  trace %s' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $n $i
  done
done
