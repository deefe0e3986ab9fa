#!/bin/bash
# bench.py on every BASELINE config at HEAD (one GPU): config 2 (world1 brute force), config 3
# (world8), the headline (world8_stress), config 5 (world16 and world16_tex at 3840x2160, 64 spp).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r04/configs; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-14s ms/frame %.4f  %s %.1f  latency %.3f  trace %s' % (sys.argv[1], d['ms_per_step'], d['unit'], d['value'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $tag; }
run world1_brute --scene world1 --spp 1 --brute --steps 20 --warmup 5
run world8 --scene world8 --spp 8 --steps 20 --warmup 5
run world8_stress --steps 20 --warmup 5
run world16_4k --scene world16 --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2
run world16_tex_4k --scene world16_tex --width 3840 --height 2160 --spp 64 --textures --steps 6 --warmup 2
