#!/bin/bash
# Brute-force sky pre-pass: its parity tests, then config 2 (world1 1080p brute force) with and
# without it (RT_NO_BRUTE_SKY), interleaved rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/bsky; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_render.py -k "brute or frame_parity or update_scene or sky_prepass or spp8_sky" tests/test_gpu_fullsize.py::test_world1_1080p_brute_force > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in on off; do
    if [ $v = off ]; then export RT_NO_BRUTE_SKY=1; else unset RT_NO_BRUTE_SKY; fi
    timeout -k 10 200 python3 -u bench.py --scene world1 --spp 1 --brute --steps 20 --warmup 5 --no-cpu-baseline --no-camera-path > $O/w1b_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/w1b_${v}_$i.log; exit 1; }
    tail -1 $O/w1b_${v}_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('brute sky %-3s round %s ms/frame %.4f latency %.4f trace %s' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $v $i
  done
done
unset RT_NO_BRUTE_SKY
