#!/bin/bash
# Round 5: LDS-staged in-order sample sums (RT_LDS_SUM) for config 5: parity tests of the
# 64-spp kernels, same-box A/B on world16 / world16_tex 4K 64 spp, write traffic per launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/g; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "config5" > $O/pytest_config5.log 2>&1 || { echo "config5 tests failed"; tail -30 $O/pytest_config5.log; exit 1; }
tail -1 $O/pytest_config5.log
run() { local tag=$1 lib=$2; shift 2; RTAMD_LIB=$R/$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-camera-path "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('%-18s ms/frame %.4f  latency %.3f  trace %s' % (sys.argv[1], d['ms_per_step'], d['frame_latency_ms'], d.get('trace_kernel_ms')))" $tag; }
W16="--scene world16 --width 3840 --height 2160 --spp 64 --steps 6 --warmup 2"
for i in 1 2; do
  for l in ls0 ls1; do run w16_${l}_$i tools/_exp/lib_$l.so $W16; done
done
for l in ls0 ls1; do run w16tex_${l} tools/_exp/lib_$l.so $W16 --textures --scene world16_tex; done
export TMPDIR=/tmp
for l in ls0 ls1; do
  (cd /tmp && RTAMD_LIB=$R/tools/_exp/lib_$l.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_INSTS_LDS SQ_INSTS_VALU --output-format csv -d $R/$O/pmc_w16_$l -o w -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-overlap --no-camera-path $W16 > $R/$O/pmc_w16_$l.log 2>&1) || { echo "pmc $l failed"; exit 1; }
  python3 tools/pmc_summary.py $O/pmc_w16_$l "trace_kernel<0, true, 692>"
done
echo "r05_g done"
