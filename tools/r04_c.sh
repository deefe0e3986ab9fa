#!/bin/bash
# Round 4, config 5: 768-thread unparked kernels (RT_B768=1, default) vs the 1024-thread spilling
# ones (RT_B768=0) on world16 / world16_tex at 3840x2160, 64 spp; config-5 parity tests; the CLI's
# frames in flight (single device and 8 virtual ranks).
set -o pipefail
mkdir -p gpurun_out/r04/ab_b768
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k config5 > gpurun_out/r04/pytest_config5.log 2>&1 || { echo "config5 tests failed"; exit 1; }
for i in 1 2; do
  for v in 0 1; do
    for sc in world16 world16_tex; do
      t=""; [ $sc = world16_tex ] && t="--textures"
      RT_B768=$v timeout -k 10 200 python3 bench.py --scene $sc --width 3840 --height 2160 --spp 64 --steps 5 --warmup 2 --no-cpu-baseline $t > gpurun_out/r04/ab_b768/${sc}_b${v}_$i.log 2>&1 || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'frame_ms %.3f trace %.3f Grays/s %.2f' % (d['frame_ms'], d['trace_kernel_ms'], d['value']/1e3))" gpurun_out/r04/ab_b768/${sc}_b${v}_$i.log "$sc RT_B768=$v round $i"
    done
  done
done
for a in "--gpus 1 --ranks 8 --in-flight 8" "--gpus 1 --ranks 8 --in-flight 1" "--in-flight 8" "--in-flight 1"; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 ./gpu-ray-tracer_amd/rtracer -c scenes/world8_stress.json --width 1920 --height 1080 --spp 8 --frames 100 $a 2>&1 | grep "ms/frame"
done
echo "r04_c done"
