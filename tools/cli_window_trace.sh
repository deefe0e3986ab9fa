#!/bin/bash
# The driver's 20-frame window as the CLI runs it (C ABI only: outside torch the host copies
# stay on the copy engines under the profiler), under a kernel + memory-copy trace: per frame
# the build / sky / trace kernels and the host copy, for tools/window_timeline.py.
# world8_stress 1920x1080 8 spp, 8 in flight, host-readable and device-resident.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-cli_window}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
C="$R/gpu-ray-tracer_amd/rtracer --width 1920 --height 1080 --spp 8 --in-flight 8 --frames ${FRAMES:-20} -c $R/scenes/${SCENE:-world8_stress}.json"
for m in readback device; do
  a=""; [ $m == readback ] && a="--readback"
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/$m -o $m -- $C $a > $O/$m.log 2>&1 || { tail $O/$m.log; exit 1; }
  grep "In flight" $O/$m.log
done
