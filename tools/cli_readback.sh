#!/bin/bash
# The CLI's frames in flight (C ABI only, no torch), device-resident and host-readable
# (--readback), world8_stress and world8 at 1920x1080 8 spp; then the host-readable run under a
# kernel + memory-copy trace (outside torch the copies stay on the copy engines under the profiler).
# Grid policies stream (the CLI's default) and half.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-cli_rb}
mkdir -p $O
C="$R/gpu-ray-tracer_amd/rtracer --width 1920 --height 1080 --spp 8 --in-flight 8 --frames ${FRAMES:-100}"
: > $O/cli_rb.log
for i in 1 2; do for sc in world8_stress world8; do for ov in stream half; do for m in "" "--readback"; do
  echo "== $sc --overlap $ov $m (run $i)" >> $O/cli_rb.log
  timeout -k 10 60 $C -c $R/scenes/$sc.json --overlap $ov $m >> $O/cli_rb.log 2>&1 || { tail $O/cli_rb.log; exit 1; }
done; done; done; done
grep -E "==|In flight" $O/cli_rb.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o prof -- $C -c $R/scenes/world8.json --readback > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
echo done
