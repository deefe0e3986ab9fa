#!/bin/bash
# The CLI's host-readable frames in flight (world8, 1080p 8 spp, 100 frames) under a kernel +
# memory-copy + HIP API trace: when each device-to-host copy was enqueued (hipMemcpyAsync)
# against when its frame's trace kernel ended and when the copy ran (tools/copy_api_lag.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-cli_api}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --output-format csv -d $O/prof -o prof -- $R/gpu-ray-tracer_amd/rtracer --width 1920 --height 1080 --spp 8 --in-flight 8 --frames ${FRAMES:-100} -c $R/scenes/${SCENE:-world8}.json --readback > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
grep "In flight" $O/prof.log
