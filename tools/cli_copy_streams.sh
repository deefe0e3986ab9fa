#!/bin/bash
# Experiment: the CLI's host-readable frames in flight with their copies on one copy stream or
# alternated over two (RT_CLI_COPY_STREAMS), interleaved, world8 and world8_stress, 100 frames.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-cli_cs}
mkdir -p $O
export GPU_MAX_HW_QUEUES=16
C="$R/gpu-ray-tracer_amd/rtracer --width 1920 --height 1080 --spp 8 --in-flight 8 --frames ${FRAMES:-100}"
for i in 1 2 3; do for sc in world8_stress world8; do
  timeout -k 10 60 $C -c $R/scenes/$sc.json > $O/dev.txt 2>&1 || exit 1
  echo "$sc device-resident: $(grep 'In flight' $O/dev.txt)"
  for n in 1 2; do
    RT_CLI_COPY_STREAMS=$n timeout -k 10 60 $C -c $R/scenes/$sc.json --readback > $O/rb.txt 2>&1 || exit 1
    echo "$sc copy streams $n: $(grep 'In flight' $O/rb.txt)"
  done
done; done
