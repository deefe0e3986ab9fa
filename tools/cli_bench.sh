#!/bin/bash
# The reference's own benchmark (main.cc:210-216: "Time: X ms" for the first update_scene after
# the scene is made) through the CLI's -b, world8_stress at 1920x1080, 1 spp (update_scene) and
# 8 spp (the build extension), three fresh processes each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-cli_b}
mkdir -p $O
: > $O/cli_b.log
for spp in 1 8; do for i in 1 2 3; do
  echo "== rtracer -c scenes/world8_stress.json --width 1920 --height 1080 --spp $spp -b (run $i)" >> $O/cli_b.log
  timeout -k 10 60 $R/gpu-ray-tracer_amd/rtracer -c $R/scenes/world8_stress.json --width 1920 --height 1080 --spp $spp -b >> $O/cli_b.log 2>&1 || { tail $O/cli_b.log; exit 1; }
done; done
grep -E "==|Time" $O/cli_b.log
