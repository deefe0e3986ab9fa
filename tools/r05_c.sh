#!/bin/bash
# Round 5: write traffic of config 2 (world1 brute force, M_BRUTE) and config 5 (world16 4K 64 spp,
# partial parking M_PART and without it), lone serial frames (tools/profile.sh QUICK).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r05/c; mkdir -p $O
QUICK=1 timeout -k 10 300 bash tools/profile.sh r05/c/prof_w1b --scene world1 --spp 1 --brute > $O/prof_w1b.log 2>&1 || { echo "profile w1b failed"; tail $O/prof_w1b.log; exit 1; }
QUICK=1 timeout -k 10 400 bash tools/profile.sh r05/c/prof_w16 --scene world16 --width 3840 --height 2160 --spp 64 > $O/prof_w16.log 2>&1 || { echo "profile w16 failed"; tail $O/prof_w16.log; exit 1; }
RT_NO_PART=1 QUICK=1 timeout -k 10 400 bash tools/profile.sh r05/c/prof_w16_nopart --scene world16 --width 3840 --height 2160 --spp 64 > $O/prof_w16_nopart.log 2>&1 || { echo "profile w16 nopart failed"; tail $O/prof_w16_nopart.log; exit 1; }
echo "r05_c done"
