#!/bin/bash
# A/B timing of library variants on the bench workload, interleaved A B A B ... so clock
# and thermal drift hit every arm alike.  Usage: tools/ab.sh ROUNDS lib1.so lib2.so ... [-- bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
for r in $(seq 1 $ROUNDS); do
  for L in "${LIBS[@]}"; do
    RTAMD_LIB=$L timeout -k 10 120 python3 "$R/bench.py" --no-cpu-baseline --steps ${AB_STEPS:-20} --warmup 3 --no-camera-path "$@" > /tmp/ab_out.txt 2>&1 || { cat /tmp/ab_out.txt; exit 1; }
    python3 - "$L" <<'PY'
import json, sys
line = [l for l in open('/tmp/ab_out.txt') if l.startswith('{')][-1]
d = json.loads(line)
print("%-40s frame %.4f ms  device-resident %.4f  trace %.4f ms  bvh %.4f  %.1f Mrays/s" % (sys.argv[1].split('/')[-1], d['ms_per_step'], (d.get('device_resident') or {}).get('ms_per_step', float('nan')), d['trace_kernel_ms'], d['bvh_build_ms'], d['value']))
PY
  done
done
