#!/bin/bash
# The timed window's length, interleaved: bench.py at 20 and at 60 steps (the driver's 20 and a
# steady-state window), ROUNDS times, same box; prints the host-readable frame, the
# device-resident frame and the box's frame copy rate of each run.  Usage: tools/steps_ab.sh ROUNDS [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-steps_ab}
mkdir -p $O
ROUNDS=$1; shift
for r in $(seq 1 $ROUNDS); do
  for K in 20 60; do
    timeout -k 10 150 python3 "$R/bench.py" --no-cpu-baseline --steps $K --no-camera-path "$@" > $O/k${K}_$r.json 2> $O/k${K}_$r.err || { tail $O/k${K}_$r.err; exit 1; }
    python3 - $O/k${K}_$r.json $K <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print("steps %3s  host-readable %.4f ms  device-resident %.4f ms  copy %.1f GB/s" % (
    sys.argv[2], d['ms_per_step'], (d.get('device_resident') or {}).get('ms_per_step', float('nan')),
    (d.get('copy_engine') or {}).get('GBs', float('nan'))), flush=True)
PY
  done
done
