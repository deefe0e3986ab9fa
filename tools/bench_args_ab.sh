#!/bin/bash
# bench.py under several argument sets, interleaved (A B C A B C ...) on one box, so that the
# box's state hits every arm alike.  Usage: tools/bench_args_ab.sh ROUNDS "args A" "args B" ...
# Prints host-readable and device-resident ms per frame and the box's frame copy rate per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG:-args_ab}
mkdir -p $O
ROUNDS=$1; shift
for r in $(seq 1 $ROUNDS); do
  i=0
  for A in "$@"; do
    i=$((i + 1))
    timeout -k 10 150 python3 "$R/bench.py" --no-cpu-baseline --no-camera-path $A > $O/a${i}_$r.json 2> $O/a${i}_$r.err || { tail $O/a${i}_$r.err; exit 1; }
    python3 - $O/a${i}_$r.json "$A" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print("%-40s host-readable %.4f ms  device-resident %.4f ms  copy %.1f GB/s" % (
    sys.argv[2], d['ms_per_step'], (d.get('device_resident') or {}).get('ms_per_step', float('nan')),
    (d.get('copy_engine') or {}).get('GBs', float('nan'))), flush=True)
PY
  done
done
