"""Per-kernel durations from a rocprofv3 rocpd database (the default output format):
python3 tools/rocpd_summary.py DIR/...db [name filter]"""
import collections, re, sqlite3, sys
c = sqlite3.connect(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
meta = {}
for name, st, en, vg, sg, grid, wg in c.execute("select name, start, end, vgpr_count, sgpr_count, grid_x, workgroup_x from kernels"):
    if pat in name:
        m = re.search(r"([A-Za-z_]\w*(?:<[^()]*>)?)\(", name.replace("(anonymous namespace)::", ""))
        k = (m.group(1) if m else name)[:60]
        d[k].append((en - st) / 1e3)
        meta[k] = (vg, sg, grid, wg)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("%-60s n=%4d avg %9.1f us  min %9.1f  vgpr %s sgpr %s grid %s wg %s" % ((k, len(v), sum(v) / len(v), min(v)) + meta[k]))
