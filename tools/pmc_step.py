"""Counters of bench.py's timed window: the kernels dispatched between
bench.py's two profile markers (rt_profile_marker tags 1 and 2, an empty kernel of 64 x tag
threads) in a rocprofv3 run of bench.py's own command, summed and divided by the timed steps.

  * PMC passes (one counter group per run, tools/profile_step.sh): each counter summed over
    every dispatch of the window, per step = sum / steps.  rocprofv3 serialises dispatches
    while it collects counters, so counts and bytes are the work's (VALU instructions, HBM
    bytes), not the overlap's.  HBM bytes = FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md
    §HBM: gfx950's FETCH_SIZE counts half of wide reads).
  * The kernel-trace pass (no counters, frames in flight as timed): GPU busy time per step =
    the union of the window's dispatch intervals / steps (<= ms_per_step by construction), and
    the summed per-kernel durations (> busy when frames overlap).

Usage: python tools/pmc_step.py PROFILE_DIR KEY STEPS [OUT_JSON]  (KEY as bench.py's
"%(scene)s_%(W)dx%(H)d_spp%(spp)d_n%(N)d")."""
import collections
import csv
import glob
import json
import os
import sys


def marker_tag(name, threads):
    return int(threads) // 64 if "profile_marker_kernel" in name else 0


def window_rows(rows, did, name, threads):
    """Rows whose dispatch lies strictly between the last tag-1 marker and the tag-2 marker after it."""
    rows = sorted(rows, key=lambda r: int(r[did]))
    lo = hi = None
    for r in rows:
        t = marker_tag(r[name], r[threads])
        if t == 1:
            lo, hi = int(r[did]), None
        elif t == 2 and lo is not None and hi is None:
            hi = int(r[did])
    if lo is None or hi is None:
        return None
    return [r for r in rows if lo < int(r[did]) < hi]


def counters(root):
    """{counter: summed value over the window's dispatches} from every counter_collection.csv."""
    out, nd = {}, {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        w = window_rows(rows, "Dispatch_Id", "Kernel_Name", "Grid_Size")
        if w is None:
            continue
        per = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in w:
            per[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for k, v in per.items():
            out[k] = v
            nd[k] = len(disp[k])
    return out, nd


def busy(root):
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        w = window_rows(rows, "Dispatch_Id", "Kernel_Name", "Grid_Size_X")
        if not w:
            continue
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in w)
        tot, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        tot += ce - cs
        by = collections.defaultdict(lambda: [0, 0])
        for r in w:
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            by[n][0] += 1
            by[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        return {"busy_ns": tot, "span_ns": max(e for _, e in iv) - iv[0][0], "dispatches": len(w),
                "kernels": {k: {"calls": c, "sum_ns": t} for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])}}
    return None


def main():
    root, key, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_step.json")
    c, nd = counters(root)
    # busy time from the kernel-trace pass only (the PMC passes' traces are serialised)
    b = busy(os.path.join(root, "kt") if os.path.isdir(os.path.join(root, "kt")) else root)
    if not c and not b:
        sys.exit("no marker-delimited window under " + root)
    ps = {k: v / steps for k, v in c.items()}
    entry = {"steps": steps, "per_step": ps, "dispatches_in_window": nd, "source": os.path.relpath(root)}
    if "FETCH_SIZE" in ps and "WRITE_SIZE" in ps:
        rd, wr = 2.0 * ps["FETCH_SIZE"] * 1024.0, ps["WRITE_SIZE"] * 1024.0
        entry.update(hbm_bytes_per_step=int(rd + wr), read_bytes_per_step=int(rd), write_bytes_per_step=int(wr))
    kt_log = os.path.join(root, "kt.log")                 # the kernel-trace pass's own bench line
    if os.path.exists(kt_log):
        for line in open(kt_log):
            if line.startswith("{") and '"ms_per_step"' in line:
                d = json.loads(line)
                entry["profiled_ms_per_step"] = d["ms_per_step"]
                # the kind of window profiled: bench.py flags per_step figures from another kind
                entry["window"] = {
                    "grid_timed_frames": d.get("config", {}).get("grid_timed_frames"),
                    "frames_in_flight": d.get("frames_in_flight"),
                    "timed_to": d.get("pmc_window", "device") if d.get("frames_in_flight", 1) > 1 else "serial",
                    "lib_sha16": d.get("build", {}).get("lib_sha16")}
    if b:
        entry["gpu_busy_ms_per_step"] = b["busy_ns"] / steps / 1e6
        entry["window_span_ms"] = b["span_ns"] / 1e6
        entry["kernel_ms_per_step"] = {k: round(v["sum_ns"] / steps / 1e6, 4) for k, v in b["kernels"].items()}
        entry["kernel_calls"] = {k: v["calls"] for k, v in b["kernels"].items()}
    try:
        db = json.load(open(out))
    except (OSError, ValueError):
        db = {}
    db[key] = entry
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


if __name__ == "__main__":
    main()
