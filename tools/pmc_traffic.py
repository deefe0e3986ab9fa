"""Turn a tools/profile.sh run into profiles/pmc_traffic.json (HBM bytes per trace stage:
the trace kernel plus the sky pre-pass of fast frames)
and a short markdown summary.

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived memory-side (TCC EA) counters in KiB.
Per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half of the bytes of wide
coalesced streaming reads, so the read side is doubled; WRITE_SIZE is calibrated here
against the known frame store (4 B per pixel of RGBA8) -- see `write_calibration`.

Usage: python tools/pmc_traffic.py PROFILE_DIR KEY W ROWS [OUT_JSON]
"""
import collections
import csv
import glob
import json
import os
import sys


def is_timed_trace(name):
    """The frame kernel bench.py times: trace_kernel<NS, LDS, MODE> without the STATS bit
    (the single counted frame bench.py renders first uses MODE 2/3) and without the PROF bit
    (rt_frame_work's untimed profiling frame, MODE bit 6)."""
    if "trace_kernel<" not in name:
        return False
    mode = name.split("trace_kernel<", 1)[1].split(">", 1)[0].split(",")[-1].strip()
    return mode.isdigit() and (int(mode) & 2) == 0 and (int(mode) & 64) == 0


def is_sky(name):
    """The sky pre-pass of the fast frames: part of the trace stage."""
    return "sky_kernel" in name


def stage(root, counter):
    """Per frame of the trace stage: the trace kernel's mean per dispatch plus the sky
    pre-pass's (when the profile has one)."""
    a, n = per_dispatch(root, counter)
    b, _ = per_dispatch(root, counter, is_sky)
    return (None, 0) if a is None else (a + (b or 0.0), n)


def per_dispatch(root, counter, sel=is_timed_trace):
    """Mean per dispatch of the selected kernel that was dispatched most often: bench.py's
    timed frames.  A lone frame of another instantiation (bench.py's untimed frame_work
    pass renders one without partial parking) is not the timed kernel and would skew the
    mean (round 5: one such frame wrote 2.46 GB and tripled world16's write figure)."""
    vals = collections.defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sel(r["Kernel_Name"]) and r["Counter_Name"] == counter:
                vals[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
                names[(f, r["Dispatch_Id"])] = r["Kernel_Name"]
    if not vals:
        return None, 0
    top = collections.Counter(names.values()).most_common(1)[0][0]
    v = [x for k, x in vals.items() if names[k] == top]
    return sum(v) / len(v), len(v)


def kernel_stats(root, sel=is_timed_trace):
    for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sel(r["Name"]):
                return {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                        "max_ns": float(r["MaxNs"])}
    return None


def main():
    root, key, W, rows = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    fetch_kib, nf = stage(root, "FETCH_SIZE")
    write_kib, nw = stage(root, "WRITE_SIZE")
    rdreq, _ = stage(root, "TCC_EA0_RDREQ_sum")
    wrreq, _ = stage(root, "TCC_EA0_WRREQ_sum")
    issue = {c: stage(root, c)[0] for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
                                           "SQ_WAIT_ANY")}
    issue_sky = {c: per_dispatch(root, c, is_sky)[0] for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU")}
    if fetch_kib is None or write_kib is None:
        sys.exit("no FETCH_SIZE/WRITE_SIZE rows for trace_kernel under " + root)
    frame_bytes = 4 * W * rows
    rd = 2.0 * fetch_kib * 1024.0                      # gfx950: FETCH_SIZE counts half of wide reads
    wr = write_kib * 1024.0
    entry = {
        "hbm_bytes_per_launch": int(rd + wr),
        "read_bytes_per_launch": int(rd), "write_bytes_per_launch": int(wr),
        "raw": {"FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib, "dispatches": [nf, nw],
                "TCC_EA0_RDREQ": rdreq, "TCC_EA0_WRREQ": wrreq},
        "write_calibration": {"frame_store_bytes": frame_bytes, "write_over_frame": wr / frame_bytes},
        "kernel_trace": kernel_stats(root),
        "kernel_trace_sky": kernel_stats(root, is_sky),
        # per frame: trace kernel + sky pre-pass (the trace stage bench.py's events span)
        "stage": "sky_kernel + trace_kernel",
        # wave-level instruction counts per launch (secondary bound: VALU issue, bench.py)
        "issue": {k: v for k, v in issue.items() if v is not None},
        "issue_sky_kernel": {k: v for k, v in issue_sky.items() if v is not None},
        "source": os.path.relpath(root),
    }
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = entry
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


if __name__ == "__main__":
    main()
