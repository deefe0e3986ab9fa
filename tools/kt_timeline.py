"""Frame timeline of a rocprofv3 --kernel-trace of pipelined frames (tools/pipe_slices.py or
bench.py): per frame the BVH build, sky pre-pass and trace kernel, their durations, the delay
from each frame's build end to its sky / trace start (dispatches waiting for whole free CUs),
and the interval between consecutive trace-kernel starts and ends (the frame rate).

Usage: python tools/kt_timeline.py KERNEL_TRACE_CSV [--last N]"""
import csv
import statistics as stt
import sys


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    for k in ("bvh_build_kernel", "sky_kernel", "trace_kernel", "large_"):
        if k in n:
            return n.split("((")[0].split("(")[0]
    return None


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 60
    rows = []
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r.get("Stream_Id", "0")))
    rows.sort()
    frames, cur = [], {}
    for s, e, k, sid in rows:                          # a frame = build, sky, trace in order on its stream
        kind = "build" if "bvh_build" in k else "sky" if "sky" in k else "trace" if "trace" in k else None
        if kind == "build":
            cur[sid] = {"build": (s, e)}
        elif kind and cur.get(sid) is not None:
            cur[sid][kind] = (s, e)
            if kind == "trace":
                cur[sid]["trace_name"] = k
                frames.append(cur[sid])
                cur[sid] = None
    frames.sort(key=lambda f: f["trace"][0])
    frames = [f for f in frames if "build" in f][-last:]
    if not frames:
        sys.exit("no frames")
    us = lambda a, b: (b - a) / 1e3
    col = lambda f: [f(x) for x in frames if f(x) is not None]
    def stats(name, vals):
        vals = [v for v in vals if v is not None]
        if vals:
            print("%-34s n=%3d  median %8.1f us  mean %8.1f  min %8.1f  max %8.1f" %
                  (name, len(vals), stt.median(vals), stt.mean(vals), min(vals), max(vals)))
    print("trace kernel:", frames[-1]["trace_name"])
    stats("build duration", col(lambda f: us(*f["build"])))
    stats("sky duration", col(lambda f: us(*f["sky"]) if "sky" in f else None))
    stats("trace duration", col(lambda f: us(*f["trace"])))
    stats("build end -> sky start", col(lambda f: us(f["build"][1], f["sky"][0]) if "sky" in f else None))
    stats("sky end -> trace start", col(lambda f: us(f["sky"][1], f["trace"][0]) if "sky" in f else None))
    stats("build start -> trace end (latency)", col(lambda f: us(f["build"][0], f["trace"][1])))
    ts = [f["trace"][0] for f in frames]
    te = [f["trace"][1] for f in frames]
    stats("trace start interval", [us(a, b) for a, b in zip(ts, ts[1:])])
    stats("trace end interval", [us(a, b) for a, b in zip(te, te[1:])])
    conc = []
    for f in frames:                                   # trace kernels resident at this one's start
        conc.append(sum(1 for g in frames if g["trace"][0] <= f["trace"][0] < g["trace"][1]))
    stats("trace kernels resident at a start", conc)
    span = us(frames[0]["build"][0], frames[-1]["trace"][1])
    print("span %.1f us over %d frames: %.1f us per frame" % (span, len(frames), span / len(frames)))


if __name__ == "__main__":
    main()
