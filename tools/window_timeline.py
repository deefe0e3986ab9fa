#!/usr/bin/env python3
"""Timeline of the last F frames of a kernel + memory-copy trace (rocprofv3 csv, e.g.
tools/cli_window_trace.sh): per frame the BVH build, sky pre-pass and trace kernels and the
host copy (start / end in us from the window's first build), then where the window's time goes:
the fill (first frame's build to its trace's end), the spacing of frame completions, the last
frame's tail and the copies' drain after the last trace.  Usage: window_timeline.py DIR F"""
import csv
import glob
import os
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    assert f, (d, pat)
    return list(csv.DictReader(open(f[0])))


def main():
    d, F = sys.argv[1], int(sys.argv[2])
    kt = load(d, "*kernel_trace.csv")
    ks = {}
    for r in kt:
        n = r["Kernel_Name"]
        key = "build" if "bvh_build_kernel" in n else "sky" if "sky_kernel" in n else "trace" if "trace_kernel" in n else None
        if key:
            ks.setdefault(key, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for k in ks:
        ks[k].sort()
        ks[k] = ks[k][-F:]
    try:
        mc = [r for r in load(d, "*memory_copy_trace.csv") if r["Direction"].endswith("DEVICE_TO_HOST")]
        cp = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in mc)[-F:]
        if len(cp) < F or cp[0][0] < ks["build"][0][0]:     # no per-frame copies in this window
            cp = []
    except AssertionError:
        cp = []
    t0 = ks["build"][0][0]
    us = lambda t: (t - t0) / 1e3
    print("frame   build            sky              trace             copy")
    for i in range(F):
        b, s, t = ks["build"][i], ks["sky"][i], ks["trace"][i]
        c = cp[i] if len(cp) == F else None
        print("%3d  %7.1f-%7.1f  %7.1f-%7.1f  %7.1f-%7.1f  %s" % (
            i, us(b[0]), us(b[1]), us(s[0]), us(s[1]), us(t[0]), us(t[1]),
            "%7.1f-%7.1f" % (us(c[0]), us(c[1])) if c else "-"))
    ends = sorted(t[1] for t in ks["trace"])
    gaps = [(ends[i + 1] - ends[i]) / 1e3 for i in range(F - 1)]
    last_trace = us(ends[-1])
    last = max(last_trace, us(max(c[1] for c in cp)) if cp else 0)
    print("window (first build -> last trace end): %.1f us = %.4f ms per frame" % (last_trace, last_trace / 1e3 / F))
    if cp:
        print("window (first build -> last copy end): %.1f us = %.4f ms per frame" % (last, last / 1e3 / F))
    print("first frame's trace ends at %.1f us; trace ends spaced (us): %s" % (us(ends[0]), " ".join("%.0f" % g for g in gaps)))
    mid = sorted(gaps[2:-2]) if F > 6 else sorted(gaps)
    print("median spacing %.1f us; %d frames x median = %.1f us" % (mid[len(mid) // 2], F, F * mid[len(mid) // 2]))
    if cp:
        print("copies after the last trace end: %d, drain %.1f us" % (sum(1 for c in cp if c[1] > ends[-1]), last - last_trace))
        # a copy can start once its frame's trace has ended and the previous copy is done
        # (one copy stream): the rest of the wait is the host's (event wait, enqueue) or the engine's
        late, lag = [], []
        for i in range(F):
            ready = max(ks["trace"][i][1], cp[i - 1][1] if i else 0)
            late.append((cp[i][0] - ready) / 1e3)
            lag.append((cp[i][1] - ks["trace"][i][1]) / 1e3)
        sl = sorted(late)
        print("copy start after it could start (us): median %.1f, p90 %.1f, max %.1f; frame end -> copy end: median %.1f, max %.1f"
              % (sl[F // 2], sl[int(F * 0.9)], sl[-1], sorted(lag)[F // 2], max(lag)))


if __name__ == "__main__":
    main()
