#!/usr/bin/env python3
"""From a kernel + memory-copy + HIP API trace (tools/cli_api_trace.sh): for each
device-to-host copy, when the host enqueued it (hipMemcpyAsync, by correlation id) against when
the copy engine started it, and how many trace kernels had ended before the enqueue but had no
copy enqueued yet (frames waiting for the host).  Usage: copy_api_lag.py DIR [LAST_N]"""
import csv
import glob
import os
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    api = {r["Correlation_Id"]: r for r in load(d, "*hip_api_trace.csv")}
    mc = sorted((r for r in load(d, "*memory_copy_trace.csv") if r["Direction"].endswith("DEVICE_TO_HOST")),
                key=lambda r: int(r["Start_Timestamp"]))[-n:]
    ends = sorted(int(r["End_Timestamp"]) for r in load(d, "*kernel_trace.csv") if "trace_kernel" in r["Kernel_Name"])
    lag, wait_q, dur = [], [], []
    for i, r in enumerate(mc):
        a = api.get(r["Correlation_Id"])
        if a is None:
            continue
        t_api = int(a["Start_Timestamp"])
        lag.append((int(r["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
        dur.append((int(a["End_Timestamp"]) - t_api) / 1e3)
        # frames finished before this enqueue whose copies were not enqueued before it
        done = sum(1 for e in ends if e < t_api)
        enq = sum(1 for q in mc[:i] if q["Correlation_Id"] in api and int(api[q["Correlation_Id"]]["Start_Timestamp"]) < t_api)
        wait_q.append(done - enq - (len(ends) - n - 0))
    s = lambda v: "median %.1f, p10 %.1f, p90 %.1f, max %.1f" % (sorted(v)[len(v) // 2], sorted(v)[len(v) // 10],
                                                              sorted(v)[int(len(v) * 0.9)], max(v))
    print("copies with an API record: %d of %d" % (len(lag), len(mc)))
    print("hipMemcpyAsync return -> copy start (us): " + s(lag))
    print("hipMemcpyAsync call duration (us): " + s(dur))
    fn = {}
    for r in api.values():
        fn.setdefault(r["Function"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(fn.items(), key=lambda x: -sum(x[1]))[:10]:
        print("  %-32s calls %5d  total %8.1f us  median %.1f us  max %.1f us" % (k, len(v), sum(v), sorted(v)[len(v) // 2], max(v)))


if __name__ == "__main__":
    main()
