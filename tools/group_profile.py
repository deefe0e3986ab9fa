"""Per-group durations of the fast frame kernel (rt_profile_groups; profiling aid).

For a slice (rows y = row0 + i*row_step, as bench.py's rank row0 of row_step renders
them) prints the group-duration distribution, the heaviest groups with their pixels,
and the critical-path bound they set; saves the durations as .npy under gpurun_out/.
Usage: python tools/group_profile.py [--scene S] [--slices 1:0,8:0,8:4]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (binds the HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="world8_stress")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=8)
    p.add_argument("--slices", default="1:0,8:0,8:4", help="row_step:row0 pairs")
    p.add_argument("--top", type=int, default=12)
    p.add_argument("--prof", action="store_true", help="PROF kernel: wave step counts per group (timing perturbed)")
    a = p.parse_args()
    L = rtamd.lib()
    L.rt_profile_groups.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    rtamd.set_device(0)
    s = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", a.scene + ".json"), a.width, a.height)
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    for sl in a.slices.split(","):
        step, row0 = (int(x) for x in sl.split(":"))
        cap = 13 * a.width * a.height
        buf = np.zeros(cap, np.uint32)
        geo = np.zeros(4, np.int32)
        ms = ctypes.c_double()
        rtamd._check(L.rt_profile_groups(s._h, a.spp, row0, step, 4, int(a.prof), buf.ctypes.data, cap, geo.ctypes.data,
                                         ctypes.byref(ms)))
        ng, gw, gh, ngx = (int(x) for x in geo)
        d = buf[:ng].astype(np.float64) / 1e5                  # ms
        cnt = buf[ng:13 * ng].reshape(ng, 12) if a.prof else None
        np.save(os.path.join(out_dir, "groups_%s_%d_%d%s.npy" % (a.scene, step, row0, "_prof" if a.prof else "")),
                buf[:13 * ng] if a.prof else buf[:ng])
        order = np.argsort(-d)
        top = []
        for g in order[:a.top]:
            gx, gy = int(g) % ngx, int(g) // ngx
            top.append({"g": int(g), "ms": round(float(d[g]), 4), "x": [gx * gw, gx * gw + gw - 1],
                        "y": [row0 + gy * gh * step, row0 + (gy * gh + gh - 1) * step]})
            if cnt is not None:
                top[-1]["queries_pairs_leaves_tris"] = [int(x) for x in cnt[g][:4]]
                top[-1]["kcyc_query_leaf_sample_post_group_light_normal_park"] = [round(int(x) / 1e3, 1) for x in cnt[g][4:]]
        print(json.dumps({"scene": a.scene, "row_step": step, "row0": row0, "kernel_ms": round(ms.value, 4),
                          "n_groups": ng, "group": [gw, gh], "sum_ms": round(float(d.sum()), 2),
                          "mean_ms": round(float(d.mean()), 5), "p50": round(float(np.percentile(d, 50)), 5),
                          "p99": round(float(np.percentile(d, 99)), 4), "p999": round(float(np.percentile(d, 99.9)), 4),
                          "max_ms": round(float(d.max()), 4), "n_over_0.1ms": int((d > 0.1).sum()),
                          "n_over_0.3ms": int((d > 0.3).sum()),
                          "mean_steps": [round(float(x), 1) for x in cnt[:, :4].mean(0)] if cnt is not None else None,
                          "cycle_split_all_groups": ([round(float(cnt[:, k].sum() / max(1, cnt[:, 8].sum())), 3) for k in (4, 5, 6, 7)]
                                                     if cnt is not None else None),
                          # live groups: more than one wave query (a sky group's one query misses)
                          "live_groups": int((cnt[:, 0] > 1).sum()) if cnt is not None else None,
                          "live_mean_steps": ([round(float(x), 2) for x in cnt[cnt[:, 0] > 1][:, :4].mean(0)]
                                              if cnt is not None else None),
                          "live_mean_kcyc_query_leaf_sample_post_group_light_normal_park": (
                              [round(float(x) / 1e3, 1) for x in cnt[cnt[:, 0] > 1][:, 4:].mean(0)] if cnt is not None else None),
                          "cycle_split_live_groups": ([round(float(cnt[cnt[:, 0] > 1][:, k].sum() / max(1, cnt[cnt[:, 0] > 1][:, 8].sum())), 3)
                                                       for k in (4, 5, 6, 7, 9, 10, 11)] if cnt is not None else None),
                          "top": top}), flush=True)


if __name__ == "__main__":
    main()
