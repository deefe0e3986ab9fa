"""Per-rank frame time of the N-GPU row-cyclic split, measured on ONE GPU.

For each N, renders the slices of ranks 0 and N-1 (rows y = r, r+N, ... as bench.py's
rank r does) with the same per-frame BVH rebuild and event timing, so the render side
of bench.py --gpus N can be predicted before the driver's 8-GPU run (the RCCL gather is
not included).  Usage: python tools/slice_bench.py [--scene S] [--steps K] [--ns 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="world8_stress")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=8)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--ns", default="1,2,4,8")
    a = p.parse_args()
    torch.cuda.set_device(0)
    rtamd.set_device(0)
    scene = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", a.scene + ".json"), a.width, a.height)
    W, H = scene.width, scene.height
    stream = torch.cuda.current_stream()
    for n in [int(x) for x in a.ns.split(",")]:
        for r in sorted({0, n - 1}):
            rows = len(range(r, H, n))
            buf = torch.zeros((rows, W), dtype=torch.int32, device="cuda")
            kw = dict(spp=a.spp, rebuild_bvh=True, row0=r, row_step=n, compact=True, rgba_ptr=buf.data_ptr(),
                      stream=stream.cuda_stream)
            st = scene.render_device(sync=True, stats=True, **kw)
            for _ in range(4):                                  # warm-up + scheduling history
                scene.render_device(**kw)
            scene.timing_collect()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                scene.render_device(timing=True, **kw)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            tm = scene.timing_collect()
            f = max(1, tm["frames"])
            print(json.dumps({"n": n, "rank": r, "rows": rows, "frame_ms": round(ms, 4),
                              "trace_ms": round(tm["trace_ms_total"] / f, 4), "bvh_ms": round(tm["bvh_ms_total"] / f, 4),
                              "rays": st["rays"], "mrays_s_rank": round(st["rays"] / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
