"""What the fast kernels do per rank for an N-way row-cyclic split (rt_frame_work): closest-hit
queries, wave-level query steps, child-pair steps and leaf visits, against the whole frame's.
Shows how much packet coherence the row-cyclic groups lose.  Usage: python tools/slice_work.py"""
import json, os, sys
import torch  # noqa: F401  (HIP runtime first)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd
S = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", "world8_stress.json"), 1920, 1080)
full = S.frame_work(spp=8)
print(json.dumps({"n": 1, **full}))
for n in (2, 4, 8):
    tot = {k: ([0] * len(v) if isinstance(v, list) else 0) for k, v in full.items()}
    for r in range(n):
        w = S.frame_work(spp=8, row0=r, row_step=n)
        for k in w:
            tot[k] = [a + b for a, b in zip(tot[k], w[k])] if isinstance(w[k], list) else tot[k] + w[k]
    print(json.dumps({"n": n, **{k: v for k, v in tot.items()},
                      "ratio_to_full": {k: round(tot[k] / max(1, full[k]), 3) for k in full
                                       if k != "scene_bytes" and not isinstance(full[k], list)}}))
