"""Latency of the drop-in call: rt_update_scene (raytracer.cu:102-120 -- BVH rebuild, one frame
at the reference's 1 spp, synchronous, frame copied into the host canvas), world8_stress at
1920x1080 by default.  Usage: python tools/update_scene_time.py [scene] [W] [H] [calls]"""
import json, os, sys, time
import torch  # noqa: F401  (binds the HIP runtime first)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd
scene = sys.argv[1] if len(sys.argv) > 1 else "world8_stress"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
n = int(sys.argv[4]) if len(sys.argv) > 4 else 40
rtamd.set_device(0)
s = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", scene + ".json"), W, H)
for _ in range(5):
    s.update_scene()
ts = []
for _ in range(n):
    t = time.perf_counter()
    s.update_scene()
    ts.append(time.perf_counter() - t)
ts.sort()
print(json.dumps({"scene": scene, "W": W, "H": H, "calls": n, "median_ms": round(ts[n // 2] * 1e3, 4),
                  "min_ms": round(ts[0] * 1e3, 4), "lib": os.path.basename(rtamd.LIB_PATH)}), flush=True)
