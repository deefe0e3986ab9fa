"""Experiment: frames in flight = 1, 2, 3 (scene replicas on separate streams)."""
import os, sys, time, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd
torch.cuda.set_device(0); rtamd.set_device(0)
p = os.path.join(ROOT, "scenes", "world8_stress.json")
S = [rtamd.Scene.load_json(p, 1920, 1080) for _ in range(3)]
for n in (1, 8):
    rows = len(range(0, 1080, n))
    bufs = [torch.zeros((rows, 1920), dtype=torch.int32, device="cuda") for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    kw = dict(spp=8, rebuild_bvh=True, row0=0, row_step=n, compact=True)
    for depth in (1, 2, 3, 1, 2, 3):
        def frame(k):
            i = k % depth
            S[i].render_device(rgba_ptr=bufs[i].data_ptr(), stream=streams[i].cuda_stream, **kw)
        for k in range(6): frame(k)
        torch.cuda.synchronize()
        K = 60
        t = time.perf_counter()
        for k in range(K): frame(k)
        torch.cuda.synchronize()
        print(json.dumps({"n": n, "depth": depth, "ms_per_frame": round((time.perf_counter() - t) / K * 1e3, 4)}), flush=True)
