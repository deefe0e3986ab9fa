"""Experiment: consecutive frames on two streams (two scene replicas = two BVH/work/history
slots), so frame k+1 starts on CUs freed by frame k's tail.  Throughput per frame vs serial."""
import os, sys, time, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd

torch.cuda.set_device(0)
rtamd.set_device(0)
p = os.path.join(ROOT, "scenes", "world8_stress.json")
A = rtamd.Scene.load_json(p, 1920, 1080)
B = rtamd.Scene.load_json(p, 1920, 1080)
for n in (1, 8):
    rows = len(range(0, 1080, n))
    bufs = [torch.zeros((rows, 1920), dtype=torch.int32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    kw = dict(spp=8, rebuild_bvh=True, row0=0, row_step=n, compact=True)
    for mode in ("serial", "overlap", "serial", "overlap"):
        def frame(k):
            sc = (A, B)[k % 2] if mode == "overlap" else A
            st = streams[k % 2] if mode == "overlap" else streams[0]
            sc.render_device(rgba_ptr=bufs[k % 2].data_ptr(), stream=st.cuda_stream, **kw)
        for k in range(6):
            frame(k)
        torch.cuda.synchronize()
        K = 40
        t = time.perf_counter()
        for k in range(K):
            frame(k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / K * 1e3
        print(json.dumps({"n": n, "mode": mode, "ms_per_frame": round(ms, 4)}), flush=True)
