"""Experiment: depth-d frames in flight, scene replicas vs one scene with d frame slots."""
import os, sys, time, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd
torch.cuda.set_device(0); rtamd.set_device(0)
p = os.path.join(ROOT, "scenes", "world8_stress.json")
R = [rtamd.Scene.load_json(p, 1920, 1080) for _ in range(3)]
S1 = rtamd.Scene.load_json(p, 1920, 1080)
bufs = [torch.zeros((1080, 1920), dtype=torch.int32, device="cuda") for _ in range(3)]
streams = [torch.cuda.Stream() for _ in range(3)]
kw = dict(spp=8, rebuild_bvh=True, compact=True)
import rtamd.dist as rtdist
pipes = {d: rtdist.FramePipeline(1920, 1080, 1, 0, "cuda", depth=d) for d in (2, 3)}
for mode, depth in (("slots", 3), ("pipe", 3), ("pipe_timed", 3), ("slots", 2), ("pipe", 2), ("slots", 3), ("pipe", 3)):
    if mode != "replicas":
        S1.set_frame_slots(depth)
    def frame(k):
        if mode.startswith("pipe"):
            pipes[depth].step(k, lambda buf, st: S1.render_device(rgba_ptr=buf.data_ptr(), stream=st.cuda_stream,
                                                                timing=mode == "pipe_timed", **kw))
            return
        i = k % depth
        sc = R[i] if mode == "replicas" else S1
        sc.render_device(rgba_ptr=bufs[i].data_ptr(), stream=streams[i].cuda_stream, **kw)
    for k in range(6): frame(k)
    torch.cuda.synchronize()
    K = 60
    t = time.perf_counter()
    for k in range(K): frame(k)
    if mode.startswith("pipe"): pipes[depth].finish()
    torch.cuda.synchronize()
    if mode == "pipe_timed": S1.timing_collect()
    print(json.dumps({"mode": mode, "depth": depth, "ms_per_frame": round((time.perf_counter() - t) / K * 1e3, 4)}), flush=True)
