"""Per-rank frame throughput of an N-way row-cyclic slice with frames in flight, on one GPU
(the render side of bench.py --gpus N; no gather).  NS / DEPTHS / RT_BENCH_HW_QUEUES env vars."""
import os, sys, time, json
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_BENCH_HW_QUEUES", "16")
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd, rtamd.dist as rtdist
torch.cuda.set_device(0); rtamd.set_device(0)
p = os.path.join(ROOT, "scenes", "world8_stress.json")
S = rtamd.Scene.load_json(p, 1920, 1080)
# one set of render streams for every configuration: streams drawn later from torch's pool can
# share a hardware queue, which serialises two frames in flight
streams = [torch.cuda.Stream() for _ in range(max(int(x) for x in os.environ.get("DEPTHS", "1,2,4").split(",")))]
for n in [int(x) for x in os.environ.get("NS", "1,2,4,8").split(",")]:
    rows = len(range(0, 1080, n))
    for depth in [int(x) for x in os.environ.get("DEPTHS", "1,2,4").split(",")]:
        S.set_frame_slots(depth)
        pipe = rtdist.FramePipeline(1920, rows, 1, 0, "cuda", depth=depth, streams=streams)
        def frame(k):
            pipe.step(k, lambda buf, st: S.render_device(spp=8, rebuild_bvh=os.environ.get("REBUILD", "1") == "1", row0=0, row_step=n, compact=True,
                                                         rgba_ptr=buf.data_ptr(), stream=st.cuda_stream))
        for k in range(8): frame(k)
        pipe.finish(); torch.cuda.synchronize()
        K = 60
        t = time.perf_counter()
        for k in range(K): frame(k)
        pipe.finish(); torch.cuda.synchronize()
        print(json.dumps({"n": n, "depth": depth, "ms_per_frame": round((time.perf_counter() - t) / K * 1e3, 4)}), flush=True)
