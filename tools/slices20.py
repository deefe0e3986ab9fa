"""Per-rank slice pipelines at the driver's 20 timed frames (bench.py's render side of --gpus N on
one GPU, no gather): grid policy `stream` against `stream` with the last 1 / 2 / 4 / 8 frames on every CU
(bench.py --grid stream-last-full: the last one).  NS / ROUNDS / POLICIES env vars; one JSON line
per measurement."""
import os, sys, time, json
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_BENCH_HW_QUEUES", "16")
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd, rtamd.dist as rtdist
torch.cuda.set_device(0); rtamd.set_device(0)
S = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", "world8_stress.json"), 1920, 1080)
depth = 8
streams = [torch.cuda.Stream() for _ in range(depth)]
S.set_frame_slots(depth)
K = int(os.environ.get("K", "20"))
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for n in [int(x) for x in os.environ.get("NS", "1,2,4,8").split(",")]:
        rows = len(range(0, 1080, n))
        pipe = rtdist.FramePipeline(1920, rows, 1, 0, "cuda", depth=depth, streams=streams)
        def frame(k):
            pipe.step(k, lambda buf, s: S.render_device(spp=8, row0=0, row_step=n, compact=True,
                                                        rgba_ptr=buf.data_ptr(), stream=s.cuda_stream))
        S.set_overlap(False)
        for k in range(6): frame(k)                        # warm-up (bench.py: 5)
        pipe.finish(); torch.cuda.synchronize()
        for policy in os.environ.get("POLICIES", "stream,stream-last-full").split(","):
            S.set_overlap(False, stream=True)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for k in range(K):
                last = {"stream-last-full": 1, "last2": 2, "last4": 4, "last8": 8}.get(policy, 0)
                if last and k == K - last:
                    S.set_overlap(True)
                frame(k)
            pipe.finish(); torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / K * 1e3
            S.set_overlap(False)
            print(json.dumps({"round": rnd, "n": n, "policy": policy, "frames": K, "ms_per_frame": round(ms, 4)}), flush=True)
