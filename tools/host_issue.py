"""Host cost of issuing frames: an N-way row-cyclic slice pipelined 8 deep on one GPU (the
render side of bench.py --gpus N), timing the issue loop alone (host returns) and the loop
plus the final wait.  When the two agree the pipeline is host-bound.  NS env var."""
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
for n in [int(x) for x in os.environ.get("NS", "1,8").split(",")]:
    rows = len(range(0, 1080, n))
    pipe = rtdist.FramePipeline(1920, rows, 1, 0, "cuda", depth=depth, streams=streams)
    def frame(k, st=None):
        pipe.step(k, lambda buf, s: S.render_device(spp=8, row0=0, row_step=n, compact=True,
                                                    rgba_ptr=buf.data_ptr(), stream=s.cuda_stream))
    for k in range(16): frame(k)
    pipe.finish(); torch.cuda.synchronize()
    for policy in ("half", "stream"):
        S.set_overlap(False, stream=policy == "stream")
        for K in (20, 60):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for k in range(K): frame(k)
            t_issue = time.perf_counter() - t
            pipe.finish(); torch.cuda.synchronize()
            t_all = time.perf_counter() - t
            print(json.dumps({"n": n, "policy": policy, "frames": K, "issue_ms_per_frame": round(t_issue / K * 1e3, 4),
                              "ms_per_frame": round(t_all / K * 1e3, 4)}), flush=True)
    S.set_overlap(False)
