"""Host-side issue cost of one pipelined frame, measured on ONE GPU.

bench.py --gpus 8 issues, per frame and rank, a render (rt_render over ctypes: BVH build +
trace launch), an asynchronous RCCL gather of the slice and (rank 0) the un-permute copy.
At 8 GPUs a rank's render takes about 0.25 ms, so the host must issue a frame in well
under that or the GPU starves.  This tool times the issue calls alone (no
synchronisation inside the loop) for rank 0's slice of an N-way split, with the gather
through a one-rank NCCL group (same ProcessGroupNCCL code path; an 8-rank gather on
rank 0 posts 8 receives instead of 1).

Usage: python tools/host_overhead.py [--ns 1,8] [--steps 200]
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="world8_stress")
    p.add_argument("--spp", type=int, default=8)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--ns", default="1,8")
    a = p.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    rtamd.set_device(0)
    scene = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", a.scene + ".json"), 1920, 1080)
    scene.set_frame_slots(4)
    W, H = scene.width, scene.height
    streams = [torch.cuda.Stream() for _ in range(4)]
    main_st = torch.cuda.current_stream()
    for n in [int(x) for x in a.ns.split(",")]:
        rows = len(range(0, H, n))
        parts = [torch.zeros((rows, W), dtype=torch.int32, device="cuda") for _ in range(4)]
        gbufs = [torch.zeros((1, rows, W), dtype=torch.int32, device="cuda") for _ in range(4)]
        out = torch.zeros((rows, W), dtype=torch.int32, device="cuda")

        def render(k):
            s = k % 4
            scene.render_device(spp=a.spp, rebuild_bvh=True, row0=0, row_step=n, compact=True,
                                rgba_ptr=parts[s].data_ptr(), stream=streams[s].cuda_stream)

        def gather(k):
            s = k % 4
            with torch.cuda.stream(streams[s]):
                w = dist.gather(parts[s], list(gbufs[s].unbind(0)), dst=0, async_op=True)
            with torch.cuda.stream(main_st):
                w.wait()
                out.copy_(gbufs[s][0])
                ev = torch.cuda.Event()
                ev.record(main_st)

        for k in range(20):
            render(k)
            gather(k)
        torch.cuda.synchronize()
        res = {"n": n, "rows": rows}
        for name, fn in (("render", lambda k: render(k)), ("gather+unpermute", lambda k: gather(k)),
                         ("frame", lambda k: (render(k), gather(k)))):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.steps):
                fn(k)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res[name + "_issue_us"] = round((t1 - t0) / a.steps * 1e6, 1)
            res[name + "_wall_us"] = round((t2 - t0) / a.steps * 1e6, 1)
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
