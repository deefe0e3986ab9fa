#!/usr/bin/env python3
"""Where the first frames' time goes: bench.py's start-up, step by step.

Prints, for each phase, the host time until the call returns (issue) and until the device is
idle again (done): scene load, the counted frame, then the first fast frame of every frame slot
/ stream of the pipeline, then a second round over the same slots.  A cost paid once per slot
or stream shows as a first round slower than the second.
"""
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402
import rtamd.dist as rtdist  # noqa: E402


def main():
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "world8_stress"
    depth = 8
    out = {}
    t = time.perf_counter()
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    out["torch_init_ms"] = (time.perf_counter() - t) * 1e3
    rtamd.set_device(0)
    t = time.perf_counter()
    scene = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", scene_name + ".json"), 1920, 1080)
    out["load_json_ms"] = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    scene.set_frame_slots(depth)
    out["set_frame_slots_ms"] = (time.perf_counter() - t) * 1e3
    fb = rtdist.FramePipeline(1920, 1080, 1, 0, "cuda", None, depth=depth)
    stream = torch.cuda.current_stream()
    t = time.perf_counter()
    scene.render_device(spp=8, use_bvh=True, rebuild_bvh=True, row0=0, row_step=1, compact=True,
                        rgba_ptr=fb.parts[0].data_ptr(), stream=stream.cuda_stream, sync=True, stats=True)
    out["counted_frame_ms"] = (time.perf_counter() - t) * 1e3

    def frame(k, st):
        t0 = time.perf_counter()
        scene.render_device(spp=8, use_bvh=True, rebuild_bvh=True, row0=0, row_step=1, compact=True,
                            rgba_ptr=fb.parts[k % depth].data_ptr(), stream=st.cuda_stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return round((t1 - t0) * 1e3, 3), round((t2 - t0) * 1e3, 3)

    for rnd in range(3):
        out["round%d_issue_done_ms" % rnd] = [frame(k, fb.streams[k % depth]) for k in range(depth)]
    # the same slots on the default stream (no new streams): isolates per-stream first-use costs
    out["default_stream_issue_done_ms"] = [frame(k, stream) for k in range(depth)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
