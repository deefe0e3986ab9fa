#!/usr/bin/env python3
"""Host issue and wait times of the host-readable frame pipeline (bench.py's headline loop):
per frame, how long the host spends issuing it (FramePipeline.step) and waiting for the frame
it reads (host_frame), and the loop's ms per frame; host-readable (copies on one copy stream)
and device-resident for comparison."""
import json
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_BENCH_HW_QUEUES", "16")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402
import rtamd.dist as rtdist  # noqa: E402


def main():
    readback = (sys.argv[1] if len(sys.argv) > 1 else "1") == "1"
    scene_name = sys.argv[2] if len(sys.argv) > 2 else "world8_stress"
    clamp = int(os.environ.get("RT_PROBE_COPY_BYTES", "0"))
    no_consumer = os.environ.get("RT_PROBE_NO_CONSUMER", "0") == "1"   # experiment: no per-frame host read
    if clamp:                             # experiment: copies cut to `clamp` bytes (sync cost vs data)
        real = rtamd.copy_to_host_async
        rtamd.copy_to_host_async = lambda h, d, n, st=None: real(h, d, min(n, clamp), st)
    n = 40
    W, H, D = 1920, 1080, 8
    pipe = rtdist.FramePipeline(W, H, 1, 0, "cuda", None, depth=D, readback=readback)
    if os.environ.get("RT_PROBE_HIPMALLOC", "0") == "1":     # experiment: frame buffers from hipMalloc
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")

        class Dev:
            def __init__(self, n):
                self.p = ctypes.c_void_p()
                assert hip.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(n * 4)) == 0
                self.__cuda_array_interface__ = {"shape": (H, W), "typestr": "<i4", "data": (self.p.value, False),
                                                 "version": 2}
        pipe._devbufs = [Dev(W * H) for _ in pipe.parts]
        pipe.parts = [torch.as_tensor(b, device="cuda") for b in pipe._devbufs]
    for st in pipe.streams + ([pipe.copy_stream] if readback else []):
        torch.cuda.Event().record(st)
    scene = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", scene_name + ".json"), W, H)
    scene.set_frame_slots(D)
    torch.cuda.synchronize()

    def render(buf, st):
        scene.render_device(spp=8, rgba_ptr=buf.data_ptr(), stream=st.cuda_stream)
    for k in range(10):
        pipe.step(k, render)
    pipe.finish()
    torch.cuda.synchronize()
    scene.set_overlap(False, stream=True)
    issue, wait = [], []
    evs = []
    if readback:                          # timing events: render done -> copy done, per frame
        def ev_timed(stream):
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            evs.append(e)
            return e
        pipe._event = ev_timed
    t0 = time.perf_counter()
    for i in range(n):
        k = 10 + i
        a = time.perf_counter()
        pipe.step(k, render)
        b = time.perf_counter()
        if readback and k - pipe.n_host + 1 >= 10 and not no_consumer:
            pipe.host_frame(k - pipe.n_host + 1)
        c = time.perf_counter()
        issue.append((b - a) * 1e3)
        wait.append((c - b) * 1e3)
    pipe.finish()
    if readback:
        pipe.host_frame(10 + n - 1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    scene.set_overlap(False)
    lat = [round(evs[2 * i].elapsed_time(evs[2 * i + 1]), 3) for i in range(len(evs) // 2)]
    gaps = [round(evs[2 * i - 1].elapsed_time(evs[2 * i + 1]), 3) for i in range(1, len(evs) // 2)]
    print(json.dumps({"readback": readback, "ms_per_frame": round(dt, 4),
                      "issue_ms": [round(x, 3) for x in issue], "wait_ms": [round(x, 3) for x in wait],
                      "render_done_to_copy_done_ms": lat, "copy_done_interval_ms": gaps}), flush=True)


if __name__ == "__main__":
    main()
