#!/usr/bin/env python3
"""Experiment (VERDICT r05 item 1's alternative): the kernels store the frame straight into
pinned host memory, against the copy-engine pipeline bench.py times.  Both: 8 frames in
flight, world8_stress 1920x1080 8 spp, a host consumer waiting for frame k - 7 as frame k is
issued, ms per frame over N frames; then the two pipelines' last frames compared.
Usage: direct_probe.py [N] [scene]"""
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_BENCH_HW_QUEUES", "16")
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402
import rtamd.dist as rtdist  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    scene_name = sys.argv[2] if len(sys.argv) > 2 else "world8_stress"
    W, H, D = 1920, 1080, 8
    lag = D - 1
    pipe = rtdist.FramePipeline(W, H, 1, 0, "cuda", None, depth=D, readback=True)
    streams = pipe.streams
    hb = [rtamd.HostBuffer((H, W), np.int32) for _ in range(2 * D)]
    for st in streams + [pipe.copy_stream]:
        torch.cuda.Event().record(st)
    torch.cuda.synchronize()
    scene = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", scene_name + ".json"), W, H)
    scene.set_frame_slots(D)
    torch.cuda.synchronize()

    def render(ptr, st):
        scene.render_device(spp=8, use_bvh=True, rebuild_bvh=True, row0=0, row_step=1, compact=True,
                            rgba_ptr=ptr, stream=st.cuda_stream)

    frame_no = [0]

    def run_copy(n):
        t0 = time.perf_counter()
        first = frame_no[0]
        for i in range(n):
            k = frame_no[0]
            frame_no[0] += 1
            pipe.step(k, lambda buf, st: render(buf.data_ptr(), st))
            if k - lag >= first:
                pipe.host_frame(k - lag)
        pipe.finish()
        for j in range(max(first, frame_no[0] - lag), frame_no[0]):
            pipe.host_frame(j)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, pipe.host_frame(frame_no[0] - 1).numpy().copy()

    ev = [None] * (2 * D)

    def run_direct(n):
        t0 = time.perf_counter()
        first = frame_no[0]
        last = None
        for i in range(n):
            k = frame_no[0]
            frame_no[0] += 1
            h = k % (2 * D)
            st = streams[k % D]
            if ev[h] is not None:
                ev[h].synchronize()                    # frame k - 2D is read (long since)
            render(hb[h].ptr, st)
            e = torch.cuda.Event()
            e.record(st)
            ev[h] = e
            if k - lag >= first:
                ev[(k - lag) % (2 * D)].synchronize()  # the consumer: frame k - lag on the host
            last = h
        for j in range(max(first, frame_no[0] - lag), frame_no[0]):
            ev[j % (2 * D)].synchronize()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, hb[last].array.copy()

    scene.set_overlap(False, stream=True)
    run_copy(16)
    run_direct(16)
    res = {"copy": [], "direct": []}
    for rep in range(3):
        for name, fn in (("copy", run_copy), ("direct", run_direct)):
            ms, fr = fn(N)
            res[name].append(ms)
            res[name + "_frame"] = fr
            print("%-7s %d frames: %.4f ms per frame" % (name, N, ms), flush=True)
    same = np.array_equal(res["copy_frame"], res["direct_frame"])
    print("copy  median %.4f ms, direct median %.4f ms; last frames equal: %s" % (
        sorted(res["copy"])[1], sorted(res["direct"])[1], same), flush=True)
    if not same:
        print("differing pixels:", int((res["copy_frame"] != res["direct_frame"]).sum()))


if __name__ == "__main__":
    main()
