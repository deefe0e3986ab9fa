"""Frames in flight (rt_scene_set_frame_slots + rtamd.dist.FramePipeline): frames
issued on rotating streams, with the per-frame state in 2-4 slots, are the frames
serial rendering gives, bit for bit -- on one GPU, and for the row-cyclic split with its
gather and un-permute (world 2, one process: the other rank's slice is supplied by a
stand-in gather)."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, scene_path
from twin import NTHREADS, assert_frames_equal, mirror_instances

pytestmark = pytest.mark.gpu


def _serial(gpu, scene, w, h, spp, row0=0, row_step=1):
    import torch
    s = gpu.Scene.load_json(scene_path(scene), w, h)
    rows = len(range(row0, h, row_step))
    buf = torch.zeros((rows, w), dtype=torch.int32, device="cuda")
    s.render_device(spp=spp, row0=row0, row_step=row_step, compact=True, rgba_ptr=buf.data_ptr(), sync=True)
    return buf


@pytest.mark.parametrize("scene,spp,depth", [("world8_stress", 4, 2), ("world16", 1, 3), ("world8", 2, 4)])
def test_frame_slots_streams_identical(gpu, scene, spp, depth):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
    import rtamd.dist as rtdist
    w, h = 240, 160
    ref = _serial(gpu, scene, w, h, spp)
    s = gpu.Scene.load_json(scene_path(scene), w, h)
    s.set_frame_slots(depth)
    pipe = rtdist.FramePipeline(w, h, 1, 0, "cuda", depth=depth)
    for k in range(9):
        pipe.step(k, lambda buf, st: s.render_device(spp=spp, rgba_ptr=buf.data_ptr(), stream=st.cuda_stream))
        if k % 3 == 2:
            torch.cuda.synchronize()
            assert torch.equal(pipe.finish(), ref), k
    torch.cuda.synchronize()
    assert torch.equal(pipe.finish(), ref)
    assert all(torch.equal(p, ref) for p in pipe.parts)


@pytest.mark.parametrize("policy", ["half", "full", "stream"])
def test_overlap_policies_identical(gpu, policy):
    """rt_scene_set_overlap (RT_OVERLAP_HALF / FULL / STREAM; four or more slots, so frames take
    half or all of the CUs) changes only the grids: the frames are the serial frame."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
    import rtamd.dist as rtdist
    w, h, spp, depth = 320, 180, 8, 8
    ref = _serial(gpu, "world8_stress", w, h, spp)
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s.set_frame_slots(depth)
    s.set_overlap(policy == "full", stream=policy == "stream")
    pipe = rtdist.FramePipeline(w, h, 1, 0, "cuda", depth=depth)
    for k in range(12):
        pipe.step(k, lambda buf, st: s.render_device(spp=spp, rgba_ptr=buf.data_ptr(), stream=st.cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(pipe.finish(), ref)
    assert all(torch.equal(p, ref) for p in pipe.parts)


class _Work:
    """Like a torch.distributed Work: wait() makes the current stream wait for the copies
    issued on the stream current at the gather."""

    def __init__(self):
        import torch
        self.ev = torch.cuda.Event()
        self.ev.record()

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_event(self.ev)


class _TwoRankGather:
    """Stand-in for dist.gather at world 2 in one process: slice 0 is this rank's buffer,
    slice 1 the other rank's precomputed one; copies are stream-ordered on the caller's
    current stream (as the collective is ordered after it)."""

    def __init__(self, other):
        self.other = other

    def gather(self, t, gl, dst=0, async_op=False):
        gl[0].copy_(t)
        gl[1].copy_(self.other)
        return _Work()


def test_pipeline_world2_gather_and_unpermute(gpu):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
    import rtamd.dist as rtdist
    w, h, spp = 200, 151, 2                                     # ragged: rows 76 + 75
    full = _serial(gpu, "world8_stress", w, h, spp)
    r1 = _serial(gpu, "world8_stress", w, h, spp, 1, 2)
    other = torch.zeros((rtdist.slice_height(2, h), w), dtype=torch.int32, device="cuda")
    other[:r1.shape[0]] = r1
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s.set_frame_slots(3)
    pipe = rtdist.FramePipeline(w, h, 2, 0, "cuda", _TwoRankGather(other), depth=3)
    for k in range(7):
        pipe.step(k, lambda buf, st: s.render_device(spp=spp, row0=0, row_step=2, compact=True,
                                                     rgba_ptr=buf.data_ptr(), stream=st.cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(pipe.finish(), full)


def _move(s, k, inst):
    """Frame k's poses: a few instances lifted / shifted (cumulative), one frame with a
    rotated instance (the general-pose kernels), so consecutive frames differ."""
    n = inst.shape[0]
    for j in range(3):
        t = (37 * k + 101 * j) % n
        p = inst[t, 4:7] + np.float32([0.25 * j, 0.5 + 0.125 * k, -0.25 * j])
        s.set_trans(t, pos=p)
    if k == 5:
        s.set_trans(11, quat=(0.0, 0.38268343, 0.0, 0.9238795))      # 45 deg about y
    if k == 7:
        s.set_trans(11, quat=(0.0, 0.0, 0.0, 1.0))


@pytest.mark.parametrize("depth", [1, 3])
def test_pipeline_moving_instances(gpu, oracle, depth):
    """rt_builder_set_trans between frames in flight: every frame of the
    pipeline equals the serial render of the same poses, and the serial frames equal the
    oracle's render of those poses (including the frames with a 45-degree rotated instance:
    the general-pose kernels); a debug_cast side entry in the middle (it rebuilds the current
    slot's BVH) disturbs no frame."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
    import rtamd.dist as rtdist
    w, h, spp, n_frames = 160, 120, 2, 9
    ser = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    o = oracle.load(scene_path("world8_stress"), w, h)
    inst = ser.export("instances").copy()
    refs = []
    for k in range(n_frames):
        _move(ser, k, inst)
        buf = torch.zeros((h, w), dtype=torch.int32, device="cuda")
        ser.render_device(spp=spp, rgba_ptr=buf.data_ptr(), sync=True)
        refs.append(buf)
        if depth == 1:                                              # the oracle once per pose sequence
            mirror_instances(ser, o)
            of = oracle.render(o, spp=spp, nthreads=NTHREADS)
            fr = ser.render(spp=spp, want=("rgba", "radiance", "hit_inst", "hit_tri"), stats=False)
            assert np.array_equal(fr["rgba"], buf.cpu().numpy().view(np.uint32)), k
            assert_frames_equal(fr, of, ctx=k)
    assert not all(torch.equal(refs[0], r) for r in refs[1:])   # the poses change the frames
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s.set_frame_slots(depth)
    pipe = rtdist.FramePipeline(w, h, 1, 0, "cuda", depth=depth)
    outs = [None] * n_frames

    def render(k):
        def f(buf, st):
            s.render_device(spp=spp, rgba_ptr=buf.data_ptr(), stream=st.cuda_stream)
            outs[k] = buf.clone()                                  # on st, after the render
        return f
    for k in range(n_frames):
        _move(s, k, inst)
        pipe.step(k, render(k))
        if k == 4:
            s.debug_cast(w // 2, h // 2)
    pipe.finish()
    torch.cuda.synchronize()
    for k in range(n_frames):
        assert torch.equal(outs[k], refs[k]), k


@pytest.mark.parametrize("world,extra", [(1, 0), (2, 0), (1, 3), (2, 3)])
def test_pipeline_host_readback(gpu, world, extra):
    """FramePipeline(readback=True): every frame reaches its pinned host buffer through the
    asynchronous copy (rank 0 of a world-2 split: after the gather and un-permute), equal to
    the serial frame, while later frames are in flight; `extra` more frames behind too (the
    default host buffers are 2 x depth: bench.py's consumer is 2 x depth - 1 behind)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
    import rtamd.dist as rtdist
    w, h, spp, depth = 200, 151, 2, 3
    full = _serial(gpu, "world8_stress", w, h, spp).cpu()
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s.set_frame_slots(depth)
    if world == 1:
        pipe = rtdist.FramePipeline(w, h, 1, 0, "cuda", depth=depth, readback=True)
        kw = dict(row0=0, row_step=1)
    else:
        r1 = _serial(gpu, "world8_stress", w, h, spp, 1, 2)
        other = torch.zeros((rtdist.slice_height(2, h), w), dtype=torch.int32, device="cuda")
        other[:r1.shape[0]] = r1
        pipe = rtdist.FramePipeline(w, h, 2, 0, "cuda", _TwoRankGather(other), depth=depth, readback=True)
        kw = dict(row0=0, row_step=2)
    seen = 0
    for k in range(8):
        pipe.step(k, lambda buf, st: s.render_device(spp=spp, compact=True, rgba_ptr=buf.data_ptr(),
                                                     stream=st.cuda_stream, **kw))
        if k >= depth - 1:
            j = (k - depth + 2 if world > 1 else k - depth + 1) - extra
            if j >= 0:
                assert torch.equal(pipe.host_frame(j), full), (k, j)
                seen += 1
    pipe.finish()
    torch.cuda.synchronize()
    assert torch.equal(pipe.host_frame(7), full)
    assert seen >= 4 - extra
