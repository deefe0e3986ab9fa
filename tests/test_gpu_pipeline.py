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


class _Work:
    def wait(self):
        pass


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
