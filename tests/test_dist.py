"""Multi-rank frame partition on CPU (gloo, world_size 2 and 3): the row-cyclic
slices each rank renders, gathered and un-permuted by rtamd.dist.RowCyclicFrame (the
code bench.py runs over RCCL), reassemble exactly the single-process frame.  Ranks
render their slices with the oracle (no GPU here); the GPU slice rendering itself is
covered by test_gpu_render.py::test_row_slices_compose."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import scene_path


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, scene, w, h, spp, out_path, slots):
    import torch.distributed as dist
    from oracle_lib import Oracle
    import rtamd.dist as rtdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = Oracle()
        fr = orc.render(orc.load(scene_path(scene), w, h), spp=spp, row0=rank, row_step=world, nthreads=2,
                        want=("rgba",))
        fb = rtdist.RowCyclicFrame(w, h, world, rank, "cpu", dist, slots=slots)
        mine = torch.from_numpy(np.ascontiguousarray(fr["rgba"].view(np.int32)[list(rtdist.rows_of(rank, world, h))]))
        # the oracle returns the full-size frame; each rank takes its rows (compact slice).
        # Three frames through the (pipelined) gather: frame k = image + k, so a stale
        # or overwritten slot shows up in the last or the middle frame.
        outs = []
        for k in range(3):
            fb.slot_part(k)[:mine.shape[0]] = mine + k
            out = fb.gather(k)
            if k == 1:
                fb.finish()
                if rank == 0:
                    outs.append(out.clone())
        out = fb.finish()
        if rank == 0:
            np.save(out_path, np.stack([outs[0].numpy(), out.numpy()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h,slots", [(2, 61, 1), (3, 61, 1), (2, 60, 2), (3, 60, 2), (3, 61, 2)])
def test_row_cyclic_gather_reassembles_frame(oracle, tmp_path, world, h, slots):
    """61 rows: ragged last slice (row loop un-permute); 60: one strided copy; slots = 2:
    double-buffered asynchronous gathers (bench.py's RCCL mode)."""
    scene, w, spp = "world8_stress", 96, 2
    out_path = str(tmp_path / "frame.npy")
    mp.spawn(_rank_main, args=(world, _free_port(), scene, w, h, spp, out_path, slots), nprocs=world, join=True)
    full = oracle.render(oracle.load(scene_path(scene), w, h), spp=spp, nthreads=4, want=("rgba",))["rgba"].view(np.int32)
    got = np.load(out_path)
    assert np.array_equal(got[0], full + 1)
    assert np.array_equal(got[1], full + 2)


def test_rows_partition_covers_frame_once():
    import rtamd.dist as rtdist
    for h in (1, 7, 1080, 2160):
        for g in (1, 2, 3, 4, 8):
            rows = sorted(y for r in range(g) for y in rtdist.rows_of(r, g, h))
            assert rows == list(range(h))
            assert all(len(rtdist.rows_of(r, g, h)) <= rtdist.slice_height(g, h) for r in range(g))


@pytest.mark.parametrize("depth,lag", [(4, 3), (8, 7), (3, 5)])
def test_frame_pipeline_copies_in_completion_order(depth, lag):
    """FramePipeline(readback=True) with frames completing out of order (as frames in flight do,
    several sharing the GPU): a frame's host copy is issued once its own frame is seen complete,
    before older frames' copies; every frame is copied exactly once, from its own frame buffer
    before that buffer is rendered again, and the consumer reads frame k - lag as frame k."""
    import torch
    import rtamd.dist as rtdist
    W, H = 8, 4
    pipe = rtdist.FramePipeline(W, H, 1, 0, "cpu", None, depth=depth, readback=True)

    class Ev:                                   # complete after `delay` completion queries
        def __init__(self, delay):
            self.delay = delay

        def synchronize(self):
            self.delay = 0

    n_ev = [0]

    def event(stream):
        n_ev[0] += 1
        return Ev((n_ev[0] * 5) % 7)

    def done(ev):
        ev.delay -= 1
        return ev.delay < 0
    pipe._event, pipe._done = event, done
    order = []
    to_host = pipe._to_host

    def logged(k, src, stream):
        assert int(src[0, 0]) == k              # the buffer still holds frame k when it is copied
        order.append(k)
        return to_host(k, src, stream)
    pipe._to_host = logged
    n = 4 * depth + 3
    got = {}
    for k in range(n):
        pipe.step(k, lambda buf, st, k=k: buf.fill_(k))
        if k - lag >= 0:
            got[k - lag] = pipe.host_frame(k - lag).clone()
    pipe.finish()
    for j in range(max(0, n - lag), n):
        got[j] = pipe.host_frame(j).clone()
    assert sorted(order) == list(range(n))
    assert order != sorted(order), "no frame was copied ahead of an older one"
    for j in range(n):
        assert torch.equal(got[j], torch.full((H, W), j, dtype=torch.int32)), j


def _pipe_main(rank, world, port, scene, w, h, spp, out_path, depth, readback, lag):
    import torch.distributed as dist
    from oracle_lib import Oracle
    import rtamd.dist as rtdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = Oracle()
        fr = orc.render(orc.load(scene_path(scene), w, h), spp=spp, row0=rank, row_step=world, nthreads=2,
                        want=("rgba",))
        mine = torch.from_numpy(np.ascontiguousarray(fr["rgba"].view(np.int32)[list(rtdist.rows_of(rank, world, h))]))
        pipe = rtdist.FramePipeline(w, h, world, rank, "cpu", dist, depth=depth, readback=readback)

        def render(k):
            def f(buf, st):
                buf[:mine.shape[0]] = mine + k               # frame k = image + k
            return f
        got = []
        n = 2 * depth + 2
        for k in range(n):
            pipe.step(k, render(k))
            j = k - lag                                      # a host consumer `lag` frames behind
            if readback and rank == 0 and j >= 0:
                got.append(pipe.host_frame(j).clone().numpy())
        last = pipe.finish()
        if rank == 0:
            if readback:
                got += [pipe.host_frame(j).clone().numpy() for j in range(n - lag, n)]
            else:
                got = [last.clone().numpy()]
            np.save(out_path, np.stack(got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h,depth,readback,lag", [(2, 61, 3, False, 0), (3, 60, 4, False, 0),
                                                        (2, 61, 3, True, 2), (3, 61, 2, True, 1),
                                                        (2, 61, 3, True, 5)])
def test_frame_pipeline_gather_across_processes(oracle, tmp_path, world, h, depth, readback, lag):
    """rtamd.dist.FramePipeline (bench.py's default N > 1 path) across processes: frames in
    flight, asynchronous gathers into per-slot buffers, the un-permute one frame later, and
    (readback) every frame's host copy -- the frame k that rank 0 reads is image + k, for a
    consumer depth - 1 frames behind and one 2 x depth - 1 behind (the default host buffers)."""
    scene, w, spp = "world8_stress", 96, 2
    out_path = str(tmp_path / "frames.npy")
    mp.spawn(_pipe_main, args=(world, _free_port(), scene, w, h, spp, out_path, depth, readback, lag), nprocs=world,
             join=True)
    full = oracle.render(oracle.load(scene_path(scene), w, h), spp=spp, nthreads=4, want=("rgba",))["rgba"].view(np.int32)
    got = np.load(out_path)
    n = 2 * depth + 2
    if readback:
        assert got.shape[0] == n
        for k in range(n):
            assert np.array_equal(got[k], full + k), k
    else:
        assert np.array_equal(got[0], full + n - 1)
