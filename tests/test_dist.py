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


def _rank_main(rank, world, port, scene, w, h, spp, out_path):
    import torch.distributed as dist
    from oracle_lib import Oracle
    import rtamd.dist as rtdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = Oracle()
        fr = orc.render(orc.load(scene_path(scene), w, h), spp=spp, row0=rank, row_step=world, nthreads=2,
                        want=("rgba",))
        fb = rtdist.RowCyclicFrame(w, h, world, rank, "cpu", dist)
        mine = fr["rgba"].view(np.int32)
        # the oracle returns the full-size frame; take this rank's rows (compact slice)
        rows = list(rtdist.rows_of(rank, world, h))
        fb.part[:len(rows)] = torch.from_numpy(np.ascontiguousarray(mine[rows]))
        out = fb.gather()
        if rank == 0:
            np.save(out_path, out.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_cyclic_gather_reassembles_frame(oracle, tmp_path, world):
    scene, w, h, spp = "world8_stress", 96, 61, 2          # 61 rows: ragged last slice for G = 2, 3
    out_path = str(tmp_path / "frame.npy")
    mp.spawn(_rank_main, args=(world, _free_port(), scene, w, h, spp, out_path), nprocs=world, join=True)
    full = oracle.render(oracle.load(scene_path(scene), w, h), spp=spp, nthreads=4, want=("rgba",))
    assert np.array_equal(np.load(out_path), full["rgba"].view(np.int32))


def test_rows_partition_covers_frame_once():
    import rtamd.dist as rtdist
    for h in (1, 7, 1080, 2160):
        for g in (1, 2, 3, 4, 8):
            rows = sorted(y for r in range(g) for y in rtdist.rows_of(r, g, h))
            assert rows == list(range(h))
            assert all(len(rtdist.rows_of(r, g, h)) <= rtdist.slice_height(g, h) for r in range(g))
