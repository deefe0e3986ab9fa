"""Multi-GPU frame partition: row-cyclic slices + one gather.

Rank r of G renders rows y = r, r+G, r+2G, ... (compact: slice row i is frame row
r + i*G), which balances lit-pixel load to within 1% on the reference scenes where
contiguous bands are 1.4-2.5x off.  The BVH and scene are replicated (each rank
rebuilds the identical tree from the same instance array), so the frame's only
exchange is gathering the packed RGBA8 slices to rank 0 (RCCL `gather` over xGMI on
GPUs; any torch.distributed backend works, the CPU tests use gloo) and the row
un-permute there.  Slices are padded to ceil(H/G) rows so every message has the
same size.
"""
import torch


def rows_of(rank, world, height):
    """Frame rows owned by `rank` (in slice order)."""
    return range(rank, height, world)


def slice_height(world, height):
    return (height + world - 1) // world


class RowCyclicFrame:
    """Per-rank slice buffer + (rank 0) the assembled frame.

    `part` is the compact slice a rank renders into (rt_render_opts.row0 = rank,
    row_step = world, compact = 1); `gather()` assembles the frame on rank 0.
    """

    def __init__(self, width, height, world, rank, device, dist=None, dtype=torch.int32, host_staging=False):
        """host_staging: gather through host memory (backends without device tensors,
        e.g. gloo when testing the multi-rank path on one GPU)."""
        self.W, self.H, self.world, self.rank, self.dist = width, height, world, rank, dist
        self.host_staging = host_staging
        self.rows = slice_height(world, height)
        self.part = torch.zeros((self.rows, width), dtype=dtype, device=device)
        gdev = "cpu" if host_staging else device
        self.gathered = ([torch.empty((self.rows, width), dtype=dtype, device=gdev) for _ in range(world)]
                         if (world > 1 and rank == 0) else None)
        # one rank: the slice is the frame (rows_of(0, 1, H) = every row, in order) -- no copy
        self.frame = (self.part if world == 1 else
                      torch.empty((height, width), dtype=dtype, device=device) if rank == 0 else None)

    def gather(self):
        """Collect every rank's slice on rank 0 and un-permute the rows into `frame`."""
        if self.world > 1:
            self.dist.gather(self.part.cpu() if self.host_staging else self.part, self.gathered, dst=0)
            if self.rank == 0:
                for r in range(self.world):
                    n = len(rows_of(r, self.world, self.H))
                    self.frame[r::self.world] = self.gathered[r][:n].to(self.frame.device)
        return self.frame
