"""Multi-GPU frame partition: row-cyclic slices + one gather.

Rank r of G renders rows y = r, r+G, r+2G, ... (compact: slice row i is frame row
r + i*G), which balances lit-pixel load to within 1% on the reference scenes where
contiguous bands are 1.4-2.5x off.  The BVH and scene are replicated (each rank
rebuilds the identical tree from the same instance array), so the frame's only
exchange is gathering the packed RGBA8 slices to rank 0 (RCCL `gather` over xGMI on
GPUs; any torch.distributed backend works, the CPU tests use gloo) and the row
un-permute there.  Slices are padded to ceil(H/G) rows so every message has the
same size.

Pipelining, two forms:
- `RowCyclicFrame(slots=2)` (serial frames, bench.py --no-overlap): frame k renders into
  slice buffer k % 2 and its gather is issued asynchronously, so it runs on the collective
  stream while frame k+1 renders; frame k's un-permute is enqueued when frame k+1's gather
  is issued (or by `finish()`), after waiting for frame k's gather.
- `FramePipeline(depth)` (bench.py default, depth 4): frames in flight on their own
  streams, see the class.
The waits are stream dependencies, not host synchronisation.
"""
import contextlib

import torch


def rows_of(rank, world, height):
    """Frame rows owned by `rank` (in slice order)."""
    return range(rank, height, world)


def slice_height(world, height):
    return (height + world - 1) // world


class RowCyclicFrame:
    """Per-rank slice buffer(s) + (rank 0) the assembled frame.

    `part` is the compact slice a rank renders into (rt_render_opts.row0 = rank,
    row_step = world, compact = 1); `gather()` assembles the frame on rank 0.
    """

    def __init__(self, width, height, world, rank, device, dist=None, dtype=torch.int32, host_staging=False,
                 slots=1):
        """host_staging: gather through host memory (backends without device tensors,
        e.g. gloo when testing the multi-rank path on one GPU).  slots = 2: double-buffered
        slices with asynchronous gathers (see the module docstring)."""
        self.W, self.H, self.world, self.rank, self.dist = width, height, world, rank, dist
        self.host_staging = host_staging
        self.rows = slice_height(world, height)
        self.slots = 1 if (world == 1 or host_staging) else max(1, slots)
        self.parts = [torch.zeros((self.rows, width), dtype=dtype, device=device) for _ in range(self.slots)]
        self.part = self.parts[0]
        gdev = "cpu" if host_staging else device
        # rank 0: one contiguous [world, rows, W] buffer; the gather list is its views
        self.gbuf = (torch.empty((world, self.rows, width), dtype=dtype, device=gdev)
                     if (world > 1 and rank == 0) else None)
        self.gathered = list(self.gbuf.unbind(0)) if self.gbuf is not None else None
        # one rank: the slice is the frame (rows_of(0, 1, H) = every row, in order) -- no copy
        self.frame = (self.part if world == 1 else
                      torch.empty((height, width), dtype=dtype, device=device) if rank == 0 else None)
        self._pending = None

    def slot_part(self, k):
        """Slice buffer frame k renders into."""
        return self.parts[k % self.slots]

    def _unpermute(self):
        if self.H % self.world == 0:       # frame row i*G + r = slice r row i: one strided copy
            self.frame.view(self.rows, self.world, self.W).copy_(self.gbuf.transpose(0, 1))
        else:
            for r in range(self.world):
                n = len(rows_of(r, self.world, self.H))
                self.frame[r::self.world] = self.gathered[r][:n].to(self.frame.device)

    def finish(self):
        """Complete an outstanding asynchronous gather (stream-ordered) and un-permute."""
        if self._pending is not None:
            self._pending.wait()
            self._pending = None
            if self.rank == 0:
                self._unpermute()
        return self.frame

    def gather(self, k=0):
        """Collect every rank's slice of frame k on rank 0 and un-permute the rows into
        `frame`.  With slots = 2 the gather is left in flight (finish() / the next call
        completes it)."""
        if self.world == 1:
            return self.frame
        self.finish()
        src = self.slot_part(k)
        if self.host_staging:
            self.dist.gather(src.cpu(), self.gathered, dst=0)
            if self.rank == 0:
                self._unpermute()
            return self.frame
        work = self.dist.gather(src, self.gathered, dst=0, async_op=self.slots > 1)
        if self.slots > 1:
            self._pending = work
        elif self.rank == 0:
            self._unpermute()
        return self.frame


class _Done:
    """A completed event (host-side copies on CPU tensors are synchronous)."""

    def synchronize(self):
        pass


class FramePipeline:
    """`depth` frames in flight (bench.py over RCCL, or one GPU): frame k renders on stream
    k % depth into slice buffer k % depth, with the scene in `depth` frame slots
    (rt_scene_set_frame_slots), so frame k+1's blocks start on the CUs that the previous
    frames' longest groups leave idle.  The RGBA8 slices of frame k are gathered
    asynchronously into gather buffer k % depth on rank 0; frame k's un-permute runs on the
    main stream once frame k+1 has been issued.  Every wait is a stream dependency:
      - frame k's render waits for frame k-depth's gather (it rewrites that slice buffer);
      - frame k's gather waits for frame k-depth's un-permute (same gather buffer);
      - frame k's un-permute waits for frame k's gather.
    Images are the ones serial frames give; only the overlap changes.

    readback=True keeps the reference's post-condition (update_scene returns with the frame
    host-readable, raytracer.cu:102-120 / canvas.cu:23-29) without giving up the overlap: the
    finished frame (rank 0) is copied into pinned host buffer k % host_buffers (rt_host_alloc)
    by a copy-engine transfer (rt_copy_to_host_async: no blit kernel, no CU taken from the
    frames in flight), issued on one copy stream once the frame (N > 1: its un-permute) has
    completed, while later frames render (see the comment in __init__).  `host_frame(k)` waits for frame k's
    copy; a host buffer is reused host_buffers frames later, after its copy (and the caller's
    read) is done, so a consumer may read frames up to host_buffers - 1 behind the last one
    issued.  host_buffers defaults to 2 x depth: the frames the consumer has not read yet are
    the frames in flight, and a consumer only depth - 1 behind caps them at depth including the
    copies (measured: DESIGN.md §4.1).

    host_staging=True (device frames, a backend without device tensors: gloo, several ranks
    sharing one GPU in the tests of bench.py's N > 1 path): each rank's slice is copied by the
    copy engine into a pinned staging buffer per slot on the render stream, and frame k's gather
    of those host slices is issued when frame k + 1 has been issued (after a host wait for frame
    k's staging copy, so that frames k and k + 1 are in flight meanwhile); rank 0 uploads the
    gathered slices into the slot's device gather buffer and un-permutes there as the RCCL path
    does.  The per-slot waits are those of the RCCL path: a slot's staging buffer is rewritten
    after its previous gather has completed, its gather buffer after its previous un-permute."""

    def __init__(self, width, height, world, rank, device, dist=None, dtype=torch.int32, depth=2, readback=False,
                 streams=None, host_buffers=None, host_staging=False, copy_lag=None, copy_streams=2):
        self.W, self.H, self.world, self.rank, self.dist = width, height, world, rank, dist
        self.depth = D = max(1, int(depth))
        self.rows = slice_height(world, height)
        # one rank copying frames to the host: twice as many frame buffers as streams, so that a
        # buffer is rewritten 2 x depth frames after its frame, long after its host copy
        self.n_parts = 2 * D if (readback and world == 1) else D
        self.parts = [torch.zeros((self.rows, width), dtype=dtype, device=device) for _ in range(self.n_parts)]
        # CPU tensors (the gloo tests of the multi-process logic): no streams, no events
        self.cuda = str(device).startswith("cuda")
        # streams: the render streams to reuse (at least `depth` of them; e.g. a later pipeline in
        # the same process).  HIP spreads streams over GPU_MAX_HW_QUEUES hardware queues in the
        # order they are created, and two render streams that share a queue serialise their
        # frames (measured: 0.354 -> 0.42-0.44 ms per 2-way slice frame).  torch's
        # stream pool hands out streams in creation order, and the first seven take distinct
        # queues of eight (the null stream holds the first): create the pipeline early and reuse
        # its streams rather than drawing new ones for each pipeline.
        if streams is not None:
            assert len(streams) >= D, (len(streams), D)
            self.streams = list(streams)[:D]
        else:
            self.streams = [torch.cuda.Stream(device=device) if self.cuda else None for _ in range(D)]
        self.main = torch.cuda.current_stream(device) if self.cuda else None
        self.gbufs = ([torch.empty((world, self.rows, width), dtype=dtype, device=device) for _ in range(D)]
                      if (world > 1 and rank == 0) else None)
        self.host_staging = bool(host_staging) and world > 1 and self.cuda
        self.np_dtype = torch.empty(0, dtype=dtype).numpy().dtype
        if self.host_staging:
            from . import HostBuffer
            self._stage = [HostBuffer((self.rows, width), self.np_dtype) for _ in range(D)]
            self.stage = [b.tensor() for b in self._stage]
            self.stage_ev = [None] * D          # staging copy of the frame last rendered in each slot
            self.hgbufs = ([torch.empty((world, self.rows, width), dtype=dtype) for _ in range(D)]
                           if rank == 0 else None)
            self.stage_pending = None           # (frame, slot) staged but not yet gathered
        self.readback = bool(readback) and (world == 1 or rank == 0)
        n_out = D if self.readback else 1                 # one un-permute target per slot when copied out
        self.outs = ([torch.empty((height, width), dtype=dtype, device=device) for _ in range(n_out)]
                     if (world > 1 and rank == 0) else None)
        self.out = self.outs[0] if self.outs else None
        self.n_host = max(D, int(host_buffers)) if host_buffers else 2 * D
        if self.readback:
            if self.cuda:                       # pinned by the library: the copy engine writes it
                from . import HostBuffer
                self._host = [HostBuffer((height, width), self.np_dtype) for _ in range(self.n_host)]
                self.host = [b.tensor() for b in self._host]
            else:
                self.host = [torch.empty((height, width), dtype=dtype) for _ in range(self.n_host)]
            self.host_ev = [None] * self.n_host     # D2H copy of the frame last copied into each host buffer
            self.host_no = [-1] * self.n_host       # its frame number
            self.out_copy = [None] * D              # world > 1: the copy that last read each un-permute target
            # Host copies are issued once their frame is complete: the host waits for frame k (rank 0
            # with N > 1: its un-permute) when it issues frame k + lag, then enqueues the copy on the
            # one copy stream.  A copy enqueued behind a frame still rendering (a stream wait on
            # the frame's event) waits on the copy engine for that frame's signal, and those waits
            # measured 0.5-5.6 ms from frame done to copy done for a 0.16-ms copy, a convoy that
            # held the frames behind it (0.68 ms per frame against 0.59 device-resident); with
            # the copies issued on completion 0.59-0.61 (profiles/r06/rbprobe/).
            # Frames' copies alternate over `copy_streams` copy streams (the runtime puts each on its
            # own copy-engine queue): consecutive copies on one queue left gaps of ~85 us between
            # them and a backlog of ~10 copies behind the frames under a trace (enqueue -> start
            # 3.1 ms median); two queues overlap those gaps (CLI, 100 frames, world8: +4-12% ->
            # +0.3-2% over device-resident; profiles/r06/cli_cs/, profiles/r06/cli_api/).
            self.copy_streams = ([torch.cuda.Stream(device=device) for _ in range(max(1, int(copy_streams)))]
                                 if self.cuda else [None])
            self.copy_stream = self.copy_streams[0]
            self.copy_done = [None] * self.n_parts  # one rank: the copy that last read parts[p]
            # copies trail the frames issued by `lag`: the host waits for frame k - lag as it issues
            # frame k, so lag + 1 frames stay in flight (one rank: depth, as device-resident frames;
            # N > 1: depth - 1, the un-permute targets are reused after depth frames)
            # (copy_lag: a longer wait before the host blocks, within the buffers: one rank up to
            # 2 depth - 2, N > 1 up to depth - 2)
            self.lag = max(0, D - 1) if world == 1 else max(0, D - 2)
            if copy_lag is not None:
                self.lag = max(0, min(int(copy_lag), self.n_parts - 2 if world == 1 else D - 2))
            self.deferred = []                      # (frame, source, ready event, ("part" | "out", slot))
            if self.cuda:
                # The runtime gives a copy issued while an earlier one still runs the next idle SDMA
                # engine, and a copy's first use of an engine creates its queue (~7 ms inside the
                # enqueue, profiles/r06/rblog/): start the engines these streams will use now.
                from . import copy_engines_warm
                copy_engines_warm([c.cuda_stream for c in self.copy_streams] + [st.cuda_stream for st in self.streams])
        self.work = [None] * D          # gather of the frame last rendered in each slot
        self.unperm = [None] * D        # event after the un-permute that last read each gather buffer
        self.pending = [False] * D      # slot's frame gathered but not yet un-permuted
        self.pend_no = [-1] * D         # its frame number
        self.last = -1

    def _on(self, stream):
        return torch.cuda.stream(stream) if self.cuda else contextlib.nullcontext()

    def _event(self, stream):
        if not self.cuda:
            return _Done()
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    @property
    def frame(self):
        """The last finished frame (rank 0; call finish() first)."""
        if self.world == 1:
            return self.parts[self.last % self.n_parts] if self.last >= 0 else None
        return self.out

    def _to_host(self, k, src, stream):
        """Frame k (device buffer src, complete on `stream`) -> pinned host buffer k % n_host."""
        h = k % self.n_host
        if self.host_ev[h] is not None:
            self.host_ev[h].synchronize()           # frame k - n_host's copy is done (and was read)
        with self._on(stream):
            if self.cuda:
                from . import copy_to_host_async
                assert src.is_contiguous()
                copy_to_host_async(self._host[h].ptr, src.data_ptr(), src.numel() * src.element_size(),
                                   stream.cuda_stream)
            else:
                self.host[h].copy_(src)
            ev = self._event(stream)
        self.host_ev[h], self.host_no[h] = ev, k
        return ev

    def _copy_deferred(self, i):
        """Issue deferred host copy i (its frame has completed)."""
        k, src, ev, (kind, s) = self.deferred.pop(i)
        done = self._to_host(k, src, self.copy_streams[k % len(self.copy_streams)])
        if kind == "part":
            self.copy_done[s] = done
        else:
            self.out_copy[s] = done

    def _copy_ready(self):
        """Issue the deferred copy of every frame that has completed, oldest first; frames in flight
        complete out of order (several share the GPU), and a copy held back for an older frame
        trailed its own by milliseconds (the CLI's trace: ~4 ms, ~6 copies left after the last
        frame, profiles/r06/cli_window/).  Each frame has its own host buffer."""
        i = 0
        while i < len(self.deferred):
            if self._done(self.deferred[i][2]):
                self._copy_deferred(i)
            else:
                i += 1

    def _flush_copies(self, upto=None, key=None):
        """Wait until the deferred host copies are issued: the one that reads `key`; or those of
        frames <= upto; with neither, all.  Polls, so that the copies of frames that complete
        meanwhile (in any order) are issued as they complete."""
        def pending():
            if key is not None:
                return any(e[3] == key for e in self.deferred)
            if upto is not None:
                return any(e[0] <= upto for e in self.deferred)
            return bool(self.deferred)
        while pending():
            self._copy_ready()

    def _done(self, ev):
        return ev.query() if self.cuda else True

    def _defer_copy(self, k, src, ready, key):
        """Frame k's host copy, issued once `ready` (an event after the frame) has completed."""
        self.deferred.append((k, src, ready, key))
        self.deferred.sort(key=lambda e: e[0])   # (finish() un-permutes slots out of frame order)

    def _unpermute(self, s):
        if not self.pending[s]:
            return
        self.pending[s] = False
        with self._on(self.main):
            self.work[s].wait()
            if self.rank == 0:
                g = self.gbufs[s]
                if self.host_staging:           # the gathered host slices -> the slot's device gather buffer
                    g.copy_(self.hgbufs[s])
                out = self.outs[s % len(self.outs)]
                if self.readback:
                    self._flush_copies(key=("out", s))     # frame k - depth's copy has been issued
                if self.readback and self.out_copy[s] is not None and self.cuda:
                    self.main.wait_event(self.out_copy[s])  # ... and has read out
                if self.H % self.world == 0:
                    out.view(self.rows, self.world, self.W).copy_(g.transpose(0, 1))
                else:
                    for r in range(self.world):
                        out[r::self.world] = g[r][:len(rows_of(r, self.world, self.H))]
                self.out = out
                ev = self._event(self.main)
                self.unperm[s] = ev
                if self.readback:
                    self._defer_copy(self.pend_no[s], out, ev, ("out", s))

    def _gather_staged(self):
        """host_staging: issue the gather of the frame staged last (after its staging copy)."""
        if self.stage_pending is None:
            return
        k, s = self.stage_pending
        self.stage_pending = None
        self.stage_ev[s].synchronize()
        gl = list(self.hgbufs[s].unbind(0)) if self.rank == 0 else None
        self.work[s] = self.dist.gather(self.stage[s], gl, dst=0, async_op=True)
        self.pending[s] = True
        self.pend_no[s] = k

    def step(self, k, render):
        """Issue frame k: render(part, stream) enqueues the render of this rank's rows."""
        s = k % self.depth
        st = self.streams[s]
        if self.host_staging:
            with self._on(st):
                if self.work[s] is not None:
                    self.work[s].wait()                 # frame k-depth's gather has read stage[s]
                render(self.parts[s], st)
                from . import copy_to_host_async
                copy_to_host_async(self._stage[s].ptr, self.parts[s].data_ptr(), self._stage[s].nbytes, st.cuda_stream)
                self.stage_ev[s] = self._event(st)
            self._gather_staged()                       # frame k - 1's gather (frame k is in flight)
            self.stage_pending = (k, s)
            if k >= 1:
                self._unpermute((k - 1) % self.depth)
            self.last = k
            return
        with self._on(st):
            if self.work[s] is not None:
                self.work[s].wait()                     # frame k-depth's gather has read parts[s]
            p = k % self.n_parts
            if self.readback and self.world == 1:
                self._flush_copies(key=("part", p))     # frame k - 2 depth's host copy has been issued
                if self.cuda and self.copy_done[p] is not None:
                    st.wait_event(self.copy_done[p])    # ... and has read parts[p]
            render(self.parts[p], st)
            if self.readback and self.world == 1:
                self._defer_copy(k, self.parts[p], self._event(st), ("part", p))
            if self.world > 1:
                if self.unperm[s] is not None and self.cuda:
                    st.wait_event(self.unperm[s])       # frame k-depth's un-permute has read gbufs[s]
                gl = list(self.gbufs[s].unbind(0)) if self.rank == 0 else None
                self.work[s] = self.dist.gather(self.parts[s], gl, dst=0, async_op=True)
                self.pending[s] = True
                self.pend_no[s] = k
        if k >= 1:
            self._unpermute((k - 1) % self.depth)
        if self.readback:
            # every copy whose frame has already completed (no wait): a copy starts as soon as the
            # host sees its frame done, so the window's last frames leave few copies behind; then
            # (polling) frame k - lag's copy
            self._copy_ready()
            self._flush_copies(upto=k - self.lag)
        self.last = k

    def host_frame(self, k):
        """Frame k on the host (readback=True; rank 0): waits for its device-to-host copy.
        Valid until frame k + host_buffers is issued."""
        s = k % self.depth
        if self.host_staging and self.stage_pending is not None and self.stage_pending[0] == k:
            self._gather_staged()
        if self.world > 1 and self.pending[s] and self.pend_no[s] == k:
            self._unpermute(s)
        self._flush_copies(upto=k)
        h = k % self.n_host
        assert self.host_no[h] == k, (k, self.host_no[h])
        self.host_ev[h].synchronize()
        return self.host[h]

    def finish(self):
        """Complete every issued frame (stream-ordered on the main stream)."""
        if self.host_staging:
            self._gather_staged()
        for s in range(self.depth):
            self._unpermute(s)
        if self.readback:
            self._flush_copies()
        if self.cuda:
            for st in self.streams:
                self.main.wait_stream(st)
        return self.frame
