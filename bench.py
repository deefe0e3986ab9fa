#!/usr/bin/env python3
"""Benchmark of the MI355X ray-tracing core on the reference's headline workload.

Metric (BASELINE.json): Mrays/s (primary + secondary, i.e. every closest-hit query
= the reference's cast_ray calls) and frame ms on world8_stress.json at
1920x1080, 8 spp, BVH, on N MI355X.

One step = one frame: per-frame BVH rebuild + the trace kernel over this rank's
rows (row-cyclic: y = rank, rank+N, ...), then (N > 1) an RCCL gather of the packed RGBA8
rows to rank 0 and the row un-permute, then the frame's copy into pinned host memory on a
DMA copy engine (rank 0), read by a host consumer: the reference's post-condition, the frame
host-readable when update_scene returns (raytracer.cu:102-120).  Frames are pipelined eight
deep (rtamd.dist.FramePipeline(readback=True), rt_scene_set_frame_slots): frame k+1 renders on
another stream and starts on the CUs that the previous frames' longest pixel groups leave idle,
frame k's gather runs on the collective stream meanwhile, and each host copy is issued once its
frame has completed.  The timed region ends when the last frame is on the host.
The same frames left in HBM are timed afterwards as `device_resident`; `frame_latency_ms` is
one host-readable frame issued alone and waited for, `cold_frame_ms` the first one after the
scene is loaded; `--no-overlap` times serial frames.

Units.  `value` counts rays in the reference's units (every cast_ray call of
propagate_ray, taken from a counted render of the same frame): reference-equivalent rays.
The fast kernels skip work the reference does when it provably cannot change the result
(unlit shadow rays, pruned subtrees); `queries_traced_per_frame` (rt_frame_work) is what they
actually issue, reported beside it.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 the driver
uses torch.distributed.run (one process per GPU, RCCL over xGMI).
"""
import argparse
import json
import os
import sys
import time

# Frames in flight run on their own streams; HIP maps streams round-robin onto
# GPU_MAX_HW_QUEUES hardware queues (4 by default), and streams sharing a queue serialise.
# Main + 4 render streams + the collective's stream need more than 4 (measured: three
# frames in flight 1.49 ms/frame on 4 queues, 1.41 on 8).
# HIP assigns streams to queues in creation order (zig-zag over the queues), so with 8 the
# first seven streams after the null stream are distinct; 16 leaves room for the collective's
# and the readback copy's streams on N > 1 ranks without a render stream sharing a queue
# (8 vs 16 on one GPU: equal frame and slice times).
# (HIP's default, also the pool's box setting, is 4; RT_BENCH_HW_QUEUES overrides the 16 used here.)
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_BENCH_HW_QUEUES", "16")
import torch  # first: the HIP runtime torch loads is the one librt_amd.so binds to

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402
import rtamd.dist as rtdist  # noqa: E402

METRIC = "Mrays/sec (primary+secondary) + frame ms, 1080p world8_stress, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s
# MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, 2400 MHz max clock, one wave64 VALU instruction per
# SIMD every 2 cycles -> peak VALU issue in wave-instructions per second
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2
B_NODE, B_LEAF = 28, 816        # SURVEY §8d uncached per-ray model: BoundingBox / leaf (pose+mesh+12 tris)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--scene", default="world8_stress")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=8)
    p.add_argument("--brute", action="store_true", help="reference -r: no BVH")
    p.add_argument("--textures", action="store_true",
                   help="build-defined textured shading with the scene's atlas (e.g. --scene world16_tex, config 5)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample-rows", type=int, default=1, help="CPU baseline renders rows y %% k == 0")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--pmc-step", default=os.path.join(ROOT, "profiles", "pmc_step.json"),
                   help="counters summed over the timed window of this command under rocprofv3 (tools/pmc_step.py)")
    p.add_argument("--dump-frame", default="",
                   help="rank 0 saves the last timed frame (gathered, un-permuted RGBA8) as .npy (tests)")
    p.add_argument("--cpu-runs", type=int, default=3, help="CPU baseline: timed 1-thread frames (median), after one warm-up")
    p.add_argument("--no-camera-path", action="store_true",
                   help="skip the moving-camera figure (camera_path: main.cc's key and mouse steps every frame)")
    p.add_argument("--no-kernel-timing", action="store_true",
                   help="no per-frame HIP events (then trace_kernel_ms / roofline are not measured)")
    p.add_argument("--no-overlap", action="store_true", help="serial frames (no frame pipeline)")
    p.add_argument("--frames-in-flight", type=int, default=8, help="frame pipeline depth (1-8)")
    p.add_argument("--copy-streams", type=int, default=2,
                   help="host-readable pipeline: copy streams the frames' copies alternate over "
                        "(rtamd.dist.FramePipeline copy_streams; DESIGN.md 4.2)")
    p.add_argument("--copy-lag", type=int, default=None,
                   help="host-readable pipeline: the host waits for frame k - L's copy as it issues frame k "
                        "(default depth - 1; rtamd.dist.FramePipeline copy_lag)")
    p.add_argument("--grid", default=os.environ.get("RT_BENCH_GRID", "stream"),
                   choices=("stream", "half", "full", "last-full", "stream-last-full"),
                   help="grid of the timed frames (rt_scene_set_overlap): stream (default: the steady state a "
                        "caller that always has another frame behind sees) = half the CUs for every frame, "
                        "the first included (RT_OVERLAP_STREAM); stream-last-full = stream, with the timed "
                        "region's last frame on every CU (no frame follows it; DESIGN.md 4.1); "
                        "half = half the CUs for a frame issued while "
                        "another runs; full = every CU; last-full = half except the timed region's last frame; "
                        "stream-last-full = stream except the timed region's last frame (every CU)")
    p.add_argument("--no-device-resident", action="store_true",
                   help="skip the device-resident figure (the same K frames left in HBM)")
    p.add_argument("--pmc-window", default="host", choices=("host", "device"),
                   help="the window bench.py's profile markers bracket (tools/pmc_step.py): the headline's "
                        "host-readable frames, or the same frames device-resident.  Under rocprofv3 a torch "
                        "process's copy-engine transfers fall back to blit kernels (DESIGN.md 4.2), so the "
                        "counters of the headline's kernels are taken from the device-resident window")
    p.add_argument("--frame-crcs", action="store_true",
                   help="rank 0 reports the CRC-32 of every timed host frame (tests: each frame the pipeline "
                        "assembles, not only the last)")
    p.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                   help="nccl = RCCL over xGMI (the driver's runs); gloo stages the gather through host "
                        "memory and lets several ranks share one GPU (testing the N > 1 path on one GPU)")
    return p.parse_args()


def lib_sha16():
    """The product library this run loaded (profiles/pmc_step.json entries record it too)."""
    import hashlib
    try:
        return hashlib.sha256(open(rtamd.LIB_PATH, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def cgroup_cpu_quota():
    """CPUs this job's cgroup may use (cgroup v2 cpu.max = "quota period", v1 cfs files), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(args, scene_path):
    """The reference's CPU path (src/raytracer.cc semantics, restated in oracle/) on a
    bounded sample of the same workload, 1 thread -- the reference's CPU path is serial
    (SURVEY §8d).  Beside it, the GPU-semantics restatement on the host cores this job
    may use (apples-to-apples work, OpenMP-style row split)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle
    orc = Oracle()
    s = orc.load(scene_path, args.width, args.height)
    k = max(1, args.cpu_sample_rows)
    bvh = 0 if args.brute else 1
    # BASELINE.md §3's protocol: one warm-up, then the median of `cpu_runs` timed 1-thread runs
    # (the warm-up renders every 8th row of the sample: it pages the scene and code in)
    orc.render(s, semantics=1, use_bvh=bvh, spp=1, row0=0, row_step=8 * k, nthreads=1, want=())
    runs = []
    for _ in range(max(1, args.cpu_runs)):
        t = time.perf_counter()
        fr = orc.render(s, semantics=1, use_bvh=bvh, spp=1, row0=0, row_step=k, nthreads=1, want=())
        runs.append(time.perf_counter() - t)
    dt = sorted(runs)[len(runs) // 2]
    rays = int(fr["stats"][0])
    rows = len(range(0, args.height, k))
    # every core this job may run on (its CPU affinity), not the machine's count: a GPU box shares
    # its host between jobs and pins each to its share
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = cgroup_cpu_quota()              # a CPU-time quota caps the job below its affinity mask
    nthr = max(1, min(affinity, quota) if quota else affinity)
    t = time.perf_counter()
    fg = orc.render(s, semantics=0, use_bvh=bvh, spp=1, row0=0, row_step=k, nthreads=nthr, want=())
    dg = time.perf_counter() - t
    # the same CPU path row-split over the job's host cores (BASELINE.md §3's all-core variant;
    # the reference's CPU path is one serial pixel loop, raytracer.cc:49-50)
    t = time.perf_counter()
    fc = orc.render(s, semantics=1, use_bvh=bvh, spp=1, row0=0, row_step=k, nthreads=nthr, want=())
    dc = time.perf_counter() - t
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        cpu_model = "unknown"
    return {
        "value": rays / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
        "sample": "%s %dx%d rows y%%%d==0 (%d rows), spp=1, CPU-path semantics of src/raytracer.cc "
                  "(oracle restatement), 1 thread; median of %d runs after a warm-up: %.1f s, %d rays; "
                  "extrapolated frame at %d spp: %.0f ms"
                  % (args.scene, args.width, args.height, k, rows, len(runs), dt, rays, args.spp, dt * k * args.spp * 1e3),
        "runs_s": [round(x, 3) for x in runs],
        "spread": round((max(runs) - min(runs)) / dt, 4),
        "cpu_path_all_cores": {"value": int(fc["stats"][0]) / dc / 1e6, "unit": "Mrays/s", "cores": nthr,
                               "seconds": round(dc, 2), "kind": "port"},
        "gpu_semantics_all_cores": {"value": int(fg["stats"][0]) / dg / 1e6, "unit": "Mrays/s", "cores": nthr,
                                    "seconds": round(dg, 2)},
        "cpu_model": cpu_model, "nproc": os.cpu_count(), "affinity_cores": affinity, "cgroup_cpu_quota": quota,
        "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
    }


# main.cc's camera steps (main.cc:19-20, 144-177): the W key translates the camera by
# (0, 0, MOVE_SPEED) in its own frame; a mouse motion of (xrel, yrel) = (1, 0) turns it by
# Quat(up, ROT_SPEED * 1) * Quat(right, ROT_SPEED * 0) (rel_mot normalized: (1, 0)).
MOVE_SPEED, ROT_SPEED = 0.2, 0.01


def _quat_axis_angle(axis, theta):
    """geometry.h:36-41 as a g++ TU computes it: double cos / sin of the float 0.5f * theta,
    rounded to float (include/rtracer_amd.hpp, tests/test_shim_math.py)."""
    import math
    import numpy as np
    h = float(np.float32(0.5) * np.float32(theta))
    hc, hs = np.float32(math.cos(h)), np.float32(math.sin(h))
    a = np.asarray(axis, np.float32)
    return np.array([a[0] * hs, a[1] * hs, a[2] * hs, hc], np.float32)


def _quat_mul(a, b):
    """geometry.h:161-174 (Hamilton product, the reference's operand order) in float32."""
    import numpy as np
    i, j, k, r = [np.float32(x) for x in a]
    bi, bj, bk, br = [np.float32(x) for x in b]
    return np.array([i * br + r * bi + j * bk - k * bj, j * br + r * bj + k * bi - i * bk,
                     k * br + r * bk + i * bj - j * bi, r * br - i * bi - j * bj - k * bk], np.float32)


def _normalized(v):
    """Vec::normalized (linear.h:159-167): (1 / len) * v above the 1e-5 threshold."""
    import numpy as np
    v = np.asarray(v, np.float32)
    n = np.float32(np.sqrt(np.float32(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]))
    return (np.float32(1.0) / n) * v if n > np.float32(1e-5) else np.zeros(3, np.float32)


def camera_move(scene):
    """One frame of main.cc's interactive caller: the W key, then a one-pixel mouse motion."""
    scene.translate_camera((0.0, 0.0, MOVE_SPEED))                         # main.cc:146-148
    r, u, _ = scene.camera_axes()
    rot = _quat_mul(_quat_axis_angle(_normalized(u), ROT_SPEED * 1.0),     # main.cc:173-177
                    _quat_axis_angle(_normalized(r), ROT_SPEED * 0.0))
    scene.rotate_camera(rot)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = max(world, 1)
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist = None
    gloo = world > 1 and args.dist_backend == "gloo"
    if world > 1:
        import torch.distributed as dist
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    rtamd.set_device(dev)
    depth = max(1, min(8, args.frames_in_flight))
    overlap = not args.no_overlap and depth > 1
    H0, W0 = args.height, args.width
    if overlap:
        # frames in flight (rtamd.dist.FramePipeline).  `fbr` copies every finished frame to pinned
        # host memory on a copy engine (the reference's post-condition: the headline); `fb` leaves
        # frames in HBM (the device-resident figure).  Both share the render streams, created and
        # first used here, before the scene exists: a torch stream's HIP stream is created at its
        # first use (1-7 ms each, profiles/r06/cold/), the caller's one-time cost, not a frame's.
        fbr = rtdist.FramePipeline(W0, H0, world, rank, "cuda", dist, depth=depth, readback=True, host_staging=gloo,
                                   copy_lag=args.copy_lag, copy_streams=args.copy_streams)
        fb = rtdist.FramePipeline(W0, H0, world, rank, "cuda", dist, depth=depth, streams=fbr.streams,
                                  host_staging=gloo)
        for st_ in fbr.streams + [c for c in getattr(fbr, "copy_streams", []) if c is not None]:
            torch.cuda.Event().record(st_)
        torch.cuda.synchronize()
    scene_path = os.path.join(ROOT, "scenes", args.scene + ".json")
    # procedural::gpu::generate: the scene goes to the device and one untimed frame warms it
    # (rt_scene_load_json with a gfx950 device present, include/rt_amd.h)
    t_load = time.perf_counter()
    scene = rtamd.Scene.load_json(scene_path, args.width, args.height)
    if args.textures:
        scene.load_atlas()
    if overlap:
        scene.set_frame_slots(depth)
    torch.cuda.synchronize()
    load_ms = (time.perf_counter() - t_load) * 1e3
    W, H = scene.width, scene.height
    assert (W, H) == (W0, H0), (W, H, W0, H0)
    my_rows = len(rtdist.rows_of(rank, world, H))
    stream = torch.cuda.current_stream()
    use_bvh = not args.brute
    frame_no = [0]
    if not overlap:                       # serial frames; RCCL gather of frame k overlaps frame k+1
        fb = rtdist.RowCyclicFrame(W, H, world, rank, "cuda", dist, host_staging=gloo, slots=2)
        fbr = None
    part = fb.parts[0]

    def render(buf, st, timing):
        scene.render_device(spp=args.spp, use_bvh=use_bvh, rebuild_bvh=True, row0=rank, row_step=world,
                            compact=True, rgba_ptr=buf.data_ptr(), stream=st.cuda_stream,
                            timing=timing, textures=args.textures)

    def step(timing, pipe=None):
        """Issue one frame (device-resident pipeline unless `pipe` is given)."""
        k = frame_no[0]
        frame_no[0] += 1
        if overlap:
            (pipe or fb).step(k, lambda buf, st: render(buf, st, timing))
        else:
            render(fb.slot_part(k), stream, timing)
            fb.gather(k)
        return k

    def host_step(timing=False):
        """Issue one host-readable frame; returns its number."""
        if overlap:
            return step(timing, fbr)
        return step(timing)

    def host_read(k):
        """Rank 0: frame k on the host (waits for its copy-engine transfer)."""
        if overlap:
            return fbr.host_frame(k)
        fb.finish()
        return fb.frame.cpu()

    def set_grid(last=False):
        if not overlap:
            return
        if args.grid == "full" or (last and args.grid in ("last-full", "stream-last-full")):
            scene.set_overlap(True)                         # nothing is issued behind the last frame
        elif args.grid in ("stream", "stream-last-full"):
            scene.set_overlap(False, stream=True)           # the timed frames are issued back to back
        else:
            scene.set_overlap(False)

    crcs = {}

    def consume(k, lag, first=0):
        """Rank 0's host consumer: reads frame k - lag (from `first` on: the frames issued through
        the host-readable pipeline), in order (the reference's caller blits the canvas after every
        update_scene, main.cc:180-196)."""
        j = k - lag
        if rank == 0 and j >= first and (overlap or lag == 0):
            h = host_read(j)
            if args.frame_crcs:
                import zlib
                crcs[j] = zlib.crc32(h.numpy().tobytes())

    lag = (fbr.n_host - 1) if overlap else 0

    def host_frames(n, moving=False, last_full=True):
        """n host-readable frames issued back to back, each read by the host consumer; returns the
        first and last frame numbers.  The caller brackets the timing."""
        set_grid()
        first = None
        for i in range(n):
            if moving:
                camera_move(scene)
            if last_full and i == n - 1:
                set_grid(last=True)
            k = host_step()
            first = k if first is None else first
            consume(k, lag, first)
        if overlap:
            fbr.finish()
        if rank == 0:
            for j in range(max(first, k - lag + 1) if overlap else k + 1, k + 1):   # the frames still unread
                consume(j, 0)
        torch.cuda.synchronize()
        if overlap:
            scene.set_overlap(False)
        return first, k

    # The reference's own benchmark (main.cc:210-216): the first frame after the scene is made,
    # host-readable (here: the first host-readable frame after load, at this run's spp and size).
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    tc = time.perf_counter()
    k0 = host_step()
    if overlap:
        fbr.finish()
    if rank == 0:
        host_read(k0)
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - tc) * 1e3
    # per-frame work counters (deterministic): one untimed counted render of this rank's rows
    st = scene.render_device(spp=args.spp, use_bvh=use_bvh, rebuild_bvh=True, row0=rank, row_step=world,
                             compact=True, rgba_ptr=part.data_ptr(), stream=stream.cuda_stream, sync=True, stats=True,
                             textures=args.textures)
    if args.warmup > 1:
        host_frames(args.warmup - 1)
    scene.timing_collect()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()

    # ---- the headline: K host-readable frames (to the framebuffer on the host,
    # gathered to rank 0 for N > 1) ----
    crcs.clear()
    if args.pmc_window == "host":
        rtamd.profile_marker(1, stream.cuda_stream)         # the timed window starts (tools/pmc_step.py)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    f_first, f_last = host_frames(args.steps, last_full=True)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if args.pmc_window == "host":
        rtamd.profile_marker(2, stream.cuda_stream)         # ... and ends
    timed_crcs = [crcs.get(j) for j in range(f_first, f_last + 1)]
    if args.dump_frame and rank == 0:
        import numpy as np
        np.save(args.dump_frame, host_read(f_last).numpy().view(np.uint32) if overlap else fb.frame.cpu().numpy().view(np.uint32))

    # ---- the same frames left in HBM (no host copy): the device-resident figure ----
    dev_s = None
    if not args.no_device_resident:
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        set_grid()
        if args.pmc_window == "device":
            rtamd.profile_marker(1, stream.cuda_stream)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for i in range(args.steps):
            if i == args.steps - 1:
                set_grid(last=True)
            step(False)
        fb.finish()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        dev_s = time.perf_counter() - t2
        if args.pmc_window == "device":
            rtamd.profile_marker(2, stream.cuda_stream)
        if overlap:
            scene.set_overlap(False)
    tm = scene.timing_collect()
    # latency of one host-readable frame issued alone (render + gather + un-permute + copy to the
    # host, waited for); with frames in flight the kernels' event-timed durations come from these
    # lone frames (a launch that overlaps other frames' kernels runs longer than its cost)
    lat = []
    for _ in range(max(3, args.steps // 2)):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        k = host_step(not args.no_kernel_timing)
        if overlap:
            fbr.finish()
        if rank == 0:
            host_read(k)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t3)
    lat_ms = sorted(lat)[len(lat) // 2] * 1e3
    tm = scene.timing_collect()
    # this box's copy-engine rate for one full frame to pinned host memory, alone (rank 0; the
    # rate is a property of the box at the time of the call -- 29 or 53 GB/s seen)
    copy_rate = None
    if overlap and rank == 0 and fbr is not None and fbr.copy_stream is not None:
        src = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        hb = rtamd.HostBuffer((H, W), "int32")
        cs = fbr.copy_stream
        cs.wait_stream(torch.cuda.current_stream())
        for rep in range(2):
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record(cs)
            for _ in range(20):
                rtamd.copy_to_host_async(hb.ptr, src.data_ptr(), 4 * W * H, cs.cuda_stream)
            c1.record(cs)
            cs.synchronize()
        cms = c0.elapsed_time(c1) / 20
        copy_rate = {"frame_copy_ms": round(cms, 4), "GBs": round(4 * W * H / (cms * 1e-3) / 1e9, 1),
                     "source": "20 back-to-back frame copies on the copy stream, event-timed, after the timed windows"}
        hb.free()
        del src
    # Moving camera (the reference's real caller moves it every frame, main.cc:140-180): the
    # same K host-readable frames with main.cc's key and mouse steps applied before each, so the
    # previous frame's heavy-group flags (history-driven scheduling) are one pose stale.
    # Rays in the reference's units from a counted replay of the same poses (untimed).
    cam_path = None
    if not args.no_camera_path:
        pos0, quat0 = scene.camera()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        tc0 = time.perf_counter()
        host_frames(args.steps, moving=True)
        if dist:
            dist.barrier()
        cam_s = time.perf_counter() - tc0
        scene.set_camera(pos0, quat0)
        cam_rays = 0
        for i in range(args.steps):
            camera_move(scene)
            cst = scene.render_device(spp=args.spp, use_bvh=use_bvh, rebuild_bvh=True, row0=rank, row_step=world,
                                      compact=True, rgba_ptr=part.data_ptr(), stream=stream.cuda_stream, sync=True,
                                      stats=True, textures=args.textures)
            cam_rays += int(cst["rays"])
        scene.set_camera(pos0, quat0)
        cam_path = (cam_s, cam_rays)
    # what the fast kernels actually do for this rank's rows (profiling run, untimed)
    try:
        work = scene.frame_work(spp=args.spp, row0=rank, row_step=world, compact=True) \
            if (use_bvh and not args.textures and args.spp <= 64) else None
    except rtamd.RtError:
        work = None

    red_dev = "cpu" if gloo else "cuda"
    local_rays = torch.tensor([st["rays"], st["nodes"], st["leaves"], st["tri_tests"],
                               work["queries"] if work else 0, work["leaf_lanes"] if work else 0],
                              dtype=torch.float64, device=red_dev)
    tmax = torch.tensor([elapsed, dev_s if dev_s is not None else 0.0], dtype=torch.float64, device=red_dev)
    if dist:
        dist.all_reduce(local_rays, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    rays, nodes, leaves, tris, queries, leaf_lanes = [float(x) for x in local_rays.cpu()]
    elapsed, dev_s = float(tmax[0].item()), (float(tmax[1].item()) if dev_s is not None else None)
    if cam_path:
        cp = torch.tensor([cam_path[0], float(cam_path[1])], dtype=torch.float64, device=red_dev)
        cps = cp[1:].clone()
        if dist:
            dist.all_reduce(cp[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(cps, op=dist.ReduceOp.SUM)
        cam_path = (float(cp[0].item()), float(cps[0].item()))
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    value = rays * args.steps / elapsed / 1e6
    # Dominant kernel: the trace stage (sky pre-pass + trace kernel) of a lone frame, event-timed
    # on the launch stream (with frames in flight a launch that overlaps other frames' kernels
    # runs longer than its cost).  This rank's rows.
    trace_ms = tm["trace_ms_total"] / max(1, tm["frames"])
    if tm["frames"] == 0:                                   # --no-kernel-timing: fall back to the step time
        trace_ms = ms_per_step
    bvh_ms = tm["bvh_ms_total"] / max(1, tm["frames"])
    frame_bytes = 4 * W * my_rows
    traffic, issue = None, {}
    if os.path.exists(args.pmc):
        try:
            pm = json.load(open(args.pmc))
            key = "%s_%dx%d_spp%d_n%d" % (args.scene, W, H, args.spp, world)
            traffic = pm.get(key, {}).get("hbm_bytes_per_launch")
            issue = pm.get(key, {}).get("issue", {})
        except Exception:
            traffic, issue = None, {}
    # Algorithmic (compulsory) bytes of one launch: the scene the kernel reads (the ordered
    # tree, instance, triangle, mesh, material and light records: rt_work.scene_bytes) plus the
    # RGBA8 frame it writes.  Everything else is re-reads the LDS/L2 serve.
    algo_bytes = frame_bytes + (work["scene_bytes"] if work else 0)
    ref_bytes = B_NODE * nodes / world + B_LEAF * leaves / world + frame_bytes   # this rank's share
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": traffic,
            "binding": None,
            "algorithmic_bytes_per_launch": int(algo_bytes),
            "algorithmic_GBs": round(algo_bytes / (trace_ms * 1e-3) / 1e9, 3),
            "launch_ms": round(trace_ms, 4)}
    if traffic:
        # measured: HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, rocprofv3 --pmc of the same
        # frame at HEAD, profiles/pmc_traffic.json) over the event-timed launch
        achieved = traffic / (trace_ms * 1e-3) / 1e9
        roof.update(achieved=round(achieved, 2), frac=round(achieved / HBM_PEAK_GBS, 4),
                    traffic_over_algorithmic=round(traffic / max(1, algo_bytes), 2),
                    source="achieved = measured HBM bytes per launch (profiles/pmc_traffic.json) / event-timed launch")
    else:
        achieved = algo_bytes / (trace_ms * 1e-3) / 1e9
        roof.update(achieved=round(achieved, 3), frac=round(achieved / HBM_PEAK_GBS, 5),
                    source="achieved = algorithmic bytes / event-timed launch (no PMC profile for this config)")
    ref_gbs = ref_bytes / (trace_ms * 1e-3) / 1e9
    roof["reference_equivalent"] = {
        "bytes_per_launch": int(ref_bytes), "GBs": round(ref_gbs, 1), "frac": round(ref_gbs / HBM_PEAK_GBS, 2),
        "note": "SURVEY 8d uncached model in the reference's units (28 B per BVH node test + 816 B per leaf, "
                "counts of the reference traversal) -- not HBM traffic: frac exceeds 1, so the kernel cannot be "
                "doing this work from HBM; LDS residency of the tree and scene and the exact pruning serve it"}
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32",
        "data": "procedural scene from the reference's %s.json (deterministic, no RNG at render time)" % args.scene,
        "config": {"workload": "%s.json %dx%d %dspp %s%s" % (args.scene, W, H, args.spp, "brute" if args.brute else "BVH",
                                                          " textured" if args.textures else ""),
                   "scene": args.scene, "width": W, "height": H, "spp": args.spp, "bvh": use_bvh,
                   "parallelism": ("row-cyclic x%d + %s gather" % (world, "gloo host-staged" if gloo else "RCCL"))
                                  if world > 1 else "single GPU",
                   # HIP hardware queues per process (HIP's and the pool's default is 4; bench.py sets 16
                   # so that four render streams + main + collective + copy each get a queue)
                   "gpu_max_hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]), "frames_in_flight": depth if overlap else 1,
                   "grid_timed_frames": args.grid if overlap else "full"},
        "build": {"lib_sha16": lib_sha16()}, "pmc_window": args.pmc_window,
        "rays_unit": "reference-equivalent rays: every cast_ray of the reference's propagate_ray (SURVEY 8d), "
                     "counted by the counted kernel on the same frame",
        "frame_ms": round(ms_per_step, 4),
        "timed_to": "host-readable frames: every timed frame (rank 0: gathered and un-permuted) copied to pinned "
                    "host memory by a copy engine and read by a host consumer; the window ends when the last "
                    "frame is on the host (the reference's update_scene post-condition, raytracer.cu:102-120)",
        "cold_frame_ms": round(cold_ms, 4), "scene_load_ms": round(load_ms, 3),
        "cold_frame_note": "the first host-readable frame after scene load (main.cc:210-216's bench: the first "
                           "update_scene after generate); scene_load_ms = load + upload + one untimed warm frame",
        "frame_latency_ms": round(lat_ms, 4), "frames_in_flight": depth if overlap else 1,
        "rays_per_frame": int(rays), "nodes_per_frame": int(nodes), "leaves_per_frame": int(leaves),
        "tri_tests_per_frame": int(tris), "trace_kernel_ms": round(trace_ms, 4), "bvh_build_ms": round(bvh_ms, 4),
        "roofline": roof,
    }
    if dev_s is not None:
        out["device_resident"] = {
            "ms_per_step": round(dev_s / args.steps * 1e3, 4), "value": round(rays * args.steps / dev_s / 1e6, 3),
            "unit": "Mrays/s", "note": "the same K frames left in HBM (no host copy), measured after the headline"}
    if copy_rate:
        out["copy_engine"] = copy_rate
    if args.frame_crcs and rank == 0:
        out["frame_crcs"] = timed_crcs
    if work:
        out["queries_traced_per_frame"] = int(queries)
        out["queries_traced_Mrays_s"] = round(queries * args.steps / elapsed / 1e6, 3)
        out["leaf_visits_traced_per_frame"] = int(leaf_lanes)
        if rank == 0 and work.get("live_wave_queries"):
            # lane occupancy of the wave-collective closest-hit query (rank 0's rows): every query,
            # and the live groups' queries only (the sky groups' one all-lane query each is answered
            # by the pre-pass in the product kernel); lanes by integrator phase; the live wave queries
            # by active lanes (buckets of 8) with their child-pair steps and leaf visits
            hw, hp, hl = work["hist_wave_queries"], work["hist_pair_steps"], work["hist_leaf_visits"]
            out["query_occupancy"] = {
                "all": round(work["queries"] / (64.0 * max(1, work["wave_queries"])), 4),
                "live_groups": round(work["live_lanes"] / (64.0 * work["live_wave_queries"]), 4),
                "lanes_by_phase": {"primary": work["lanes_primary"], "secondary": work["lanes_secondary"],
                                   "shadow": work["lanes_shadow"], "unlit_skipped": work["lanes_unlit"]},
                "live_wave_queries": work["live_wave_queries"],
                "live_hist_active_lanes": ["%d-%d" % (8 * i + 1, 8 * i + 8) for i in range(8)],
                "live_hist_wave_queries": hw, "live_hist_pair_steps": hp, "live_hist_leaf_visits": hl,
                "pair_steps_below_half_occupancy": round(sum(hp[:4]) / max(1, sum(hp)), 4),
                "source": "rt_frame_work (the fast kernel's profiling variant, untimed)"}
    if issue.get("SQ_INSTS_VALU"):
        # what bounds the kernel in fact: VALU issue plus dependent latency.
        # VALU wave-instructions per launch from the committed PMC profile, over this run's
        # event-timed kernel duration
        rate = issue["SQ_INSTS_VALU"] / (trace_ms * 1e-3)
        out["issue_bound"] = {"bound": "valu_issue", "achieved": round(rate / 1e9, 2), "peak": VALU_ISSUE_PEAK / 1e9,
                              "unit": "G wave-instr/s", "frac": round(rate / VALU_ISSUE_PEAK, 4),
                              "valu_insts_per_launch": int(issue["SQ_INSTS_VALU"]),
                              "source": "profiles/pmc_traffic.json (SQ_INSTS_VALU)"}
    # The timed step itself: counters summed over every dispatch between
    # this command's profile markers under rocprofv3 (tools/profile_step.sh, tools/pmc_step.py;
    # profiles/pmc_step.json), per step, over this run's ms_per_step.  The lone-launch figures
    # above describe one frame alone; these describe the pipelined step the metric times.
    pst = None
    if os.path.exists(args.pmc_step):
        try:
            pst = json.load(open(args.pmc_step)).get("%s_%dx%d_spp%d_n%d" % (args.scene, W, H, args.spp, world))
        except Exception:
            pst = None
    if pst and pst.get("hbm_bytes_per_step"):
        b = pst["hbm_bytes_per_step"]
        a = b / (ms_per_step * 1e-3) / 1e9
        roof["per_step"] = {"traffic": int(b), "achieved": round(a, 2), "frac": round(a / HBM_PEAK_GBS, 5),
                            "traffic_over_algorithmic": round(b / max(1, algo_bytes), 2),
                            "gpu_busy_ms_per_step": round(pst.get("gpu_busy_ms_per_step", 0.0), 4),
                            "profiled_ms_per_step": pst.get("profiled_ms_per_step"),
                            "kernel_ms_per_step": pst.get("kernel_ms_per_step"),
                            "source": "FETCH_SIZE x 2 + WRITE_SIZE summed over the timed window's dispatches "
                                      "(bench.py's markers, %d steps) / steps, over this run's ms_per_step; "
                                      "busy = union of the window's kernel intervals / steps (%s)"
                                      % (pst["steps"], pst.get("source", "profiles/pmc_step.json"))}
    if pst and pst.get("per_step", {}).get("SQ_INSTS_VALU") and "issue_bound" in out:
        ps = pst["per_step"]
        rate = ps["SQ_INSTS_VALU"] / (ms_per_step * 1e-3)
        d = {"valu_insts_per_step": int(ps["SQ_INSTS_VALU"]), "achieved": round(rate / 1e9, 2),
             "frac": round(rate / VALU_ISSUE_PEAK, 4)}
        if ps.get("SQ_WAVE_CYCLES"):
            d["wave_time_split"] = {k: round(ps[c] / ps["SQ_WAVE_CYCLES"], 4) for k, c in
                                    (("issuing", "SQ_ACTIVE_INST_ANY"), ("waiting", "SQ_WAIT_ANY"),
                                     ("issue_stalled", "SQ_WAIT_INST_ANY")) if c in ps}
        d["source"] = "SQ counters summed over the timed window's dispatches / steps (profiles/pmc_step.json)"
        out["issue_bound"]["per_step"] = d
    if pst:
        # the profiled window must be this run's kind of window: grid policy, frames in
        # flight, what the timed region ends on, and the library build
        # (the window may be the device-resident one: same frames and kernels, the host copies run
        # on copy engines that these counters do not see)
        want = {"grid_timed_frames": out["config"]["grid_timed_frames"], "frames_in_flight": out["frames_in_flight"],
                "lib_sha16": lib_sha16()}
        have = pst.get("window", {})
        stale = sorted(k for k, v in want.items() if have.get(k) != v)
        for blk in (roof.get("per_step"), out.get("issue_bound", {}).get("per_step")):
            if blk is not None:
                blk["matches_this_run"] = not stale
                blk["profiled_window"] = have.get("timed_to")
                if stale:
                    blk["differs_in"] = {k: [have.get(k), want[k]] for k in stale}
    # What binds.  HBM is far below its roof (roofline.frac); the kernel is
    # bound by VALU issue plus the traversal step's dependent latency, so the
    # binding fraction is VALU wave-instructions issued over the CU array's issue peak.
    if "issue_bound" in out:
        ib = out["issue_bound"]
        ps = ib.get("per_step")
        src = ps if (ps and ps.get("matches_this_run", True)) else ib
        roof["binding"] = {
            "resource": "valu_issue", "frac": src["frac"], "achieved": src["achieved"], "peak": ib["peak"],
            "unit": ib["unit"], "over": "the pipelined step (timed window's counters)" if src is ps else
            "the lone trace launch", "lone_launch_frac": ib["frac"],
            "note": "HBM frac above is the roofline the contract names; the kernel's binding resource is "
                    "instruction issue (wave time: issuing / waiting on LDS and scalar loads / issue-stalled)"}
    if cam_path:
        out["camera_path"] = {
            "ms_per_step": round(cam_path[0] / args.steps * 1e3, 4), "steps": args.steps,
            "Mrays_s": round(cam_path[1] / cam_path[0] / 1e6, 3), "rays_per_frame_mean": int(cam_path[1] / args.steps),
            "move": "per frame: Camera::translate({0, 0, %g}) and rotate(Quat(up, %g) * Quat(right, 0)) -- main.cc's W "
                    "key and a one-pixel mouse motion (main.cc:144-177)" % (MOVE_SPEED, ROT_SPEED),
            "note": "same pipeline as the headline with the camera moved before every frame; rays from a counted "
                    "replay of the same poses; value stays on the static headline camera (BASELINE config)"}
    if not args.no_cpu_baseline and world == 1:       # the CPU baseline: rank 0 at N = 1 only
        out["cpu_baseline"] = cpu_baseline(args, scene_path)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
