"""Parity at the sizes the bench and BASELINE.json's configs run, against the
oracle (raytracer.cu:17-43 sample semantics: build-defined spp offsets, per-sample clamp,
k-ordered sum, truncating RGBA8):

- config 4 / the bench's headline: world8_stress 1920x1080 8 spp rendered exactly as bench.py
  renders it -- eight frame slots, frames on rotating streams (FramePipeline), fast kernels with
  the sky pre-pass -- on one GPU, and as 2 / 8 row-cyclic rank slices reassembled;
- config 3: world8 1920x1080 8 spp; config 2: world1 1920x1080 brute force (counters too);
- config 5 at its own size: world16 and world16_tex (textured mode) at 3840x2160, 64 spp, the
  fast frame (pipelined as bench.py renders it, and with every output) against the oracle on
  every 45th row, and the counted kernel on the same rows (fast == counted bit for bit, counters
  equal the oracle's);
- config 5's sample mapping at a reduced size: world16 and world16_tex (textured mode) at
  320x180 with spp = 64 (64 lanes per pixel, one pixel per wave, 1x1 sky cones, the generic
  reduction) and spp = 96 (the M_MULTI rounds), fast and counted kernels.
The oracle runs on up to 16 host threads (a few seconds per 1080p frame)."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, scene_path
from twin import NTHREADS, assert_frames_equal

pytestmark = pytest.mark.gpu
WANT = ("rgba", "radiance", "hit_inst", "hit_tri")
W, H = 1920, 1080


@pytest.fixture(scope="module")
def stress_1080p(oracle):
    return oracle.render(oracle.load(scene_path("world8_stress"), W, H), spp=8, nthreads=NTHREADS)


def _pipelined(gpu, scene, spp, world=1, rank=0, depth=8, n_frames=11, textures=False, size=(W, H), stream=True,
               host=False):
    """This rank's rows of the last of n_frames frames issued as bench.py issues them (its timed
    frames: RT_OVERLAP_STREAM).  host=True: the frames as bench.py's headline times them, each
    copied by a copy engine into pinned host memory and read there by a consumer that trails the
    pipeline (FramePipeline(readback=True)): the list of every frame's host copy."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
    import rtamd.dist as rtdist
    W, H = size
    s = gpu.Scene.load_json(scene_path(scene), W, H)
    if textures:
        s.load_atlas()
    s.set_frame_slots(depth)
    s.set_overlap(False, stream=stream)
    pipe = rtdist.FramePipeline(W, H, 1, 0, "cuda", depth=depth, readback=host)
    n = len(range(rank, H, world))
    frames = []
    for k in range(n_frames):
        pipe.step(k, lambda buf, st: s.render_device(spp=spp, row0=rank, row_step=world, compact=True,
                                                     rgba_ptr=buf.data_ptr(), stream=st.cuda_stream,
                                                     textures=textures))
        if host and k - pipe.n_host + 1 >= 0:
            frames.append(pipe.host_frame(k - pipe.n_host + 1)[:n].numpy().view(np.uint32).copy())
    out = pipe.finish()
    torch.cuda.synchronize()
    if host:
        for j in range(max(0, n_frames - pipe.n_host + 1), n_frames):
            frames.append(pipe.host_frame(j)[:n].numpy().view(np.uint32).copy())
        assert len(frames) == n_frames
        return frames
    return out[:n].cpu().numpy().view(np.uint32)


def test_bench_frame_world8_stress_1080p(gpu, stress_1080p):
    """The headline frame: pipelined fast frames as the bench times them (each copied to pinned
    host memory by a copy engine and read from there; every one of them checked), then one fast
    frame with every output, against the oracle."""
    host = _pipelined(gpu, "world8_stress", 8, n_frames=20, host=True)
    for k, f in enumerate(host):
        assert_frames_equal({"rgba": f}, stress_1080p, keys=("rgba",), ctx="host frame %d" % k)
    rgba = _pipelined(gpu, "world8_stress", 8)
    assert np.array_equal(rgba, host[-1])
    s = gpu.Scene.load_json(scene_path("world8_stress"), W, H)
    fr = s.render(spp=8, want=WANT, stats=False)
    assert np.array_equal(fr["rgba"], rgba)
    assert_frames_equal(fr, stress_1080p, ctx="fast")
    assert (fr["hit_inst"] >= 0).mean() > 0.1
    # the next lone frames run the previous frame's heavy groups first, dealt out statically
    # over the grid's waves (several rounds at this size): every group still exactly once
    for k in range(2):
        fr2 = s.render(spp=8, want=WANT, stats=False)
        for key in fr:
            assert np.array_equal(fr2[key], fr[key]), (k, key)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_rank_slices_world8_stress_1080p(gpu, stress_1080p, world):
    """Every rank's slice (rows r, r+N, ...; compact; one-row pixel groups at N = 8) rendered
    through its own four-deep pipeline, reassembled as rank 0's un-permute does."""
    frame = np.zeros((H, W), np.uint32)
    for r in range(world):
        frame[r::world] = _pipelined(gpu, "world8_stress", 8, world=world, rank=r, n_frames=9)
    assert_frames_equal({"rgba": frame}, stress_1080p, keys=("rgba",), ctx=world)


def test_world8_1080p_8spp(gpu, oracle):
    s = gpu.Scene.load_json(scene_path("world8"), W, H)
    fr = s.render(spp=8, want=WANT, stats=False)
    assert_frames_equal(fr, oracle.render(oracle.load(scene_path("world8"), W, H), spp=8, nthreads=NTHREADS))
    assert np.array_equal(_pipelined(gpu, "world8", 8, n_frames=9), fr["rgba"])


def test_world1_1080p_brute_force(gpu, oracle):
    """Config 2 (reference -r): every ray tests both instances; counters equal the oracle's."""
    s = gpu.Scene.load_json(scene_path("world1"), W, H)
    of = oracle.render(oracle.load(scene_path("world1"), W, H), use_bvh=0, spp=1, nthreads=NTHREADS)
    full = s.render(spp=1, use_bvh=False, want=WANT, stats=True)
    assert_frames_equal(full, of, ctx="counted")
    st = full["stats"]
    assert (st["rays"], st["nodes"], st["leaves"], st["tri_tests"]) == tuple(int(x) for x in of["stats"])
    assert st["rays"] == 2084662                               # SURVEY Appendix D (the reference's count)
    fast = s.render(spp=1, use_bvh=False, want=WANT, stats=False)
    for k in WANT:
        assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), k


@pytest.mark.parametrize("scene,textures", [("world16", False), ("world16_tex", True)])
@pytest.mark.parametrize("spp", [16, 32, 48, 64, 96])
def test_config5_sample_mapping(gpu, oracle, scene, textures, spp):
    """Config 5 (world16, 64 spp, textured) at 320x180: the 16/32/48/64-lanes-per-pixel mappings
    and the multi-round (spp > 64) kernels, fast and counted, against the oracle; counters too.
    spp 16-64 run the partially parked kernel's LDS-staged sample sums, with
    (radiance requested) and without (RGBA only) the raw-radiance channel lanes."""
    w, h = 320, 180
    s = gpu.Scene.load_json(scene_path(scene), w, h)
    o = oracle.load(scene_path(scene), w, h)
    if textures:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import make_atlas
        s.load_atlas()
        o.set_atlas(make_atlas.atlas())
        o.set_textures(True)
    of = oracle.render(o, spp=spp, nthreads=NTHREADS)
    full = s.render(spp=spp, want=WANT, stats=True, textures=textures)
    assert_frames_equal(full, of, ctx="counted")
    st = full["stats"]
    assert (st["rays"], st["nodes"], st["leaves"], st["tri_tests"]) == tuple(int(x) for x in of["stats"])
    fast = s.render(spp=spp, want=WANT, stats=False, textures=textures)
    for k in WANT:
        assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), k
    only = s.render(spp=spp, want=("rgba",), stats=False, textures=textures)
    assert np.array_equal(only["rgba"], full["rgba"])
    assert (full["hit_inst"] >= 0).mean() > 0.2


@pytest.mark.parametrize("scene,textures", [("world16", False), ("world16_tex", True)])
def test_config5_full_size(gpu, oracle, scene, textures):
    """Config 5 (BASELINE.json: world16, 3840x2160, 64 spp, textured) at its own size.  The fast
    frame -- the unparked ordered-tree kernel world16's 93 KB tree leaves room for -- rendered as
    bench.py renders it (eight frame slots, rotating streams) and once with every output; rows
    y % 45 == 0 (48 rows, 11.8 M samples) against the oracle; the counted kernel on the same rows
    equals the fast frame bit for bit and its counters equal the oracle's."""
    w, h, spp, step = 3840, 2160, 64, 45
    s = gpu.Scene.load_json(scene_path(scene), w, h)
    o = oracle.load(scene_path(scene), w, h)
    if textures:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import make_atlas
        s.load_atlas()
        o.set_atlas(make_atlas.atlas())
        o.set_textures(True)
    piped = _pipelined(gpu, scene, spp, n_frames=9, textures=textures, size=(w, h))
    fast = s.render(spp=spp, want=WANT, stats=False, textures=textures)
    assert np.array_equal(piped, fast["rgba"])
    rows = slice(0, None, step)
    of = oracle.render(o, spp=spp, row0=0, row_step=step, nthreads=NTHREADS)
    assert_frames_equal({k: fast[k][rows] for k in WANT}, {k: of[k][rows] for k in WANT}, ctx=scene)
    counted = s.render(spp=spp, row0=0, row_step=step, compact=True, want=WANT, stats=True, textures=textures)
    for k in WANT:
        assert np.array_equal(counted[k].view(np.uint32), fast[k][rows].view(np.uint32)), k
    st = counted["stats"]
    assert (st["rays"], st["nodes"], st["leaves"], st["tri_tests"]) == tuple(int(x) for x in of["stats"])
    assert (fast["hit_inst"] >= 0).mean() > 0.2


@pytest.mark.parametrize("w,h", [(203, 45), (37, 29)])
def test_config5_wide_store_runs(gpu, oracle, w, h):
    """Config 5's one-pixel groups store RGBA 16 consecutive pixels at a time (DESIGN §3.2 item 31:
    live tickets in runs of 16, a run flushed when the next pixel is not adjacent, after 64
    pixels, or when the wave leaves its loop).  Widths that are no multiple of 16, row ends inside
    a run, and compact row slices (each slice row ends a run) against the oracle, RGBA only (the
    wide path) and with every output; pipelined as bench.py issues frames."""
    spp = 64
    s = gpu.Scene.load_json(scene_path("world16"), w, h)
    of = oracle.render(oracle.load(scene_path("world16"), w, h), spp=spp, nthreads=NTHREADS)
    only = s.render(spp=spp, want=("rgba",), stats=False)
    assert np.array_equal(only["rgba"], of["rgba"]), int((only["rgba"] != of["rgba"]).sum())
    fast = s.render(spp=spp, want=WANT, stats=False)
    assert_frames_equal(fast, of, ctx="world16 %dx%d" % (w, h))
    for row0, step in [(1, 3), (0, 2)]:
        sl = s.render(spp=spp, row0=row0, row_step=step, compact=True, want=("rgba",), stats=False)
        assert np.array_equal(sl["rgba"], of["rgba"][row0::step]), (row0, step)
    piped = _pipelined(gpu, "world16", spp, world=3, rank=1, n_frames=10, size=(w, h))
    assert np.array_equal(piped, of["rgba"][1::3])
