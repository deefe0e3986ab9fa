"""GPU parity tests of the hot path: full frames from the HIP trace kernel (through
the C ABI) against the oracle on the same scenes.

Bar (BASELINE north_star): primary hit indices (instance, triangle) identical
pixel-for-pixel; radiance within 1e-5 relative; counters (rays / BVH nodes /
leaves / triangle tests) identical; RGBA8 identical except where a 1-ulp
radiance difference crosses a byte boundary (pow is not bit-reproducible,
DESIGN.md §Exactness) — such bytes may differ by exactly 1.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, scene_path
from twin import NTHREADS, Twin, assert_frames_equal, mirror_camera

pytestmark = pytest.mark.gpu
WANT = ("rgba", "radiance", "hit_inst", "hit_tri")


def orc_check(oracle, o, fr, spp, row0=0, row_step=1, compact=False, use_bvh=1, ctx=""):
    """fr (a product frame) against the oracle's render of the same rows of scene o."""
    of = oracle.render(o, spp=spp, use_bvh=use_bvh, row0=row0, row_step=row_step, nthreads=NTHREADS)
    if compact:
        of = {k: (v[row0::row_step] if k != "stats" else v) for k, v in of.items()}
    assert_frames_equal(fr, of, keys=[k for k in WANT if k in fr], ctx=ctx)
    return of

RAD_RTOL = 1e-5


def check_frame(gpu_fr, orc_fr, spp=1):
    assert np.array_equal(gpu_fr["hit_inst"], orc_fr["hit_inst"])
    assert np.array_equal(gpu_fr["hit_tri"], orc_fr["hit_tri"])
    a, b = gpu_fr["radiance"].astype(np.float64), orc_fr["radiance"].astype(np.float64)
    err = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
    err[(a == b)] = 0
    assert err.max() <= RAD_RTOL, float(err.max())
    ga = gpu_fr["rgba"].view(np.uint8).astype(int)
    oa = orc_fr["rgba"].view(np.uint8).astype(int)
    d = np.abs(ga - oa)
    assert d.max() == 0, (int(d.max()), int((d > 0).sum()))     # RGBA8 byte-exact (twin.assert_frames_equal)
    return 0


@pytest.mark.parametrize("scene,w,h,bvh,spp", [
    ("world1", 256, 256, 1, 1),
    ("world1", 320, 240, 0, 1),          # brute force (config 2 mode)
    ("world8", 320, 240, 1, 1),
    ("world8_stress", 320, 240, 1, 1),
    ("world8_stress", 160, 120, 1, 8),
    ("world16", 256, 192, 1, 1),
    ("config", 200, 150, 1, 2),
])
def test_frame_parity(gpu, oracle, scene, w, h, bvh, spp):
    s = gpu.Scene.load_json(scene_path(scene), w, h)
    fr = s.render(spp=spp, use_bvh=bool(bvh), want=("rgba", "radiance", "hit_inst", "hit_tri"))
    o = oracle.render(oracle.load(scene_path(scene), w, h), use_bvh=bvh, spp=spp, nthreads=8)
    check_frame(fr, o, spp)
    st = fr["stats"]
    assert (st["rays"], st["nodes"], st["leaves"], st["tri_tests"]) == tuple(int(x) for x in o["stats"])


def test_golden_fixture_frames(gpu):
    """The committed oracle frames (GPU semantics) reproduce on the device."""
    import glob
    for f in sorted(glob.glob(os.path.join(GOLDEN, "frame_*_gpu.npz"))):
        name = os.path.basename(f)[len("frame_"):-4].split("_")
        spp, bvh = int(name[-2][3:]), name[-3] == "bvh"
        w, h = map(int, name[-4].split("x"))
        scene = "_".join(name[:-4])
        g = np.load(f)
        s = gpu.Scene.load_json(scene_path(scene), w, h)
        fr = s.render(spp=spp, use_bvh=bvh, want=("rgba", "radiance", "hit_inst", "hit_tri"))
        check_frame(fr, {k: g[k] for k in ("rgba", "radiance", "hit_inst", "hit_tri")}, spp)


def test_update_scene_postcondition(gpu, oracle):
    """rt_update_scene == rtracer::gpu::update_scene: frame complete and host-readable on return."""
    s = gpu.Scene.load_json(scene_path("world8"), 200, 120)
    s.update_scene(kernel_dim=16, optimize=True)
    c = s.canvas()
    o = oracle.render(oracle.load(scene_path("world8"), 200, 120), spp=1, nthreads=8, want=("rgba",))
    assert np.array_equal(c, o["rgba"])
    y, x = 60, 100
    v = int(c[y, x])
    assert s.get_color(x, y) == ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)
    s.update_scene(kernel_dim=8, optimize=False)          # brute force gives the same image
    assert np.array_equal(s.canvas(), c)


@pytest.mark.parametrize("G,spp", [(3, 2), (8, 8)])
def test_row_slices_compose(gpu, G, spp):
    """Row-cyclic slices (multi-GPU partition) rendered separately equal the full frame
    (G = 8 also switches the slices to one-row pixel groups)."""
    s = gpu.Scene.load_json(scene_path("world8_stress"), 160, 96)
    full = s.render(spp=spp, want=("rgba", "hit_inst"))
    out = np.zeros_like(full["rgba"])
    for r in range(G):
        part = s.render(spp=spp, row0=r, row_step=G, compact=True, want=("rgba",))
        out[r::G] = part["rgba"]
    assert np.array_equal(out, full["rgba"])


def test_camera_move_rerender(gpu, oracle):
    """Interactive camera (main.cc:140-180): after each translate / rotate the frame (counted
    and fast kernels) equals the oracle's render of the same camera pose."""
    import math
    s = gpu.Scene.load_json(scene_path("world8"), 128, 96)
    o = oracle.load(scene_path("world8"), 128, 96)
    first = s.render(want=("rgba",))["rgba"]
    for d, a in (([0.5, -2.0, 1.0], 0.05), ([0.0, 0.0, 3.0], -0.2), ([-1.0, 0.5, 0.0], 0.7)):
        s.translate_camera(d)
        s.rotate_camera([math.sin(a / 2), 0, 0, math.cos(a / 2)])
        mirror_camera(s, o)
        for stats in (True, False):
            fr = s.render(spp=2, want=WANT, stats=stats)
            of = orc_check(oracle, o, fr, 2, ctx=(d, a, stats))
        if stats:
            assert tuple(fr["stats"][k] for k in ("rays", "nodes", "leaves", "tri_tests")) == tuple(int(x) for x in of["stats"])
    assert not np.array_equal(fr["rgba"], first)


def test_debug_cast_log(gpu, oracle):
    """debug_cast's whole event log (raytracer.cu:91-100; printf sites scene.cu:107-153 and
    light.cu:38-39, in order) equals the oracle's for lit, mirror, sky and -- world1 seen from
    a moved camera -- refraction pixels (shadow segments through the Kt cube)."""
    s = gpu.Scene.load_json(scene_path("world8_stress"), 320, 240)
    o = oracle.load(scene_path("world8_stress"), 320, 240)
    fr = s.render(want=("hit_inst",))
    ys, xs = np.nonzero(fr["hit_inst"] >= 0)
    log = s.debug_cast(int(xs[0]), int(ys[0]))
    assert log[0] == "shooting a ray" and "shooting shadow ray" in log
    ys, xs = np.nonzero(fr["hit_inst"] < 0)
    assert s.debug_cast(int(xs[0]), int(ys[0])) == ["shooting a ray"]
    kinds = set()
    for x in range(3, 320, 17):
        for y in range(5, 240, 13):
            g = s.debug_cast(x, y)
            assert g == o.debug_cast(x, y), (x, y)
            kinds |= set(g)
    assert "preparing to shoot a reflection ray" in kinds
    w = gpu.Scene.load_json(scene_path("world1"), 64, 48)
    ow = oracle.load(scene_path("world1"), 64, 48)
    w.set_camera([0.5, 2.0, -3.0], [0.2, 0.0, 0.0, 0.98])
    mirror_camera(w, ow)
    refr = 0
    for x in range(0, 64, 3):
        for y in range(0, 48, 3):
            g = w.debug_cast(x, y)
            assert g == ow.debug_cast(x, y), (x, y)
            refr += "preparing to shoot a refraction ray" in g
    assert refr >= 10


def test_empty_scene_renders_black(gpu, tmp_path):
    p = tmp_path / "empty.json"
    p.write_text('{"atlas": "x", "grid_size": 0, "cubes": [], "width": 40, "height": 30}')
    s = gpu.Scene.load_json(str(p))
    fr = s.render(want=("rgba", "hit_inst"))
    assert (fr["rgba"] == 0).all() and (fr["hit_inst"] == -1).all()


@pytest.mark.parametrize("scene,spp", [("world8_stress", 4), ("world16", 1), ("world1", 2), ("world8", 2),
                                       ("config", 2)])
def test_occlusion_early_exit_is_exact(gpu, oracle, scene, spp):
    """Frames rendered without statistics use the fast kernel: shadow-ray occlusion early
    exit (all-opaque scenes) and distance pruning of subtrees beyond the current closest
    hit.  They must equal the counted (full closest-hit, reference traversal) frames bit
    for bit, and the oracle."""
    s = gpu.Scene.load_json(scene_path(scene), 240, 160)
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    fast = s.render(spp=spp, want=want, stats=False)
    full = s.render(spp=spp, want=want, stats=True)
    for k in want:
        assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), k
    o = oracle.render(oracle.load(scene_path(scene), 240, 160), spp=spp, nthreads=8)
    check_frame(fast, o, spp)


def test_fast_kernel_exact_close_camera(gpu, oracle):
    """Distance pruning with the camera inside the cube field (rays start next to boxes,
    many near-ties between overlapping leaves)."""
    s = gpu.Scene.load_json(scene_path("world8_stress"), 200, 150)
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    _, rot = s.camera()
    # the cubes fill x, z in [-4, 3], y in [0, 11]; the camera looks down at ~58 degrees
    o = oracle.load(scene_path("world8_stress"), 200, 150)
    for pos in ([0.5, 14.0, -0.5], [0.37, 6.21, -1.13], [-3.9, 10.5, 2.9], [0.0, 3.0, -6.5]):
        s.set_camera(pos, rot)
        fast = s.render(spp=2, want=want, stats=False)
        full = s.render(spp=2, want=want, stats=True)
        for k in want:
            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), k
        assert (full["hit_inst"] >= 0).mean() > 0.05, pos
        mirror_camera(s, o)
        orc_check(oracle, o, fast, 2, ctx=pos)


def test_fast_kernel_exact_grazing_rays(gpu, oracle):
    """Distance pruning and the triangle skip near their worst case: level cameras placed
    exactly on cube face planes and edges (faces at k +- 0.4995), so rays graze faces and
    run along edges at shallow angles, where the slack's max|1/d| factor matters."""
    import math
    s = gpu.Scene.load_json(scene_path("world8_stress"), 160, 120)
    o = oracle.load(scene_path("world8_stress"), 160, 120)
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    e = 0.4995
    for pos, yaw in (([e, 3 + e, -8.0], 0.0), ([-1.0, 5 + e, -7.3], 0.0), ([e, 3 + e, -8.0], 1e-3),
                     ([-4 - e, 1 + e, -6.0], 2e-4), ([0.25, 11 + e, -6.5], -5e-4)):
        s.set_camera(pos, [0.0, math.sin(yaw / 2), 0.0, math.cos(yaw / 2)])
        fast = s.render(spp=2, want=want, stats=False)
        full = s.render(spp=2, want=want, stats=True)
        for k in want:
            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (pos, yaw, k)
        assert (full["hit_inst"] >= 0).mean() > 0.05, pos
        mirror_camera(s, o)
        orc_check(oracle, o, fast, 2, ctx=(pos, yaw))


def test_fast_kernel_exact_zero_direction_axes(gpu, oracle):
    """Zero-direction-axis cut (closest_hit): rays with d_x == 0 (centre column, sample 0)
    and d_y == 0 (centre row) from origins on and around cube face planes, offset by
    fractions and multiples of the pruning slack (~1.4e-3 here), so leaves whose slab is
    skipped by the reference sit just inside and just outside the cut.  Every shadow ray
    of world8_stress's directional light (0, -1, 1) has d_x == 0 as well."""
    s = gpu.Scene.load_json(scene_path("world8_stress"), 160, 120)
    o = oracle.load(scene_path("world8_stress"), 160, 120)
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    e = 0.4995
    for off in (0.0, 1e-6, -1e-6, 7e-4, -7e-4, 1.4e-3, -1.4e-3, 3e-3, -3e-3):
        for pos in ([e + off, 3 + e + off, -8.0], [-2 - e + off, 6 - e - off, -7.5]):
            s.set_camera(pos, [0.0, 0.0, 0.0, 1.0])
            fast = s.render(spp=2, want=want, stats=False)
            full = s.render(spp=2, want=want, stats=True)
            for k in want:
                assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (pos, k)
            assert (full["hit_inst"] >= 0).mean() > 0.05, pos          # (a centre row may run in a gap)
            mirror_camera(s, o)
            orc_check(oracle, o, fast, 2, ctx=pos)


def test_fast_kernel_exact_tiny_direction_components(gpu, oracle):
    """Rays outside the filtered slab test's range (0 < |d_a| < 2^-64: ray_inv's exact flag),
    which the fast traversal sends to the exact reference test at every node (NaN
    reciprocals, pair_hit_tt2): level cameras turned by 1e-25..1e-21 rad, so the centre
    column's / row's sample-0 rays carry such a component, among ordinary rays."""
    import math
    s = gpu.Scene.load_json(scene_path("world8_stress"), 160, 120)
    o = oracle.load(scene_path("world8_stress"), 160, 120)
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    e = 0.4995
    for pos in ([e, 3 + e, -8.0], [-2 - e, 6 - e, -7.5], [0.3, 4.2, -6.0]):
        for ax, ang in ((1, 1e-25), (0, -3e-22), (1, -7e-21), (2, 1e-23)):
            q = [0.0, 0.0, 0.0, math.cos(ang / 2)]
            q[ax] = math.sin(ang / 2)
            s.set_camera(pos, q)
            fast = s.render(spp=2, want=want, stats=False)
            full = s.render(spp=2, want=want, stats=True)
            for k in want:
                assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (pos, ax, ang, k)
            assert (full["hit_inst"] >= 0).mean() > 0.05, pos
            mirror_camera(s, o)
            orc_check(oracle, o, fast, 2, ctx=(pos, ax, ang))


def test_fast_kernel_exact_random_cameras(gpu, oracle):
    """Fast kernel (ordered LBVH, pruning, axis-plane triangle path with its shared-plane
    skip and in-plane reject) == counted reference-heap kernel, bit for bit, from seeded
    random camera poses in and around the cube field (any orientation)."""
    rng = np.random.default_rng(1234)
    s = gpu.Scene.load_json(scene_path("world8_stress"), 96, 64)
    o = oracle.load(scene_path("world8_stress"), 96, 64)
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    lit = 0.0
    for _ in range(16):
        pos = [float(rng.uniform(-7, 7)), float(rng.uniform(-1, 16)), float(rng.uniform(-7, 7))]
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        s.set_camera(pos, [float(x) for x in q])
        fast = s.render(spp=2, want=want, stats=False)
        full = s.render(spp=2, want=want, stats=True)
        for k in want:
            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (pos, k)
        lit += (full["hit_inst"] >= 0).mean()
        mirror_camera(s, o)
        orc_check(oracle, o, fast, 2, ctx=pos)
    assert lit / 16 > 0.1


def test_timed_frames(gpu):
    """timing=1 (events on the dispatches themselves): one duration pair per frame, both
    positive, a frame without a BVH rebuild has a zero-length build span, and the image
    is the one an untimed render produces."""
    import torch
    s = gpu.Scene.load_json(scene_path("world8_stress"), 192, 128)
    ref = s.render(spp=2, want=("rgba",), stats=False)["rgba"]
    buf = torch.zeros((128, 192), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    s.timing_collect()
    for f in range(3):
        s.render_device(spp=2, rebuild_bvh=(f < 2), rgba_ptr=buf.data_ptr(), stream=stream, timing=True)
    tm = s.timing_collect()
    assert tm["frames"] == 3
    assert tm["bvh_ms_total"] > 0 and tm["trace_ms_total"] > 0
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    s.render_device(spp=2, rebuild_bvh=False, rgba_ptr=buf.data_ptr(), stream=stream, timing=True)
    one = s.timing_collect()
    assert one["frames"] == 1 and one["bvh_ms_total"] < 0.01 and one["trace_ms_total"] > 0
    assert s.timing_collect()["frames"] == 0


@pytest.mark.parametrize("spp,w,h", [(8, 240, 160), (3, 240, 160), (16, 160, 120), (64, 64, 48)])
def test_fast_kernel_exact_spp8_sky_and_horizon(gpu, oracle, spp, w, h):
    """The bench's sample mapping (8 samples per pixel: one-round-trip exchange, clamp before
    the exchange) and the whole-group miss test: fast frames == counted frames bit for bit
    with the camera at the scene's pose, turned to the sky (every group a miss group), at
    the horizon (groups straddling it) and from random poses; with every output, and with
    the colour alone (the raw-sum exchange skipped).  spp = 3 takes the generic exchange; spp =
    16 two pixels per lane row, spp = 64 one pixel per wave (config 5's mapping, 1 x 1 sky
    cones).  Every pose is also put against the oracle."""
    import torch
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    o = oracle.load(scene_path("world8_stress"), w, h)
    pos0, q0 = s.camera()
    rng = np.random.default_rng(77)
    poses = [(pos0, q0), (pos0, (-0.3826834, 0.0, 0.0, 0.9238795)), (pos0, (0.0, 0.0, 0.0, 1.0)),
             ((0.5, 3.0, -12.0), (0.0, 0.0, 0.0, 1.0))]
    for _ in range(3):
        q = rng.normal(size=4)
        poses.append(([float(rng.uniform(-6, 6)), float(rng.uniform(0, 12)), float(rng.uniform(-9, 9))],
                      [float(x) for x in q / np.linalg.norm(q)]))
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    sky_seen = lit_seen = False
    buf = torch.zeros((h, w), dtype=torch.int32, device="cuda")
    for pos, q in poses:
        s.set_camera(pos, q)
        full = s.render(spp=spp, want=want, stats=True)
        fast = s.render(spp=spp, want=want, stats=False)
        for k in want:
            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (pos, q, k)
        s.render_device(spp=spp, rgba_ptr=buf.data_ptr(), compact=False, sync=True)
        assert np.array_equal(buf.cpu().numpy().view(np.uint32), full["rgba"]), (pos, q)
        mirror_camera(s, o)
        orc_check(oracle, o, fast, spp, ctx=(pos, q))
        hit = full["hit_inst"] >= 0
        sky_seen |= bool((~hit).all())
        lit_seen |= bool(hit.any() and (~hit).any())
    assert sky_seen and lit_seen


def _scene_bounds(s):
    """World bounds of the scene's triangles (instance translations + mesh vertices; the cube
    worlds have identity rotations)."""
    v = s.export("vertices")
    inst = s.export("instances")
    lo = inst[:, 4:7].min(0) + v.min(0)                       # instances: quat (4), position (3)
    hi = inst[:, 4:7].max(0) + v.max(0)
    return lo, hi


@pytest.mark.parametrize("spp,row_step", [(8, 1), (2, 1), (8, 3), (16, 1), (64, 2)])
def test_sky_prepass_grazing_cones(gpu, oracle, spp, row_step):
    """The sky pre-pass decides most groups by their ray cone (cone_misses_root: side planes
    and box faces with conservative margins) and writes their outputs itself.  Cameras on and
    just beside the scene's bounding planes, looking along them, put group cones within
    rounding of the root boxes: fast frames (pre-pass) == counted frames (no pre-pass) bit
    for bit, whole frames and row slices."""
    w, h = (64, 48) if spp <= 16 else (32, 24)
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    o = oracle.load(scene_path("world8_stress"), w, h)
    lo, hi = _scene_bounds(s)
    mid = 0.5 * (lo + hi)
    c, sn = np.cos, np.sin
    quats = [(0.0, 0.0, 0.0, 1.0)]
    for a in (0.25, 0.5, 0.75, 1.0, 1.5):                      # about y (level views)
        quats.append((0.0, float(sn(0.5 * np.pi * a)), 0.0, float(c(0.5 * np.pi * a))))
    for a in (-0.2, 0.2):                                      # tilted up / down
        quats.append((float(sn(0.5 * np.pi * a)), 0.0, 0.0, float(c(0.5 * np.pi * a))))
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    n = 0
    for axis in range(3):
        for side, plane in ((0, lo[axis]), (1, hi[axis])):
            for off in (0.0, 2e-3, -2e-3, 0.3):
                pos = mid.copy()
                pos[axis] = plane + (off if side else -off)
                for q in quats[:: (1 if axis == 1 else 2)]:
                    s.set_camera([float(x) for x in pos], q)
                    kw = dict(spp=spp, want=want, row0=row_step - 1, row_step=row_step, compact=True)
                    fast = s.render(stats=False, **kw)         # first: the staging buffers hold another pose
                    full = s.render(stats=True, **kw)
                    for k in want:
                        assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (axis, side, off, q, k)
                    mirror_camera(s, o)
                    orc_check(oracle, o, fast, spp, row0=row_step - 1, row_step=row_step, compact=True,
                              ctx=(axis, side, off, q))
                    n += 1
    assert n > 60


@pytest.mark.parametrize("scene,spp,row_step", [("world1", 1, 1), ("world1", 4, 3), ("world1", 16, 1)])
def test_brute_sky_prepass_grazing(gpu, oracle, scene, spp, row_step):
    """Brute-force frames (the reference's -r) with the sky pre-pass testing each instance's box
    grown by the pruning slack (grown_box_maybe): cameras on, just beside
    and away from every instance box's face planes, looking along them and across, so rays
    pass within rounding of the grown boxes; fast frames (pre-pass) == counted frames (no
    pre-pass) bit for bit and == the oracle's brute-force frames, whole frames and row slices."""
    w, h = (64, 48) if spp <= 4 else (32, 24)
    s = gpu.Scene.load_json(scene_path(scene), w, h)
    o = oracle.load(scene_path(scene), w, h)
    v = s.export("vertices")
    inst = s.export("instances")
    c, sn = np.cos, np.sin
    quats = [(0.0, 0.0, 0.0, 1.0)]
    for a in (0.25, 0.5, 1.0, 1.5):                            # about y (level views)
        quats.append((0.0, float(sn(0.5 * np.pi * a)), 0.0, float(c(0.5 * np.pi * a))))
    for a in (-0.25, 0.25):                                    # tilted down / up
        quats.append((float(sn(0.5 * np.pi * a)), 0.0, 0.0, float(c(0.5 * np.pi * a))))
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    n = skies = 0
    for i in range(min(len(inst), 3)):
        lo, hi = inst[i, 4:7] + v.min(0), inst[i, 4:7] + v.max(0)
        mid = 0.5 * (lo + hi)
        for axis in range(3):
            for side, plane in ((0, lo[axis]), (1, hi[axis])):
                for off in (0.0, 1e-3, -1e-3, 2.0):
                    pos = mid.copy()
                    pos[axis] = plane + (off if side else -off)
                    for q in quats[:: (1 if axis == 1 else 3)]:
                        s.set_camera([float(x) for x in pos], q)
                        kw = dict(spp=spp, use_bvh=False, want=want, row0=row_step - 1, row_step=row_step, compact=True)
                        fast = s.render(stats=False, **kw)
                        full = s.render(stats=True, **kw)
                        for k in want:
                            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (i, axis, side, off, q, k)
                        mirror_camera(s, o)
                        orc_check(oracle, o, fast, spp, row0=row_step - 1, row_step=row_step, compact=True, use_bvh=0,
                                  ctx=(i, axis, side, off, q))
                        n += 1
                        skies += int((full["hit_inst"] < 0).all())
    assert n > 50 and skies < n


def _opaque_cubes(gpu, oracle, w, h):
    """A built opaque scene of 12 cube instances (3 meshes: diffuse, specular, mirror) on a
    ragged grid: the brute-force sky pre-pass tests every instance's grown box (<= 64)."""
    m = gpu.material
    mats = [m(Ka=(0.1, 0.1, 0.1, 1), Kd=(0.6, 0.3, 0.1, 1)),
            m(Ka=(0.1, 0.1, 0.1, 1), Kd=(0.2, 0.5, 0.2, 1), Ks=(0.8, 0.8, 0.8, 1), alpha=6.0),
            m(Kd=(0.3, 0.3, 0.3, 1), Ks=(0.5, 0.5, 0.5, 1), Kr=(0.7, 0.7, 0.7, 1), alpha=8.0)]
    t = Twin(gpu, oracle)
    meshes = [t.build_cube(1.0, mt) for mt in mats]
    rng = np.random.default_rng(11)
    for i in range(4):
        for j in range(3):
            k = t.add_trans(meshes[(i + j) % 3])
            t.set_trans(k, pos=(2.5 * i - 3.75 + float(rng.uniform(-0.3, 0.3)), float(rng.integers(0, 3)),
                                3.0 * j - 3.0))
    t.add_point_light((0.5, 6.0, 0.3), (1.0, 1.0, 1.0, 1.0))
    t.add_directional_light((0.3, -1.0, 0.8), (0.9, 0.8, 0.7, 1.0))
    t.finish(w, h, 60.0, 100.0, cam_pos=(0.0, 9.0, -12.0), cam_quat=(-0.3826834, 0.0, 0.0, 0.9238795),
             dist_atten=(0.1, 0.05, 0.01), ambience=(0.2, 0.2, 0.2, 1.0), depth=3)
    return t.gpu, t.orc


@pytest.mark.parametrize("scene,spp,row_step", [("world8", 1, 1), ("world8", 8, 3), ("world8_stress", 2, 1),
                                                ("world8_stress", 8, 8), ("cubes", 1, 1), ("cubes", 8, 2)])
def test_brute_fast_opaque(gpu, oracle, scene, spp, row_step):
    """the opaque brute-force kernel (trace_kernel<0, true, M_BRUTE | ...>, NS = 0: no
    refraction code, the occlusion early exit `b.time <= occl_t`) on opaque scenes -- world8 (380
    instances) and world8_stress (570; both above the sky pre-pass's 64) and the built 12-instance
    scene (with the brute-force sky pre-pass) -- fast == counted bit for bit == the oracle's
    use_bvh = 0 frame, whole frames and row slices, from the scene's camera and two others."""
    w, h = 96, 64
    if scene == "cubes":
        s, o = _opaque_cubes(gpu, oracle, w, h)
    else:
        s = gpu.Scene.load_json(scene_path(scene), w, h)
        o = oracle.load(scene_path(scene), w, h)
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    poses = [None, ((1.0, 6.0, -8.0), (-0.2588190, 0.0, 0.0, 0.9659258)), ((-4.0, 2.0, 3.0), (0.0, 0.7071068, 0.0, 0.7071068))]
    hits = 0
    for pose in poses:
        if pose:
            s.set_camera(*pose)
        kw = dict(spp=spp, use_bvh=False, want=want, row0=row_step - 1, row_step=row_step, compact=True)
        fast = s.render(stats=False, **kw)
        full = s.render(stats=True, **kw)
        for k in want:
            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (pose, k)
        mirror_camera(s, o)
        orc_check(oracle, o, fast, spp, row0=row_step - 1, row_step=row_step, compact=True, use_bvh=0, ctx=(scene, pose))
        hits += int((full["hit_inst"] >= 0).sum())
    assert hits > 0


@pytest.mark.parametrize("spp,row_step", [(1, 1), (4, 3)])
def test_brute_sky_prepass_grazing_many(gpu, oracle, spp, row_step):
    """the brute-force sky pre-pass over many instances (the built 12-cube opaque
    scene; world1 has two): cameras on, beside and away from the face planes of six instance
    boxes, looking along them and across, so that rays pass within rounding of several grown
    boxes at once; fast (pre-pass) == counted (none) bit for bit == the oracle."""
    w, h = 48, 32
    s, o = _opaque_cubes(gpu, oracle, w, h)
    v = s.export("vertices")
    inst = s.export("instances")
    c, sn = np.cos, np.sin
    quats = [(0.0, 0.0, 0.0, 1.0)]
    for a in (0.5, 1.0, 1.5):
        quats.append((0.0, float(sn(0.5 * np.pi * a)), 0.0, float(c(0.5 * np.pi * a))))
    quats.append((float(sn(-0.125 * np.pi)), 0.0, 0.0, float(c(-0.125 * np.pi))))
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    n = skies = 0
    for i in range(0, len(inst), 2):
        lo, hi = inst[i, 4:7] + v.min(0), inst[i, 4:7] + v.max(0)
        mid = 0.5 * (lo + hi)
        for axis in range(3):
            for side, plane in ((0, lo[axis]), (1, hi[axis])):
                for off in (0.0, 1e-3, 3.0):
                    pos = mid.copy()
                    pos[axis] = plane + (off if side else -off)
                    for q in quats[:: (1 if axis == 1 else 2)]:
                        s.set_camera([float(x) for x in pos], q)
                        kw = dict(spp=spp, use_bvh=False, want=want, row0=row_step - 1, row_step=row_step, compact=True)
                        fast = s.render(stats=False, **kw)
                        full = s.render(stats=True, **kw)
                        for k in want:
                            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (i, axis, side, off, q, k)
                        mirror_camera(s, o)
                        orc_check(oracle, o, fast, spp, row0=row_step - 1, row_step=row_step, compact=True, use_bvh=0,
                                  ctx=(i, axis, side, off, q))
                        n += 1
                        skies += int((full["hit_inst"] < 0).all())
    assert n > 100 and skies < n


@pytest.mark.parametrize("col1", [(0.9, 0.8, 0.7, 1.0), (0.9, -0.0, 0.7, 1.0)])
def test_unlit_skip_exact(gpu, oracle, col1):
    """The fast kernels trace no shadow segments for a light whose phong factor (diffuse +
    specular) is zero in every channel; the light's term is then that signed zero whatever the
    shadow, so frames equal the counted kernel's (every shadow ray traced) bit for bit.  A
    built scene with opaque, specular (small and large alpha), refractive (Kt in (0, 1)) and
    reflective cubes, lights from above and below (back-facing for many faces) and cameras
    all around.  A light colour with a -0 channel makes the skip unsound (-0 x 0 vs +0 x 0)
    and the host turns it off: the frames must still agree."""
    m = gpu.material
    mats = [m(Ka=(0.1, 0.1, 0.1, 1), Kd=(0.6, 0.3, 0.1, 1)),
            m(Ka=(0.1, 0.1, 0.1, 1), Kd=(0.2, 0.5, 0.2, 1), Ks=(0.8, 0.8, 0.8, 1), alpha=0.3),
            m(Kd=(0.2, 0.2, 0.6, 1), Kt=(0.5, 0.6, 0.7, 1), eta=1.3),
            m(Kd=(0.3, 0.3, 0.3, 1), Ks=(0.5, 0.5, 0.5, 1), Kr=(0.7, 0.7, 0.7, 1), alpha=8.0)]
    s = Twin(gpu, oracle)
    meshes = [s.build_cube(1.0, mt) for mt in mats]
    rng = np.random.default_rng(5)
    for i in range(5):
        for j in range(5):
            t = s.add_trans(meshes[(i + 2 * j) % 4])
            s.set_trans(t, pos=(1.6 * i - 3.2, float(rng.integers(0, 3)), 1.6 * j - 3.2))
    s.add_point_light((0.5, 6.0, 0.3), (1.0, 1.0, 1.0, 1.0))
    s.add_directional_light((0.3, -1.0, 0.8), col1)
    s.add_directional_light((-0.2, 1.0, -0.4), (0.4, 0.5, 0.6, 1.0))   # from below
    s.finish(96, 64, 60.0, 100.0, cam_pos=(0.0, 9.0, -9.0), cam_quat=(-0.3826834, 0.0, 0.0, 0.9238795),
             dist_atten=(0.1, 0.05, 0.01), ambience=(0.2, 0.2, 0.2, 1.0), depth=3)
    o, s = s.orc, s.gpu
    want = ("rgba", "radiance", "hit_inst", "hit_tri")
    poses = [((0.0, 9.0, -9.0), (-0.3826834, 0.0, 0.0, 0.9238795))]
    for _ in range(6):
        q = rng.normal(size=4)
        poses.append(((float(rng.uniform(-6, 6)), float(rng.uniform(-2, 8)), float(rng.uniform(-6, 6))),
                      tuple(float(x) for x in q / np.linalg.norm(q))))
    lit = 0.0
    for pos, q in poses:
        s.set_camera(pos, q)
        fast = s.render(spp=4, want=want, stats=False)
        full = s.render(spp=4, want=want, stats=True)
        for k in want:
            assert np.array_equal(fast[k].view(np.uint32), full[k].view(np.uint32)), (pos, q, k)
        lit += (full["hit_inst"] >= 0).mean()
        mirror_camera(s, o)
        of = orc_check(oracle, o, full, 4, ctx=(pos, q))
        assert tuple(full["stats"][k] for k in ("rays", "nodes", "leaves", "tri_tests")) == tuple(int(x) for x in of["stats"])
    assert lit / len(poses) > 0.05
