"""CPU tests: pin the oracle (test infrastructure) before trusting it.

1. Math primitives: bit-exact against known-answer vectors produced by the
   reference's own raymath headers, z_order.cu, bounding_box.cu and entity.cu
   (tests/golden/kat_*.npz, made by tests/golden/make_golden.py from oracle/_ref/kat_ref).
2. Whole-frame behaviour: ray / node / leaf / triangle counters and CPU-vs-GPU
   semantic image differences equal the measurements of the reference code
   recorded in SURVEY.md Appendix D and §8d.
3. Committed frame fixtures re-render identically.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, scene_path


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.mark.parametrize("op,inputs", [
    ("normalize3", ["v"]), ("cross", ["a", "b"]), ("reflect", ["d", "n"]), ("quat_rotate", ["q", "v"]),
    ("quat_inverse", ["q"]), ("quat_mul", ["a", "b"]), ("ray_ctor", ["ray"]), ("zorder", ["v"]),
    ("axis_angle", ["a"]), ("to_mat3", ["q"]),
])
def test_oracle_kat_bit_exact(oracle, op, inputs):
    g = golden(f"kat_{op}.npz")
    out = oracle.kat(op, *[g[k] for k in inputs])
    assert np.array_equal(_bits(out), _bits(g["out"])), op


def test_oracle_kat_refract(oracle):
    g = golden("kat_refract.npz")
    out, tir = oracle.kat("refract", g["d"], g["n"], g["n12"])
    assert np.array_equal(tir, g["tir"])
    assert np.array_equal(_bits(out), _bits(g["out"]))
    assert 0.05 < g["tir"].mean() < 0.95          # both branches exercised


def test_oracle_kat_triangle(oracle):
    g = golden("kat_tri_hit.npz")
    hit, tuv = oracle.kat("tri_hit", g["tri"], g["ray"])
    assert np.array_equal(hit, g["hit"])
    assert np.array_equal(_bits(tuv), _bits(g["out"]))
    assert 0.2 < g["hit"].mean() < 0.9            # edge cases on both sides of the 1e-5 test


def test_oracle_kat_slab_test(oracle):
    """BoundingBox::intersects (bounding_box.cu:62-104) as the reference's own TU computes it
    (kat_box_hit.npz, round 5): hit and entry time, on face / edge / corner targets, zero and
    negative-zero direction components, flat and degenerate boxes, origins inside."""
    g = golden("kat_box_hit.npz")
    hit, t = oracle.kat("box_hit", g["box"], g["ray"])
    assert np.array_equal(hit, g["hit"])
    h = g["hit"] == 1
    assert np.array_equal(_bits(t[h]), _bits(g["t"][h]))
    assert 0.2 < g["hit"].mean() < 0.9


@pytest.mark.parametrize("op,inputs", [("box_from_local", ["box", "entity"]), ("box_merge", ["a", "b"])])
def test_oracle_kat_boxes(oracle, op, inputs):
    """from_local (create_boxes' instance boxes) and merge (the BVH level merges),
    bounding_box.cu:5-60, against the reference's TU."""
    g = golden(f"kat_{op}.npz")
    out, nd = oracle.kat(op, *[g[k] for k in inputs])
    assert np.array_equal(nd, g["nd"])
    assert np.array_equal(_bits(out), _bits(g["out"]))


def test_oracle_kat_entity(oracle):
    """Entity::point/vec_to/from_local (entity.cu:5-37): cast_local's and Hitable::hit's pose
    chain, against the reference's TU."""
    g = golden("kat_entity.npz")
    assert np.array_equal(_bits(oracle.kat("entity", g["entity"], g["v"])), _bits(g["out"]))


def test_oracle_kat_hitable(oracle):
    """Hitable::hit's HitHandle (hitable.cu:7-38: the mesh pose's local ray, then the normal and
    time of a local hit brought back), against the reference's TU around a known local hit."""
    g = golden("kat_hitable.npz")
    assert np.array_equal(_bits(oracle.kat("hitable", g["entity"], g["ray"], g["hit"])), _bits(g["out"]))


# counters measured on the reference's GPU-semantics path (1080p, spp=1)
APPENDIX_D = {
    ("world1", 0): (2084662, 0, 4169324, 50031888),
    ("world1", 1): (2084636, 2098420, 8004, 96048),
    ("world8", 1): (2770208, 47422214, 4550509, 54606108),
    ("world8_stress", 1): (3250153, 109186219, 8928838, 107146056),
    ("world16", 1): (4182940, 328876154, 21388083, 256656996),
}


@pytest.mark.parametrize("scene,bvh", list(APPENDIX_D))
def test_oracle_counters_match_reference_measurements(oracle, scene, bvh):
    s = oracle.load(scene_path(scene), 1920, 1080)
    st = oracle.render(s, semantics=0, use_bvh=bvh, spp=1, nthreads=8, want=())["stats"]
    assert tuple(int(x) for x in st) == APPENDIX_D[(scene, bvh)]


@pytest.mark.parametrize("scene,w,h,ndiff,maxd,cpu_rays", [
    ("world1", 640, 480, 1406, 12, 327352),
    ("world8", 640, 480, 0, 0, 403598),
    ("world8_stress", 640, 480, 7993, 109, 573334),
])
def test_oracle_cpu_vs_gpu_semantics(oracle, scene, w, h, ndiff, maxd, cpu_rays):
    """the reference's CPU path differs from its GPU path on Kr/Kt scenes."""
    s = oracle.load(scene_path(scene), w, h)
    g = oracle.render(s, semantics=0, nthreads=8, want=("rgba",))
    c = oracle.render(s, semantics=1, nthreads=8, want=("rgba",))
    a = g["rgba"].view(np.uint8).reshape(-1, 4).astype(int)
    b = c["rgba"].view(np.uint8).reshape(-1, 4).astype(int)
    d = np.abs(a - b).max(1)
    assert int((d > 0).sum()) == ndiff and int(d.max()) == maxd
    assert int(c["stats"][0]) == cpu_rays


def test_oracle_frames_reproduce(oracle):
    import glob
    files = sorted(glob.glob(os.path.join(GOLDEN, "frame_*.npz")))
    assert len(files) >= 5
    for f in files:
        name = os.path.basename(f)[len("frame_"):-4]
        parts = name.split("_")
        sem = 1 if parts[-1] == "cpu" else 0
        spp = int(parts[-2][3:])
        bvh = parts[-3] == "bvh"
        w, h = map(int, parts[-4].split("x"))
        scene = "_".join(parts[:-4])
        g = np.load(f)
        s = oracle.load(scene_path(scene), w, h)
        fr = oracle.render(s, semantics=sem, use_bvh=int(bvh), spp=spp, nthreads=4)
        for k in ("rgba", "radiance", "hit_inst", "hit_tri", "stats"):
            assert np.array_equal(_bits(fr[k]), _bits(g[k])), (name, k)


def test_oracle_bvh_is_heap_complete(oracle):
    """BVH invariants of bvh.cu:43-91: parents are exact unions, padding leaves degenerate."""
    s = oracle.load(scene_path("world8_stress"), 64, 64)
    boxes, order = s.bvh()
    n = order.size
    assert n == 1024 and sorted(order.tolist()) == list(range(n))
    for k in range(1, n):                 # heap node k at storage 2n-1-k
        p = boxes[2 * n - 1 - k]
        l, r = boxes[2 * n - 1 - 2 * k], boxes[2 * n - 2 - 2 * k]
        live = [c for c in (l, r) if c[6]]
        if not live:
            assert p[6] == 0
            continue
        assert np.array_equal(p[:3], np.min([c[:3] for c in live], 0))
        assert np.array_equal(p[3:6], np.max([c[3:6] for c in live], 0))
    assert int(boxes[:n, 6].sum()) == s.n_instances
