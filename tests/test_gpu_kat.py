"""GPU known-answer tests: the device math (the same inline functions the trace
kernel uses, run on gfx950 through the C ABI) against vectors produced by the
reference's own raymath sources.  Bit-exact except pow (1 ulp)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def g(name):
    return np.load(os.path.join(GOLDEN, f"kat_{name}.npz"))


@pytest.mark.parametrize("op,inputs", [
    ("normalize3", ["v"]), ("cross", ["a", "b"]), ("reflect", ["d", "n"]), ("quat_rotate", ["q", "v"]),
    ("quat_inverse", ["q"]), ("quat_mul", ["a", "b"]), ("ray_ctor", ["ray"]), ("to_mat3", ["q"]),
])
def test_device_math_bit_exact(gpu, op, inputs):
    k = g(op)
    out = gpu.kat_device(op, *[k[i] for i in inputs])
    ref = k["out"]
    assert np.array_equal(_bits(out.reshape(ref.shape)), _bits(ref)), op


def test_device_slab_tests_equal_reference(gpu, oracle):
    """Every device box test (exact, filtered, packed pair) against the reference-built slab
    test vectors (kat_box_hit.npz: bounding_box.cu:62-104 compiled from the reference)."""
    k = g("box_hit")
    box, ray = k["box"], k["ray"]
    assert np.array_equal(gpu.kat_device("box_hit", box, ray), k["hit"])
    assert np.array_equal(gpu.kat_device("box_hit_f", box, ray), k["hit"])
    other = np.roll(box, 1, axis=0)
    pair = gpu.kat_device("box_pair", np.concatenate([box, other], 1), ray)
    assert np.array_equal(pair[:, 0], k["hit"])
    ref1, _ = oracle.kat("box_hit", other, ray)             # the oracle: pinned to the same TU (test_oracle.py)
    assert np.array_equal(pair[:, 1], ref1)


@pytest.mark.parametrize("op,inputs", [("box_from_local", ["box", "entity"]), ("box_merge", ["a", "b"])])
def test_device_boxes_equal_reference(gpu, op, inputs):
    """The BVH build's box arithmetic (rt_math.h from_local / merge, run by bvh_build_kernel)
    against the reference-built vectors (bounding_box.cu:5-60)."""
    k = g(op)
    out, nd = gpu.kat_device(op, *[k[i] for i in inputs])
    assert np.array_equal(nd, k["nd"])
    assert np.array_equal(_bits(out), _bits(k["out"]))


def test_device_entity_equal_reference(gpu):
    """Pose transforms (rt_math.h Pose, identity specialisation included) against entity.cu."""
    k = g("entity")
    assert np.array_equal(_bits(gpu.kat_device("entity", k["entity"], k["v"])), _bits(k["out"]))


def test_device_zorder(gpu):
    k = g("zorder")
    assert np.array_equal(gpu.kat_device("zorder", k["v"]), k["out"])


def test_device_refract(gpu):
    k = g("refract")
    out, tir = gpu.kat_device("refract", k["d"], k["n"], k["n12"])
    assert np.array_equal(tir, k["tir"])
    assert np.array_equal(_bits(out), _bits(k["out"]))


def test_device_triangle_test(gpu):
    k = g("tri_hit")
    out, hit = gpu.kat_device("tri_hit", k["tri"], k["ray"])
    assert np.array_equal(hit, k["hit"])
    assert np.array_equal(_bits(out), _bits(k["out"]))


def test_device_identity_pose_specialisation(gpu, oracle):
    """qrot_identity == the general Quat*Vec3 for q = (0,0,0,1), incl. signed zeros and tiny vectors."""
    rng = np.random.default_rng(7)
    v = (rng.normal(size=(20000, 3)) * 10.0 ** rng.uniform(-8, 3, size=(20000, 1))).astype(np.float32)
    v[rng.random(v.shape) < 0.1] = 0.0
    v[rng.random(v.shape) < 0.1] = -0.0
    q = np.tile(np.array([0, 0, 0, 1], np.float32), (len(v), 1))
    assert np.array_equal(_bits(gpu.kat_device("quat_rotate", q, v)), _bits(oracle.kat("quat_rotate", q, v)))
    qi = np.tile(np.array([-0.0, -0.0, -0.0, 1], np.float32), (len(v), 1))
    assert np.array_equal(_bits(gpu.kat_device("quat_rotate", qi, v)), _bits(oracle.kat("quat_rotate", qi, v)))


def test_device_box_test_matches_oracle(gpu, oracle):
    rng = np.random.default_rng(11)
    n = 20000
    mn = rng.normal(size=(n, 3)).astype(np.float32)
    mx = (mn + np.abs(rng.normal(size=(n, 3)))).astype(np.float32)
    box = np.concatenate([mn, mx, (rng.random((n, 1)) < 0.9).astype(np.float32)], 1)
    o = (rng.normal(size=(n, 3)) * 3).astype(np.float32)
    tgt = mn + (mx - mn) * rng.uniform(-0.1, 1.1, size=(n, 3)).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d[rng.random((n, 3)) < 0.05] = 0.0
    ray = np.concatenate([o, d], 1)
    hit = gpu.kat_device("box_hit", box, ray)
    ref, _ = oracle.kat("box_hit", box, ray)
    assert np.array_equal(hit, ref)
    assert 0.2 < ref.mean() < 0.95


def test_device_pow_within_one_ulp(gpu):
    rng = np.random.default_rng(3)
    x = rng.uniform(0, 20, 100000).astype(np.float32)
    y = rng.choice(np.array([0.6, 0.7, 0.8, 1.0, 2.5], np.float32), 100000)
    out = gpu.kat_device("pow", x, y)[:, 0]
    ref = np.power(x.astype(np.float64), y.astype(np.float64)).astype(np.float32)
    ulp = np.abs(out.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1


def test_device_pow_shading_domain(gpu):
    """pow as the shading uses it (phong.cu:27-32: max(dot, 0) ** alpha, x in [0, 1]; light.cu:18-25
    and scene.cu:14-22: Kt ** t and t ** Kt): within 1 ulp of the correctly rounded value and of the
    oracle's glibc powf, on dense grids of x."""
    x = np.concatenate([np.linspace(0, 1, 200001, dtype=np.float32), np.geomspace(1e-30, 1, 50000).astype(np.float32),
                        np.linspace(1, 50, 50000, dtype=np.float32)])
    for yv in (0.6, 0.7, 0.8, 1.5, 2.5, 10.0):
        y = np.full_like(x, yv)
        out = gpu.kat_device("pow", x, y)[:, 0]
        exact = np.power(x.astype(np.float64), y.astype(np.float64)).astype(np.float32)
        glibc = np.power(x, y)                    # float32 numpy power is libm powf (the oracle's pow)
        for ref in (exact, glibc):
            ulp = np.abs(out.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
            assert ulp.max() <= 1, (yv, int(ulp.max()))
        # pow_pos (rt_math.h) rounds a double within 2^-44 of x^y: the same float as the library's
        # double pow rounded, bar midpoint cases far rarer than these grids (0 of 4e7 on the host)
        assert np.array_equal(out.view(np.int32), exact.view(np.int32)), yv


def test_device_pow_wide_domain(gpu):
    """pow over random positive floats and exponents, including the ranges pow_pos hands to the
    library (|y ln x| > 700, x = 0, inf): equal to (float)pow(double, double), within 1 ulp of powf."""
    rng = np.random.default_rng(11)
    bits = rng.integers(0, 0x7f800000, 400000, dtype=np.int64).astype(np.uint32)
    x = bits.view(np.float32)
    y = (rng.uniform(-40, 40, x.size) * np.where(np.arange(x.size) % 3 == 0, 1.0, 0.05)).astype(np.float32)
    x[:4] = [0.0, np.inf, 1.0, 3.0]
    y[:4] = [0.7, 0.7, 1e30, 1e30]
    out = gpu.kat_device("pow", x, y)[:, 0]
    with np.errstate(over="ignore", under="ignore"):
        exact = np.power(x.astype(np.float64), y.astype(np.float64)).astype(np.float32)
        glibc = np.power(x, y)
    assert np.array_equal(out.view(np.int32), exact.view(np.int32))
    ulp = np.abs(out.view(np.int32).astype(np.int64) - glibc.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1


def test_filtered_triangle_equals_exact(gpu):
    """tri_accept_f (filtered) == Triangle::hit + the t >= 1e-5 acceptance, bit for bit, on the
    edge-dense golden vectors (the reference's own geometry.h produced them)."""
    k = g("tri_hit")
    out, hit = gpu.kat_device("tri_hit_f", k["tri"], k["ray"])
    exp_hit = (k["hit"] == 1) & (k["out"][:, 0] >= np.float32(1e-5))
    assert np.array_equal(hit.astype(bool), exp_hit)
    assert np.array_equal(_bits(out[exp_hit]), _bits(k["out"][exp_hit]))


def _adversarial_boxes(rng, n):
    mn = (rng.normal(size=(n, 3)) * 4).astype(np.float32)
    mx = (mn + np.abs(rng.normal(size=(n, 3))) + np.float32(1e-3)).astype(np.float32)
    box = np.concatenate([mn, mx, np.ones((n, 1), np.float32)], 1)
    o = (rng.normal(size=(n, 3)) * 20).astype(np.float32)
    # targets exactly on faces, edges and corners (the slab test's ties)
    t = rng.uniform(-0.05, 1.05, size=(n, 3)).astype(np.float32)
    snap = rng.random((n, 3))
    t[snap < 0.3] = 0.0
    t[(snap >= 0.3) & (snap < 0.6)] = 1.0
    tgt = (mn + (mx - mn) * t).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d[rng.random((n, 3)) < 0.03] = 0.0
    return box, np.concatenate([o, d], 1).astype(np.float32)


def test_filtered_box_equals_exact(gpu, oracle):
    rng = np.random.default_rng(2024)
    box, ray = _adversarial_boxes(rng, 200000)
    ref, _ = oracle.kat("box_hit", box, ray)
    assert np.array_equal(gpu.kat_device("box_hit_f", box, ray), ref)
    assert np.array_equal(gpu.kat_device("box_hit", box, ray), ref)
    assert 0.2 < ref.mean() < 0.9


def test_filtered_triangle_adversarial(gpu, oracle):
    """Rays aimed at triangle vertices/edges (barycentric sum right at the 1e-5 boundary)."""
    rng = np.random.default_rng(99)
    n = 100000
    tri = (rng.normal(size=(n, 3, 3)) * 2).astype(np.float32)
    w = rng.dirichlet([1, 1, 1], size=n).astype(np.float32)
    e = rng.integers(0, 3, n)
    w[np.arange(n), e] = rng.normal(scale=3e-6, size=n)      # just inside / outside an edge
    p = np.einsum("ni,nij->nj", w, tri).astype(np.float32)
    o = (p + rng.normal(size=(n, 3)) * 5).astype(np.float32)
    ray = np.concatenate([o, p - o], 1).astype(np.float32)
    tri = tri.reshape(n, 9)
    h_ref, tuv = oracle.kat("tri_hit", tri, ray)
    exp = (h_ref == 1) & (tuv[:, 0] >= np.float32(1e-5))
    out, hit = gpu.kat_device("tri_hit_f", tri, ray)
    assert np.array_equal(hit.astype(bool), exp)
    assert np.array_equal(_bits(out[exp]), _bits(tuv[exp]))
    assert 0.1 < exp.mean() < 0.9


def test_packed_pair_box_test_equals_exact(gpu, oracle):
    """pair_hit (both children of a BVH pair, packed slab arithmetic, filtered with a
    self-relative bound) == the reference slab test for each box, on face/edge/corner
    targets, degenerate slots and rays with zero direction components."""
    rng = np.random.default_rng(4242)
    n = 200000
    box, ray = _adversarial_boxes(rng, n)
    box[rng.random(n) < 0.05, 6] = 0.0                        # degenerate (padding) boxes
    other = np.roll(box, 1, axis=0)
    ref0, _ = oracle.kat("box_hit", box, ray)
    ref1, _ = oracle.kat("box_hit", other, ray)
    out = gpu.kat_device("box_pair", np.concatenate([box, other], 1), ray)
    assert np.array_equal(out[:, 0], ref0)
    assert np.array_equal(out[:, 1], ref1)
    assert 0.2 < ref0.mean() < 0.9


def test_device_cr_rcp_sqrt(gpu):
    """rt_math.h rcp_cr/sqrt_cr (the device's correctly rounded reciprocal and sqrt, the
    compiler's sequences) against IEEE float32 (numpy), bit for bit: every significand of the binades [1, 4)
    (rounding depends only on the significand, and for sqrt on the exponent's parity),
    both signs for rcp, plus 4M random bit patterns over the whole float range (the
    out-of-range inputs take the compiler's general sequences)."""
    sig = (np.arange(1 << 24, dtype=np.uint32) + np.uint32(0x3F800000)).view(np.float32)   # [1, 4)
    rng = np.random.default_rng(5)
    rnd = rng.integers(0, 1 << 32, size=1 << 22, dtype=np.uint64).astype(np.uint32).view(np.float32)
    edges = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 2.0 ** -125, 2.0 ** 125, 2.0 ** -126, 2.0 ** 126,
                      2.0 ** -100, 2.0 ** 100, 1e-45, 3.4e38], np.float32)
    with np.errstate(all="ignore"):
        for x in (sig, -sig, rnd, edges):
            x = np.ascontiguousarray(x.reshape(-1, 1))
            got = gpu.kat_device("rcp_cr", x).reshape(-1)
            ref = (np.float32(1.0) / x).reshape(-1)
            nan = np.isnan(ref)
            assert np.array_equal(np.isnan(got), nan)
            assert np.array_equal(_bits(got[~nan]), _bits(ref[~nan])), "rcp_cr"
            xs = np.abs(x)
            got = gpu.kat_device("sqrt_cr", xs).reshape(-1)
            ref = np.sqrt(xs).reshape(-1)
            nan = np.isnan(ref)
            assert np.array_equal(np.isnan(got), nan)
            assert np.array_equal(_bits(got[~nan]), _bits(ref[~nan])), "sqrt_cr"
