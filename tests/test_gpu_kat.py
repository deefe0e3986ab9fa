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
