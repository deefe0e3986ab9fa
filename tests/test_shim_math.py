"""The C++ shim's host math (include/rtracer_amd.hpp, rmath) against the reference-built KAT
fixtures, bit for bit (CPU only).

main.cc moves and turns the camera with rmath (main.cc:144-177): Quat(axis, theta) for a mouse
turn, Quat * Quat to compose it, Vec arithmetic / normalized for a key move.  The fixtures'
outputs come from the reference's own geometry.h / linear.h compiled with g++
(oracle/ref_kat/kat_driver.cpp), where the unqualified cos / sin in Quat(axis, theta)
(geometry.h:36-41) are the C double functions rounded to float."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def shim_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("shim") / "shim_rmath")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "shim_rmath.cpp"), "-o", exe],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return exe


def run_op(exe, tmp_path, op, n, *arrays, width):
    src, dst = str(tmp_path / (op + ".in")), str(tmp_path / (op + ".out"))
    np.concatenate([np.ascontiguousarray(a, np.float32).ravel() for a in arrays]).tofile(src)
    r = subprocess.run([exe, op, str(n), src, dst], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return np.fromfile(dst, np.float32).reshape(n, width)


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("op,keys,width", [("axis_angle", ["a"], 4), ("quat_mul", ["a", "b"], 4),
                                           ("normalize3", ["v"], 3), ("ray_ctor", ["ray"], 6)])
def test_shim_rmath_equals_reference_kat(shim_exe, tmp_path, op, keys, width):
    d = np.load(os.path.join(GOLD, "kat_%s.npz" % op))
    n = d[keys[0]].shape[0]
    out = run_op(shim_exe, tmp_path, op, n, *[d[k] for k in keys], width=width)
    exp = d["out"].reshape(n, width)
    assert np.array_equal(bits(out), bits(exp)), op


def test_shim_axis_angle_double_libm(shim_exe, tmp_path):
    """A dense theta sweep: the shim's Quat(axis, theta) equals (float) cos / sin (double) of the
    float 0.5f * theta (glibc, the functions a g++ TU calls), and the sweep holds angles where
    the float overloads round differently, so the test tells the two apart."""
    libm = ctypes.CDLL("libm.so.6")
    libm.cos.restype = libm.sin.restype = ctypes.c_double
    libm.cos.argtypes = libm.sin.argtypes = [ctypes.c_double]
    libm.cosf.restype = libm.sinf.restype = ctypes.c_float
    libm.cosf.argtypes = libm.sinf.argtypes = [ctypes.c_float]
    rng = np.random.default_rng(5)
    theta = np.concatenate([rng.uniform(-8, 8, 3000), np.linspace(-0.05, 0.05, 1000),
                            np.float32([0.785398163, 3.14159265, 1.57079633, 0.1, -0.1])]).astype(np.float32)
    axis = np.tile(np.float32([0.6, 0.0, 0.8]), (theta.size, 1))
    a = np.concatenate([axis, theta[:, None]], 1).astype(np.float32)
    out = run_op(shim_exe, tmp_path, "axis_angle", theta.size, a, width=4)
    half = (np.float32(0.5) * theta).astype(np.float32)
    c_d = np.float32([libm.cos(float(h)) for h in half])
    s_d = np.float32([libm.sin(float(h)) for h in half])
    c_f = np.float32([libm.cosf(float(h)) for h in half])
    s_f = np.float32([libm.sinf(float(h)) for h in half])
    assert np.array_equal(bits(out[:, 3]), bits(c_d))
    assert np.array_equal(bits(out[:, 0]), bits(np.float32(0.6) * s_d))
    assert np.array_equal(bits(out[:, 2]), bits(np.float32(0.8) * s_d))
    assert (bits(c_d) != bits(c_f)).any() or (bits(s_d) != bits(s_f)).any()
