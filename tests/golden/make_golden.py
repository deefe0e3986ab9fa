#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz).

Two families:

1. ``kat_<op>.npz`` — known-answer vectors for the math primitives on the hot
   path, produced by ``oracle/_ref/kat_ref``: the REFERENCE's own
   include/raymath/{linear.h,geometry.h}, src/rayopt/{z_order,bounding_box}.cu and
   src/rayprimitives/entity.cu compiled unmodified with g++ (``make -C oracle ref``).  Inputs are seeded numpy draws
   concentrated on the numerically delicate regions (grazing rays, triangle
   edges, tiny vectors under the 1e-5 threshold, signed zeros).

2. ``frame_<scene>_<w>x<h>_<mode>.npz`` — oracle frames (RGBA8, radiance, hit
   ids, counters).  These are produced by the oracle restatement and are pinned
   indirectly: their ray/node/leaf/triangle counters equal the measurements of
   the reference recorded in SURVEY.md Appendix D (checked by
   tests/test_oracle.py).

Run in the build container (needs /root/reference for family 1):
    make -C oracle ref && python tests/golden/make_golden.py
"""
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
KAT = os.path.join(ROOT, "oracle", "_ref", "kat_ref")

N = 4096


def _run(op, n, inputs, n_f=0, n_i=0, n_u=0):
    with tempfile.TemporaryDirectory() as d:
        fi, fo = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fi, "wb") as f:
            for a in inputs:
                f.write(np.ascontiguousarray(a, dtype=np.float32).tobytes())
        subprocess.check_call([KAT, op, str(n), fi, fo])
        raw = open(fo, "rb").read()
    of = np.frombuffer(raw[: 4 * n_f], dtype=np.float32)
    oi = np.frombuffer(raw[4 * n_f: 4 * n_f + 4 * n_i], dtype=np.int32)
    ou = np.frombuffer(raw[4 * n_f + 4 * n_i: 4 * n_f + 4 * n_i + 8 * n_u], dtype=np.uint64)
    assert len(raw) == 4 * n_f + 4 * n_i + 8 * n_u, (op, len(raw))
    return of, oi, ou


def _vecs(rng, n, scale_pow=(-7, 3)):
    mag = 10.0 ** rng.uniform(*scale_pow, size=(n, 1))
    v = rng.normal(size=(n, 3)) * mag
    # sprinkle exact zeros / negative zeros / axis-aligned vectors
    m = rng.random(size=(n, 3))
    v[m < 0.08] = 0.0
    v[(m >= 0.08) & (m < 0.12)] = -0.0
    return v.astype(np.float32)


def _quats(rng, n):
    q = rng.normal(size=(n, 4)).astype(np.float32)
    q[: n // 8] = [0, 0, 0, 1]                                  # identity (the cube world's poses)
    q[n // 8: n // 4] = [-0.0, -0.0, -0.0, 1]                   # inverse of identity
    sc = rng.choice([1.0, 0.5, 2.0, 1e-3, 1e-4], size=(n, 1))
    q[n // 4:] = (q[n // 4:] / np.linalg.norm(q[n // 4:], axis=1, keepdims=True) * sc[n // 4:]).astype(np.float32)
    return q


def _tri_rays(rng, n):
    """Triangles (cube-face triangles + random) and rays aimed at points near their edges."""
    s = np.float32(0.999) * np.float32(0.5)
    cube = np.array([[-s, s, -s], [s, s, -s], [-s, -s, -s], [s, -s, -s], [-s, s, s], [s, s, s], [-s, -s, s], [s, -s, s]], np.float32)
    faces = [(3, 0, 1), (2, 0, 3), (0, 4, 1), (4, 5, 1), (3, 1, 7), (1, 5, 7), (2, 6, 0), (0, 6, 4), (6, 7, 4), (4, 7, 5), (6, 2, 3), (3, 7, 6)]
    tris = np.empty((n, 3, 3), np.float32)
    half = n // 2
    for i in range(half):
        tris[i] = cube[list(faces[i % 12])]
    tris[half:] = rng.normal(size=(n - half, 3, 3)).astype(np.float32)
    # barycentric targets around the triangle, dense near the edges
    u = rng.uniform(-0.02, 1.02, size=n)
    v = rng.uniform(-0.02, 1.02, size=n)
    near = rng.random(n) < 0.5
    v[near] = (1 - u[near]) + rng.normal(scale=1e-6, size=near.sum())
    w = 1 - u - v
    p = tris[:, 0] * w[:, None] + tris[:, 1] * u[:, None] + tris[:, 2] * v[:, None]
    o = (p + rng.normal(size=(n, 3)) * 4).astype(np.float32)
    d = (p - o).astype(np.float32)
    graze = rng.random(n) < 0.1                                # nearly parallel to the plane
    nrm = np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0])
    d[graze] -= (np.sum(d[graze] * nrm[graze], 1) / np.maximum(np.sum(nrm[graze] ** 2, 1), 1e-30))[:, None] * nrm[graze] * 0.9999
    return tris.reshape(n, 9), np.concatenate([o, d], 1).astype(np.float32)


def make_kats():
    rng = np.random.default_rng(20261015)
    out = {}
    v = _vecs(rng, N)
    of, _, _ = _run("normalize3", N, [v], n_f=3 * N)
    out["normalize3"] = dict(v=v, out=of.reshape(N, 3))
    a, b = _vecs(rng, N), _vecs(rng, N)
    of, _, _ = _run("cross", N, [a, b], n_f=3 * N)
    out["cross"] = dict(a=a, b=b, out=of.reshape(N, 3))
    d, nn = _vecs(rng, N, (-2, 2)), _vecs(rng, N, (-2, 2))
    of, _, _ = _run("reflect", N, [d, nn], n_f=3 * N)
    out["reflect"] = dict(d=d, n=nn, out=of.reshape(N, 3))
    n12 = rng.choice(np.array([1.0, 0.8, 1.25, 1.5, 0.6667], np.float32), size=(N, 2)).astype(np.float32)
    of, oi, _ = _run("refract", N, [d, nn, n12], n_f=3 * N, n_i=N)
    out["refract"] = dict(d=d, n=nn, n12=n12, out=of.reshape(N, 3), tir=oi)
    q, vv = _quats(rng, N), _vecs(rng, N, (-3, 2))
    of, _, _ = _run("quat_rotate", N, [q, vv], n_f=3 * N)
    out["quat_rotate"] = dict(q=q, v=vv, out=of.reshape(N, 3))
    of, _, _ = _run("quat_inverse", N, [q], n_f=4 * N)
    out["quat_inverse"] = dict(q=q, out=of.reshape(N, 4))
    q2 = _quats(rng, N)
    of, _, _ = _run("quat_mul", N, [q, q2], n_f=4 * N)
    out["quat_mul"] = dict(a=q, b=q2, out=of.reshape(N, 4))
    tris, rays = _tri_rays(rng, N)
    of, oi, _ = _run("tri_hit", N, [tris, rays], n_f=3 * N, n_i=N)
    out["tri_hit"] = dict(tri=tris, ray=rays, out=of.reshape(N, 3), hit=oi)
    rr = np.concatenate([_vecs(rng, N, (-1, 2)), _vecs(rng, N, (-3, 1))], 1)
    of, _, _ = _run("ray_ctor", N, [rr], n_f=6 * N)
    out["ray_ctor"] = dict(ray=rr, out=of.reshape(N, 6))
    zv = (rng.normal(size=(N, 3)) * 10 ** rng.uniform(-3, 3, size=(N, 1))).astype(np.float32)
    zv[:16] = 0.0
    zv[16:32] = -0.0
    _, _, ou = _run("zorder", N, [zv], n_u=N)
    out["zorder"] = dict(v=zv, out=ou)
    at = np.concatenate([_vecs(rng, 256, (-1, 1)), rng.uniform(-100, 100, size=(256, 1)).astype(np.float32)], 1)
    at[0] = [1, 0, 0, 45]                                        # the cube-world camera orientation
    of, _, _ = _run("axis_angle", 256, [at], n_f=4 * 256)
    out["axis_angle"] = dict(a=at, out=of.reshape(256, 4))
    of, _, _ = _run("to_mat3", N, [q], n_f=9 * N)
    out["to_mat3"] = dict(q=q, out=of.reshape(N, 9))
    for k, dct in out.items():
        np.savez_compressed(os.path.join(HERE, f"kat_{k}.npz"), **dct)
        print("kat", k, {kk: vv.shape for kk, vv in dct.items()})


def _adv_boxes(rng, n):
    """Boxes with rays aimed at points near them, dense on faces, edges and corners (the slab
    test's ties), zero direction components, degenerate boxes, negative-zero coordinates."""
    mn = (rng.normal(size=(n, 3)) * 4).astype(np.float32)
    mx = (mn + np.abs(rng.normal(size=(n, 3))) + np.float32(1e-3)).astype(np.float32)
    mx[: n // 16] = mn[: n // 16]                                 # flat / point boxes
    nd = (rng.random((n, 1)) < 0.95).astype(np.float32)
    box = np.concatenate([mn, mx, nd], 1).astype(np.float32)
    o = (rng.normal(size=(n, 3)) * 20).astype(np.float32)
    t = rng.uniform(-0.05, 1.05, size=(n, 3)).astype(np.float32)
    snap = rng.random((n, 3))
    t[snap < 0.3] = 0.0
    t[(snap >= 0.3) & (snap < 0.6)] = 1.0
    tgt = (mn + (mx - mn) * t).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d[rng.random((n, 3)) < 0.04] = 0.0
    d[rng.random((n, 3)) < 0.01] = -0.0
    inside = rng.random(n) < 0.05                                  # origins inside the box
    o[inside] = ((mn + mx) * np.float32(0.5))[inside]
    return box, np.concatenate([o, d], 1).astype(np.float32)


def make_kats_geometry():
    """Round 5: the slab test (BoundingBox::intersects), from_local / merge (create_boxes and the
    BVH level merges) and the Entity pose transforms (cast_local, Hitable::hit), from the
    reference's bounding_box.cu / entity.cu compiled unmodified with g++ (oracle/Makefile ref)."""
    rng = np.random.default_rng(20261018)
    out = {}
    n = 8192
    box, ray = _adv_boxes(rng, n)
    of, oi, _ = _run("box_hit", n, [box, ray], n_f=n, n_i=n)
    out["box_hit"] = dict(box=box, ray=ray, t=of, hit=oi)
    q = _quats(rng, N)
    q[N // 4: N // 2] = [0, 0, 0, 1]                              # the cube world's identity poses
    ent = np.concatenate([q, _vecs(rng, N, (-1, 3))], 1).astype(np.float32)
    b0, _ = _adv_boxes(rng, N)
    of, oi, _ = _run("box_from_local", N, [b0, ent], n_f=6 * N, n_i=N)
    out["box_from_local"] = dict(box=b0, entity=ent, out=of.reshape(N, 6), nd=oi)
    b1, _ = _adv_boxes(rng, N)
    b1[: N // 8, :6] = b0[: N // 8, :6]                           # equal boxes / shared faces
    of, oi, _ = _run("box_merge", N, [b0, b1], n_f=6 * N, n_i=N)
    out["box_merge"] = dict(a=b0, b=b1, out=of.reshape(N, 6), nd=oi)
    v = _vecs(rng, N, (-3, 3))
    of, _, _ = _run("entity", N, [ent, v], n_f=12 * N)
    out["entity"] = dict(entity=ent, v=v, out=of.reshape(N, 12))
    # Hitable::hit's pose step around a local hit (hitable.cu:7-38): rays from _vecs, local hits
    # at random times (zeros, tiny, large) with random normals (tiny ones under the threshold)
    rr = np.concatenate([_vecs(rng, N, (-1, 2)), _vecs(rng, N, (-3, 1))], 1).astype(np.float32)
    hit = np.concatenate([(10.0 ** rng.uniform(-6, 3, size=(N, 1))).astype(np.float32), _vecs(rng, N, (-7, 1))], 1)
    hit[: N // 32, 0] = 0.0
    of, _, _ = _run("hitable", N, [ent, rr, hit], n_f=10 * N)
    out["hitable"] = dict(entity=ent, ray=rr, hit=hit.astype(np.float32), out=of.reshape(N, 10))
    for k, dct in out.items():
        np.savez_compressed(os.path.join(HERE, f"kat_{k}.npz"), **dct)
        print("kat", k, {kk: vv.shape for kk, vv in dct.items()})


FRAMES = [  # (scene, w, h, use_bvh, spp, semantics)
    ("world1", 256, 256, 1, 1, 1),      # config 1: CPU path (raytracer.cc)
    ("world1", 256, 256, 1, 1, 0),
    ("world1", 160, 120, 0, 1, 0),      # brute force (config 2 mode)
    ("world8", 160, 120, 1, 1, 0),
    ("world8_stress", 160, 120, 1, 1, 0),
    ("world8_stress", 96, 64, 1, 4, 0),
    ("world16", 128, 96, 1, 1, 0),
]


def make_frames():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle  # noqa: E402
    orc = Oracle()
    for scene, w, h, bvh, spp, sem in FRAMES:
        s = orc.load(os.path.join(ROOT, "scenes", scene + ".json"), w, h)
        fr = orc.render(s, semantics=sem, use_bvh=bvh, spp=spp, nthreads=8)
        name = f"frame_{scene}_{w}x{h}_{'bvh' if bvh else 'brute'}_spp{spp}_{'cpu' if sem else 'gpu'}.npz"
        np.savez_compressed(os.path.join(HERE, name), **fr)
        print("frame", name, fr["stats"])


if __name__ == "__main__":
    what = sys.argv[1:] or ["kats", "frames"]
    if "kats" in what:
        make_kats()
    if "kats" in what or "geometry" in what:
        make_kats_geometry()
    if "frames" in what:
        make_frames()
