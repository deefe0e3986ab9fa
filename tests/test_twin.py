"""CPU tests of the oracle's SceneBuilder, camera and pose setters (the checker the GPU
tests use for built scenes, moved cameras and moved / rotated instances): the oracle's
builder reproduces its own JSON loader, and the product's host-side scene arrays equal the
oracle's for the same builder calls and poses (no GPU: device upload is lazy)."""
import json

import numpy as np
import pytest

from conftest import scene_path
from twin import Twin, mirror_camera, mirror_instances


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def _world_by_builder(b, ref_arrays, doc, W, H, depth):
    R = ref_arrays
    meshes = [b.build_cube(0.999, m) for m in R["materials"]]
    for q, m in zip(R["instances"], R["inst_mesh"]):
        t = b.add_trans(meshes[m])
        b.set_trans(t, pos=q[4:7])
    inv = np.float32(1) / np.float32(255)
    for l in doc["lights"].get("directional", []):           # raw direction: DirLight normalizes (light.cuh:62)
        b.add_directional_light(l["dir"], inv * np.float32(l["col"]))
    for l in R["lights"]:
        if l[3] == 0:
            b.add_point_light(l[:3], l[4:8])
    cam, env = R["camera"], R["env"]
    fov = np.float32(np.float32(45 * np.pi) / np.float32(180))
    b.finish(W, H, float(fov), float(cam[8]), cam_pos=cam[:3], cam_quat=cam[3:7], dist_atten=env[:3],
             ambience=env[3:7], depth=depth)


@pytest.mark.parametrize("name", ["world1", "world8_stress"])
def test_oracle_builder_reproduces_oracle_loader(oracle, name):
    W, H = 48, 32
    ref = oracle.load(scene_path(name), W, H)
    b = oracle.create()
    _world_by_builder(b, ref.arrays(), json.load(open(scene_path(name))), W, H, ref.depth)
    A, B = ref.arrays(), b.arrays()
    for k in A:
        assert np.array_equal(_bits(A[k]), _bits(B[k])), k
    fa = oracle.render(ref, spp=2, nthreads=4)
    fb = oracle.render(b, spp=2, nthreads=4)
    for k in ("rgba", "radiance", "hit_inst", "hit_tri"):
        assert np.array_equal(_bits(fa[k]), _bits(fb[k])), k
    assert np.array_equal(fa["stats"], fb["stats"])


def _mixed_scene(tw):
    """Meshes with their own poses, triangles added to meshes out of order, per-triangle
    materials and texture coordinates, instances with rotations, both light kinds."""
    m = lambda **k: np.array(list(k.get("Ke", (0, 0, 0, 0))) + list(k.get("Ka", (.1, .1, .1, 1))) +
                             list(k.get("Kd", (.5, .4, .3, 1))) + list(k.get("Ks", (0, 0, 0, 0))) +
                             list(k.get("Kt", (0, 0, 0, 0))) + list(k.get("Kr", (0, 0, 0, 0))) +
                             [k.get("alpha", 0.0), k.get("eta", 1.0)], np.float32)
    v = [tw.add_vertex(*p) for p in ((0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 1), (-1, 0.5, 0.25))]
    m0 = tw.create_mesh((0.1, 0.0, -0.2), (0.0, 0.3826834, 0.0, 0.9238795))
    m1 = tw.create_mesh()
    tw.add_triangle(m0, v[0], v[1], v[2], m(Kd=(.9, .1, .1, 1)))
    tw.add_triangle(m1, v[0], v[2], v[3], m(Kr=(.5, .5, .5, 1)))
    tw.add_triangle(m0, v[1], v[4], v[2], m(Kt=(.6, .7, .8, 1), eta=1.4))
    tw.add_triangle(m1, v[3], v[4], v[5], m(Ks=(.5, .5, .5, 1), alpha=4.0))
    c = tw.build_cube(0.75, m(Kd=(.2, .8, .2, 1)), tile=(10.0, 20.0, 32.0))
    for k, mesh in enumerate((m0, m1, c, c, m0)):
        t = tw.add_trans(mesh)
        q = np.array([0.1 * k, 0.2, -0.05 * k, 1.0], np.float32)
        tw.set_trans(t, pos=(1.5 * k - 3.0, 0.25 * k, 2.0), quat=q / np.linalg.norm(q))
    tw.add_directional_light((0.2, -1.0, 0.4), (0.9, 0.9, 0.8, 1.0))
    tw.add_point_light((0.0, 4.0, -1.0), (1.0, 0.9, 0.7, 1.0))
    tw.add_directional_light((-0.3, -0.2, 1.0), (0.3, 0.3, 0.5, 1.0))
    tw.finish(40, 30, 0.7, 25.0, cam_pos=(0.0, 1.0, -8.0), cam_quat=(0.05, 0.0, 0.0, 0.99875),
              dist_atten=(0.5, 0.1, 0.01), ambience=(0.2, 0.2, 0.25, 1.0), depth=3)


def test_twin_builder_arrays_equal(rt, oracle):
    tw = Twin(rt, oracle)
    _mixed_scene(tw)
    A, B = tw.gpu.arrays(), tw.orc.arrays()
    for k in B:
        assert np.array_equal(_bits(A[k]), _bits(B[k])), k


def test_mirrored_camera_and_poses(rt, oracle):
    s = rt.Scene.load_json(scene_path("world8"), 64, 48)
    o = oracle.load(scene_path("world8"), 64, 48)
    s.translate_camera([0.5, -2.0, 1.0])
    s.rotate_camera([0.0247, 0.0, 0.0, 0.99969])
    mirror_camera(s, o)
    assert np.array_equal(_bits(s.export("camera")), _bits(o.arrays()["camera"]))
    s.set_trans(7, pos=(0.5, 9.0, -1.0), quat=(0.0, 0.38268343, 0.0, 0.9238795))
    mirror_instances(s, o)
    assert np.array_equal(_bits(s.export("instances")), _bits(o.arrays()["instances"]))


def test_oracle_setters_reject_bad_input(oracle):
    o = oracle.load(scene_path("world1"), 16, 16)
    with pytest.raises(AssertionError):
        o.set_trans(99, pos=(0, 0, 0))
    b = oracle.create()
    with pytest.raises(AssertionError):
        b.add_triangle(0, 0, 1, 2, np.zeros(26, np.float32))     # no mesh yet
    with pytest.raises(RuntimeError):
        oracle.render(b)                                         # not finished
