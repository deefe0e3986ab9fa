"""CPU tests of the product's host side: worldN.json loading, the cube-world
generator and SceneBuilder (no GPU needed: device upload is lazy)."""
import numpy as np
import pytest

from conftest import scene_path

SCENES = ["world1", "world2", "world4", "world8", "world8_stress", "world16", "config"]


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("res", [(0, 0), (1920, 1080), (3840, 2160)])
def test_loader_matches_oracle_bitwise(rt, oracle, name, res):
    a = rt.Scene.load_json(scene_path(name), *res)
    b = oracle.load(scene_path(name), *res)
    A, B = a.arrays(), b.arrays()
    for k in B:
        assert np.array_equal(_bits(A[k]), _bits(B[k])), (name, k)
    assert a.info()["n_instances"] == b.n_instances


def test_instance_counts(rt):
    counts = {n: rt.Scene.load_json(scene_path(n)).info()["n_instances"] for n in ["world1", "world8", "world8_stress", "world16"]}
    assert counts == {"world1": 2, "world8": 380, "world8_stress": 570, "world16": 1452}


def test_global_near_uses_float_tan(rt):
    """camera.cu:7 is an nvcc TU: tan(float) -> tanf.  SURVEY App. C: 1-ulp sensitive at 1920/1000."""
    s = rt.Scene.load_json(scene_path("world8_stress"), 1920, 1080)
    cam = s.export("camera")
    fov = np.float32(np.float32(45 * np.pi) / np.float32(180))
    tanf = np.float32(np.tan(np.float64(fov)))    # tanf is correctly rounded for this argument
    near = np.float32(np.float32(np.float32(0.5) * np.float32(1920)) / np.float32(1000)) / tanf
    assert cam[7] == near


def test_missing_and_malformed_files(rt, tmp_path):
    with pytest.raises(rt.RtError) as e:
        rt.Scene.load_json(str(tmp_path / "nope.json"))
    assert e.value.code == rt.RT_ERR_IO
    bad = tmp_path / "bad.json"
    bad.write_text('{"cubes": [ {"Ka": [1,2,3,4]} ')
    with pytest.raises(rt.RtError) as e:
        rt.Scene.load_json(str(bad))
    assert e.value.code == rt.RT_ERR_PARSE
    deep = tmp_path / "deep.json"
    deep.write_text('{"atlas": "x", "depth": 10}')
    with pytest.raises(rt.RtError) as e:            # frames[MAX_DEPTH=10] would overflow (scene.cu:25,95)
        rt.Scene.load_json(str(deep))
    assert e.value.code == rt.RT_ERR_PARSE


def test_empty_world_loads(rt, tmp_path):
    p = tmp_path / "empty.json"
    p.write_text('{"atlas": "x", "grid_size": 0, "cubes": [], "width": 8, "height": 4}')
    s = rt.Scene.load_json(str(p))
    assert s.info()["n_instances"] == 0 and s.width == 8 and s.height == 4


def test_builder_matches_loader(rt):
    """SceneBuilder API reproduces the JSON loader's world1 scene."""
    ref = rt.Scene.load_json(scene_path("world1"), 64, 48)
    R = ref.arrays()
    b = rt.Scene.create("assets/sus.png")
    mats = R["materials"]
    meshes = [b.build_cube(0.999, m) for m in mats]
    for q, m in zip(R["instances"], R["inst_mesh"]):
        t = b.add_trans(meshes[m])
        b.set_trans(t, pos=q[4:7])
    import json
    doc = json.load(open(scene_path("world1")))
    inv = np.float32(1) / np.float32(255)
    for l in doc["lights"]["directional"]:                  # raw direction: DirLight normalizes (light.cuh:62)
        b.add_directional_light(l["dir"], inv * np.float32(l["col"]))
    for l in R["lights"]:
        if l[3] == 0:
            b.add_point_light(l[:3], l[4:8])
    cam, env = R["camera"], R["env"]
    fov = np.float32(np.float32(45 * np.pi) / np.float32(180))
    b.finish(64, 48, float(fov), float(cam[8]), cam_pos=cam[:3], cam_quat=cam[3:7], dist_atten=env[:3],
             ambience=env[3:7], depth=ref.info()["depth"])
    B = b.arrays()
    for k in R:
        assert np.array_equal(_bits(B[k]), _bits(R[k])), k


def test_builder_errors(rt):
    b = rt.Scene.create()
    with pytest.raises(rt.RtError):
        b.add_triangle(0, 0, 1, 2, rt.material())          # no mesh yet
    m = b.create_mesh()
    with pytest.raises(rt.RtError):
        b.add_triangle(m, 0, 1, 2, rt.material())          # no vertices yet
    with pytest.raises(rt.RtError):
        b.info()                                             # not finished


def test_camera_translate_rotate(rt, oracle):
    s = rt.Scene.load_json(scene_path("world8"), 32, 32)
    p0, q0 = s.camera()
    s.translate_camera([0, 0, 1])
    p1, _ = s.camera()
    assert np.linalg.norm(p1 - p0) == pytest.approx(1.0, abs=1e-5)
    s.rotate_camera([0, 0, 0, 1])                            # identity rotation: o = dr * o
    _, q1 = s.camera()
    assert np.allclose(q1, q0)
    r, u, f = s.camera_axes()
    assert abs(np.dot(r, u)) < 1e-6 and abs(np.dot(u, f)) < 1e-6


def test_spp_offsets_match_oracle(rt, oracle):
    for k in range(0, 300, 7):
        assert rt.spp_offset(k) == oracle.spp_offset(k)
    assert rt.spp_offset(0) == (0.0, 0.0)


@pytest.mark.parametrize("name", ["world1", "world8", "world8_stress", "world16_tex"])
def test_triangle_exports_one_record_per_triangle(rt, name):
    """ABI 3: RT_EXPORT_TRIS / RT_EXPORT_TEXCOORDS list every triangle once, in the flattened
    mesh order (the index space of hit_tri): as many records as rt_scene_info's n_tris, and each
    triangle's vertex indices appear exactly once."""
    s = rt.Scene.load_json(scene_path(name), 32, 24)
    n = s.info()["n_tris"]
    tris, tex = s.export("tris"), s.export("texcoords")
    assert tris.shape == (n, 4) and tex.shape == (n, 7)
    assert len({tuple(r) for r in tris[:, :3]}) == n or n == 0
