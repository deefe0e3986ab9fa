"""Textured shading mode (build-defined and parity-unpinned: the
reference leaves texture mapping a TODO, cube_world.cc:79-81 / phong.cu:18-23).
CPU side: the atlas PNG decoder, the cube tile mapping, the scene description with
the mode off, and the oracle's restatement of the mode."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, scene_path
from png_lib import read_png_rgba8

sys.path.insert(0, os.path.join(ROOT, "tools"))
import make_atlas  # noqa: E402

ATLAS = os.path.join(ROOT, "scenes", "assets", "atlas_synth.png")


def test_atlas_decoder_matches_independent_reader(rt):
    s = rt.Scene.load_json(scene_path("world8_tex"), 64, 48)
    assert not s.atlas_info()["loaded"]
    s.load_atlas()                                   # the JSON's "atlas", resolved against scenes/
    a = s.atlas()
    assert a.shape == (377, 285, 4)
    assert np.array_equal(a, read_png_rgba8(ATLAS))
    assert np.array_equal(a, make_atlas.atlas())     # the generator's pixels (all five PNG filters used)


def test_atlas_errors(rt, tmp_path):
    s = rt.Scene.load_json(scene_path("world8"), 32, 24)
    with pytest.raises(rt.RtError) as e:
        s.load_atlas(str(tmp_path / "missing.png"))
    assert e.value.code == rt.RT_ERR_IO
    bad = tmp_path / "bad.png"
    bad.write_bytes(b"not a png at all")
    with pytest.raises(rt.RtError) as e:
        s.load_atlas(str(bad))
    assert e.value.code == rt.RT_ERR_PARSE
    with pytest.raises(rt.RtError):
        s.set_atlas(np.zeros((0, 4, 4), np.uint8))
    s.set_atlas(np.full((3, 5, 4), 7, np.uint8))
    assert s.atlas_info() == {"width": 5, "height": 3, "loaded": True}


def test_cube_tiles_map_faces_onto_the_tile(rt):
    s = rt.Scene.load_json(scene_path("world8_stress_tex"), 32, 24)
    tc = s.export("texcoords")
    tris = s.export("tris")
    mats = tris[:, 3]
    tiles = {0: (0, 0, 64), 1: (128, 128, 64)}
    for m in range(s.info()["n_mats"]):
        rows = tc[mats == m]
        if m not in tiles:                            # the third cube kind has no "texture" key
            assert (rows == 0).all()
            continue
        assert (rows[:, 0] == 1).all()
        tx, ty, size = tiles[m]
        corners = np.concatenate([rows[:, 1:3], rows[:, 1:3] + rows[:, 3:5], rows[:, 1:3] + rows[:, 5:7]])
        # every vertex lands on the tile square (scale 0.999 cube: corners at +-0.4995 of the unit)
        assert corners[:, 0].min() >= tx - 1e-3 and corners[:, 0].max() <= tx + size + 1e-3
        assert corners[:, 1].min() >= ty - 1e-3 and corners[:, 1].max() <= ty + size + 1e-3
        assert np.unique(np.round(corners, 3), axis=0).shape[0] == 4      # the tile's 4 corners


def test_texture_keys_change_nothing_by_default(rt, oracle):
    a, b = rt.Scene.load_json(scene_path("world8"), 64, 48), rt.Scene.load_json(scene_path("world8_tex"), 64, 48)
    A, B = a.arrays(), b.arrays()
    for k in A:
        if k != "texcoords":
            assert np.array_equal(A[k].view(np.uint8), B[k].view(np.uint8)), k
    o1 = oracle.render(oracle.load(scene_path("world8"), 96, 72), spp=1, nthreads=8, want=("rgba",))
    o2 = oracle.render(oracle.load(scene_path("world8_tex"), 96, 72), spp=1, nthreads=8, want=("rgba",))
    assert np.array_equal(o1["rgba"], o2["rgba"])


def test_oracle_textured_mode_samples_the_atlas(oracle):
    sc = oracle.load(scene_path("world8_tex"), 96, 72)
    plain = oracle.render(sc, spp=1, nthreads=8)
    sc.set_atlas(make_atlas.atlas())
    sc.set_textures(True)
    tex = oracle.render(sc, spp=1, nthreads=8)
    assert np.array_equal(plain["hit_inst"], tex["hit_inst"])        # geometry unchanged
    lit = plain["hit_inst"] >= 0
    assert lit.any() and (tex["rgba"][lit] != plain["rgba"][lit]).mean() > 0.3
    assert np.array_equal(tex["rgba"][~lit], plain["rgba"][~lit])
