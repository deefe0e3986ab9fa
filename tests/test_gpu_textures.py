"""Textured shading mode on the GPU (build-defined; see tests/test_textures.py): frames
must equal the oracle's restatement of the same mode; with the mode off, textured
scenes render exactly as the reference."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, scene_path
from test_gpu_render import check_frame

sys.path.insert(0, os.path.join(ROOT, "tools"))
import make_atlas  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scene,w,h,spp", [("world8_tex", 200, 150, 2), ("world8_stress_tex", 160, 120, 4),
                                           ("world16_tex", 128, 96, 1)])
def test_textured_frame_parity(gpu, oracle, scene, w, h, spp):
    s = gpu.Scene.load_json(scene_path(scene), w, h)
    s.load_atlas()
    fr = s.render(spp=spp, textures=True, want=("rgba", "radiance", "hit_inst", "hit_tri"))
    o = oracle.load(scene_path(scene), w, h)
    o.set_atlas(make_atlas.atlas())
    o.set_textures(True)
    ofr = oracle.render(o, spp=spp, nthreads=8)
    check_frame(fr, ofr, spp)
    st = fr["stats"]
    assert (st["rays"], st["nodes"], st["leaves"], st["tri_tests"]) == tuple(int(x) for x in ofr["stats"])
    fast = s.render(spp=spp, textures=True, want=("rgba", "radiance"), stats=False)
    for k in ("rgba", "radiance"):
        assert np.array_equal(fast[k].view(np.uint32), fr[k].view(np.uint32)), k


def test_textures_off_is_the_reference(gpu, oracle):
    s = gpu.Scene.load_json(scene_path("world8_tex"), 160, 120)
    s.load_atlas()
    fr = s.render(spp=1, want=("rgba", "radiance", "hit_inst", "hit_tri"))
    check_frame(fr, oracle.render(oracle.load(scene_path("world8"), 160, 120), spp=1, nthreads=8))


def test_textures_need_an_atlas(gpu):
    s = gpu.Scene.load_json(scene_path("world8_tex"), 32, 24)
    with pytest.raises(gpu.RtError) as e:
        s.render(textures=True)
    assert e.value.code == gpu.RT_ERR_STATE
