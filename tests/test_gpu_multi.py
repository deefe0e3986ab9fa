"""Multi-GPU frames from one host process (rt_scene_set_devices): whole frames
split into row-cyclic slices, gathered with RCCL and un-permuted on the first device.  On a
one-GPU box every slice renders on device 0 and the gather runs over a one-rank
communicator: the frame must be the single-device frame, bit for bit, and the oracle's.
(Replicas on other devices -- camera / instance / environment sync -- need a multi-GPU
node; the driver's 8-GPU runs use one process per GPU through torch.distributed.)"""
import numpy as np
import pytest

from conftest import scene_path
from twin import NTHREADS, assert_frames_equal, mirror_camera

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ranks", [2, 5, 8])
def test_multi_device_frames(gpu, oracle, ranks):
    w, h, spp = 240, 161, 4                                     # ragged: 161 rows
    one = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s.set_devices([0], ranks)
    o = oracle.load(scene_path("world8_stress"), w, h)
    for k, (d, a) in enumerate((([0, 0, 0], 0.0), ([0.5, -1.0, 2.0], 0.05), ([-1.0, 0.0, 0.5], -0.1))):
        for sc in (one, s):
            sc.translate_camera(d)
            sc.rotate_camera([np.sin(a / 2), 0, 0, np.cos(a / 2)])
        ref = one.render(spp=spp, want=("rgba",), stats=True)
        fr = s.render(spp=spp, want=("rgba",), stats=True)
        assert np.array_equal(fr["rgba"], ref["rgba"]), k
        st, rs = fr["stats"], ref["stats"]
        assert (st["rays"], st["nodes"], st["leaves"], st["tri_tests"]) == \
               (rs["rays"], rs["nodes"], rs["leaves"], rs["tri_tests"])
        mirror_camera(s, o)
        assert_frames_equal(fr, oracle.render(o, spp=spp, nthreads=NTHREADS), keys=("rgba",), ctx=k)
    # rt_update_scene (the reference's entry) goes through the split too; then back to one GPU
    s.update_scene(16, True)
    one.update_scene(16, True)
    assert np.array_equal(s.canvas(), one.canvas())
    s.set_devices([0], 1)
    assert np.array_equal(s.render(spp=spp)["rgba"], ref["rgba"])


def test_multi_device_rejects(gpu):
    s = gpu.Scene.load_json(scene_path("world8"), 64, 48)
    for devs, n in (([0, 0], 2), ([0], -1), ([99], 1), ([0], 49)):
        with pytest.raises(gpu.RtError) as e:
            s.set_devices(devs, n)
        assert e.value.code == gpu.RT_ERR_ARG, (devs, n)
    s.set_devices([0], 4)
    with pytest.raises(gpu.RtError) as e:                        # RGBA8 only
        s.render(want=("rgba", "hit_inst"))
    assert e.value.code == gpu.RT_ERR_ARG
