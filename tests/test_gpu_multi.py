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


@pytest.mark.parametrize("ranks,depth", [(2, 4), (8, 8), (3, 4)])
def test_multi_device_frames_in_flight(gpu, oracle, ranks, depth):
    """rt_scene_set_devices with frame slots: frame f renders, gathers and un-permutes on its
    slot's streams while later frames start; each frame is issued asynchronously on the caller's
    stream into one of `depth` device buffers, which the caller copies to pinned host memory on
    that stream before the buffer is reused `depth` frames later (the un-permute must wait for
    that copy).  Every frame, each from its own camera, equals the oracle's frame."""
    import torch
    w, h, spp = 120, 81, 2
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s.set_frame_slots(depth)
    s.set_devices([0], ranks)
    o = oracle.load(scene_path("world8_stress"), w, h)
    st = torch.cuda.Stream()
    bufs = [torch.empty((h, w), dtype=torch.int32, device="cuda") for _ in range(depth)]
    n = 2 * depth + 1
    host = [torch.empty((h, w), dtype=torch.int32, pin_memory=True) for _ in range(n)]
    poses = []
    for f in range(n):
        a = 0.02 * f
        s.translate_camera([0.1 * (f % 3) - 0.1, 0.0, 0.15])
        s.rotate_camera([0.0, np.sin(a / 2), 0.0, np.cos(a / 2)])
        poses.append(s.camera())
        with torch.cuda.stream(st):
            bufs[f % depth].fill_(-1)                        # caller work on the buffer before the frame
            s.render_device(spp=spp, rgba_ptr=bufs[f % depth].data_ptr(), stream=st.cuda_stream)
            host[f].copy_(bufs[f % depth], non_blocking=True)
    st.synchronize()
    for f in range(n):
        o.set_camera(*poses[f])
        exp = oracle.render(o, spp=spp, nthreads=NTHREADS, want=("rgba",))
        got = {"rgba": host[f].numpy().view(np.uint32)}
        assert_frames_equal(got, exp, keys=("rgba",), ctx=f)
    # the synchronous entry (rt_update_scene) after asynchronous frames: its own frame only
    s.update_scene(16, True)
    o.set_camera(*s.camera())
    one = oracle.render(o, spp=1, nthreads=NTHREADS, want=("rgba",))
    assert_frames_equal({"rgba": s.canvas()}, one, keys=("rgba",))


def test_multi_device_replicas(gpu, oracle):
    """Real replicas (n_devices = 2): scene upload on device 1, camera / instance-pose sync to the
    replica, the cross-device ncclGather, with frames in flight.  Needs two GPUs; on a one-GPU box
    it is skipped, and multi-device parity (n_devices > 1) is then unpinned on hardware
    (DESIGN.md §6)."""
    if gpu.device_count() < 2:
        pytest.skip("needs two GPUs (the driver's GPU tests run on one)")
    import torch
    w, h, spp = 160, 97, 2
    s = gpu.Scene.load_json(scene_path("world8_stress"), w, h)
    s.set_frame_slots(4)
    s.set_devices([0, 1], 4)
    o = oracle.load(scene_path("world8_stress"), w, h)
    st = torch.cuda.Stream()
    buf = torch.empty((h, w), dtype=torch.int32, device="cuda")
    for f in range(6):
        s.translate_camera([0.0, 0.05 * f, 0.1])
        if f == 3:                                       # an instance moves: replicas rebuild from it
            p = s.export("instances")[5]
            s.set_trans(5, pos=p[4:7] + np.float32([0.5, 0.0, 0.0]))
            o.set_trans(5, pos=p[4:7] + np.float32([0.5, 0.0, 0.0]))
        with torch.cuda.stream(st):
            s.render_device(spp=spp, rgba_ptr=buf.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        mirror_camera(s, o)
        exp = oracle.render(o, spp=spp, nthreads=NTHREADS, want=("rgba",))
        assert_frames_equal({"rgba": buf.cpu().numpy().view(np.uint32)}, exp, keys=("rgba",), ctx=f)
