"""Host-readable frames (ABI 4): pinned host buffers from rt_host_alloc,
device -> host copies on a copy engine (rt_copy_to_host_async), the engine warm-up, and
update_scene's canvas copy -- bytes equal to the device data, every size, stream-ordered."""
import ctypes

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [4, 4096 + 12, 1 << 20, 1920 * 1080 * 4, 3840 * 2160 * 4])
def test_copy_to_host_async_bytes(gpu, nbytes):
    import torch
    n = nbytes // 4
    g = torch.Generator(device="cpu").manual_seed(nbytes)
    src = torch.randint(-2 ** 31, 2 ** 31 - 1, (n,), dtype=torch.int32, generator=g)
    dev = src.cuda()
    hb = gpu.HostBuffer((n,), np.int32)
    hb.array[:] = 0
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    gpu.copy_to_host_async(hb.ptr, dev.data_ptr(), nbytes, st.cuda_stream)
    st.synchronize()
    assert np.array_equal(hb.array, src.numpy())
    hb.free()


def test_copy_is_stream_ordered_after_a_frame(gpu):
    """A frame rendered on a stream, then its copy on the same stream: the host sees the frame."""
    import torch
    W, H = 320, 180
    s = gpu.Scene.load_json(scene_path("world8_stress"), W, H)
    ref = s.render(spp=2, want=("rgba",))["rgba"]
    dev = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    hb = gpu.HostBuffer((H, W), np.int32)
    st = torch.cuda.Stream()
    for _ in range(3):
        hb.array[:] = 0
        s.render_device(spp=2, rgba_ptr=dev.data_ptr(), stream=st.cuda_stream)
        gpu.copy_to_host_async(hb.ptr, dev.data_ptr(), W * H * 4, st.cuda_stream)
        st.synchronize()
        assert np.array_equal(hb.array.view(np.uint32), ref)


def test_copy_engines_warm_idempotent(gpu):
    import torch
    streams = [torch.cuda.Stream() for _ in range(3)]
    gpu.copy_engines_warm([st.cuda_stream for st in streams])
    gpu.copy_engines_warm([st.cuda_stream for st in streams])      # once per process: returns at once
    L = gpu.lib()
    assert L.rt_copy_engines_warm(None, 1) == gpu.RT_ERR_ARG
    assert L.rt_copy_engines_warm((ctypes.c_void_p * 1)(None), 0) == gpu.RT_ERR_ARG


def test_update_scene_canvas_is_the_frame(gpu):
    """update_scene's post-condition (raytracer.cu:102-120): the pinned canvas holds the frame the
    renderer produces, after every call, including after the camera moved."""
    W, H = 256, 144
    s = gpu.Scene.load_json(scene_path("world8_stress"), W, H)
    for k in range(3):
        if k:
            s.translate_camera((0.0, 0.0, 0.5 * k))
        s.update_scene()
        ref = s.render(spp=1, want=("rgba",))["rgba"]
        assert np.array_equal(s.canvas(), ref), k
