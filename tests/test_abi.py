"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
symbol include/rt_amd.h declares, and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, scene_path

HEADER = os.path.join(ROOT, "include", "rt_amd.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_listed(rt):
    assert declared_symbols() == sorted(rt.SYMBOLS)


def test_library_exports_every_declared_symbol(rt):
    L = ctypes.CDLL(rt.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_abi_version(rt):
    assert rt.lib().rt_abi_version() == 4


def test_library_is_gfx950_code(rt):
    """The shared object carries a gfx950 code object (built by hipcc --offload-arch=gfx950)."""
    blob = open(rt.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_render_without_gpu_fails_loudly(rt):
    if rt.device_count() > 0:
        pytest.skip("a GPU is present")
    s = rt.Scene.load_json(scene_path("world1"), 16, 16)
    with pytest.raises(rt.RtError) as e:
        s.render()
    assert e.value.code == rt.RT_ERR_NODEV
    with pytest.raises(rt.RtError):
        s.update_scene()


def test_oracle_not_linked_into_product(rt):
    """The product library must not depend on or embed the oracle."""
    blob = open(rt.LIB_PATH, "rb").read()
    assert b"orc_render" not in blob and b"liboracle" not in blob


def test_cpp_shim_and_cli_compile_against_the_abi(tmp_path):
    """include/rtracer_amd.hpp (the reference's rtracer/renv/procedural C++ API over the C
    ABI) compiles and links with a reference-style caller and with the CLI; nothing is
    run here (no GPU in this container)."""
    import subprocess
    inc = os.path.join(ROOT, "include")
    libdir = os.path.join(ROOT, "gpu-ray-tracer_amd")
    for src in (os.path.join(ROOT, "tests", "shim_world.cpp"), os.path.join(ROOT, "tests", "shim_main.cpp"),
                os.path.join(libdir, "cli", "rtracer.cpp")):
        hip = ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-L/opt/rocm/lib", "-lamdhip64"] \
            if src.endswith("rtracer.cpp") else []
        r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", inc, src, "-o", str(tmp_path / "a.out"),
                            "-L", libdir, "-lrt_amd"] + hip, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_frame_slots_arguments(rt):
    """rt_scene_set_frame_slots takes 1 to 8 (host-side state; no GPU needed)."""
    s = rt.Scene.load_json(scene_path("world1"), 16, 16)
    for n in (2, 4, 8, 3, 1):
        s.set_frame_slots(n)
    for n in (0, 9):
        with pytest.raises(rt.RtError) as e:
            s.set_frame_slots(n)
        assert e.value.code == rt.RT_ERR_ARG


def test_overlap_policy_arguments(rt):
    """rt_scene_set_overlap takes RT_OVERLAP_HALF (0), RT_OVERLAP_FULL (1) or RT_OVERLAP_STREAM (2)
    (host-side state)."""
    s = rt.Scene.load_json(scene_path("world1"), 16, 16)
    s.set_frame_slots(4)
    s.set_overlap(True)
    s.set_overlap(False, stream=True)
    s.set_overlap(False)
    for bad in (3, -1):
        assert rt.lib().rt_scene_set_overlap(s._h, bad) == rt.RT_ERR_ARG


def test_host_copy_entries_without_gpu(rt):
    """ABI 4's host-readable frame entries: argument checks, and no pinned memory without a GPU
    (no CPU stand-in: the copy is a copy-engine transfer or nothing)."""
    L = rt.lib()
    assert L.rt_copy_to_host_async(None, None, 16, None) == rt.RT_ERR_ARG
    p = ctypes.c_void_p()
    assert L.rt_host_alloc(0, ctypes.byref(p)) == rt.RT_ERR_ARG
    assert L.rt_host_free(None) == rt.RT_OK
    assert L.rt_copy_engines_warm(None, 1) == rt.RT_ERR_ARG
    if rt.device_count() > 0:
        pytest.skip("a GPU is present")
    assert L.rt_host_alloc(4096, ctypes.byref(p)) == rt.RT_ERR_NODEV
    assert L.rt_copy_engines_warm((ctypes.c_void_p * 2)(None, None), 2) == rt.RT_ERR_NODEV
