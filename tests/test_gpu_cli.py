"""The reference-facing front ends on the GPU: the headless CLI with the reference's
flags (gpu-ray-tracer_amd/cli/rtracer.cpp, main.cc:31-79) and a program written
against the C++ shim (include/rtracer_amd.hpp: SceneBuilder / update_scene /
get_canvas) -- both must produce the oracle's frame."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, scene_path

pytestmark = pytest.mark.gpu
CLI = os.path.join(ROOT, "gpu-ray-tracer_amd", "rtracer")


def _run(args, timeout=120):
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout)


def _ppm_rgb(path):
    data = open(path, "rb").read()
    head = data.split(b"\n", 3)
    w, h = map(int, head[1].split())
    return np.frombuffer(head[3], np.uint8).reshape(h, w, 3)


@pytest.mark.parametrize("flags,bvh", [(["-b"], 1), (["-b", "-r"], 0), (["--frames", "3", "-d", "8"], 1)])
def test_cli_frame_matches_oracle(oracle, tmp_path, flags, bvh):
    out = str(tmp_path / "f.ppm")
    r = _run([CLI, "-c", scene_path("world8"), "--width", "200", "--height", "120", "--out", out] + flags)
    assert r.returncode == 0, r.stderr
    assert "Loaded scene" in r.stdout
    assert ("Time: " in r.stdout) if "-b" in flags else ("FPS: " in r.stdout)
    o = oracle.render(oracle.load(scene_path("world8"), 200, 120), use_bvh=bvh, spp=1, nthreads=8, want=("rgba",))
    rgba = o["rgba"]
    exp = np.stack([(rgba >> 24) & 255, (rgba >> 16) & 255, (rgba >> 8) & 255], -1).astype(np.uint8)
    assert np.array_equal(_ppm_rgb(out), exp)


def test_cli_multisample_and_debug(tmp_path):
    out = str(tmp_path / "f.ppm")
    r = _run([CLI, "-c", scene_path("world8_stress"), "--width", "160", "--height", "90", "--spp", "4", "-b",
              "--out", out, "--debug", "80,45"])
    assert r.returncode == 0, r.stderr
    assert "shooting debug ray at 80, 45" in r.stdout and "shooting a ray" in r.stdout
    assert _ppm_rgb(out).shape == (90, 160, 3)


def test_cli_rejects_serial_and_bad_args():
    r = _run([CLI, "-c", scene_path("world1"), "-s"])
    assert r.returncode == 2 and "serial" in r.stderr
    assert _run([CLI]).returncode == 2
    r = _run([CLI, "-c", "/nonexistent.json", "-b"])
    assert r.returncode == 1 and "cannot load" in r.stderr


def _write_desc(path, rt):
    """world1 as a SceneBuilder description (the same construction test_scene.py checks)."""
    ref = rt.Scene.load_json(scene_path("world1"), 96, 72)
    R = ref.arrays()
    doc = json.load(open(scene_path("world1")))
    inv = np.float32(1) / np.float32(255)
    fov = np.float32(np.float32(45 * np.pi) / np.float32(180))
    cam, env = R["camera"], R["env"]
    g = lambda xs: " ".join("%.9g" % float(x) for x in xs)
    lines = ["96 72 %.9g %.9g %d" % (fov, cam[8], ref.info()["depth"]), g(cam[:7]), g(env[:7]), str(len(R["materials"]))]
    lines += [g(m) for m in R["materials"]]
    lines.append(str(len(R["instances"])))
    lines += ["%d %s" % (m, g(q[4:7])) for q, m in zip(R["instances"], R["inst_mesh"])]
    dirs = doc["lights"]["directional"]
    lines.append(str(len(dirs)))
    lines += [g(list(l["dir"]) + list(inv * np.float32(l["col"]))) for l in dirs]
    pts = [l for l in R["lights"] if l[3] == 0]
    lines.append(str(len(pts)))
    lines += [g(list(l[:3]) + list(l[4:8])) for l in pts]
    open(path, "w").write("\n".join(lines) + "\n")


def test_cpp_shim_scene_builder_frame(gpu, oracle, tmp_path):
    exe = str(tmp_path / "shim_world")
    inc = os.path.join(ROOT, "include")
    libdir = os.path.join(ROOT, "gpu-ray-tracer_amd")
    r = _run(["g++", "-O1", "-std=c++17", "-I", inc, os.path.join(ROOT, "tests", "shim_world.cpp"), "-o", exe,
              "-L", libdir, "-lrt_amd", "-Wl,-rpath," + libdir])
    assert r.returncode == 0, r.stderr
    desc, out = str(tmp_path / "w.txt"), str(tmp_path / "c.bin")
    _write_desc(desc, gpu)
    r = _run([exe, desc, out])
    assert r.returncode == 0, r.stdout + r.stderr
    frame = np.fromfile(out, np.uint32).reshape(72, 96)
    o = oracle.render(oracle.load(scene_path("world1"), 96, 72), spp=1, nthreads=8, want=("rgba",))
    assert np.array_equal(frame, o["rgba"])
    assert (frame != 0).any()


def test_cli_textured_mode(oracle, tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_atlas
    out = str(tmp_path / "t.ppm")
    r = _run([CLI, "-c", scene_path("world8_tex"), "--width", "160", "--height", "120", "-b", "--textures",
              "--out", out])
    assert r.returncode == 0, r.stderr
    o = oracle.load(scene_path("world8_tex"), 160, 120)
    o.set_atlas(make_atlas.atlas())
    o.set_textures(True)
    rgba = oracle.render(o, spp=1, nthreads=8, want=("rgba",))["rgba"]
    exp = np.stack([(rgba >> 24) & 255, (rgba >> 16) & 255, (rgba >> 8) & 255], -1).astype(np.uint8)
    got = _ppm_rgb(out)
    assert np.array_equal(got, exp), int((got != exp).sum())


@pytest.mark.parametrize("ranks", [2, 3, 8])
def test_cli_multi_device_slices(oracle, tmp_path, ranks):
    """--gpus 1 --ranks R: the reference caller's update_scene through rtracer::gpu::use_devices
    (rt_scene_set_devices) -- R row-cyclic slices, the RCCL gather (one-rank communicator on a
    one-GPU box) and the un-permute -- gives the oracle's frame."""
    out = str(tmp_path / "m.ppm")
    r = _run([CLI, "-c", scene_path("world8"), "--width", "200", "--height", "121", "--out", out, "--frames", "3",
              "--gpus", "1", "--ranks", str(ranks)])
    assert r.returncode == 0, r.stderr
    assert "slices" in r.stdout
    o = oracle.render(oracle.load(scene_path("world8"), 200, 121), spp=1, nthreads=8, want=("rgba",))
    rgba = o["rgba"]
    exp = np.stack([(rgba >> 24) & 255, (rgba >> 16) & 255, (rgba >> 8) & 255], -1).astype(np.uint8)
    assert np.array_equal(_ppm_rgb(out), exp)


def test_cpp_shim_main_cc_calls(oracle, tmp_path):
    """The reference front end's GPU-path calls through the shim (tests/shim_main.cpp: generate,
    update_scene, Canvas::get_surface over an SDL test double, main.cc's key and mouse camera
    moves, debug_cast): the frame the surface shows after the moves is the oracle's frame at the
    camera pose the program reports."""
    exe = str(tmp_path / "shim_main")
    inc = os.path.join(ROOT, "include")
    libdir = os.path.join(ROOT, "gpu-ray-tracer_amd")
    r = _run(["g++", "-O1", "-std=c++17", "-I", inc, os.path.join(ROOT, "tests", "shim_main.cpp"), "-o", exe,
              "-L", libdir, "-lrt_amd", "-Wl,-rpath," + libdir])
    assert r.returncode == 0, r.stderr
    out = str(tmp_path / "m.bin")
    W, H = 160, 100
    r = _run([exe, scene_path("world8_stress"), str(W), str(H), out])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Loaded scene" in r.stdout and "shooting a ray" in r.stdout
    raw = np.fromfile(out, np.uint8)
    frame = raw[:4 * W * H].view(np.uint32).reshape(H, W)
    pose = raw[4 * W * H:].view(np.float32)
    o = oracle.load(scene_path("world8_stress"), W, H)
    o.set_camera(pose[:3], pose[3:7])
    exp = oracle.render(o, spp=1, nthreads=8, want=("rgba",))["rgba"]
    assert np.array_equal(frame, exp)
    assert (frame != 0).any()


@pytest.mark.parametrize("extra", [["--in-flight", "4"], ["--gpus", "1", "--ranks", "8", "--in-flight", "8"],
                                   ["--in-flight", "8", "--readback"], ["--in-flight", "3", "--readback"]])
def test_cli_frames_in_flight(oracle, tmp_path, extra):
    """--in-flight D: frames issued asynchronously, D in flight, each into its own device buffer on
    its own stream (single device, and 8 row-cyclic slices through rt_scene_set_devices with one
    slot's streams per frame); --readback: every frame copied to pinned host memory by a copy
    engine once complete (the written frame is the host copy); the last frame equals the oracle's."""
    out = str(tmp_path / "p.ppm")
    r = subprocess.run([CLI, "-c", scene_path("world8_stress"), "--width", "240", "--height", "136", "--spp", "2",
                        "--frames", "12", "--out", out] + extra, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, GPU_MAX_HW_QUEUES="16"))
    assert r.returncode == 0, r.stderr
    assert "ms/frame" in r.stdout
    o = oracle.render(oracle.load(scene_path("world8_stress"), 240, 136), spp=2, nthreads=8, want=("rgba",))
    rgba = o["rgba"]
    exp = np.stack([(rgba >> 24) & 255, (rgba >> 16) & 255, (rgba >> 8) & 255], -1).astype(np.uint8)
    got = _ppm_rgb(out)
    assert np.array_equal(got, exp), int((got != exp).sum())
