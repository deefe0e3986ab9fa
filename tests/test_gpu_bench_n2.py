"""bench.py's N > 1 code path on one GPU: N ranks launched the
way the driver launches them (python -m torch.distributed.run, one process per rank,
MASTER_ADDR 127.0.0.1), with the gloo backend so that the ranks may share the one GPU (RCCL
refuses two ranks on one device).  This runs bench.py's rank logic, its all-reduces and the
frame pipeline with frames in flight (FramePipeline's host-staged gather: per-slot staging,
gather and un-permute ordering as on RCCL) end to end, at N = 2, 4 (the quarter-grid policy of
small slices) and 8 (one-row pixel groups); rank 0 reports the CRC-32 of every timed frame it
assembled on the host, and each must equal the one-process frame's, as must the dumped last
frame bit for bit.  Named to run first among the GPU tests: the ranks start before this test
process has touched the GPU."""
import json
import os
import socket
import subprocess
import sys
import zlib

import numpy as np
import pytest

from conftest import ROOT, scene_path

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("ranks,size", [(2, (320, 180, 2)), (2, (1920, 1080, 8)), (4, (1920, 1080, 8)),
                                        (8, (1920, 1080, 8))])
def test_bench_ranks_gloo(request, tmp_path, ranks, size):
    W, H, spp = size
    steps = 6
    dump = str(tmp_path / "frame.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--dist-backend", "gloo", "--steps", str(steps),
           "--warmup", "2", "--frames-in-flight", "4", "--no-cpu-baseline", "--no-camera-path",
           "--no-device-resident", "--width", str(W), "--height", str(H), "--spp", str(spp), "--frame-crcs",
           "--dump-frame", dump]
    # several processes share the GPU here: fewer hardware queues each (HIP's default, 4)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", RT_BENCH_HW_QUEUES="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    log = r.stdout + r.stderr
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_n%d_gloo_%dx%d.log" % (ranks, W, H)), "w") as f:
        f.write(" ".join(cmd) + "\n" + log)
    assert r.returncode == 0, log[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, log[-3000:]                       # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == ranks and d["steps"] == steps and d["warmup"] == 2
    assert d["config"]["parallelism"].startswith("row-cyclic x%d" % ranks)
    assert d["frames_in_flight"] == 4
    assert d["value"] > 0 and d["ms_per_step"] > 0
    frame = np.load(dump)
    gpu = request.getfixturevalue("gpu")                      # this process's first GPU call
    one = gpu.Scene.load_json(scene_path("world8_stress"), W, H)
    ref = one.render(spp=spp, want=("rgba",), stats=True)
    assert frame.shape == (H, W)
    assert np.array_equal(frame, ref["rgba"])
    # every timed frame rank 0 assembled and read on the host, not only the last
    crc = zlib.crc32(np.ascontiguousarray(ref["rgba"]).view(np.int32).tobytes())
    assert d["frame_crcs"] == [crc] * steps, (d["frame_crcs"], crc)
    # the rays every rank counted (all-reduced) are the one-process frame's
    assert d["rays_per_frame"] == ref["stats"]["rays"]
