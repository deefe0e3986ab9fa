"""bench.py's N > 1 code path on one GPU: two ranks launched the way the
driver launches them (python -m torch.distributed.run, one process per rank, MASTER_ADDR
127.0.0.1), with the gloo backend so that both ranks may share the one GPU (RCCL refuses two
ranks on one device).  This runs bench.py's rank logic, its all-reduces and the row-cyclic
gather / un-permute end to end; rank 0's gathered frame must equal the one-process frame bit
for bit.  Named to run first among the GPU tests: the ranks start before this test process
has touched the GPU."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, scene_path

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("size", [(320, 180, 2), (1920, 1080, 8)])
def test_bench_two_ranks_gloo(request, tmp_path, size):
    W, H, spp = size
    dump = str(tmp_path / "frame.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-camera-path", "--width", str(W), "--height", str(H), "--spp", str(spp),
           "--dump-frame", dump]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    log = r.stdout + r.stderr
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_n2_gloo_%dx%d.log" % (W, H)), "w") as f:
        f.write(" ".join(cmd) + "\n" + log)
    assert r.returncode == 0, log[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, log[-3000:]                       # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1
    assert d["config"]["parallelism"].startswith("row-cyclic x2")
    assert d["value"] > 0 and d["ms_per_step"] > 0
    frame = np.load(dump)
    gpu = request.getfixturevalue("gpu")                      # this process's first GPU call
    one = gpu.Scene.load_json(scene_path("world8_stress"), W, H)
    ref = one.render(spp=spp, want=("rgba",), stats=True)
    assert frame.shape == (H, W)
    assert np.array_equal(frame, ref["rgba"])
    # the rays both ranks counted (all-reduced) are the one-process frame's
    assert d["rays_per_frame"] == ref["stats"]["rays"]
