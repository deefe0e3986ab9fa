#!/usr/bin/env python3
"""Copy-engine rate inside a torch process (torch's own HIP runtime), for host buffers made
with different hipHostMalloc flags: 40 device -> pinned-host copies of one 1080p RGBA8 frame
through rt_copy_to_host_async, timed by events on the copy stream.  Compare with
tools/copy_probe.hip (the /opt/rocm runtime) on the same box."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402

FLAGS = {"default": 0x0, "coherent": 0x40000000, "noncoherent": 0x80000000, "writecombined": 0x4}


def main():
    n = 1920 * 1080 * 4
    dev = torch.randint(0, 1 << 30, (n // 4,), dtype=torch.int32, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    st = torch.cuda.Stream()
    rtamd.copy_engines_warm([st.cuda_stream])
    order = sys.argv[1].split(",") if len(sys.argv) > 1 else list(FLAGS)
    for name in order:
        fl = FLAGS[name]
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), ctypes.c_uint(fl)) == 0, name
        for rep in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(40):
                rtamd.copy_to_host_async(p.value, dev.data_ptr(), n, st.cuda_stream)
            e1.record(st)
            st.synchronize()
            ms = e0.elapsed_time(e1) / 40
        ok = bytes((ctypes.c_uint8 * 64).from_address(p.value)) == dev[:16].cpu().numpy().tobytes()
        print("%-14s %.4f ms per copy, %.1f GB/s, data %s" % (name, ms, n / (ms * 1e-3) / 1e9, "ok" if ok else "WRONG"),
              flush=True)
        hip.hipHostFree(p)
    # one default buffer, 8 fresh streams in turn (a fresh stream may get another engine)
    hb = rtamd.HostBuffer((n // 4,), "int32")
    for k in range(8):
        sk = torch.cuda.Stream()
        for rep in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sk)
            for _ in range(40):
                rtamd.copy_to_host_async(hb.ptr, dev.data_ptr(), n, sk.cuda_stream)
            e1.record(sk)
            sk.synchronize()
        ms = e0.elapsed_time(e1) / 40
        print("fresh stream %d: %.4f ms per copy, %.1f GB/s" % (k, ms, n / (ms * 1e-3) / 1e9), flush=True)
    hb.free()


if __name__ == "__main__":
    main()
