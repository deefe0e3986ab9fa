#!/usr/bin/env python3
"""Which device -> pinned-host copies run as blit kernels in a bench-like process.

Variants (argv[1]): a torch process with GPU_MAX_HW_QUEUES = 16 (or RT_BENCH_HW_QUEUES), eight
torch streams, a kernel then rt_copy_to_host_async on the same stream, one copy per stream, with
or without a trace kernel in flight.  Run under rocprofv3 --kernel-trace --memory-copy-trace and
under AMD_LOG_LEVEL to see the runtime's choice (tools/copy_probe2.sh)."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", os.environ.get("RT_BENCH_HW_QUEUES", "16"))
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402


def main():
    n_streams = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    after_kernel = (sys.argv[2] if len(sys.argv) > 2 else "1") == "1"
    W, H = 1920, 1080
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    dev = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in range(n_streams)]
    host = [rtamd.HostBuffer((H, W)) for _ in range(n_streams)]
    torch.cuda.synchronize()
    t = time.perf_counter()
    for rep in range(4):
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                if after_kernel:
                    dev[i].fill_(rep * 100 + i)
                rtamd.copy_to_host_async(host[i].ptr, dev[i].data_ptr(), host[i].nbytes, st.cuda_stream)
        torch.cuda.synchronize()
    dt = time.perf_counter() - t
    ok = all(int(host[i].array[7, 9]) == (300 + i if after_kernel else 0) for i in range(n_streams))
    print("streams %d after_kernel %d: %.3f ms per round of %d copies, data %s"
          % (n_streams, after_kernel, dt / 4 * 1e3, n_streams, "ok" if ok else "WRONG"), flush=True)


if __name__ == "__main__":
    main()
