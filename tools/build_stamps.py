"""Phase timestamps of the BVH build kernel (experiment library built with
-DRT_BUILD_STAMPS; wall_clock64 at 100 MHz).  Usage:
RTAMD_LIB=tools/_exp/librt_stamps.so python tools/build_stamps.py [scene]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402

PHASES = ["zero work + boxes/morton", "bitonic sort", "reorder boxes", "level merges", "heap scatter", "ordered LBVH"]


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "world8_stress"
    torch.cuda.set_device(0)
    rtamd.set_device(0)
    s = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", scene + ".json"), 1920, 1080)
    buf = torch.zeros((1080, 1920), dtype=torch.int32, device="cuda")
    fn = rtamd.lib().rt_exp_build_stamps
    acc = [0.0] * len(PHASES)
    K = 20
    for k in range(K + 3):
        s.render_device(spp=1, rebuild_bvh=True, rgba_ptr=buf.data_ptr(), stream=torch.cuda.current_stream().cuda_stream,
                        sync=True, timing=True)
        st = (ctypes.c_ulonglong * 16)()
        fn(st)
        if k >= 3:
            for i in range(len(PHASES)):
                acc[i] += (st[i + 1] - st[i]) * 10e-3          # 100 MHz ticks -> us
    tm = s.timing_collect()
    print("%s: bvh event-timed %.1f us/frame" % (scene, tm["bvh_ms_total"] / max(1, tm["frames"]) * 1e3))
    for i, p in enumerate(PHASES):
        print("  %-28s %6.2f us" % (p, acc[i] / K))
    print("  %-28s %6.2f us" % ("total in kernel", sum(acc) / K))


if __name__ == "__main__":
    main()
