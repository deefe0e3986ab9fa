"""Trace-kernel time of the bench workload under other camera poses (profiling aid): e.g. a
camera turned to the sky makes every pixel group a one-query miss group, which prices the
per-group fixed cost.  Usage: python tools/cam_probe.py [--quat i j k r] [--frames N]"""
import argparse, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd

p = argparse.ArgumentParser()
p.add_argument("--scene", default="world8_stress")
p.add_argument("--quat", type=float, nargs=4, action="append", default=None)
p.add_argument("--frames", type=int, default=10)
p.add_argument("--spp", type=int, default=8)
p.add_argument("--no-base", action="store_true", help="skip the scene's own camera pose")
a = p.parse_args()
torch.cuda.set_device(0); rtamd.set_device(0)
s = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", a.scene + ".json"), 1920, 1080)
pos0, q0 = s.camera()
buf = torch.zeros((1080, 1920), dtype=torch.int32, device="cuda")
for q in (([] if a.no_base else [None]) + (a.quat or [])):
    s.set_camera(pos=pos0, quat=q0 if q is None else q)
    st = s.render_device(spp=a.spp, rgba_ptr=buf.data_ptr(), sync=True, stats=True)
    for _ in range(3):
        s.render_device(spp=a.spp, rgba_ptr=buf.data_ptr(), sync=True)
    s.timing_collect()
    for _ in range(a.frames):
        s.render_device(spp=a.spp, rgba_ptr=buf.data_ptr(), sync=True, timing=True)
    tm = s.timing_collect()
    lit = float((buf != buf[0, 0]).float().mean())
    print(json.dumps({"quat": list(map(float, q0 if q is None else q)), "trace_ms": round(tm["trace_ms_total"] / tm["frames"], 4),
                      "rays": st["rays"], "nodes": st["nodes"], "leaves": st["leaves"], "non_bg_frac": round(lit, 4)}), flush=True)
