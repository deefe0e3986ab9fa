"""Trace-kernel time of the bench workload with scene variations (profiling aid, results not
the reference's): integrator depth (reflections), lights removed, ...
Usage: python tools/variant_probe.py"""
import json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd

torch.cuda.set_device(0); rtamd.set_device(0)
path = os.path.join(ROOT, "scenes", "world8_stress.json")
buf = torch.zeros((1080, 1920), dtype=torch.int32, device="cuda")


def run(tag, s, frames=10):
    st = s.render_device(spp=8, rgba_ptr=buf.data_ptr(), sync=True, stats=True)
    for _ in range(3):
        s.render_device(spp=8, rgba_ptr=buf.data_ptr(), sync=True)
    s.timing_collect()
    for _ in range(frames):
        s.render_device(spp=8, rgba_ptr=buf.data_ptr(), sync=True, timing=True)
    tm = s.timing_collect()
    print(json.dumps({"variant": tag, "trace_ms": round(tm["trace_ms_total"] / tm["frames"], 4), "rays": st["rays"],
                      "nodes": st["nodes"], "leaves": st["leaves"]}), flush=True)


s = rtamd.Scene.load_json(path, 1920, 1080)
run("base", s)
for d in (1, 0):
    s.set_env(depth=d)
    run("depth%d" % d, s)
