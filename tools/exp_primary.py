"""Profiling aid: time the primary-ray closest-hit kernel alone (experiment 0)."""
import ctypes, os, sys, json
import torch  # noqa
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd
L = rtamd.lib()
L.rt_experiment.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p]
scene = sys.argv[1] if len(sys.argv) > 1 else "world8_stress"
for which, spp in [(int(w), 8) for w in (sys.argv[2].split(',') if len(sys.argv) > 2 else ['3', '2', '4'])]:
    s = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", scene + ".json"), 1920, 1080)
    ms = ctypes.c_double(); c = (ctypes.c_uint64 * 4)()
    rtamd._check(L.rt_experiment(s._h, which, spp, 6, ctypes.byref(ms), c))
    print(json.dumps({"scene": scene, "which": which, "lib": os.path.basename(rtamd.LIB_PATH), "spp": spp, "ms": ms.value, "rays": c[0], "nodes": c[1], "leaves": c[2],
                      "Mrays_s": c[0] / ms.value / 1e3}))
