"""Triangle-test work of the fast kernel's profiling variant (rt_experiment 6): wave-level leaf
visits and triangle-loop iterations, and the exact inside tests actually run (wave-level and
lane-level), for one frame.  Sizes the triangle filters.  Usage: python tools/tri_work.py [scene]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (binds the HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "world8_stress"
L = rtamd.lib()
L.rt_experiment.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                            ctypes.c_void_p]
s = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", scene + ".json"), 1920, 1080)
c = np.zeros(64, np.uint64)
ms = ctypes.c_double()
rtamd._check(L.rt_experiment(s._h, 6, 8, 2, ctypes.byref(ms), c.ctypes.data))
names = {0: "queries", 2: "leaf_lanes", 4: "wave_queries", 5: "pair_steps", 6: "leaf_visits", 7: "tri_iters",
         13: "inside_tests_wave", 14: "inside_tests_lanes"}
print(json.dumps({"scene": scene, "prof_kernel_ms": round(ms.value, 4), **{v: int(c[k]) for k, v in names.items()}}))
