"""Profiling aid (rt_experiment): 0-3 primary-ray closest-hit kernels alone (atomic/static
work, with/without leaves), 4/5 the full counted frame kernel with/without the occlusion
exit, plus wave-level step counters (SIMD work) next to the per-lane reference counters."""
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
    ms = ctypes.c_double(); c = (ctypes.c_uint64 * 22)()
    rtamd._check(L.rt_experiment(s._h, which, spp, 6, ctypes.byref(ms), c))
    print(json.dumps({"scene": scene, "which": which, "lib": os.path.basename(rtamd.LIB_PATH), "spp": spp, "ms": ms.value, "rays": c[0], "nodes": c[1], "leaves": c[2],
                      "Mrays_s": c[0] / ms.value / 1e3,
                      "wave_queries": c[4], "wave_pair_steps": c[5], "wave_leaf_visits": c[6], "wave_tri_iters": c[7],
                      "lane_util_queries": c[0] / max(1, 64 * c[4]), "lane_util_pairs": c[1] / max(1, 128 * c[5] + 64 * c[4]),
                      "lane_util_leaves": c[2] / max(1, 64 * c[6]),
                      "frac_cycles_in_queries": c[8] / max(1, c[10]), "frac_cycles_in_leaves": c[9] / max(1, c[10]),
                      "frac_cycles_in_samples": c[11] / max(1, c[10]), "frac_cycles_post_query": c[12] / max(1, c[10]),
                      "wave_inside_tests": c[13], "lane_inside_tests": c[14],
                      "wave_busy_over_span": c[17] / max(1, (c[16] - c[15]) * 3072),
                      "span_ms": (c[16] - c[15]) / 1e5, "latest_start_ms": (c[18] - c[15]) / 1e5,
                      "earliest_end_ms": (c[19] - c[15]) / 1e5, "max_group_ms": c[20] / 1e5,
                      "max_group_wave_queries": c[21]}))
