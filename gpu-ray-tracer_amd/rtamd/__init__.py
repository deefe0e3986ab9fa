"""rtamd — Python host side of the MI355X ray-tracing core.

Thin ctypes binding over the C ABI in include/rt_amd.h (librt_amd.so, built by
``make -C gpu-ray-tracer_amd``).  There is no CPU fallback: if the library or a
gfx950 device is missing, the calls raise.

Mirrors the reference's render-path API (wtzhang23/gpu-ray-tracer):
  Scene.load_json(path)          ~ procedural::gpu::generate (cube_world.h:20-23)
  Scene.builder(...) methods     ~ rtracer::SceneBuilder (scene_builder.h:29-117)
  Scene.update_scene(kd, opt)    ~ rtracer::gpu::update_scene (raytracer.h:18-22)
  Scene.debug_cast(x, y)         ~ rtracer::gpu::debug_cast (raytracer.h:21)
  Scene.render(...)              the spp / row-slice / device-output extension
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB_PATH = os.environ.get("RTAMD_LIB", os.path.join(PKG, "librt_amd.so"))

RT_OK, RT_ERR_ARG, RT_ERR_IO, RT_ERR_PARSE, RT_ERR_HIP, RT_ERR_STATE, RT_ERR_NODEV, RT_ERR_LIMIT = 0, -1, -2, -3, -4, -5, -6, -7
EXPORTS = {"vertices": 0, "normals": 1, "tris": 2, "materials": 3, "instances": 4, "inst_mesh": 5,
           "lights": 6, "camera": 7, "env": 8, "texcoords": 9}

# Every symbol include/rt_amd.h declares (checked by tests/test_abi.py).
SYMBOLS = [
    "rt_abi_version", "rt_last_error", "rt_device_count", "rt_set_device", "rt_scene_load_json", "rt_scene_create",
    "rt_scene_free", "rt_builder_add_vertex", "rt_builder_create_mesh", "rt_builder_add_triangle",
    "rt_builder_add_trans", "rt_builder_set_trans", "rt_builder_build_cube", "rt_builder_add_point_light",
    "rt_builder_add_directional_light", "rt_builder_finish", "rt_scene_info", "rt_scene_export", "rt_camera_get",
    "rt_camera_set", "rt_camera_translate", "rt_camera_rotate", "rt_camera_axes", "rt_env_set",
    "rt_render_opts_default", "rt_render", "rt_update_scene", "rt_canvas_read", "rt_canvas_host_ptr",
    "rt_canvas_get_color", "rt_debug_cast", "rt_kat_device", "rt_spp_offset", "rt_timing_collect",
    "rt_builder_add_triangle_tex", "rt_builder_build_cube_tex", "rt_scene_set_atlas", "rt_scene_load_atlas",
    "rt_scene_atlas_info", "rt_scene_set_frame_slots", "rt_scene_set_overlap", "rt_frame_work",
    "rt_scene_set_devices", "rt_profile_marker", "rt_host_alloc", "rt_host_free", "rt_copy_to_host_async",
    "rt_copy_engines_warm",
]


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("rt error %d: %s" % (code, msg))
        self.code = code


class RenderOpts(ctypes.Structure):
    _fields_ = [("spp", ctypes.c_int), ("use_bvh", ctypes.c_int), ("rebuild_bvh", ctypes.c_int),
                ("row0", ctypes.c_int), ("row_step", ctypes.c_int), ("compact", ctypes.c_int),
                ("kernel_dim", ctypes.c_int), ("stream", ctypes.c_void_p), ("rgba", ctypes.c_void_p),
                ("radiance", ctypes.c_void_p), ("hit_inst", ctypes.c_void_p), ("hit_tri", ctypes.c_void_p),
                ("sync", ctypes.c_int), ("host_outputs", ctypes.c_int), ("timing", ctypes.c_int),
                ("textures", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_uint64), ("nodes", ctypes.c_uint64), ("leaves", ctypes.c_uint64),
                ("tri_tests", ctypes.c_uint64), ("bvh_ms", ctypes.c_double), ("trace_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Work(ctypes.Structure):
    _fields_ = [("queries", ctypes.c_uint64), ("wave_queries", ctypes.c_uint64), ("pair_steps", ctypes.c_uint64),
                ("leaf_visits", ctypes.c_uint64), ("leaf_lanes", ctypes.c_uint64), ("tri_iters", ctypes.c_uint64),
                ("scene_bytes", ctypes.c_uint64),
                # query occupancy (ABI 3)
                ("lanes_primary", ctypes.c_uint64), ("lanes_secondary", ctypes.c_uint64),
                ("lanes_shadow", ctypes.c_uint64), ("lanes_unlit", ctypes.c_uint64),
                ("live_wave_queries", ctypes.c_uint64), ("live_lanes", ctypes.c_uint64),
                ("hist_wave_queries", ctypes.c_uint64 * 8), ("hist_pair_steps", ctypes.c_uint64 * 8),
                ("hist_leaf_visits", ctypes.c_uint64 * 8)]

    def as_dict(self):
        d = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            d[k] = [int(x) for x in v] if k.startswith("hist_") else int(v)
        return d


_lib = None


def lib():
    """Load librt_amd.so (once).  If torch is already imported, the library binds to
    torch's HIP runtime (same soname), so device pointers/streams are shared."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RtError(RT_ERR_STATE, "librt_amd.so not built (%s): run `make -C gpu-ray-tracer_amd`" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, ip, fp = ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float)
    L.rt_last_error.restype = ctypes.c_char_p
    L.rt_scene_load_json.argtypes = [ctypes.c_char_p, ip, ip, ctypes.POINTER(vp)]
    L.rt_scene_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
    L.rt_scene_free.argtypes = [vp]
    L.rt_builder_add_vertex.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.POINTER(ip)]
    L.rt_builder_create_mesh.argtypes = [vp, vp, vp, ctypes.POINTER(ip)]
    L.rt_builder_add_triangle.argtypes = [vp, ip, ip, ip, ip, vp]
    L.rt_builder_add_trans.argtypes = [vp, ip, ctypes.POINTER(ip)]
    L.rt_builder_set_trans.argtypes = [vp, ip, vp, vp]
    L.rt_builder_build_cube.argtypes = [vp, ctypes.c_float, vp, ctypes.POINTER(ip)]
    L.rt_builder_build_cube_tex.argtypes = [vp, ctypes.c_float, vp, vp, ctypes.POINTER(ip)]
    L.rt_builder_add_triangle_tex.argtypes = [vp, ip, ip, ip, ip, vp, vp]
    L.rt_scene_set_atlas.argtypes = [vp, vp, ip, ip]
    L.rt_scene_load_atlas.argtypes = [vp, ctypes.c_char_p]
    L.rt_scene_atlas_info.argtypes = [vp, vp]
    L.rt_builder_add_point_light.argtypes = [vp, vp, vp]
    L.rt_builder_add_directional_light.argtypes = [vp, vp, vp]
    L.rt_builder_finish.argtypes = [vp, ip, ip, ctypes.c_float, ctypes.c_float, vp, vp, vp, vp, ip]
    L.rt_scene_info.argtypes = [vp, vp]
    L.rt_scene_export.argtypes = [vp, ip, vp, ctypes.c_int64]
    L.rt_camera_get.argtypes = [vp, vp, vp]
    L.rt_camera_set.argtypes = [vp, vp, vp]
    L.rt_camera_translate.argtypes = [vp, vp]
    L.rt_camera_rotate.argtypes = [vp, vp]
    L.rt_camera_axes.argtypes = [vp, vp, vp, vp]
    L.rt_env_set.argtypes = [vp, vp, vp, ip]
    L.rt_render_opts_default.argtypes = [ctypes.POINTER(RenderOpts)]
    L.rt_render_opts_default.restype = None
    L.rt_render.argtypes = [vp, ctypes.POINTER(RenderOpts), ctypes.POINTER(Stats)]
    L.rt_update_scene.argtypes = [vp, ip, ip]
    L.rt_canvas_read.argtypes = [vp, vp, ctypes.c_int64]
    L.rt_canvas_host_ptr.argtypes = [vp]
    L.rt_canvas_host_ptr.restype = vp
    L.rt_canvas_get_color.argtypes = [vp, ip, ip, vp]
    L.rt_debug_cast.argtypes = [vp, ip, ip, ctypes.c_char_p, ctypes.c_int64]
    L.rt_kat_device.argtypes = [ctypes.c_char_p, ip, vp, vp, vp, vp, vp, vp]
    L.rt_spp_offset.argtypes = [ip, fp, fp]
    L.rt_set_device.argtypes = [ip]
    L.rt_timing_collect.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ip)]
    L.rt_device_count.argtypes = [ctypes.POINTER(ip)]
    L.rt_scene_set_frame_slots.argtypes = [vp, ip]
    L.rt_scene_set_overlap.argtypes = [vp, ip]
    L.rt_frame_work.argtypes = [vp, ctypes.POINTER(RenderOpts), ctypes.POINTER(Work)]
    L.rt_scene_set_devices.argtypes = [vp, vp, ip, ip]
    if hasattr(L, "rt_profile_marker"):         # (absent from libraries older than ABI 3's round 5: A/B runs)
        L.rt_profile_marker.argtypes = [ip, vp]
    if hasattr(L, "rt_copy_to_host_async"):     # ABI 4
        L.rt_host_alloc.argtypes = [ctypes.c_int64, ctypes.POINTER(vp)]
        L.rt_host_free.argtypes = [vp]
        L.rt_copy_to_host_async.argtypes = [vp, vp, ctypes.c_int64, vp]
        L.rt_copy_engines_warm.argtypes = [ctypes.POINTER(vp), ip]
    _lib = L
    return L


def _check(code):
    if code != RT_OK:
        raise RtError(code, lib().rt_last_error().decode(errors="replace"))


def _f(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if n is not None:
        assert a.size == n, (a.size, n)
    return a


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def device_count():
    n = ctypes.c_int()
    _check(lib().rt_device_count(ctypes.byref(n)))
    return n.value


def set_device(d):
    _check(lib().rt_set_device(int(d)))


def spp_offset(k):
    dx, dy = ctypes.c_float(), ctypes.c_float()
    _check(lib().rt_spp_offset(k, ctypes.byref(dx), ctypes.byref(dy)))
    return dx.value, dy.value


def profile_marker(tag, stream=None):
    """An empty marker kernel of `tag` workgroups on `stream` (an int hipStream_t, None = the
    default stream): tools/pmc_step.py finds a timed region between two markers."""
    if hasattr(lib(), "rt_profile_marker"):
        _check(lib().rt_profile_marker(int(tag), stream))


class HostBuffer:
    """Pinned host memory from rt_host_alloc (hipHostMalloc), viewed as a torch / numpy array.
    The frame's host copy lands here through a copy engine (copy_to_host_async)."""

    def __init__(self, shape, dtype=np.int32):
        self.shape, self.dtype = tuple(shape), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = ctypes.c_void_p()
        _check(lib().rt_host_alloc(self.nbytes, ctypes.byref(p)))
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr)) \
            .view(self.dtype).reshape(self.shape)

    def tensor(self):
        import torch
        return torch.from_numpy(self.array)

    def free(self):
        if self.ptr:
            self.array = None
            _check(lib().rt_host_free(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def copy_to_host_async(host_ptr, dev_ptr, nbytes, stream=None):
    """Device -> pinned-host copy on a DMA copy engine, enqueued on `stream` (an int
    hipStream_t; None = the null stream).  No CU is used (rt_copy_to_host_async)."""
    _check(lib().rt_copy_to_host_async(host_ptr, dev_ptr, int(nbytes), stream))


def copy_engines_warm(streams):
    """Start the SDMA engines a host-copy pipeline will use: one gated copy from each of
    `streams` (int hipStream_t handles; rt_copy_engines_warm)."""
    arr = (ctypes.c_void_p * len(streams))(*streams)
    _check(lib().rt_copy_engines_warm(arr, len(streams)))


def material(Ke=(0, 0, 0, 0), Ka=(0, 0, 0, 0), Kd=(0, 0, 0, 0), Ks=(0, 0, 0, 0), Kt=(0, 0, 0, 0), Kr=(0, 0, 0, 0),
             alpha=0.0, eta=1.0):
    """material26 record (material.h:14-31)."""
    return np.array(list(Ke) + list(Ka) + list(Kd) + list(Ks) + list(Kt) + list(Kr) + [alpha, eta], np.float32)


class Scene:
    """A scene resident on one GPU (renv::gpu::Scene equivalent)."""

    def __init__(self, handle):
        self._h = handle
        self._info = None

    # ---- creation ----
    @classmethod
    def load_json(cls, path, width=0, height=0):
        h = ctypes.c_void_p()
        _check(lib().rt_scene_load_json(os.fspath(path).encode(), int(width), int(height), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def create(cls, atlas=""):
        h = ctypes.c_void_p()
        _check(lib().rt_scene_create(atlas.encode(), ctypes.byref(h)))
        return cls(h)

    def close(self):
        if self._h:
            lib().rt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- SceneBuilder ----
    def add_vertex(self, x, y, z):
        i = ctypes.c_int()
        _check(lib().rt_builder_add_vertex(self._h, x, y, z, ctypes.byref(i)))
        return i.value

    def create_mesh(self, pos=(0, 0, 0), quat=(0, 0, 0, 1)):
        i = ctypes.c_int()
        _check(lib().rt_builder_create_mesh(self._h, _ptr(_f(pos, 3)), _ptr(_f(quat, 4)), ctypes.byref(i)))
        return i.value

    def add_triangle(self, mesh, i0, i1, i2, mat):
        _check(lib().rt_builder_add_triangle(self._h, mesh, i0, i1, i2, _ptr(_f(mat, 26))))

    def add_trans(self, mesh):
        i = ctypes.c_int()
        _check(lib().rt_builder_add_trans(self._h, mesh, ctypes.byref(i)))
        return i.value

    def set_trans(self, t, pos=None, quat=None):
        _check(lib().rt_builder_set_trans(self._h, t, _ptr(None if pos is None else _f(pos, 3)),
                                          _ptr(None if quat is None else _f(quat, 4))))

    def build_cube(self, scale, mat, tile=None):
        """tile=(tx, ty, size): every face mapped onto that atlas square (textured mode)."""
        i = ctypes.c_int()
        if tile is None:
            _check(lib().rt_builder_build_cube(self._h, scale, _ptr(_f(mat, 26)), ctypes.byref(i)))
        else:
            _check(lib().rt_builder_build_cube_tex(self._h, scale, _ptr(_f(mat, 26)), _ptr(_f(tile, 3)),
                                                   ctypes.byref(i)))
        return i.value

    def add_triangle_tex(self, mesh, i0, i1, i2, mat, tex6):
        _check(lib().rt_builder_add_triangle_tex(self._h, mesh, i0, i1, i2, _ptr(_f(mat, 26)), _ptr(_f(tex6, 6))))

    # ---- texture atlas (textured shading mode) ----
    def load_atlas(self, path=None):
        _check(lib().rt_scene_load_atlas(self._h, None if path is None else path.encode()))

    def set_atlas(self, rgba8):
        a = np.ascontiguousarray(rgba8, dtype=np.uint8)
        assert a.ndim == 3 and a.shape[2] == 4
        _check(lib().rt_scene_set_atlas(self._h, _ptr(a), a.shape[1], a.shape[0]))

    def atlas(self):
        """The loaded atlas as (H, W, 4) uint8 (empty array if none)."""
        a = self.atlas_info()
        out = np.zeros((a["height"], a["width"], 4), np.uint8)
        if out.size:
            _check(lib().rt_scene_export(self._h, 10, _ptr(out), out.nbytes))
        return out

    def atlas_info(self):
        v = np.zeros(3, np.int32)
        _check(lib().rt_scene_atlas_info(self._h, _ptr(v)))
        return {"width": int(v[0]), "height": int(v[1]), "loaded": bool(v[2])}

    def add_point_light(self, pos, col):
        _check(lib().rt_builder_add_point_light(self._h, _ptr(_f(pos, 3)), _ptr(_f(col, 4))))

    def add_directional_light(self, d, col):
        _check(lib().rt_builder_add_directional_light(self._h, _ptr(_f(d, 3)), _ptr(_f(col, 4))))

    def finish(self, width, height, fov, unit, cam_pos=(0, 0, 0), cam_quat=(0, 0, 0, 1), dist_atten=(0, 0, 0),
               ambience=(0, 0, 0, 0), depth=0):
        _check(lib().rt_builder_finish(self._h, width, height, fov, unit, _ptr(_f(cam_pos, 3)), _ptr(_f(cam_quat, 4)),
                                       _ptr(_f(dist_atten, 3)), _ptr(_f(ambience, 4)), depth))
        self._info = None

    # ---- introspection ----
    def info(self):
        if self._info is None:
            c = np.zeros(10, np.int32)
            _check(lib().rt_scene_info(self._h, _ptr(c)))
            keys = ["W", "H", "n_vertices", "n_tris", "n_meshes", "n_instances", "n_lights", "n_point", "depth", "n_mats"]
            self._info = dict(zip(keys, [int(x) for x in c]))
        return self._info

    @property
    def width(self):
        return self.info()["W"]

    @property
    def height(self):
        return self.info()["H"]

    def export(self, what):
        i = self.info()
        shapes = {"vertices": ((i["n_vertices"], 3), np.float32), "normals": ((i["n_vertices"], 3), np.float32),
                  "tris": ((i["n_tris"], 4), np.int32), "materials": ((i["n_mats"], 26), np.float32),
                  "instances": ((i["n_instances"], 7), np.float32), "inst_mesh": ((i["n_instances"],), np.int32),
                  "lights": ((i["n_lights"], 8), np.float32), "camera": ((21,), np.float32), "env": ((7,), np.float32),
                  "texcoords": ((i["n_tris"], 7), np.float32)}
        shp, dt = shapes[what]
        a = np.zeros(shp, dt)
        _check(lib().rt_scene_export(self._h, EXPORTS[what], _ptr(a), a.nbytes))
        return a

    def arrays(self):
        return {k: self.export(k) for k in EXPORTS}

    # ---- camera / env ----
    def camera(self):
        p, q = np.zeros(3, np.float32), np.zeros(4, np.float32)
        _check(lib().rt_camera_get(self._h, _ptr(p), _ptr(q)))
        return p, q

    def set_camera(self, pos=None, quat=None):
        _check(lib().rt_camera_set(self._h, _ptr(None if pos is None else _f(pos, 3)),
                                   _ptr(None if quat is None else _f(quat, 4))))

    def translate_camera(self, d):
        _check(lib().rt_camera_translate(self._h, _ptr(_f(d, 3))))

    def rotate_camera(self, dq):
        _check(lib().rt_camera_rotate(self._h, _ptr(_f(dq, 4))))

    def camera_axes(self):
        r, u, f = np.zeros(3, np.float32), np.zeros(3, np.float32), np.zeros(3, np.float32)
        _check(lib().rt_camera_axes(self._h, _ptr(r), _ptr(u), _ptr(f)))
        return r, u, f

    def set_env(self, ambience=None, dist_atten=None, depth=None):
        d = self.info()["depth"] if depth is None else depth
        _check(lib().rt_env_set(self._h, _ptr(None if ambience is None else _f(ambience, 4)),
                                _ptr(None if dist_atten is None else _f(dist_atten, 3)), int(d)))
        self._info = None

    # ---- rendering ----
    def render(self, spp=1, use_bvh=True, rebuild_bvh=True, row0=0, row_step=1, compact=False,
               want=("rgba",), stats=True, textures=False):
        """Render to host numpy arrays (outputs staged through device buffers)."""
        W, H = self.width, self.height
        rows = len(range(row0, H, row_step)) if compact else H
        o = RenderOpts()
        lib().rt_render_opts_default(ctypes.byref(o))
        o.spp, o.use_bvh, o.rebuild_bvh, o.row0, o.row_step, o.compact = spp, int(use_bvh), int(rebuild_bvh), row0, row_step, int(compact)
        o.host_outputs, o.sync, o.textures = 1, 1, int(textures)
        out = {}
        if "rgba" in want:
            out["rgba"] = np.zeros((rows, W), np.uint32)
            o.rgba = _ptr(out["rgba"])
        if "radiance" in want:
            out["radiance"] = np.zeros((rows, W, 4), np.float32)
            o.radiance = _ptr(out["radiance"])
        if "hit_inst" in want:
            out["hit_inst"] = np.full((rows, W), -1, np.int32)
            o.hit_inst = _ptr(out["hit_inst"])
        if "hit_tri" in want:
            out["hit_tri"] = np.full((rows, W), -1, np.int32)
            o.hit_tri = _ptr(out["hit_tri"])
        st = Stats()
        _check(lib().rt_render(self._h, ctypes.byref(o), ctypes.byref(st) if stats else None))
        if stats:
            out["stats"] = st.as_dict()
        return out

    def render_device(self, spp=1, use_bvh=True, rebuild_bvh=True, row0=0, row_step=1, compact=True,
                      rgba_ptr=None, radiance_ptr=None, hit_inst_ptr=None, hit_tri_ptr=None, stream=None,
                      sync=False, stats=False, timing=False, textures=False):
        """Render into caller-owned DEVICE buffers (e.g. torch tensors' data_ptr())."""
        o = RenderOpts()
        lib().rt_render_opts_default(ctypes.byref(o))
        o.spp, o.use_bvh, o.rebuild_bvh, o.row0, o.row_step, o.compact = spp, int(use_bvh), int(rebuild_bvh), row0, row_step, int(compact)
        o.rgba, o.radiance, o.hit_inst, o.hit_tri = rgba_ptr, radiance_ptr, hit_inst_ptr, hit_tri_ptr
        o.stream, o.sync, o.host_outputs, o.timing, o.textures = stream, int(sync), 0, int(timing), int(textures)
        st = Stats()
        _check(lib().rt_render(self._h, ctypes.byref(o), ctypes.byref(st) if stats else None))
        return st.as_dict() if stats else None

    def frame_work(self, spp=1, row0=0, row_step=1, compact=True):
        """What the fast kernels do for this frame (rt_frame_work): queries issued after the
        exact skips, wave-level traversal steps."""
        o = RenderOpts()
        lib().rt_render_opts_default(ctypes.byref(o))
        o.spp, o.row0, o.row_step, o.compact = spp, row0, row_step, int(compact)
        w = Work()
        _check(lib().rt_frame_work(self._h, ctypes.byref(o), ctypes.byref(w)))
        return w.as_dict()

    def set_devices(self, devices, n_ranks=None):
        """Split every whole frame row-cyclically over `devices` from this process (n_ranks
        slices, RCCL gather to devices[0]; rt_scene_set_devices).  [d], 1 = back to one GPU."""
        d = np.ascontiguousarray(devices, np.int32)
        _check(lib().rt_scene_set_devices(self._h, _ptr(d), int(d.size), int(n_ranks or d.size)))

    def set_frame_slots(self, n):
        """1 (default) to 8: consecutive frames rotate through n copies of the per-frame
        state (BVH, work counters, scheduling history), so frames issued on different streams
        overlap (rt_scene_set_frame_slots)."""
        _check(lib().rt_scene_set_frame_slots(self._h, int(n)))

    def set_overlap(self, full, stream=False):
        """Grid of a frame issued while another frame of the scene runs (four or more slots): False =
        half the CUs (default; device-resident pipelines), True = every CU (pipelines that
        copy each frame to the host); stream=True: half the CUs for every frame, the first
        included, while frames are issued back to back (rt_scene_set_overlap)."""
        _check(lib().rt_scene_set_overlap(self._h, 2 if stream else 1 if full else 0))

    def timing_collect(self):
        a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _check(lib().rt_timing_collect(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
        return {"bvh_ms_total": a.value, "trace_ms_total": b.value, "frames": n.value}

    def update_scene(self, kernel_dim=16, optimize=True):
        _check(lib().rt_update_scene(self._h, kernel_dim, int(optimize)))

    def canvas(self):
        a = np.zeros((self.height, self.width), np.uint32)
        _check(lib().rt_canvas_read(self._h, _ptr(a), a.size))
        return a

    def get_color(self, x, y):
        c = np.zeros(4, np.uint8)
        _check(lib().rt_canvas_get_color(self._h, x, y, _ptr(c)))
        return tuple(int(v) for v in c)

    def debug_cast(self, x, y):
        buf = ctypes.create_string_buffer(1 << 16)
        _check(lib().rt_debug_cast(self._h, x, y, buf, len(buf)))
        return buf.value.decode().splitlines()


def kat_device(op, *inputs):
    """Evaluate a math primitive on the GPU (test hook; see rt_amd.h rt_kat_device)."""
    sizes = {"normalize3": (3, 0, 0), "cross": (3, 0, 0), "reflect": (3, 0, 0), "refract": (3, 1, 0),
             "quat_rotate": (3, 0, 0), "quat_inverse": (4, 0, 0), "quat_mul": (4, 0, 0), "tri_hit": (3, 1, 0),
             "ray_ctor": (6, 0, 0), "zorder": (0, 0, 1), "to_mat3": (9, 0, 0), "box_hit": (0, 1, 0), "pow": (1, 0, 0),
             "tri_hit_f": (3, 1, 0), "box_hit_f": (0, 1, 0), "box_pair": (0, 2, 0),
             "rcp_cr": (1, 0, 0), "sqrt_cr": (1, 0, 0), "box_from_local": (6, 1, 0), "box_merge": (6, 1, 0),
             "entity": (12, 0, 0)}
    nf, ni, nu = sizes[op]
    ins = [_f(a) for a in inputs] + [None] * (3 - len(inputs))
    n = inputs[0].shape[0]
    of = np.zeros((n, nf), np.float32) if nf else None
    oi = (np.zeros(n, np.int32) if ni == 1 else np.zeros((n, ni), np.int32)) if ni else None
    ou = np.zeros(n, np.uint64) if nu else None
    _check(lib().rt_kat_device(op.encode(), n, _ptr(ins[0]), _ptr(ins[1]), _ptr(ins[2]), _ptr(of), _ptr(oi), _ptr(ou)))
    res = [x for x in (of, oi, ou) if x is not None]
    return res[0] if len(res) == 1 else tuple(res)
