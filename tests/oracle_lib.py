"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int32)
_u = ctypes.POINTER(ctypes.c_uint64)
_u32 = ctypes.POINTER(ctypes.c_uint32)


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


class Oracle:
    def __init__(self, path=LIB):
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.orc_last_error.restype = ctypes.c_char_p
        L.orc_load.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, _u32, _f, _i, _i, _u]
        L.orc_build_bvh.argtypes = [ctypes.c_void_p, _f, _i, ctypes.c_int]
        for name in ["orc_scene_counts", "orc_scene_vertices", "orc_scene_normals", "orc_scene_tris",
                     "orc_scene_materials", "orc_scene_lights"]:
            getattr(L, name).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_scene_instances.argtypes = [ctypes.c_void_p, _f, _i]
        L.orc_scene_camera.argtypes = [ctypes.c_void_p, _f, _f]
        L.orc_spp_offset.argtypes = [ctypes.c_int, _f, _f]
        L.orc_set_atlas.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.orc_set_textures.argtypes = [ctypes.c_void_p, ctypes.c_int]
        vp, fl = ctypes.c_void_p, ctypes.c_float
        L.orc_scene_create.argtypes = [ctypes.POINTER(vp)]
        L.orc_builder_add_vertex.argtypes = [vp, fl, fl, fl]
        L.orc_builder_create_mesh.argtypes = [vp, vp, vp]
        L.orc_builder_add_triangle.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]
        L.orc_builder_add_trans.argtypes = [vp, ctypes.c_int]
        L.orc_builder_build_cube.argtypes = [vp, fl, vp, vp]
        L.orc_builder_add_point_light.argtypes = [vp, vp, vp]
        L.orc_builder_add_directional_light.argtypes = [vp, vp, vp]
        L.orc_builder_finish.argtypes = [vp, ctypes.c_int, ctypes.c_int, fl, fl, vp, vp, vp, vp, ctypes.c_int]
        L.orc_set_camera.argtypes = [vp, vp, vp]
        L.orc_set_trans.argtypes = [vp, ctypes.c_int, vp, vp]
        L.orc_set_env.argtypes = [vp, vp, vp, ctypes.c_int]
        L.orc_debug_cast.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int64]
        self.L = L

    # -- scenes ---------------------------------------------------------------
    def load(self, path, width=0, height=0):
        s = ctypes.c_void_p()
        r = self.L.orc_load(path.encode(), int(width), int(height), ctypes.byref(s))
        if r != 0:
            raise RuntimeError("oracle load failed: %s" % self.L.orc_last_error().decode())
        return OracleScene(self, s)

    def create(self):
        """Empty scene for the SceneBuilder calls (OracleScene.add_vertex ... finish)."""
        s = ctypes.c_void_p()
        assert self.L.orc_scene_create(ctypes.byref(s)) == 0
        return OracleScene(self, s, building=True)

    def spp_offset(self, k):
        dx, dy = ctypes.c_float(), ctypes.c_float()
        self.L.orc_spp_offset(k, ctypes.byref(dx), ctypes.byref(dy))
        return dx.value, dy.value

    def render(self, scene, semantics=0, use_bvh=1, spp=1, row0=0, row_step=1, nthreads=8,
               want=("rgba", "radiance", "hit_inst", "hit_tri")):
        W, H = scene.W, scene.H
        rgba = np.zeros(W * H, np.uint32) if "rgba" in want else None
        rad = np.zeros(W * H * 4, np.float32) if "radiance" in want else None
        hi = np.full(W * H, -1, np.int32) if "hit_inst" in want else None
        ht = np.full(W * H, -1, np.int32) if "hit_tri" in want else None
        st = np.zeros(4, np.uint64)
        r = self.L.orc_render(scene.h, semantics, use_bvh, spp, row0, row_step, nthreads,
                              _p(rgba, _u32), _p(rad, _f), _p(hi, _i), _p(ht, _i), _p(st, _u))
        if r != 0:
            raise RuntimeError(self.L.orc_last_error().decode())
        out = {"stats": st}
        if rgba is not None:
            out["rgba"] = rgba.reshape(H, W)
        if rad is not None:
            out["radiance"] = rad.reshape(H, W, 4)
        if hi is not None:
            out["hit_inst"] = hi.reshape(H, W)
        if ht is not None:
            out["hit_tri"] = ht.reshape(H, W)
        return out

    # -- KATs -----------------------------------------------------------------
    def kat(self, op, *arrays, n_out=None):
        L = self.L
        arrs = [np.ascontiguousarray(a, np.float32) for a in arrays]
        n = arrs[0].shape[0]
        P = lambda a: a.ctypes.data_as(_f)
        if op in ("normalize3", "reflect", "cross", "quat_rotate"):
            o = np.zeros((n, 3), np.float32)
            getattr(L, "orc_kat_" + op)(n, *[P(a) for a in arrs], P(o))
            return o
        if op in ("quat_inverse", "quat_mul", "axis_angle"):
            o = np.zeros((n, 4), np.float32)
            getattr(L, "orc_kat_" + op)(n, *[P(a) for a in arrs], P(o))
            return o
        if op == "to_mat3":
            o = np.zeros((n, 9), np.float32)
            L.orc_kat_to_mat3(n, P(arrs[0]), P(o))
            return o
        if op == "ray_ctor":
            o = np.zeros((n, 6), np.float32)
            L.orc_kat_ray_ctor(n, P(arrs[0]), P(o))
            return o
        if op == "refract":
            o = np.zeros((n, 3), np.float32)
            t = np.zeros(n, np.int32)
            L.orc_kat_refract(n, P(arrs[0]), P(arrs[1]), P(arrs[2]), P(o), t.ctypes.data_as(_i))
            return o, t
        if op == "tri_hit":
            o = np.zeros((n, 3), np.float32)
            h = np.zeros(n, np.int32)
            L.orc_kat_tri_hit(n, P(arrs[0]), P(arrs[1]), h.ctypes.data_as(_i), P(o))
            return h, o
        if op in ("box_from_local", "box_merge"):
            o = np.zeros((n, 6), np.float32)
            nd = np.zeros(n, np.int32)
            getattr(L, "orc_kat_" + op)(n, P(arrs[0]), P(arrs[1]), P(o), nd.ctypes.data_as(_i))
            return o, nd
        if op == "hitable":
            o = np.zeros((n, 10), np.float32)
            L.orc_kat_hitable(n, P(arrs[0]), P(arrs[1]), P(arrs[2]), P(o))
            return o
        if op == "entity":
            o = np.zeros((n, 12), np.float32)
            L.orc_kat_entity(n, P(arrs[0]), P(arrs[1]), P(o))
            return o
        if op == "box_hit":
            t = np.zeros(n, np.float32)
            h = np.zeros(n, np.int32)
            L.orc_kat_box_hit(n, P(arrs[0]), P(arrs[1]), h.ctypes.data_as(_i), P(t))
            return h, t
        if op == "zorder":
            o = np.zeros(n, np.uint64)
            L.orc_kat_zorder(n, P(arrs[0]), o.ctypes.data_as(_u))
            return o
        raise KeyError(op)


def _fa(a, n):
    if a is None:
        return None
    a = np.ascontiguousarray(a, np.float32)
    assert a.size == n, (a.size, n)
    return a


def _vp(a):
    return None if a is None else a.ctypes.data


class OracleScene:
    def __init__(self, orc, h, building=False):
        self.orc, self.h = orc, h
        self.W = self.H = self.depth = 0
        if not building:
            self._counts()

    def _counts(self):
        orc, h = self.orc, self.h
        c = np.zeros(10, np.int32)
        orc.L.orc_scene_counts(h, c.ctypes.data)
        (self.W, self.H, self.n_vertices, self.n_tris, self.n_meshes, self.n_instances, self.n_lights,
         self.n_point, self.depth, self.n_mats) = [int(x) for x in c]

    def set_atlas(self, rgba8):
        """Build extension: (H, W, 4) uint8 atlas for the textured shading mode."""
        self._atlas = np.ascontiguousarray(rgba8, np.uint8)
        assert self.orc.L.orc_set_atlas(self.h, self._atlas.ctypes.data, self._atlas.shape[1], self._atlas.shape[0]) == 0

    def set_textures(self, on=True):
        assert self.orc.L.orc_set_textures(self.h, int(on)) == 0

    # -- SceneBuilder (scene_builder.h:29-117) ---------------------------------
    def _idx(self, r):
        assert r >= 0, r
        return r

    def add_vertex(self, x, y, z):
        return self._idx(self.orc.L.orc_builder_add_vertex(self.h, x, y, z))

    def create_mesh(self, pos=(0, 0, 0), quat=(0, 0, 0, 1)):
        p, q = _fa(pos, 3), _fa(quat, 4)
        return self._idx(self.orc.L.orc_builder_create_mesh(self.h, _vp(p), _vp(q)))

    def add_triangle(self, mesh, i0, i1, i2, mat, tex6=None):
        m, t = _fa(mat, 26), _fa(tex6, 6)
        assert self.orc.L.orc_builder_add_triangle(self.h, mesh, i0, i1, i2, _vp(m), _vp(t)) == 0

    def add_trans(self, mesh):
        return self._idx(self.orc.L.orc_builder_add_trans(self.h, mesh))

    def build_cube(self, scale, mat, tile=None):
        m, t = _fa(mat, 26), _fa(tile, 3)
        return self._idx(self.orc.L.orc_builder_build_cube(self.h, scale, _vp(m), _vp(t)))

    def add_point_light(self, pos, col):
        p, c = _fa(pos, 3), _fa(col, 4)
        assert self.orc.L.orc_builder_add_point_light(self.h, _vp(p), _vp(c)) == 0

    def add_directional_light(self, d, col):
        p, c = _fa(d, 3), _fa(col, 4)
        assert self.orc.L.orc_builder_add_directional_light(self.h, _vp(p), _vp(c)) == 0

    def finish(self, width, height, fov, unit, cam_pos=(0, 0, 0), cam_quat=(0, 0, 0, 1), dist_atten=(0, 0, 0),
               ambience=(0, 0, 0, 0), depth=0):
        a = [_fa(cam_pos, 3), _fa(cam_quat, 4), _fa(dist_atten, 3), _fa(ambience, 4)]
        assert self.orc.L.orc_builder_finish(self.h, width, height, fov, unit, *[_vp(x) for x in a], depth) == 0
        self._counts()

    def debug_cast(self, x, y, use_bvh=True):
        """debug_cast's event log of pixel (x, y) (raytracer.cu:91-100), one event per line."""
        buf = ctypes.create_string_buffer(1 << 16)
        assert self.orc.L.orc_debug_cast(self.h, x, y, int(use_bvh), buf, len(buf)) == 0
        return buf.value.decode().splitlines()

    # -- poses / environment (Entity setters, entity.h:49-74) -------------------
    def set_camera(self, pos=None, quat=None):
        p, q = _fa(pos, 3), _fa(quat, 4)
        assert self.orc.L.orc_set_camera(self.h, _vp(p), _vp(q)) == 0

    def set_trans(self, t, pos=None, quat=None):
        p, q = _fa(pos, 3), _fa(quat, 4)
        assert self.orc.L.orc_set_trans(self.h, t, _vp(p), _vp(q)) == 0

    def set_env(self, ambience=None, dist_atten=None, depth=None):
        a, d = _fa(ambience, 4), _fa(dist_atten, 3)
        assert self.orc.L.orc_set_env(self.h, _vp(a), _vp(d), self.depth if depth is None else depth) == 0
        self._counts()

    def __del__(self):
        try:
            self.orc.L.orc_free(self.h)
        except Exception:
            pass

    def arrays(self):
        L = self.orc.L
        v = np.zeros((self.n_vertices, 3), np.float32); L.orc_scene_vertices(self.h, v.ctypes.data)
        n = np.zeros((self.n_vertices, 3), np.float32); L.orc_scene_normals(self.h, n.ctypes.data)
        t = np.zeros((self.n_tris, 4), np.int32); L.orc_scene_tris(self.h, t.ctypes.data)
        m = np.zeros((self.n_mats, 26), np.float32); L.orc_scene_materials(self.h, m.ctypes.data)
        q = np.zeros((self.n_instances, 7), np.float32); mi = np.zeros(self.n_instances, np.int32)
        L.orc_scene_instances(self.h, q.ctypes.data_as(_f), mi.ctypes.data_as(_i))
        li = np.zeros((self.n_lights, 8), np.float32); L.orc_scene_lights(self.h, li.ctypes.data)
        cam = np.zeros(21, np.float32); env = np.zeros(7, np.float32)
        L.orc_scene_camera(self.h, cam.ctypes.data_as(_f), env.ctypes.data_as(_f))
        return dict(vertices=v, normals=n, tris=t, materials=m, instances=q, inst_mesh=mi, lights=li,
                    camera=cam, env=env)

    def bvh(self):
        n = 1
        while n < max(self.n_instances, 1):
            n *= 2
        boxes = np.zeros((2 * n - 1, 7), np.float32)
        order = np.zeros(n, np.int32)
        r = self.orc.L.orc_build_bvh(self.h, boxes.ctypes.data_as(_f), order.ctypes.data_as(_i), n)
        assert r == n, r
        return boxes, order
