// rt_oracle.cpp — CPU ORACLE for the MI355X ray-tracing core.  TEST INFRASTRUCTURE ONLY.
//
// A plain C++ restatement of wtzhang23/gpu-ray-tracer (reference mounted at
// /root/reference).  Every routine cites the reference file:line it follows.  It
// restates BOTH integrators:
//   * ORC_SEM_GPU — renv::gpu::propagate_ray (src/rayenv/scene.cu:92-188) driven by
//     rtracer::gpu::trace/update_scene (src/raytracer.cu:17-43, 102-120) with the
//     Morton BVH of ropt::gpu::BVH (src/rayopt/bvh.cu:11-156).  This is the
//     north-star semantics the HIP path must reproduce.
//   * ORC_SEM_CPU — rtracer::cpu::update_scene (src/raytracer.cc:41-62), the serial
//     CPU path, bug for bug (all-ULONG_MAX Morton keys, bvh.cc:17; dead recursion
//     cap, scene.cu:224).  This is the timing baseline only.
//
// Floating point: every expression keeps the reference's operand order; the file
// must be built with -ffp-contract=off and without -ffast-math / -march flags
// (see oracle/Makefile).  Functions the reference calls unqualified inside nvcc
// translation units (abs, pow, sqrt on floats) resolve to fabsf/powf/sqrtf there;
// those in g++ translation units (cos/sin in cube_world.cc) run in double.
//
// Parity status: math primitives pinned by the reference's own raymath/z_order
// sources (oracle/ref_kat); integrator/BVH/loader glue "parity unpinned" (their
// reference sources need CUDA/Thrust/rapidjson/SDL headers absent here).

#include "rt_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>
#include <pthread.h>

namespace {

thread_local std::string g_err;

const float THRESH = 1e-5f;  // rmath::THRESHOLD is `constexpr double = 1E-5f` (linear.h:15)
const int MAX_DEPTH = 10;    // renv::gpu::MAX_DEPTH (scene.cu:25)

// ----------------------------------------------------------------------------
// raymath (include/raymath/linear.h, geometry.h)
// ----------------------------------------------------------------------------
struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };

inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }   // linear.h:68-74,104-109
inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }   // linear.h:76-82,111-116
inline V3 mul(float c, V3 v) { return v3(v.x * c, v.y * c, v.z * c); }      // linear.h:100-106,132-137 (coords[i] *= coef)
inline V3 neg(V3 v) { return mul(-1.0f, v); }                               // linear.h:139-142 ((T)-1 * vec)
inline float dot(V3 a, V3 b) {                                              // linear.h:197-205
    float s = 0; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s;
}
inline float len(V3 v) { return sqrtf(dot(v, v)); }                         // linear.h:150-157 (sqrt -> sqrtf in .cu TUs)
inline V3 normalized(V3 v) {                                                // linear.h:159-167
    float l = len(v);
    if (l > THRESH) return mul(1 / l, v);
    return v3(0, 0, 0);
}
inline V3 cross(V3 a, V3 b) {                                               // linear.h:207-215
    float x = a.y * b.z - a.z * b.y;
    float y = a.z * b.x - a.x * b.z;
    float z = a.x * b.y - a.y * b.x;
    return v3(x, y, z);
}
inline V4 add4(V4 a, V4 b) { return V4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline V4 mul4(V4 a, V4 b) { return V4{a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }  // linear.h:84-90
inline V4 smul4(float c, V4 v) { return V4{v.x * c, v.y * c, v.z * c, v.w * c}; }
inline float dot4(V4 a, V4 b) {
    float s = 0; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; s += a.w * b.w; return s;
}

V3 reflect(V3 dir, V3 nrm) {                                                // linear.h:217-226
    float d_len = len(dir);
    V3 d_norm = normalized(dir);
    V3 n_norm = normalized(nrm);
    V3 projection = mul(dot(d_norm, n_norm), n_norm);
    V3 r_norm = normalized(sub(d_norm, mul(2.0f, projection)));
    return mul(d_len, r_norm);
}

V3 refract(V3 dir, V3 nrm, float from, float to, bool& tir) {               // linear.h:228-243
    float d_len = len(dir);
    V3 d_norm = normalized(dir);
    V3 n_norm = normalized(nrm);
    float ratio = from / to;
    float cosi = dot(d_norm, n_norm);
    float sint_2 = ratio * ratio * (1 - cosi * cosi);
    if (sint_2 > 1) {
        tir = true;
        return mul(d_len, reflect(d_norm, n_norm));
    }
    tir = false;
    return mul(d_len, add(mul(ratio, d_norm), mul(ratio * cosi - sqrtf(1 - sint_2), n_norm)));
}

struct Quat { float i, j, k, r; };                                          // geometry.h:17-26 (inner = {i,j,k,r})

inline V4 qv(Quat q) { return V4{q.i, q.j, q.k, q.r}; }
Quat qnormalized(Quat q) {                                                  // geometry.h:142-145 -> Vec4::normalized
    V4 v = qv(q);
    float l = sqrtf(dot4(v, v));
    if (l > THRESH) { float c = 1 / l; return Quat{q.i * c, q.j * c, q.k * c, q.r * c}; }
    return Quat{0, 0, 0, 0};
}
Quat qinverse(Quat q) {                                                     // geometry.h:129-139
    float sq = dot4(qv(q), qv(q));
    if (sq < THRESH) return Quat{0, 0, 0, 0};
    float inv = 1 / sq;
    return Quat{q.i * -inv, q.j * -inv, q.k * -inv, q.r * inv};
}
Quat qmul(Quat a, Quat b) {                                                 // geometry.h:148-155
    return Quat{a.i * b.r + a.r * b.i + a.j * b.k - a.k * b.j,
                a.j * b.r + a.r * b.j + a.k * b.i - a.i * b.k,
                a.k * b.r + a.r * b.k + a.i * b.j - a.j * b.i,
                a.r * b.r - a.i * b.i - a.j * b.j - a.k * b.k};
}
V3 qrot(Quat q, V3 v) {                                                     // geometry.h:176-181 (Quat * Vec3)
    float length = len(v);
    Quat prod = qmul(qmul(qnormalized(q), Quat{v.x, v.y, v.z, 0}), qinverse(q));
    return mul(length, normalized(v3(prod.i, prod.j, prod.k)));
}
Quat qaxis_angle_g(V3 axis, float theta) {                                  // geometry.h:36-41 in a g++ TU: double cos/sin
    float hc = (float)std::cos((double)(0.5f * theta));
    float hs = (float)std::sin((double)(0.5f * theta));
    return Quat{axis.x * hs, axis.y * hs, axis.z * hs, hc};
}
void to_mat3(Quat q, float m[3][3]) {                                       // geometry.h:183-198
    float length = sqrtf(dot4(qv(q), qv(q)));
    float ni = q.i / length, nj = q.j / length, nk = q.k / length, nr = q.r / length;
    float ii = 2.0f * ni * ni, jj = 2.0f * nj * nj, kk = 2.0f * nk * nk;
    float ri = 2.0f * nr * ni, rj = 2.0f * nr * nj, rk = 2.0f * nr * nk, ij = 2.0f * ni * nj,
          ik = 2.0f * ni * nk, jk = 2.0f * nj * nk;
    float t[3][3] = {{1 - (jj + kk), ij - rk, ik + rj},
                     {ij + rk, 1 - (ii + kk), jk - ri},
                     {ik - rj, jk + ri, 1 - (ii + jj)}};
    memcpy(m, t, sizeof t);
}

struct Ray { V3 o, d; };
inline Ray make_ray(V3 o, V3 d) { return Ray{o, normalized(d)}; }           // geometry.h:207-208
inline V3 ray_at(const Ray& r, float t) { return add(r.o, mul(t, r.d)); }   // geometry.h:220-222

bool plane_hit(V3 po, V3 pn_unnorm, const Ray& r, float& time) {           // geometry.h:229-262
    V3 n = normalized(pn_unnorm);
    float denom = dot(r.d, n);
    if (fabsf(denom) < THRESH) return false;                                 // abs(float) -> fabsf (nvcc TU)
    time = (1.0f / denom) * dot(sub(po, r.o), n);
    return true;
}
bool triangle_hit(V3 a, V3 b, V3 c, const Ray& r, float& time, float& u, float& v) {  // geometry.h:273-290
    V3 plane_norm = cross(sub(b, a), sub(c, a));
    if (plane_hit(a, plane_norm, r, time)) {
        V3 p = ray_at(r, time);
        float area = len(plane_norm);
        float b0 = len(cross(sub(c, p), sub(b, p))) / area;
        float b1 = len(cross(sub(c, p), sub(a, p))) / area;
        float b2 = len(cross(sub(a, p), sub(b, p))) / area;
        if (fabsf(b0 + b1 + b2 - 1.0f) <= THRESH) { u = b1; v = b2; return true; }
    }
    return false;
}

// ----------------------------------------------------------------------------
// Entity (src/rayprimitives/entity.cu:5-37)
// ----------------------------------------------------------------------------
struct Entity { Quat o; V3 p; };
inline V3 point_to_local(const Entity& e, V3 v) { return qrot(e.o, sub(v, e.p)); }
inline V3 point_from_local(const Entity& e, V3 v) { return add(qrot(qinverse(e.o), v), e.p); }
inline V3 vec_to_local(const Entity& e, V3 v) { return qrot(e.o, v); }
inline V3 vec_from_local(const Entity& e, V3 v) { return qrot(qinverse(e.o), v); }
inline Ray ray_to_local(const Entity& e, const Ray& r) {                    // entity.cu:25-29
    V3 ld = vec_to_local(e, r.d);
    V3 lp = point_to_local(e, r.o);
    return make_ray(lp, ld);
}

// ----------------------------------------------------------------------------
// BoundingBox (src/rayopt/bounding_box.cu, include/rayopt/bounding_box.h)
// ----------------------------------------------------------------------------
struct Box { V3 mn, mx; bool nd; };
inline Box box_empty() { return Box{v3(0, 0, 0), v3(0, 0, 0), false}; }
void fit_vertex(Box& b, V3 v) {                                             // bounding_box.cu:5-22
    if (!b.nd) { b.mn = v; b.mx = v; b.nd = true; return; }
    float* mn = &b.mn.x; float* mx = &b.mx.x; const float* vv = &v.x;
    for (int i = 0; i < 3; i++) {
        if (vv[i] < mn[i]) mn[i] = vv[i];
        if (vv[i] > mx[i]) mx[i] = vv[i];
    }
}
Box merge(const Box& a, const Box& b) {                                     // bounding_box.cu:24-49
    Box r = a;
    if (!r.nd) { r = b; return r; }
    if (!b.nd) return r;
    float* rmn = &r.mn.x; float* rmx = &r.mx.x; const float* bmn = &b.mn.x; const float* bmx = &b.mx.x;
    for (int i = 0; i < 3; i++) {
        if (rmn[i] > bmn[i]) rmn[i] = bmn[i];
        if (rmx[i] < bmx[i]) rmx[i] = bmx[i];
    }
    return r;
}
Box from_local(const Box& a, const Entity& e) {                             // bounding_box.cu:51-60
    Box r = box_empty();
    if (!a.nd) return r;
    fit_vertex(r, point_from_local(e, a.mn));
    fit_vertex(r, point_from_local(e, a.mx));
    return r;
}
bool box_intersects(const Box& b, const Ray& r, float& time) {              // bounding_box.cu:62-104
    if (!b.nd) return false;
    const float* d = &r.d.x; const float* o = &r.o.x; const float* mn = &b.mn.x; const float* mx = &b.mx.x;
    float tmin = -INFINITY, tmax = INFINITY;
    for (int a = 0; a < 3; a++) {
        if (d[a] == 0) continue;
        float tn = (mn[a] - o[a]) / d[a];
        float tf = (mx[a] - o[a]) / d[a];
        if (tn > tf) { float t = tn; tn = tf; tf = t; }
        if (tn > tmin) tmin = tn;
        if (tf < tmax) tmax = tf;
        if (tmin > tmax || tmax < THRESH) return false;
    }
    time = tmin >= 0 ? tmin : tmax;
    return true;
}
inline V3 box_center(const Box& b) { return mul(0.5f, add(b.mn, b.mx)); }  // bounding_box.h:37-39

uint64_t z_order(V3 vec) {                                                  // z_order.cu:5-36
    V3 inv = neg(vec);
    uint32_t x, y, z;
    memcpy(&x, &inv.x, 4); memcpy(&y, &inv.y, 4); memcpy(&z, &inv.z, 4);
    uint32_t xo = 31, yo = 31, zo = 31;
    uint64_t t = 0;
    for (unsigned i = 0; i < 64; i++) {
        t <<= 1;
        switch (i % 3) {
            case 0: t |= (x >> xo) & 1u; xo--; break;
            case 1: t |= (y >> yo) & 1u; yo--; break;
            case 2: t |= (z >> zo) & 1u; zo--; break;
        }
    }
    return t;
}

// ----------------------------------------------------------------------------
// Scene model (SceneBuilder, scene_builder.h:29-117; gpu/scene.h:32-110)
// ----------------------------------------------------------------------------
struct Material { V4 Ke{}, Ka{}, Kd{}, Ks{}, Kt{}, Kr{}; float alpha = 0, eta = 1; };  // material.h:14-31
inline bool reflective(const Material& m) { return m.Kr.x > 0.0f || m.Kr.y > 0.0f || m.Kr.z > 0.0f || m.Kr.w > 0.0f; }
inline bool refractive(const Material& m) { return m.Kt.x > 0.0f || m.Kt.y > 0.0f || m.Kt.z > 0.0f || m.Kt.w > 0.0f; }

// TextureCoords (texture_coords.h:12-29) of the build-defined textured mode (the
// reference never samples them, phong.cu:18-23): texel = t + u*U + v*V
struct Tex { int has = 0; float tx = 0, ty = 0, ux = 0, uy = 0, vx = 0, vy = 0; };
struct Tri { int i0, i1, i2; int mat; Tex tex; };
struct Mesh { Entity e; int begin, count; };
struct Inst { Entity e; int mesh; };
struct Light { int type; V3 v; V4 col; };   // type 0 point (pos), 1 directional (normalized dir)

struct Camera { Entity e; float near_, unit, W, H; };                       // camera.h:14-20

}  // namespace

struct orc_scene {
    int W = 0, H = 0;
    std::vector<V3> verts, norms;
    std::vector<Tri> tris;
    std::vector<Material> mats;
    std::vector<Mesh> meshes;
    std::vector<Inst> insts;
    std::vector<Light> lights;       // point lights first, then directional (scene_builder.cu:61-81)
    int n_point = 0;
    V3 dist_atten{0, 0, 0};
    V4 ambience{0, 0, 0, 0};
    int depth = 0;
    Camera cam;
    std::vector<uint8_t> atlas;      // textured mode (build extension): RGBA8 atlas
    int atlas_w = 0, atlas_h = 0;
    int textures = 0;
    // SceneBuilder state (scene_builder.h:29-117) until orc_builder_finish flattens it:
    // triangles per MeshBuilder, lights by kind (build_gpu_scene puts point lights first)
    bool building = false;
    std::vector<std::vector<Tri>> mesh_tris;
    std::vector<Light> b_points, b_dirs;
};

namespace {

// ----------------------------------------------------------------------------
// Minimal JSON (subset used by cube_world.cc via rapidjson: objects, arrays,
// numbers parsed with strtod, strings).
// ----------------------------------------------------------------------------
struct JV {
    enum T { NUL, NUM, STR, ARR, OBJ, BOOL } t = NUL;
    double num = 0; std::string str; std::vector<JV> arr; std::map<std::string, JV> obj; bool b = false;
    bool has(const char* k) const { return t == OBJ && obj.count(k); }
    const JV& operator[](const char* k) const { return obj.at(k); }
    const JV& operator[](int i) const { return arr.at((size_t)i); }
};
struct JP {
    const char* p; const char* e;
    void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) p++; }
    JV parse() {
        ws(); JV v;
        if (p >= e) throw std::runtime_error("json: unexpected end");
        if (*p == '{') {
            v.t = JV::OBJ; p++; ws();
            if (*p == '}') { p++; return v; }
            for (;;) { ws(); JV k = parse(); ws(); if (*p != ':') throw std::runtime_error("json: ':'"); p++;
                       v.obj[k.str] = parse(); ws(); if (*p == ',') { p++; continue; } if (*p == '}') { p++; break; }
                       throw std::runtime_error("json: object"); }
        } else if (*p == '[') {
            v.t = JV::ARR; p++; ws();
            if (*p == ']') { p++; return v; }
            for (;;) { v.arr.push_back(parse()); ws(); if (*p == ',') { p++; continue; } if (*p == ']') { p++; break; }
                       throw std::runtime_error("json: array"); }
        } else if (*p == '"') {
            v.t = JV::STR; p++;
            while (p < e && *p != '"') { if (*p == '\\') p++; v.str.push_back(*p++); }
            p++;
        } else if (!strncmp(p, "true", 4)) { v.t = JV::BOOL; v.b = true; p += 4; }
        else if (!strncmp(p, "false", 5)) { v.t = JV::BOOL; p += 5; }
        else if (!strncmp(p, "null", 4)) { p += 4; }
        else { char* end; v.t = JV::NUM; v.num = strtod(p, &end); if (end == p) throw std::runtime_error("json: number"); p = end; }
        return v;
    }
};
inline float gf(const JV& v) { return (float)v.num; }        // rapidjson GetFloat = (float)GetDouble
inline int gi(const JV& v) { return (int)v.num; }
V3 read_vec3(const JV& v) { return v3(gf(v[0]), gf(v[1]), gf(v[2])); }     // cube_world.cc:23-25
V4 read_vec4(const JV& v) { return V4{gf(v[0]), gf(v[1]), gf(v[2]), gf(v[3])}; }

// Perlin (src/procedural/perlin.cu; an nvcc host TU: float overloads of acos/cos/sin/floor)
struct Perlin {
    float amplitude = 1.0f, period = 1.0f;
    std::vector<V3> vecs; std::vector<int> perm; int n;
    Perlin(int seed, int n_vecs) : n(n_vecs) {                              // perlin.cu:80-103
        std::mt19937 generator(seed);
        auto rng = std::bind(std::uniform_real_distribution<float>{}, generator);
        vecs.resize(n); perm.resize(n);
        for (int i = 0; i < n; i++) {
            float theta = acosf(2 * rng() - 1);
            float phi = (float)(2 * rng() * M_PI);                           // perlin.cu:91 (double product, float var)
            vecs[i] = normalized(v3(cosf(phi) * sinf(theta), sinf(phi) * sinf(theta), cosf(theta)));
            perm[i] = i;
        }
        auto rng_int = std::bind(std::uniform_int_distribution<unsigned>{}, generator);
        for (int i = 0; i < n; i++) {
            int swap_idx = rng_int() % n;
            int t = perm[i]; perm[i] = perm[swap_idx]; perm[swap_idx] = t;
        }
    }
    const V3& hash(int x, int y, int z) const {                              // perlin.cu:12-23
        int hx = x % n; int hxy = (perm[hx] + y) % n; int hxyz = (perm[hxy] + z) % n;
        return vecs[perm[hxyz]];
    }
    static float smooth(float d) { return d * d * (3 - 2 * d); }            // perlin.cu:33-35
    static float interp(float a, float b, float w) { return w * a + (1 - w) * b; }  // perlin.cu:7-9
    float sample(float x, float y, float z) const {                         // perlin.cu:59-78
        float gx = x * n / period, gy = y * n / period, gz = z * n / period;
        int ix = (int)floorf(gx) % n, iy = (int)floorf(gy) % n, iz = (int)floorf(gz) % n;
        float mx = smooth(gx - floorf(gx)), my = smooth(gy - floorf(gy)), mz = smooth(gz - floorf(gz));
        auto w = [&](int dx, int dy, int dz) {                               // perlin.cu:45-52
            float cx = ix + dx, cy = iy + dy, cz = iz + dz;
            V3 off = v3(dx - mx, dy - my, dz - mz);
            const V3& wv = hash((int)cx, (int)cy, (int)cz);
            return dot(wv, normalized(off));
        };
        float w000 = w(0, 0, 0), w001 = w(0, 0, 1), w010 = w(0, 1, 0), w011 = w(0, 1, 1);
        float w100 = w(1, 0, 0), w101 = w(1, 0, 1), w110 = w(1, 1, 0), w111 = w(1, 1, 1);
        float x00 = interp(w000, w100, mx), x01 = interp(w001, w101, mx);
        float x10 = interp(w010, w110, mx), x11 = interp(w011, w111, mx);
        float xy0 = interp(x00, x10, my), xy1 = interp(x01, x11, my);
        return amplitude * interp(xy0, xy1, mz);
    }
};

// SceneBuilder::build_cube (scene_builder.cu:181-239)
// tile (build extension): {tx, ty, size}: face-local (s, t) in [-scale/2, scale/2] ->
// [tx, tx+size] x [ty, ty+size], image rows downwards; front/back faces use (x, y),
// top/bottom (x, z), right/left (z, y) -- the build's documented mapping.
void build_cube(orc_scene& s, float scale, const Material& mat, const float* tile = nullptr) {
    V3 A = mul(scale, v3(-0.5f, 0.5f, -0.5f)), B = mul(scale, v3(0.5f, 0.5f, -0.5f));
    V3 C = mul(scale, v3(-0.5f, -0.5f, -0.5f)), D = mul(scale, v3(0.5f, -0.5f, -0.5f));
    V3 E = mul(scale, v3(-0.5f, 0.5f, 0.5f)), F = mul(scale, v3(0.5f, 0.5f, 0.5f));
    V3 G = mul(scale, v3(-0.5f, -0.5f, 0.5f)), Hh = mul(scale, v3(0.5f, -0.5f, 0.5f));
    int mi = (int)s.mats.size(); s.mats.push_back(mat);
    Mesh m; m.e = Entity{Quat{0, 0, 0, 1}, v3(0, 0, 0)}; m.begin = (int)s.tris.size(); m.count = 0;
    if (s.building) s.mesh_tris.emplace_back();
    const V3* faces[12][3] = {{&D, &A, &B}, {&C, &A, &D}, {&A, &E, &B}, {&E, &F, &B}, {&D, &B, &Hh}, {&B, &F, &Hh},
                              {&C, &G, &A}, {&A, &G, &E}, {&G, &Hh, &E}, {&E, &Hh, &F}, {&G, &C, &D}, {&D, &Hh, &G}};
    static const int axes[6][2] = {{0, 1}, {0, 2}, {2, 1}, {2, 1}, {0, 1}, {0, 2}};
    for (int k = 0; k < 12; k++) {
        const V3* const* f = faces[k];
        Tri t; int base = (int)s.verts.size();
        s.verts.push_back(*f[0]); s.verts.push_back(*f[1]); s.verts.push_back(*f[2]);
        t.i0 = base; t.i1 = base + 1; t.i2 = base + 2; t.mat = mi;
        if (tile) {
            float c[3][2];
            for (int j = 0; j < 3; j++) {
                const float p[3] = {f[j]->x, f[j]->y, f[j]->z};
                c[j][0] = tile[0] + (p[axes[k / 2][0]] / scale + 0.5f) * tile[2];
                c[j][1] = tile[1] + (0.5f - p[axes[k / 2][1]] / scale) * tile[2];
            }
            t.tex.has = 1; t.tex.tx = c[0][0]; t.tex.ty = c[0][1];
            t.tex.ux = c[1][0] - c[0][0]; t.tex.uy = c[1][1] - c[0][1];
            t.tex.vx = c[2][0] - c[0][0]; t.tex.vy = c[2][1] - c[0][1];
        }
        if (s.building) s.mesh_tris.back().push_back(t);
        else { s.tris.push_back(t); m.count++; }
    }
    if (s.building) m.begin = m.count = 0;
    s.meshes.push_back(m);
}

// SceneBuilder::generate_normals (scene_builder.cc:11-29)
void generate_normals(orc_scene& s) {
    s.norms.assign(s.verts.size(), v3(0, 0, 0));
    for (const Mesh& m : s.meshes)
        for (int t = m.begin; t < m.begin + m.count; t++) {
            const Tri& tr = s.tris[t];
            V3 a = sub(s.verts[tr.i1], s.verts[tr.i0]);
            V3 b = sub(s.verts[tr.i2], s.verts[tr.i0]);
            V3 n = normalized(cross(a, b));
            s.norms[tr.i0] = add(s.norms[tr.i0], n);
            s.norms[tr.i1] = add(s.norms[tr.i1], n);
            s.norms[tr.i2] = add(s.norms[tr.i2], n);
        }
    for (V3& n : s.norms) n = normalized(n);
}

// procedural::generate_config + finish_env (cube_world.cc:38-191)
void load_cube_world(orc_scene& s, const JV& doc, int w_over, int h_over) {
    int seed = 42, grid = 8, width = 640, height = 480;
    float fov = (float)M_PI / 4, unit = 200;
    if (doc.has("seed")) seed = gi(doc["seed"]);
    if (doc.has("grid_size")) grid = gi(doc["grid_size"]);
    if (doc.has("width")) width = gi(doc["width"]);
    if (doc.has("height")) height = gi(doc["height"]);
    if (doc.has("fov")) fov = (float)(doc["fov"].num * M_PI) / 180;       // cube_world.cc:56-58
    if (doc.has("unit_length")) unit = (float)doc["unit_length"].num;
    if (w_over > 0) width = w_over;
    if (h_over > 0) height = h_over;
    s.W = width; s.H = height;
    // Camera (camera.cu:6-9; an nvcc TU -> tanf)
    s.cam.e = Entity{Quat{0, 0, 0, 1}, v3(0, 0, 0)};
    s.cam.near_ = 0.5f * width / unit / tanf(fov);
    s.cam.unit = unit; s.cam.W = (float)width; s.cam.H = (float)height;

    int n_cubes = 0;
    const float inv255 = 1.0f / 255;                                        // 1.0f / UINT8_MAX
    if (doc.has("cubes")) {
        const JV& cubes = doc["cubes"];
        n_cubes = (int)cubes.arr.size();
        for (int i = 0; i < n_cubes; i++) {
            const JV& c = cubes[i];
            Material m;
            if (c.has("Ke")) m.Ke = smul4(inv255, read_vec4(c["Ke"]));
            if (c.has("Ka")) m.Ka = smul4(inv255, read_vec4(c["Ka"]));
            if (c.has("Kd")) m.Kd = smul4(inv255, read_vec4(c["Kd"]));
            if (c.has("Ks")) m.Ks = smul4(inv255, read_vec4(c["Ks"]));
            if (c.has("Kt")) m.Kt = read_vec4(c["Kt"]);
            if (c.has("Kr")) m.Kr = read_vec4(c["Kr"]);
            if (c.has("alpha")) m.alpha = (float)c["alpha"].num;
            if (c.has("eta")) m.eta = (float)c["eta"].num;
            float tile[3];
            const bool tx = c.has("texture") && c["texture"].arr.size() == 3;
            if (tx) for (int k = 0; k < 3; k++) tile[k] = (float)c["texture"][k].num;
            build_cube(s, .999f, m, tx ? tile : nullptr);
        }
    }
    std::vector<Light> pts, dirs;
    if (doc.has("lights")) {
        const JV& L = doc["lights"];
        if (L.has("directional"))
            for (const JV& l : L["directional"].arr)                         // DirLight::set_shine_dir normalizes (light.cuh:62)
                dirs.push_back(Light{1, normalized(read_vec3(l["dir"])), smul4(inv255, read_vec4(l["col"]))});
        if (L.has("point"))
            for (const JV& l : L["point"].arr)
                pts.push_back(Light{0, read_vec3(l["pos"]), smul4(inv255, read_vec4(l["col"]))});
    }
    s.lights = pts; s.n_point = (int)pts.size();
    s.lights.insert(s.lights.end(), dirs.begin(), dirs.end());

    float amplitude = 1.0f;
    if (doc.has("amplitude")) amplitude = (float)doc["amplitude"].num;
    std::vector<float> last(grid * grid, 0.0f);
    float max_h = 0.0f;
    for (int c = 0; c < n_cubes; c++) {                                     // cube_world.cc:149-170
        Perlin perlin(seed, (grid + 4) / 5);
        perlin.amplitude = amplitude; perlin.period = (float)grid;
        for (int i = 0; i < grid; i++)
            for (int j = 0; j < grid; j++) {
                float x = i - grid / 2.0f, z = j - grid / 2.0f;
                float y_off = (float)(std::floor((double)(0.5f * (perlin.sample((float)i, (float)j, 0.0f) + amplitude))) + 1);
                for (int d = 0; d < y_off; d++) {
                    float y = last[i * grid + j] + d;
                    s.insts.push_back(Inst{Entity{Quat{0, 0, 0, 1}, v3(x, y, z)}, c});
                }
                last[i * grid + j] += y_off;
                max_h = std::max(max_h, last[i * grid + j]);
            }
    }
    s.cam.e.p = v3(0.0f, max_h + 10.0f, -(float)grid / 2);                  // cube_world.cc:172-173
    s.cam.e.o = qaxis_angle_g(v3(1.0f, 0.0f, 0.0f), 45);
    generate_normals(s);
    if (doc.has("ambience")) s.ambience = read_vec4(doc["ambience"]);      // finish_env :177-191
    if (doc.has("depth")) s.depth = gi(doc["depth"]);
    if (doc.has("distance_attenuation")) {
        const JV& a = doc["distance_attenuation"];
        s.dist_atten = v3((float)a["constant_term"].num, (float)a["linear_term"].num, (float)a["quadratic_term"].num);
    }
}

// Camera::at (camera.cu:33-42)
struct CamBasis { V3 r, u, f; };
CamBasis cam_basis(const Camera& c) {
    float m[3][3]; to_mat3(c.e.o, m);
    return CamBasis{normalized(v3(m[0][0], m[1][0], m[2][0])), normalized(v3(m[0][1], m[1][1], m[2][1])),
                    normalized(v3(m[0][2], m[1][2], m[2][2]))};
}
Ray cam_at(const Camera& c, const CamBasis& b, float cx, float cy) {
    float gx = (cx - (0.5f * c.W)) / c.unit;
    float gy = (0.5f * c.H - cy) / c.unit;
    V3 dir = add(add(mul(c.near_, b.f), mul(gx, b.r)), mul(gy, b.u));
    return make_ray(c.e.p, dir);
}

// ----------------------------------------------------------------------------
// BVH (GPU flavour: bvh.cu:74-91 / raytracer.cu:54-89; CPU flavour: bvh.cc:12-46)
// ----------------------------------------------------------------------------
struct BVH { std::vector<Box> tree; std::vector<int> ordering; int n = 0; };

Box mesh_box(const orc_scene& s, const Mesh& m) {                           // trimesh.cu:21-32
    Box rv = box_empty();
    for (int t = m.begin; t < m.begin + m.count; t++) {
        const Tri& tr = s.tris[t];
        fit_vertex(rv, s.verts[tr.i0]); fit_vertex(rv, s.verts[tr.i1]); fit_vertex(rv, s.verts[tr.i2]);
    }
    return from_local(rv, m.e);
}
int padded_count(int n_t) { return 1 << (int)std::ceil(std::log2((double)n_t)); }  // raytracer.cu:79

BVH build_bvh(const orc_scene& s, bool cpu_flavour) {
    BVH b;
    int nt = (int)s.insts.size();
    if (nt == 0) return b;
    int n = padded_count(nt);
    std::vector<Box> org(n, box_empty());
    for (int i = 0; i < nt; i++) org[i] = from_local(mesh_box(s, s.meshes[s.insts[i].mesh]), s.insts[i].e);  // create_boxes
    std::vector<uint64_t> codes(n);
    b.ordering.resize(n);
    for (int i = 0; i < n; i++) {
        b.ordering[i] = i;
        // GPU: gen_morton on the real boxes (bvh.cu:20-32).  CPU: bvh.cc:17 tests the
        // freshly default-constructed `boxes` vector, so every key is ULONG_MAX.
        bool degenerate = cpu_flavour ? true : !org[i].nd;
        codes[i] = degenerate ? UINT64_MAX : z_order(neg(box_center(org[i])));
    }
    if (cpu_flavour)
        std::sort(b.ordering.begin(), b.ordering.end(), [&](int a, int c) { return codes[a] < codes[c]; });  // bvh.cc:29-31
    else
        std::stable_sort(b.ordering.begin(), b.ordering.end(), [&](int a, int c) { return codes[a] < codes[c]; });  // thrust radix (stable)
    b.tree.resize(2 * n - 1);
    for (int i = 0; i < n; i++) b.tree[i] = org[b.ordering[i]];             // reorder (bvh.cu:34-41)
    int lvl = 0, size = n, out = n;
    while (size >= 2) {                                                     // build_bvh_layer (bvh.cu:43-61)
        for (int i = 0; i < size / 2; i++) b.tree[out + i] = merge(b.tree[lvl + 2 * i], b.tree[lvl + 2 * i + 1]);
        lvl += size; out += size / 2; size >>= 1;
    }
    b.n = n;
    return b;
}

// ----------------------------------------------------------------------------
// Intersection (scene.cu:27-73, hitable.cu:7-38, trimesh.cu:11-68)
// ----------------------------------------------------------------------------
struct Isect { float time; V3 norm; float u, v; int mat; int inst, tri; };
// debug_cast's event log (raytracer.cu:91-100: env.set_debug_mode(true) around one ray; the
// printf sites scene.cu:107-108, 134-135, 152-153 and light.cu:38-39), NULL otherwise
thread_local std::string* g_dbg = nullptr;
inline void dbg_event(const char* e) { if (g_dbg) { *g_dbg += e; *g_dbg += '\n'; } }
struct Counters { uint64_t rays = 0, nodes = 0, leaves = 0, tris = 0; };

struct Ctx {
    const orc_scene* s; const BVH* bvh; bool use_bvh; bool cpu_sem; Counters* c;
};

bool tri_hit(const Ctx& x, int t, const Ray& lr, Isect& is) {               // trimesh.cu:46-68
    const orc_scene& s = *x.s; const Tri& tr = s.tris[t];
    x.c->tris++;
    float time, u, v;
    if (triangle_hit(s.verts[tr.i0], s.verts[tr.i1], s.verts[tr.i2], lr, time, u, v) && time >= THRESH && time < is.time) {
        is.mat = tr.mat; is.u = u; is.v = v;
        V3 n0 = s.norms[tr.i0], n1 = s.norms[tr.i1], n2 = s.norms[tr.i2];
        float b0 = 1.0f - u - v;
        is.norm = normalized(add(add(mul(b0, n0), mul(u, n1)), mul(v, n2)));
        is.time = time;
        is.tri = t;
        return true;
    }
    return false;
}

// Hitable::hit (hitable.cu:7-38, HitHandle): the entity's local ray, hit_local, then the
// normal and time brought back (fix_isect).  hit_local(lr, is) -> bool.
template <class F>
bool hitable_hit(const Entity& e, const Ray& ray, Isect& is, F&& hit_local) {
    float scale = len(vec_to_local(e, ray.d));                                 // get_local_ray
    Ray lr = ray_to_local(e, ray);
    bool hit = hit_local(lr, is);
    if (hit) { is.norm = normalized(vec_from_local(e, is.norm)); is.time *= scale; }   // fix_isect
    return hit;
}

bool mesh_hit(const Ctx& x, const Mesh& m, const Ray& ray, Isect& is) {
    return hitable_hit(m.e, ray, is, [&](const Ray& lr, Isect& li) {
        bool hit = false;
        for (int t = m.begin; t < m.begin + m.count; t++) hit |= tri_hit(x, t, lr, li);   // trimesh.cu:11-19
        return hit;
    });
}

bool cast_local(const Ctx& x, const Ray& r, Isect& is, int ti) {            // scene.cu:27-40
    const Inst& t = x.s->insts[ti];
    x.c->leaves++;
    V3 ld = vec_to_local(t.e, r.d);
    float dir_len = len(ld);
    Ray lr = make_ray(point_to_local(t.e, r.o), ld);
    bool rv = mesh_hit(x, x.s->meshes[t.mesh], lr, is);
    if (rv) { is.norm = vec_from_local(t.e, is.norm); is.time *= dir_len; is.inst = ti; }
    return rv;
}

// CPU BVH traversal (bvh.cc:48-67): recursive, both children when a node is hit.
void traverse_cpu(const Ctx& x, const Ray& r, Isect& is, bool& hit, int k) {
    const BVH& b = *x.bvh;
    int idx = (2 * b.n - 1) - k;
    x.c->nodes++;
    float t;
    if (box_intersects(b.tree[idx], r, t)) {
        if (2 * k > 2 * b.n - 1) hit |= cast_local(x, r, is, b.ordering[idx]);
        else { traverse_cpu(x, r, is, hit, 2 * k); traverse_cpu(x, r, is, hit, 2 * k + 1); }
    }
}

bool cast_ray(const Ctx& x, const Ray& r, Isect& is) {                      // scene.cu:42-73
    x.c->rays++;
    bool hit = false;
    int nt = (int)x.s->insts.size();
    if (!x.use_bvh || nt == 0) {
        for (int i = 0; i < nt; i++) hit |= cast_local(x, r, is, i);
        return hit;
    }
    if (x.cpu_sem) { traverse_cpu(x, r, is, hit, 1); return hit; }
    // Stackless heap walk of BVHIterator (bvh.h:43-100, bvh.cu:98-156) with a
    // single lane: __ballot_sync(mask, p) == p.
    const BVH& b = *x.bvh;
    const int n = b.n;
    int k = 1;
    while (k >= 1) {
        x.c->nodes++;
        int idx = 2 * n - 1 - k;
        float t;
        bool hb = box_intersects(b.tree[idx], r, t);
        bool leaf = k >= n;                                                  // at_child: 2k >= 2n-1
        if (hb && leaf) { if (cast_local(x, r, is, b.ordering[idx])) hit = true; }
        if (hb && !leaf) { k = 2 * k; continue; }                            // step_next
        while (k % 2 == 1) k /= 2;                                          // step_up
        if (k == 0) break;
        k = k + 1;                                                           // parent()*2+1
    }
    return hit;
}

// ----------------------------------------------------------------------------
// Shading (phong.cu:14-53, light.cu:11-77, scene.cu:14-22)
// ----------------------------------------------------------------------------
V4 trans_atten(const Material& m, float time) {                             // scene.cu:14-22 (pow -> powf)
    return V4{powf(time, m.Kt.x), powf(time, m.Kt.y), powf(time, m.Kt.z), powf(time, m.Kt.w)};
}
float calc_dist_atten(const orc_scene& s, float dist) {                     // light.cu:11-16
    float quad = s.dist_atten.x + s.dist_atten.y * dist + s.dist_atten.z * dist * dist;
    return quad < 1.0f ? 1.0f : 1.0f / quad;
}
V4 calc_shadow_atten(V4 kt, float dist) {                                   // light.cu:18-25
    return V4{powf(kt.x, dist), powf(kt.y, dist), powf(kt.z, dist), powf(kt.w, dist)};
}
V4 attenuate(const Ctx& x, const Light& L, const Ray& to_light, float max_t) {  // light.cu:29-61 (gpu) / :81-114 (cpu)
    V4 rv = L.col;
    Ray cur = make_ray(ray_at(to_light, THRESH), to_light.d);
    for (;;) {
        Isect si; si.time = INFINITY; si.mat = -1; si.inst = -1; si.tri = -1; si.norm = v3(0, 0, 0);
        dbg_event("shooting shadow ray");                                    // light.cu:38-39
        if (cast_ray(x, cur, si)) {
            if (si.time > max_t) return rv;
            const Material& m = x.s->mats[si.mat];
            if (!refractive(m)) return V4{0, 0, 0, 0};
            if (dot(si.norm, cur.d) > 0) rv = mul4(rv, calc_shadow_atten(m.Kt, si.time));
            cur = make_ray(ray_at(cur, si.time), cur.d);
            max_t -= si.time;
        } else return rv;
    }
}
V4 shine(const Ctx& x, const Light& L, V3 hit_pos, V3& dir_to_light) {       // light.cu:63-77
    if (L.type == 0) {
        V3 disp = sub(L.v, hit_pos);
        float dist = len(disp);
        float da = calc_dist_atten(*x.s, dist);
        dir_to_light = normalized(disp);
        Ray to = make_ray(hit_pos, dir_to_light);
        return smul4(da, attenuate(x, L, to, dist));
    }
    dir_to_light = neg(L.v);
    return attenuate(x, L, make_ray(hit_pos, dir_to_light), INFINITY);
}
inline float fmax_std(float a, float b) { return (a < b) ? b : a; }          // std::max semantics
V4 phong(const Material& m, V4 kd, V3 nrm, V4 incoming, V3 ray_dir, V3 to_light) { // phong.cu:14-33
    float nd = fmax_std(dot(to_light, nrm), 0.0f);
    V4 diffuse = smul4(nd, kd);
    V3 reflected = reflect(neg(to_light), nrm);
    float rd = dot(neg(reflected), ray_dir);
    V4 specular = smul4(powf(fmax_std(rd, 0.0f), m.alpha), m.Ks);
    return mul4(add4(diffuse, specular), incoming);
}
V4 illuminate(const Ctx& x, const Ray& org, const Isect& is) {              // phong.cu:42-53 / :58-66
    const orc_scene& s = *x.s;
    const Material& m = s.mats[is.mat];
    V4 kd = m.Kd;                                                            // the reference
    const Tri& ht = s.tris[is.tri];
    if (s.textures && ht.tex.has && !s.atlas.empty()) {                      // build extension: point-sampled texel
        const float xf = (ht.tex.tx + is.u * ht.tex.ux) + is.v * ht.tex.vx;
        const float yf = (ht.tex.ty + is.u * ht.tex.uy) + is.v * ht.tex.vy;
        const int ix = (int)std::fmin(std::fmax(xf, 0.0f), (float)(s.atlas_w - 1));
        const int iy = (int)std::fmin(std::fmax(yf, 0.0f), (float)(s.atlas_h - 1));
        const uint8_t* px = &s.atlas[4 * ((size_t)iy * s.atlas_w + ix)];
        kd = V4{(float)px[0] / 255, (float)px[1] / 255, (float)px[2] / 255, (float)px[3] / 255};
    }
    V4 sum = add4(m.Ke, mul4(m.Ka, s.ambience));                             // org_light (phong.cu:36-39)
    for (const Light& L : s.lights) {
        V3 dtl;
        V4 inc = shine(x, L, ray_at(org, is.time), dtl);
        sum = add4(sum, phong(m, kd, is.norm, inc, org.d, dtl));
    }
    return sum;
}

// ----------------------------------------------------------------------------
// Integrators
// ----------------------------------------------------------------------------
enum FrameType { NORMAL, REFLECT, REFRACT };
struct RayFrame { Ray ray; V3 hit_pt, norm; V4 atten; int last_mat; FrameType type; int depth; bool in_obj; };

V4 propagate_gpu(const Ctx& x, const Ray& r, Isect& is) {                   // scene.cu:92-188
    const orc_scene& s = *x.s;
    RayFrame frames[MAX_DEPTH];
    frames[0] = RayFrame{r, v3(0, 0, 0), v3(0, 0, 0), V4{1, 1, 1, 1}, -1, NORMAL, s.depth, false};
    int top_i = 0;
    V4 acc{0, 0, 0, 0};
    while (top_i >= 0) {
        RayFrame& top = frames[top_i];
        switch (top.type) {
            case NORMAL: {
                is.time = INFINITY;
                dbg_event("shooting a ray");                                     // scene.cu:107-108
                if (cast_ray(x, top.ray, is)) {
                    if (top.depth > 0) {
                        if (top.in_obj) top.atten = mul4(top.atten, trans_atten(s.mats[is.mat], is.time));
                        top.type = REFLECT;
                        top.hit_pt = ray_at(top.ray, is.time);
                        top.last_mat = is.mat;
                        top.norm = is.norm;
                    } else {
                        top_i--;
                    }
                    acc = add4(acc, mul4(top.atten, illuminate(x, top.ray, is)));
                } else {
                    top_i--;
                }
                break;
            }
            case REFLECT: {
                const Material& m = s.mats[is.mat];
                top.type = REFRACT;
                if (reflective(m)) {
                    dbg_event("preparing to shoot a reflection ray");            // scene.cu:134-135
                    top_i++;
                    RayFrame& nt = frames[top_i];
                    nt.type = NORMAL; nt.last_mat = top.last_mat; nt.in_obj = top.in_obj;
                    nt.atten = mul4(top.atten, m.Kr);
                    nt.depth = top.depth - 1;
                    nt.ray = make_ray(top.hit_pt, reflect(top.ray.d, normalized(top.norm)));
                }
                break;
            }
            case REFRACT: {
                const Material& m = s.mats[is.mat];
                if (refractive(m)) {
                    dbg_event("preparing to shoot a refraction ray");            // scene.cu:152-153
                    top.type = NORMAL;
                    float n1, n2; bool tir;
                    if (top.in_obj) { n1 = s.mats[top.last_mat].eta; n2 = 1.0f; }
                    else { n1 = 1.0f; n2 = s.mats[top.last_mat].eta; }
                    V3 rd = refract(top.ray.d, normalized(top.norm), n1, n2, tir);
                    if (tir) top_i--;
                    else { top.ray = make_ray(top.hit_pt, rd); top.in_obj = !top.in_obj; top.depth--; }
                } else top_i--;
                break;
            }
        }
    }
    return acc;
}

V4 propagate_cpu(const Ctx& x, const Ray& r, Isect& is, float& last_time, bool in_obj, int depth) {  // scene.cu:222-268
    const orc_scene& s = *x.s;
    if (depth > s.depth) return V4{0, 0, 0, 0};   // dead code in practice: depth only decreases (scene.cu:224)
    is.time = INFINITY;
    if (cast_ray(x, r, is)) {
        V4 acc = illuminate(x, r, is);
        last_time = is.time;
        float next_time = 0;
        if (reflective(s.mats[is.mat])) {
            V3 rd = reflect(r.d, is.norm);
            Ray rr = make_ray(ray_at(r, is.time), rd);
            acc = add4(acc, propagate_cpu(x, rr, is, next_time, in_obj, depth - 1));
        }
        if (refractive(s.mats[is.mat])) {
            float n1, n2; bool tir;
            if (in_obj) { n1 = s.mats[is.mat].eta; n2 = 1.0f; }
            else { n1 = 1.0f; n2 = s.mats[is.mat].eta; }
            V3 rd = refract(r.d, is.norm, n1, n2, tir);
            if (!tir) {
                next_time = 0;
                Ray rr = make_ray(ray_at(r, is.time), rd);
                V4 un = propagate_cpu(x, rr, is, next_time, in_obj, depth - 1);
                acc = add4(acc, mul4(trans_atten(s.mats[is.mat], next_time), un));
            }
        }
        return acc;
    }
    return V4{0, 0, 0, 0};
}

inline uint8_t to_u8(float c) { return (uint8_t)((float)255 * c); }         // color.h:41-42
inline uint32_t encode(float r, float g, float b, float a) {                // color.cu:23-26
    return ((uint32_t)to_u8(r) << 24) + ((uint32_t)to_u8(g) << 16) + ((uint32_t)to_u8(b) << 8) + (uint32_t)to_u8(a);
}
inline float clamp1(float c) { return c > 1.0f ? 1.0f : c; }                // raytracer.cu:37-40

struct RenderJob {
    const orc_scene* s; const BVH* bvh; int sem; int use_bvh; int spp;
    const std::vector<int>* rows; size_t r_begin, r_end;
    uint32_t* rgba; float* rad; int32_t* hi; int32_t* ht;
    Counters cnt;
};

void render_rows(RenderJob* J) {
    const orc_scene& s = *J->s;
    CamBasis cb = cam_basis(s.cam);
    Ctx x{&s, J->bvh, J->use_bvh != 0, J->sem == ORC_SEM_CPU, &J->cnt};
    for (size_t ri = J->r_begin; ri < J->r_end; ri++) {
        int y = (*J->rows)[ri];
        for (int xx = 0; xx < s.W; xx++) {
            float sum[4] = {0, 0, 0, 0}, rsum[4] = {0, 0, 0, 0};
            int32_t hinst = -1, htri = -1;
            for (int k = 0; k < J->spp; k++) {
                float dx, dy; orc_spp_offset(k, &dx, &dy);
                Ray r = cam_at(s.cam, cb, (float)xx + dx, (float)y + dy);
                Isect is; is.time = INFINITY; is.mat = -1; is.inst = -1; is.tri = -1; is.norm = v3(0, 0, 0);
                V4 c;
                if (J->sem == ORC_SEM_CPU) { float t; c = propagate_cpu(x, r, is, t, false, s.depth); }
                else {
                    if (k == 0 && (J->hi || J->ht)) {
                        // primary hit ids: an extra probe of the primary ray (not counted)
                        Counters dummy; Ctx px = x; px.c = &dummy;
                        Isect ps = is; ps.time = INFINITY;
                        if (cast_ray(px, r, ps)) { hinst = ps.inst; htri = ps.tri; }
                    }
                    c = propagate_gpu(x, r, is);
                }
                float cc[4] = {c.x, c.y, c.z, c.w};
                for (int q = 0; q < 4; q++) { sum[q] += clamp1(cc[q]); rsum[q] += cc[q]; }
            }
            size_t p = (size_t)y * s.W + xx;
            float inv = (float)J->spp;
            float m[4] = {sum[0] / inv, sum[1] / inv, sum[2] / inv, sum[3] / inv};
            if (J->rgba) J->rgba[p] = encode(m[0], m[1], m[2], m[3]);
            if (J->rad) for (int q = 0; q < 4; q++) J->rad[4 * p + q] = rsum[q] / inv;
            if (J->hi) J->hi[p] = hinst;
            if (J->ht) J->ht[p] = htri;
        }
    }
}

void* thread_entry(void* a) { render_rows((RenderJob*)a); return nullptr; }

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

const char* orc_last_error(void) { return g_err.c_str(); }

void orc_spp_offset(int k, float* dx, float* dy) {
    // R2 low-discrepancy sequence, evaluated in IEEE double then rounded (build-defined; k=0 -> (0,0)).
    const double a1 = 0.7548776662466927, a2 = 0.5698402909980532;
    double u = (double)k * a1, v = (double)k * a2;
    *dx = (float)(u - std::floor(u));
    *dy = (float)(v - std::floor(v));
}

int orc_load(const char* path, int width, int height, orc_scene** out) {
    try {
        std::ifstream f(path);
        if (!f) { g_err = std::string("cannot open ") + path; return -1; }
        std::stringstream ss; ss << f.rdbuf(); std::string txt = ss.str();
        JP p{txt.data(), txt.data() + txt.size()};
        JV doc = p.parse();
        std::unique_ptr<orc_scene> s(new orc_scene);
        load_cube_world(*s, doc, width, height);
        if (s->depth >= MAX_DEPTH) { g_err = "depth >= MAX_DEPTH overflows the reference frame stack"; return -2; }
        *out = s.release();
        return 0;
    } catch (std::exception& e) { g_err = e.what(); return -1; }
}

void orc_free(orc_scene* s) { delete s; }

int orc_set_atlas(orc_scene* s, const uint8_t* rgba8, int w, int h) {
    if (!s || !rgba8 || w <= 0 || h <= 0) return -1;
    s->atlas.assign(rgba8, rgba8 + (size_t)w * h * 4);
    s->atlas_w = w; s->atlas_h = h;
    return 0;
}
int orc_set_textures(orc_scene* s, int on) {
    if (!s) return -1;
    s->textures = on ? 1 : 0;
    return 0;
}

// ---- SceneBuilder (scene_builder.h:29-117, scene_builder.cc:11-29, scene_builder.cu:21-239) ----
static Material mat26(const float* m) {                                      // material.h:14-31
    Material r;
    r.Ke = V4{m[0], m[1], m[2], m[3]}; r.Ka = V4{m[4], m[5], m[6], m[7]}; r.Kd = V4{m[8], m[9], m[10], m[11]};
    r.Ks = V4{m[12], m[13], m[14], m[15]}; r.Kt = V4{m[16], m[17], m[18], m[19]}; r.Kr = V4{m[20], m[21], m[22], m[23]};
    r.alpha = m[24]; r.eta = m[25];
    return r;
}
int orc_scene_create(orc_scene** out) {
    if (!out) return -1;
    orc_scene* s = new orc_scene;
    s->building = true;
    *out = s;
    return 0;
}
int orc_builder_add_vertex(orc_scene* s, float x, float y, float z) {       // SceneBuilder::add_vertex
    if (!s || !s->building) return -1;
    s->verts.push_back(v3(x, y, z));
    return (int)s->verts.size() - 1;
}
int orc_builder_create_mesh(orc_scene* s, const float* pos, const float* q) {   // create_mesh(pos, rot)
    if (!s || !s->building) return -1;
    Mesh m;
    m.e = Entity{q ? Quat{q[0], q[1], q[2], q[3]} : Quat{0, 0, 0, 1}, pos ? v3(pos[0], pos[1], pos[2]) : v3(0, 0, 0)};
    m.begin = m.count = 0;
    s->meshes.push_back(m);
    s->mesh_tris.emplace_back();
    return (int)s->meshes.size() - 1;
}
int orc_builder_add_triangle(orc_scene* s, int mesh, int i0, int i1, int i2, const float* m, const float* tex6) {
    if (!s || !s->building || !m || mesh < 0 || mesh >= (int)s->meshes.size()) return -1;   // MeshBuilder::add_triangle
    Tri t; t.i0 = i0; t.i1 = i1; t.i2 = i2;
    t.mat = (int)s->mats.size(); s->mats.push_back(mat26(m));               // one Material per triangle
    if (tex6) { t.tex.has = 1; t.tex.tx = tex6[0]; t.tex.ty = tex6[1]; t.tex.ux = tex6[2]; t.tex.uy = tex6[3]; t.tex.vx = tex6[4]; t.tex.vy = tex6[5]; }
    s->mesh_tris[mesh].push_back(t);
    return 0;
}
int orc_builder_add_trans(orc_scene* s, int mesh) {                          // add_trans: Transformation{hitable_idx}
    if (!s || !s->building || mesh < 0 || mesh >= (int)s->meshes.size()) return -1;
    s->insts.push_back(Inst{Entity{Quat{0, 0, 0, 1}, v3(0, 0, 0)}, mesh});
    return (int)s->insts.size() - 1;
}
int orc_builder_build_cube(orc_scene* s, float scale, const float* m, const float* tile3) {
    if (!s || !s->building || !m) return -1;
    build_cube(*s, scale, mat26(m), tile3);
    return (int)s->meshes.size() - 1;
}
int orc_builder_add_point_light(orc_scene* s, const float* pos, const float* col) {
    if (!s || !s->building || !pos || !col) return -1;
    s->b_points.push_back(Light{0, v3(pos[0], pos[1], pos[2]), V4{col[0], col[1], col[2], col[3]}});
    return 0;
}
int orc_builder_add_directional_light(orc_scene* s, const float* dir, const float* col) {
    if (!s || !s->building || !dir || !col) return -1;                      // DirLight::set_shine_dir normalizes
    s->b_dirs.push_back(Light{1, normalized(v3(dir[0], dir[1], dir[2])), V4{col[0], col[1], col[2], col[3]}});
    return 0;
}
// build_gpu_scene(Canvas, Camera) + Environment (scene_builder.cu:21-100, camera.cu:6-9,
// environment.h:19-93): meshes flattened in creation order, normals generated, point lights
// before directional ones.
int orc_builder_finish(orc_scene* s, int W, int H, float fov, float unit, const float* cpos, const float* cq,
                       const float* da, const float* amb, int depth) {
    if (!s || !s->building || W <= 0 || H <= 0 || !(unit > 0) || depth < 0 || depth >= MAX_DEPTH) return -1;
    for (size_t m = 0; m < s->meshes.size(); m++) {
        s->meshes[m].begin = (int)s->tris.size();
        s->meshes[m].count = (int)s->mesh_tris[m].size();
        for (const Tri& t : s->mesh_tris[m]) {
            if (t.i0 < 0 || t.i1 < 0 || t.i2 < 0 || t.i0 >= (int)s->verts.size() || t.i1 >= (int)s->verts.size() ||
                t.i2 >= (int)s->verts.size()) return -1;
            s->tris.push_back(t);
        }
    }
    s->lights = s->b_points; s->n_point = (int)s->b_points.size();
    s->lights.insert(s->lights.end(), s->b_dirs.begin(), s->b_dirs.end());
    s->W = W; s->H = H;
    s->cam.e = Entity{cq ? Quat{cq[0], cq[1], cq[2], cq[3]} : Quat{0, 0, 0, 1}, cpos ? v3(cpos[0], cpos[1], cpos[2]) : v3(0, 0, 0)};
    s->cam.near_ = 0.5f * W / unit / tanf(fov);                              // camera.cu:7 (nvcc TU: tanf)
    s->cam.unit = unit; s->cam.W = (float)W; s->cam.H = (float)H;
    if (da) s->dist_atten = v3(da[0], da[1], da[2]);
    if (amb) s->ambience = V4{amb[0], amb[1], amb[2], amb[3]};
    s->depth = depth;
    generate_normals(*s);
    s->building = false;
    s->mesh_tris.clear();
    return 0;
}
// Entity::set_position / set_orientation of the camera (entity.h:49-74; Camera::at reads them,
// camera.cu:33-42) and of instance i's Transformation (get_transformation(i), entity.cu:5-37).
int orc_set_camera(orc_scene* s, const float* pos, const float* q) {
    if (!s || s->building) return -1;
    if (pos) s->cam.e.p = v3(pos[0], pos[1], pos[2]);
    if (q) s->cam.e.o = Quat{q[0], q[1], q[2], q[3]};
    return 0;
}
int orc_set_trans(orc_scene* s, int i, const float* pos, const float* q) {
    if (!s || i < 0 || i >= (int)s->insts.size()) return -1;
    if (pos) s->insts[i].e.p = v3(pos[0], pos[1], pos[2]);
    if (q) s->insts[i].e.o = Quat{q[0], q[1], q[2], q[3]};
    return 0;
}
int orc_set_env(orc_scene* s, const float* amb, const float* da, int depth) {   // Environment setters
    if (!s || depth < 0 || depth >= MAX_DEPTH) return -1;
    if (amb) s->ambience = V4{amb[0], amb[1], amb[2], amb[3]};
    if (da) s->dist_atten = v3(da[0], da[1], da[2]);
    s->depth = depth;
    return 0;
}

int orc_scene_counts(const orc_scene* s, int32_t* c) {
    c[0] = s->W; c[1] = s->H; c[2] = (int)s->verts.size(); c[3] = (int)s->tris.size(); c[4] = (int)s->meshes.size();
    c[5] = (int)s->insts.size(); c[6] = (int)s->lights.size(); c[7] = s->n_point; c[8] = s->depth; c[9] = (int)s->mats.size();
    return 0;
}
int orc_scene_vertices(const orc_scene* s, float* o) { for (auto& v : s->verts) { *o++ = v.x; *o++ = v.y; *o++ = v.z; } return 0; }
int orc_scene_normals(const orc_scene* s, float* o) { for (auto& v : s->norms) { *o++ = v.x; *o++ = v.y; *o++ = v.z; } return 0; }
int orc_scene_tris(const orc_scene* s, int32_t* o) { for (auto& t : s->tris) { *o++ = t.i0; *o++ = t.i1; *o++ = t.i2; *o++ = t.mat; } return 0; }
int orc_scene_materials(const orc_scene* s, float* o) {
    for (auto& m : s->mats) {
        const V4* vs[6] = {&m.Ke, &m.Ka, &m.Kd, &m.Ks, &m.Kt, &m.Kr};
        for (auto* v : vs) { *o++ = v->x; *o++ = v->y; *o++ = v->z; *o++ = v->w; }
        *o++ = m.alpha; *o++ = m.eta;
    }
    return 0;
}
int orc_scene_instances(const orc_scene* s, float* q, int32_t* mesh) {
    for (auto& t : s->insts) {
        *q++ = t.e.o.i; *q++ = t.e.o.j; *q++ = t.e.o.k; *q++ = t.e.o.r; *q++ = t.e.p.x; *q++ = t.e.p.y; *q++ = t.e.p.z;
        *mesh++ = t.mesh;
    }
    return 0;
}
int orc_scene_lights(const orc_scene* s, float* o) {
    for (auto& l : s->lights) { *o++ = l.v.x; *o++ = l.v.y; *o++ = l.v.z; *o++ = (float)l.type; *o++ = l.col.x; *o++ = l.col.y; *o++ = l.col.z; *o++ = l.col.w; }
    return 0;
}
int orc_scene_camera(const orc_scene* s, float* c, float* env) {
    const Camera& k = s->cam; CamBasis b = cam_basis(k);
    float v[21] = {k.e.p.x, k.e.p.y, k.e.p.z, k.e.o.i, k.e.o.j, k.e.o.k, k.e.o.r, k.near_, k.unit, k.W, k.H,
                   b.r.x, b.r.y, b.r.z, b.u.x, b.u.y, b.u.z, b.f.x, b.f.y, b.f.z, 0};
    memcpy(c, v, 21 * sizeof(float));
    float e[7] = {s->dist_atten.x, s->dist_atten.y, s->dist_atten.z, s->ambience.x, s->ambience.y, s->ambience.z, s->ambience.w};
    memcpy(env, e, sizeof e);
    return 0;
}

// debug_cast (raytracer.cu:45-52, 91-100): one ray through pixel (x, y) -- Camera::at with
// the integer pixel, propagate_ray with the debug printfs on -- its event log into buf.
int orc_debug_cast(const orc_scene* s, int x, int y, int use_bvh, char* buf, int64_t cap) {
    if (!s || s->building || x < 0 || y < 0 || x >= s->W || y >= s->H || !buf || cap <= 0) return -1;
    BVH bvh = build_bvh(*s, false);
    Counters c;
    Ctx cx{s, &bvh, use_bvh != 0, false, &c};
    CamBasis cb = cam_basis(s->cam);
    Ray r = cam_at(s->cam, cb, (float)x, (float)y);
    Isect is; is.time = INFINITY; is.mat = -1; is.inst = -1; is.tri = -1; is.norm = v3(0, 0, 0);
    std::string log;
    g_dbg = &log;
    (void)propagate_gpu(cx, r, is);
    g_dbg = nullptr;
    const size_t m = std::min(log.size(), (size_t)cap - 1);
    memcpy(buf, log.data(), m);
    buf[m] = 0;
    return 0;
}

int orc_build_bvh(const orc_scene* s, float* boxes, int32_t* ordering, int max_n) {
    BVH b = build_bvh(*s, false);
    if (b.n > max_n) return -1;
    for (size_t i = 0; i < b.tree.size(); i++) {
        const Box& x = b.tree[i];
        float v[7] = {x.mn.x, x.mn.y, x.mn.z, x.mx.x, x.mx.y, x.mx.z, x.nd ? 1.0f : 0.0f};
        memcpy(boxes + 7 * i, v, sizeof v);
    }
    for (int i = 0; i < b.n; i++) ordering[i] = b.ordering[i];
    return b.n;
}

int orc_render(const orc_scene* s, int sem, int use_bvh, int spp, int row0, int row_step, int nthreads,
               uint32_t* rgba, float* rad, int32_t* hi, int32_t* ht, uint64_t* stats) {
    if (spp < 1 || row_step < 1 || row0 < 0) { g_err = "bad arguments"; return -1; }
    if (s->building) { g_err = "builder scene not finished"; return -1; }
    BVH bvh = build_bvh(*s, sem == ORC_SEM_CPU);
    std::vector<int> rows;
    for (int y = row0; y < s->H; y += row_step) rows.push_back(y);
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > rows.size()) nthreads = rows.empty() ? 1 : (int)rows.size();
    std::vector<RenderJob> jobs(nthreads);
    // interleave rows across threads in chunks for balance
    std::vector<std::vector<int>> per(nthreads);
    for (size_t i = 0; i < rows.size(); i++) per[i % nthreads].push_back(rows[i]);
    std::vector<pthread_t> th(nthreads);
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = RenderJob{s, &bvh, sem, use_bvh, spp, &per[t], 0, per[t].size(), rgba, rad, hi, ht, Counters{}};
    }
    if (nthreads == 1 && sem == ORC_SEM_GPU) {
        render_rows(&jobs[0]);
    } else {
        // Large stacks: the CPU-path recursion is unbounded (measured 4,418 levels).
        pthread_attr_t attr; pthread_attr_init(&attr); pthread_attr_setstacksize(&attr, 256u << 20);
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], &attr, thread_entry, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], nullptr);
        pthread_attr_destroy(&attr);
    }
    if (stats) {
        stats[0] = stats[1] = stats[2] = stats[3] = 0;
        for (auto& j : jobs) { stats[0] += j.cnt.rays; stats[1] += j.cnt.nodes; stats[2] += j.cnt.leaves; stats[3] += j.cnt.tris; }
    }
    return 0;
}

// ---- KATs ----
static inline V3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }
static inline void st3(float* p, V3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
void orc_kat_normalize3(int n, const float* v, float* o) { for (int i = 0; i < n; i++) st3(o + 3 * i, normalized(ld3(v + 3 * i))); }
void orc_kat_cross(int n, const float* a, const float* b, float* o) { for (int i = 0; i < n; i++) st3(o + 3 * i, cross(ld3(a + 3 * i), ld3(b + 3 * i))); }
void orc_kat_reflect(int n, const float* d, const float* m, float* o) { for (int i = 0; i < n; i++) st3(o + 3 * i, reflect(ld3(d + 3 * i), ld3(m + 3 * i))); }
void orc_kat_refract(int n, const float* d, const float* m, const float* nn, float* o, int32_t* tir) {
    for (int i = 0; i < n; i++) { bool t; st3(o + 3 * i, refract(ld3(d + 3 * i), ld3(m + 3 * i), nn[2 * i], nn[2 * i + 1], t)); tir[i] = t; }
}
void orc_kat_quat_rotate(int n, const float* q, const float* v, float* o) {
    for (int i = 0; i < n; i++) st3(o + 3 * i, qrot(Quat{q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]}, ld3(v + 3 * i)));
}
void orc_kat_quat_inverse(int n, const float* q, float* o) {
    for (int i = 0; i < n; i++) { Quat r = qinverse(Quat{q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]}); o[4 * i] = r.i; o[4 * i + 1] = r.j; o[4 * i + 2] = r.k; o[4 * i + 3] = r.r; }
}
void orc_kat_quat_mul(int n, const float* a, const float* b, float* o) {
    for (int i = 0; i < n; i++) {
        Quat r = qmul(Quat{a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]}, Quat{b[4 * i], b[4 * i + 1], b[4 * i + 2], b[4 * i + 3]});
        o[4 * i] = r.i; o[4 * i + 1] = r.j; o[4 * i + 2] = r.k; o[4 * i + 3] = r.r;
    }
}
void orc_kat_tri_hit(int n, const float* t9, const float* r6, int32_t* hit, float* o) {
    for (int i = 0; i < n; i++) {
        const float* t = t9 + 9 * i; const float* r = r6 + 6 * i;
        Ray ray = make_ray(ld3(r), ld3(r + 3));
        float time = NAN, u = NAN, v = NAN;
        hit[i] = triangle_hit(ld3(t), ld3(t + 3), ld3(t + 6), ray, time, u, v);
        o[3 * i] = hit[i] ? time : NAN; o[3 * i + 1] = hit[i] ? u : NAN; o[3 * i + 2] = hit[i] ? v : NAN;
    }
}
void orc_kat_box_hit(int n, const float* b7, const float* r6, int32_t* hit, float* t) {
    for (int i = 0; i < n; i++) {
        const float* b = b7 + 7 * i; const float* r = r6 + 6 * i;
        Box bx{ld3(b), ld3(b + 3), b[6] != 0};
        Ray ray = make_ray(ld3(r), ld3(r + 3));
        float tt = NAN;
        hit[i] = box_intersects(bx, ray, tt);
        t[i] = tt;
    }
}
void orc_kat_box_from_local(int n, const float* b7, const float* e7, float* o6, int32_t* nd) {
    for (int i = 0; i < n; i++) {
        const float* b = b7 + 7 * i; const float* e = e7 + 7 * i;
        Box r = from_local(Box{ld3(b), ld3(b + 3), b[6] != 0}, Entity{Quat{e[0], e[1], e[2], e[3]}, ld3(e + 4)});
        st3(o6 + 6 * i, r.mn); st3(o6 + 6 * i + 3, r.mx); nd[i] = r.nd ? 1 : 0;
    }
}
void orc_kat_box_merge(int n, const float* a7, const float* b7, float* o6, int32_t* nd) {
    for (int i = 0; i < n; i++) {
        const float* a = a7 + 7 * i; const float* b = b7 + 7 * i;
        Box r = merge(Box{ld3(a), ld3(a + 3), a[6] != 0}, Box{ld3(b), ld3(b + 3), b[6] != 0});
        st3(o6 + 6 * i, r.mn); st3(o6 + 6 * i + 3, r.mx); nd[i] = r.nd ? 1 : 0;
    }
}
void orc_kat_entity(int n, const float* e7, const float* v3, float* o12) {
    for (int i = 0; i < n; i++) {
        const float* e = e7 + 7 * i;
        const Entity en{Quat{e[0], e[1], e[2], e[3]}, ld3(e + 4)};
        const V3 v = ld3(v3 + 3 * i);
        st3(o12 + 12 * i, point_to_local(en, v)); st3(o12 + 12 * i + 3, vec_to_local(en, v));
        st3(o12 + 12 * i + 6, point_from_local(en, v)); st3(o12 + 12 * i + 9, vec_from_local(en, v));
    }
}
void orc_kat_hitable(int n, const float* e7, const float* ray6, const float* hit4, float* o10) {
    for (int i = 0; i < n; i++) {
        const float* e = e7 + 7 * i; const float* h = hit4 + 4 * i;
        const Entity en{Quat{e[0], e[1], e[2], e[3]}, ld3(e + 4)};
        Isect is{};
        is.time = INFINITY;
        Ray seen{};
        hitable_hit(en, make_ray(ld3(ray6 + 6 * i), ld3(ray6 + 6 * i + 3)), is, [&](const Ray& lr, Isect& li) {
            seen = lr; li.time = h[0]; li.norm = ld3(h + 1); return true;     // a local hit at (t, n)
        });
        st3(o10 + 10 * i, seen.o); st3(o10 + 10 * i + 3, seen.d); o10[10 * i + 6] = is.time; st3(o10 + 10 * i + 7, is.norm);
    }
}
void orc_kat_axis_angle(int n, const float* a4, float* o) {
    for (int i = 0; i < n; i++) { Quat q = qaxis_angle_g(ld3(a4 + 4 * i), a4[4 * i + 3]); o[4 * i] = q.i; o[4 * i + 1] = q.j; o[4 * i + 2] = q.k; o[4 * i + 3] = q.r; }
}
void orc_kat_to_mat3(int n, const float* q, float* o) {
    for (int i = 0; i < n; i++) { float m[3][3]; to_mat3(Quat{q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]}, m); memcpy(o + 9 * i, m, sizeof m); }
}
void orc_kat_zorder(int n, const float* v, uint64_t* o) { for (int i = 0; i < n; i++) o[i] = z_order(ld3(v + 3 * i)); }
void orc_kat_ray_ctor(int n, const float* r6, float* o) {
    for (int i = 0; i < n; i++) { Ray r = make_ray(ld3(r6 + 6 * i), ld3(r6 + 6 * i + 3)); st3(o + 6 * i, r.o); st3(o + 6 * i + 3, r.d); }
}

}  // extern "C"
