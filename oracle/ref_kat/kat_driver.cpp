// kat_driver.cpp — known-answer harness over the REFERENCE's own math sources.
//
// Compiled (oracle/Makefile target `ref`) with g++ directly against the
// reference's headers include/raymath/{linear.h,geometry.h}, include/rayopt/bounding_box.h,
// include/rayprimitives/{entity.h,gpu/hitable.cuh} and its translation units
// src/rayopt/z_order.cu, src/rayopt/bounding_box.cu, src/rayprimitives/entity.cu and
// src/rayprimitives/hitable.cu, unmodified, read in place from
// /root/reference.  entity.h includes <cuda.h> / <cuda_runtime.h>: those are the CUDA 12.8
// toolkit headers this image ships (Triton's copy, CUDA_INC in the Makefile), used as they
// are -- under g++ they only declare the host runtime, and nothing here calls or links it.
// Output binary: oracle/_ref/kat_ref (git-ignored).  It reads raw little-endian
// input arrays and writes raw outputs; tests/golden/make_golden.py drives it and
// commits the (inputs, outputs) pairs as fixtures.
//
// The reference's render path lives in nvcc translation units, where the CUDA
// math headers put float overloads of abs/sqrt/pow in scope (so `abs(float)` in
// Plane::hit / Triangle::hit is fabsf).  Under plain g++ that unqualified call
// would bind to C `int abs(int)`.  The using-declarations below reproduce the
// nvcc overload set for this driver's translation unit; nothing else is
// substituted.  cos/sin are deliberately left as the C double functions: the
// only caller of Quat(axis, theta) on the path is cube_world.cc, a g++ TU.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
using std::abs;
using std::sqrt;
using std::pow;

#include "raymath/linear.h"
#include "raymath/geometry.h"
#include "rayopt/z_order.h"
#include "rayopt/bounding_box.h"        // + src/rayopt/bounding_box.cu (slab test, from_local, merge)
#include "rayprimitives/entity.h"       // + src/rayprimitives/entity.cu (pose transforms)

// Hitable::hit (hitable.cu:29-38) around a known local hit: a subclass whose hit_local (the
// virtual the reference's Trimesh implements, trimesh.cu:11-19) records the local ray it is
// given and reports a hit at a given local time and normal.
#include "rayprimitives/gpu/hitable.cuh"
struct KatHitable : rprimitives::gpu::Hitable {
    rmath::Ray<float> seen;
    float t_local = 0;
    rmath::Vec3<float> n_local;
    KatHitable(rmath::Vec3<float> p, rmath::Quat<float> o) : Hitable(p, o), seen(rmath::Vec3<float>(), rmath::Vec3<float>()) {}
    bool hit_local(const rmath::Ray<float>& lr, renv::gpu::Scene*, rprimitives::Isect& is) override {
        seen = lr; is.time = t_local; is.norm = n_local; return true;
    }
};

using V3 = rmath::Vec3<float>;
using V4 = rmath::Vec4<float>;
using Q = rmath::Quat<float>;
using R = rmath::Ray<float>;

static std::vector<char> slurp(const char* p) {
    FILE* f = fopen(p, "rb");
    if (!f) { perror(p); exit(2); }
    std::vector<char> b;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    fclose(f);
    return b;
}
static const float* F(const std::vector<char>& b, size_t off) { return reinterpret_cast<const float*>(b.data()) + off; }
static V3 v3(const float* p) { return V3({p[0], p[1], p[2]}); }
static void put3(std::vector<float>& o, const V3& v) { o.push_back(v[0]); o.push_back(v[1]); o.push_back(v[2]); }

int main(int argc, char** argv) {
    if (argc != 5) { fprintf(stderr, "usage: kat_ref <op> <n> <in.bin> <out.bin>\n"); return 2; }
    std::string op = argv[1];
    int n = atoi(argv[2]);
    std::vector<char> in = slurp(argv[3]);
    std::vector<float> of;
    std::vector<int32_t> oi;
    std::vector<uint64_t> ou;
    for (int i = 0; i < n; i++) {
        if (op == "normalize3") {
            put3(of, v3(F(in, 3 * i)).normalized());
        } else if (op == "cross") {
            put3(of, rmath::cross(v3(F(in, 3 * i)), v3(F(in, 3 * (n + i)))));
        } else if (op == "reflect") {
            put3(of, rmath::reflect(v3(F(in, 3 * i)), v3(F(in, 3 * (n + i)))));
        } else if (op == "refract") {
            const float* nn = F(in, 6 * n + 2 * i);
            bool tir = false;
            put3(of, rmath::refract(v3(F(in, 3 * i)), v3(F(in, 3 * (n + i))), nn[0], nn[1], tir));
            oi.push_back(tir ? 1 : 0);
        } else if (op == "quat_rotate") {
            const float* q = F(in, 4 * i);
            put3(of, Q(q[0], q[1], q[2], q[3]) * v3(F(in, 4 * n + 3 * i)));
        } else if (op == "quat_inverse") {
            const float* q = F(in, 4 * i);
            V4 r = Q(q[0], q[1], q[2], q[3]).inverse().to_Vec4();
            for (int c = 0; c < 4; c++) of.push_back(r[c]);
        } else if (op == "quat_mul") {
            const float* a = F(in, 4 * i);
            const float* b = F(in, 4 * (n + i));
            V4 r = (Q(a[0], a[1], a[2], a[3]) * Q(b[0], b[1], b[2], b[3])).to_Vec4();
            for (int c = 0; c < 4; c++) of.push_back(r[c]);
        } else if (op == "tri_hit") {
            const float* t = F(in, 9 * i);
            const float* r = F(in, 9 * n + 6 * i);
            rmath::Triangle<float> tri(v3(t), v3(t + 3), v3(t + 6));
            R ray(v3(r), v3(r + 3));
            float time = NAN;
            rmath::Vec<float, 2> uv({NAN, NAN});
            bool h = tri.hit(ray, time, uv);
            oi.push_back(h ? 1 : 0);
            of.push_back(h ? time : NAN); of.push_back(h ? uv[0] : NAN); of.push_back(h ? uv[1] : NAN);
        } else if (op == "ray_ctor") {
            const float* r = F(in, 6 * i);
            R ray(v3(r), v3(r + 3));
            put3(of, ray.origin()); put3(of, ray.direction());
        } else if (op == "zorder") {
            ou.push_back((uint64_t)ropt::z_order(v3(F(in, 3 * i))));
        } else if (op == "box_hit") {              // BoundingBox::intersects (bounding_box.cu:62-104)
            const float* b = F(in, 7 * i);
            const float* r = F(in, 7 * n + 6 * i);
            ropt::BoundingBox bx;
            bx.min = v3(b); bx.max = v3(b + 3); bx.nondegenerate = b[6] != 0;
            R ray(v3(r), v3(r + 3));
            float t = NAN;
            const bool h = bx.intersects(ray, t);
            of.push_back(h ? t : NAN);
            oi.push_back(h ? 1 : 0);
        } else if (op == "box_from_local" || op == "box_merge") {   // bounding_box.cu:5-60
            const float* a = F(in, 7 * i);
            const float* c = F(in, 7 * n + 7 * i);
            ropt::BoundingBox ba;
            ba.min = v3(a); ba.max = v3(a + 3); ba.nondegenerate = a[6] != 0;
            ropt::BoundingBox r;
            if (op == "box_from_local") {
                rprimitives::Entity e(v3(c + 4), Q(c[0], c[1], c[2], c[3]));   // entity = (quat i j k r, pos)
                r = ropt::from_local(ba, e);
            } else {
                ropt::BoundingBox bb;
                bb.min = v3(c); bb.max = v3(c + 3); bb.nondegenerate = c[6] != 0;
                r = ropt::merge(ba, bb);
            }
            put3(of, r.min); put3(of, r.max);
            oi.push_back(r.nondegenerate ? 1 : 0);
        } else if (op == "entity") {               // Entity point/vec to/from local (entity.cu:5-37)
            const float* c = F(in, 7 * i);
            const V3 v = v3(F(in, 7 * n + 3 * i));
            rprimitives::Entity e(v3(c + 4), Q(c[0], c[1], c[2], c[3]));
            put3(of, e.point_to_local(v)); put3(of, e.vec_to_local(v));
            put3(of, e.point_from_local(v)); put3(of, e.vec_from_local(v));
        } else if (op == "hitable") {              // Hitable::hit / HitHandle (hitable.cu:7-38)
            const float* c = F(in, 7 * i);
            const float* r = F(in, 7 * n + 6 * i);
            const float* h = F(in, 13 * n + 4 * i);
            KatHitable e(v3(c + 4), Q(c[0], c[1], c[2], c[3]));
            e.t_local = h[0]; e.n_local = v3(h + 1);
            float time = INFINITY;
            rprimitives::Isect is(time);
            R ray(v3(r), v3(r + 3));
            e.hit(ray, nullptr, is);
            put3(of, e.seen.origin()); put3(of, e.seen.direction()); of.push_back(time); put3(of, is.norm);
        } else if (op == "axis_angle") {
            const float* a = F(in, 4 * i);
            V4 r = Q(v3(a), a[3]).to_Vec4();
            for (int c = 0; c < 4; c++) of.push_back(r[c]);
        } else if (op == "to_mat3") {
            const float* q = F(in, 4 * i);
            rmath::Mat3<float> m = Q(q[0], q[1], q[2], q[3]).to_Mat3();
            for (int a = 0; a < 3; a++) for (int b = 0; b < 3; b++) of.push_back(m(a, b));
        } else {
            fprintf(stderr, "unknown op %s\n", op.c_str());
            return 2;
        }
    }
    FILE* f = fopen(argv[4], "wb");
    if (!f) { perror(argv[4]); return 2; }
    fwrite(of.data(), sizeof(float), of.size(), f);
    fwrite(oi.data(), sizeof(int32_t), oi.size(), f);
    fwrite(ou.data(), sizeof(uint64_t), ou.size(), f);
    fclose(f);
    return 0;
}
