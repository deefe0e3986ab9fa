// shim_rmath.cpp — the C++ shim's host math (include/rtracer_amd.hpp, namespace rmath) on the
// inputs of the reference-built KAT fixtures (tests/golden/kat_*.npz), for
// tests/test_shim_math.py.  main.cc turns and moves the camera with these operations
// (main.cc:144-177: Quat(axis, theta), Quat * Quat, Vec arithmetic, normalized, Ray), so the
// shim must round them as the reference's g++ translation unit does.
//   shim_rmath OP N IN OUT   (IN: raw float32 inputs in the fixture's order; OUT: raw float32)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rtracer_amd.hpp"

using V3 = rmath::Vec3<float>;
using Q = rmath::Quat<float>;

int main(int argc, char** argv) {
    if (argc != 5) { std::fprintf(stderr, "usage: shim_rmath OP N IN OUT\n"); return 2; }
    const std::string op = argv[1];
    const long n = std::atol(argv[2]);
    std::vector<float> in;
    {
        FILE* f = std::fopen(argv[3], "rb");
        if (!f) { std::perror(argv[3]); return 2; }
        float x;
        while (std::fread(&x, 4, 1, f) == 1) in.push_back(x);
        std::fclose(f);
    }
    std::vector<float> out;
    auto v3 = [&](long off) { return V3({in[off], in[off + 1], in[off + 2]}); };
    auto put3 = [&](const V3& v) { for (int c = 0; c < 3; c++) out.push_back(v[c]); };
    auto put4 = [&](const Q& q) { out.push_back(q.i); out.push_back(q.j); out.push_back(q.k); out.push_back(q.r); };
    for (long i = 0; i < n; i++) {
        if (op == "axis_angle") {                  // a = (axis xyz, theta)
            const float* a = &in[4 * i];
            put4(Q(V3({a[0], a[1], a[2]}), a[3]));
        } else if (op == "quat_mul") {            // a, b stacked
            const float* a = &in[4 * i];
            const float* b = &in[4 * (n + i)];
            put4(Q(a[0], a[1], a[2], a[3]) * Q(b[0], b[1], b[2], b[3]));
        } else if (op == "normalize3") {
            put3(v3(3 * i).normalized());
        } else if (op == "ray_ctor") {             // ray = (origin, direction)
            rmath::Ray<float> r(v3(6 * i), v3(6 * i + 3));
            put3(r.origin());
            put3(r.direction());
        } else {
            std::fprintf(stderr, "unknown op %s\n", op.c_str());
            return 2;
        }
    }
    FILE* f = std::fopen(argv[4], "wb");
    if (!f) { std::perror(argv[4]); return 2; }
    std::fwrite(out.data(), 4, out.size(), f);
    std::fclose(f);
    return 0;
}
