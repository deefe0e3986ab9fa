// Host check of pow_pos (gpu-ray-tracer_amd/csrc/rt_math.h, the device pow of the shading):
// the same float as (float)pow((double)x, (double)y) with glibc, and within 1 ulp of glibc
// powf (the oracle's pow), on the shading's domain (x in (0, 1] and [1, 50], the scenes'
// exponents) and on random positive floats with exponents in [-40, 40].
//   pow_host N_RANDOM  -> prints "n diff_vs_double max_ulp_vs_powf outside_domain"
#include "rt_math.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
using namespace rtm;
static long ulps(float a, float b) {
    int32_t x, y;
    std::memcpy(&x, &a, 4); std::memcpy(&y, &b, 4);
    return std::labs((long)x - (long)y);
}
int main(int argc, char** argv) {
    const long n_random = argc > 1 ? std::atol(argv[1]) : 1000000;
    long n = 0, diff = 0, max_ulp = 0, outside = 0;
    auto check = [&](float x, float y) {
        float o;
        if (!pow_pos(x, y, o)) { outside++; return; }
        n++;
        if (o != (float)pow((double)x, (double)y)) diff++;
        const long u = ulps(o, powf(x, y));
        if (u > max_ulp) max_ulp = u;
    };
    const float ys[] = {0.6f, 0.7f, 0.8f, 1.5f, 2.5f, 10.0f};
    for (float y : ys)
        for (int i = 1; i <= 200000; i++) { check(i / 200000.0f, y); check(1.0f + 49.0f * i / 200000.0f, y); }
    std::mt19937_64 g(7);
    std::uniform_real_distribution<float> U(-40.0f, 40.0f);
    for (long i = 0; i < n_random; i++) {
        uint32_t b = (uint32_t)g() & 0x7fffffffu;
        float x;
        std::memcpy(&x, &b, 4);
        if (!(x > 0.0f) || !std::isfinite(x)) continue;
        check(x, U(g) * (i % 3 == 0 ? 1.0f : 0.05f));
    }
    std::printf("%ld %ld %ld %ld\n", n, diff, max_ulp, outside);
    return 0;
}
