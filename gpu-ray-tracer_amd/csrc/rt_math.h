// rt_math.h — bit-exact float32 math of the reference's raymath layer, usable on
// the host (scene preparation) and on gfx950 (kernels).
//
// Semantics follow include/raymath/linear.h and geometry.h of
// wtzhang23/gpu-ray-tracer operand-for-operand, because the renderer's integer
// outputs (hit instance / triangle) depend on last-ulp comparisons (the 1e-5
// barycentric tolerance, strict `<` on hit times).  Build rules that make this
// hold: -ffp-contract=off everywhere, no fast-math, HIP's default correctly
// rounded f32 division and sqrt, f32 denormals preserved (gfx950 default).
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rtm {

constexpr float THRESH = 1e-5f;   // rmath::THRESHOLD (linear.h:15): a double holding 1e-5f

struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };
struct Q { float i, j, k, r; };   // geometry.h: inner = {i, j, k, r}

RT_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
RT_HD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
// scalar * vector multiplies each coordinate by the scalar (linear.h:100-106, 132-137)
RT_HD V3 operator*(float c, V3 v) { return v3(v.x * c, v.y * c, v.z * c); }
RT_HD V3 neg(V3 v) { return (-1.0f) * v; }                           // (T)-1 * vec (linear.h:139-142)
RT_HD float dot(V3 a, V3 b) {                                       // linear.h:197-205: 0 + x*x + ...
    float s = 0.0f; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s;
}
// Correctly rounded sqrt and reciprocal (IEEE, the HIP defaults on gfx950: the compiler's
// exact sequences).  A shorter exact device form (v_rcp / v_sqrt with Newton and residual
// corrections) measured no faster while growing the code by a quarter and was
// removed; tests/test_gpu_kat.py still checks these bit for bit against IEEE.
RT_HD float rcp_cr(float x) { return 1.0f / x; }
RT_HD float sqrt_cr(float x) { return sqrtf(x); }

RT_HD float len(V3 v) { return sqrt_cr(dot(v, v)); }
RT_HD V3 normalized(V3 v) {                                         // linear.h:159-167
    float l = len(v);
    if (l > THRESH) return rcp_cr(l) * v;
    return v3(0.0f, 0.0f, 0.0f);
}
RT_HD V3 cross(V3 a, V3 b) {                                        // linear.h:207-215
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
RT_HD V4 v4(float x, float y, float z, float w) { return V4{x, y, z, w}; }
RT_HD V4 operator+(V4 a, V4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
RT_HD V4 operator*(V4 a, V4 b) { return v4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
RT_HD V4 operator*(float c, V4 v) { return v4(v.x * c, v.y * c, v.z * c, v.w * c); }
RT_HD float dot4(V4 a, V4 b) {
    float s = 0.0f; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; s += a.w * b.w; return s;
}

// reflect's tail with |dir| and normalized(dir), normalized(nrm) given
RT_HD V3 reflect_pre(float d_len, V3 dn, V3 nn) {
    V3 proj = dot(dn, nn) * nn;
    return d_len * normalized(dn - 2.0f * proj);
}
RT_HD V3 reflect(V3 dir, V3 nrm) {                                   // linear.h:217-226
    return reflect_pre(len(dir), normalized(dir), normalized(nrm));
}
RT_HD V3 refract(V3 dir, V3 nrm, float from, float to, bool& tir) {  // linear.h:228-243
    float d_len = len(dir);
    V3 dn = normalized(dir), nn = normalized(nrm);
    float ratio = from / to;
    float cosi = dot(dn, nn);
    float sint_2 = ratio * ratio * (1 - cosi * cosi);
    if (sint_2 > 1) { tir = true; return d_len * reflect(dn, nn); }
    tir = false;
    return d_len * (ratio * dn + (ratio * cosi - sqrtf(1 - sint_2)) * nn);
}

// ---- quaternions (geometry.h:17-199) ----
RT_HD V4 qv(Q q) { return v4(q.i, q.j, q.k, q.r); }
RT_HD Q qnormalized(Q q) {
    float l = sqrtf(dot4(qv(q), qv(q)));
    if (l > THRESH) { float c = 1 / l; return Q{q.i * c, q.j * c, q.k * c, q.r * c}; }
    return Q{0.0f, 0.0f, 0.0f, 0.0f};
}
RT_HD Q qinverse(Q q) {
    float sq = dot4(qv(q), qv(q));
    if (sq < THRESH) return Q{0.0f, 0.0f, 0.0f, 0.0f};
    float inv = 1 / sq;
    return Q{q.i * -inv, q.j * -inv, q.k * -inv, q.r * inv};
}
RT_HD Q qmul(Q a, Q b) {
    return Q{a.i * b.r + a.r * b.i + a.j * b.k - a.k * b.j,
             a.j * b.r + a.r * b.j + a.k * b.i - a.i * b.k,
             a.k * b.r + a.r * b.k + a.i * b.j - a.j * b.i,
             a.r * b.r - a.i * b.i - a.j * b.j - a.k * b.k};
}
// Quat * Vec3 with the two quaternion-only factors precomputed:
//   qn = normalized(q), qi = inverse(q)       (geometry.h:176-181)
RT_HD V3 qrot_pre(Q qn, Q qi, V3 v) {
    float length = len(v);
    Q p = qmul(qmul(qn, Q{v.x, v.y, v.z, 0.0f}), qi);
    return length * normalized(v3(p.i, p.j, p.k));
}
RT_HD V3 qrot(Q q, V3 v) { return qrot_pre(qnormalized(q), qinverse(q), v); }

// Exact specialisation of qrot_pre for q == (0,0,0,1) or its inverse (-0,-0,-0,1)
// (every pose in the cube world).  Proof sketch: both
// quaternion products return the input coordinates unchanged except that a
// zero comes back as +0; `x + 0.0f` performs exactly that canonicalisation
// and is not folded without fast-math.  Then |v| * normalize(v') follows.
RT_HD V3 qrot_identity(V3 v) {
    // = length * normalized(c).  len(c) == len(v) bit for bit: c differs from v only by
    // -0 -> +0, whose square is the same +0, so normalized(c)'s length is `length`.
    float length = len(v);
    V3 c = v3(v.x + 0.0f, v.y + 0.0f, v.z + 0.0f);
    V3 nc = length > THRESH ? rcp_cr(length) * c : v3(0.0f, 0.0f, 0.0f);
    return length * nc;
}

// ---- entity pose (entity.cu:5-37) with precomputed quaternion factors ----
struct Pose {
    V3 p;
    int identity;   // 1 when o == (0,0,0,1) bitwise: use qrot_identity
    Q tn, ti;       // to_local:   normalized(o),          inverse(o)
    Q fn, fi;       // from_local: normalized(inverse(o)), inverse(inverse(o))
};
RT_HD V3 vec_to_local(const Pose& e, V3 v) { return e.identity ? qrot_identity(v) : qrot_pre(e.tn, e.ti, v); }
RT_HD V3 vec_from_local(const Pose& e, V3 v) { return e.identity ? qrot_identity(v) : qrot_pre(e.fn, e.fi, v); }
RT_HD V3 point_to_local(const Pose& e, V3 v) { return vec_to_local(e, v - e.p); }
RT_HD V3 point_from_local(const Pose& e, V3 v) { return vec_from_local(e, v) + e.p; }

inline bool bits_eq(float a, float b) { union { float f; uint32_t u; } x{a}, y{b}; return x.u == y.u; }
inline Pose make_pose(Q o, V3 p) {
    Pose e;
    e.p = p;
    e.identity = bits_eq(o.i, 0.0f) && bits_eq(o.j, 0.0f) && bits_eq(o.k, 0.0f) && bits_eq(o.r, 1.0f);
    e.tn = qnormalized(o); e.ti = qinverse(o);
    Q inv = qinverse(o);
    e.fn = qnormalized(inv); e.fi = qinverse(inv);
    return e;
}

// ---- rays (geometry.h:201-223) ----
struct Ray { V3 o, d; };
RT_HD Ray make_ray(V3 o, V3 d) { return Ray{o, normalized(d)}; }
RT_HD V3 at(const Ray& r, float t) { return r.o + t * r.d; }

// ---- bounding boxes (bounding_box.cu:5-104) ----
struct Box { V3 mn, mx; int nd; };
RT_HD void fit_vertex(Box& b, V3 v) {
    if (!b.nd) { b.mn = v; b.mx = v; b.nd = 1; return; }
    if (v.x < b.mn.x) b.mn.x = v.x;
    if (v.x > b.mx.x) b.mx.x = v.x;
    if (v.y < b.mn.y) b.mn.y = v.y;
    if (v.y > b.mx.y) b.mx.y = v.y;
    if (v.z < b.mn.z) b.mn.z = v.z;
    if (v.z > b.mx.z) b.mx.z = v.z;
}
RT_HD Box merge(const Box& a, const Box& b) {
    Box r = a;
    if (!r.nd) return b;
    if (!b.nd) return r;
    if (r.mn.x > b.mn.x) r.mn.x = b.mn.x;
    if (r.mx.x < b.mx.x) r.mx.x = b.mx.x;
    if (r.mn.y > b.mn.y) r.mn.y = b.mn.y;
    if (r.mx.y < b.mx.y) r.mx.y = b.mx.y;
    if (r.mn.z > b.mn.z) r.mn.z = b.mn.z;
    if (r.mx.z < b.mx.z) r.mx.z = b.mx.z;
    return r;
}
RT_HD Box from_local(const Box& a, const Pose& e) {
    Box r; r.nd = 0; r.mn = r.mx = v3(0.0f, 0.0f, 0.0f);
    if (!a.nd) return r;
    fit_vertex(r, point_from_local(e, a.mn));
    fit_vertex(r, point_from_local(e, a.mx));
    return r;
}
// Kay–Kajiya slab test, bounding_box.cu:62-104 (true divisions; zero-direction axes skipped)
RT_HD bool slab_axis(float mn, float mx, float o, float d, float& tmin, float& tmax) {
    if (d == 0) return true;
    float tn = (mn - o) / d;
    float tf = (mx - o) / d;
    if (tn > tf) { float t = tn; tn = tf; tf = t; }
    if (tn > tmin) tmin = tn;
    if (tf < tmax) tmax = tf;
    return !(tmin > tmax || tmax < THRESH);
}
RT_HD bool box_hit(V3 mn, V3 mx, const Ray& r) {
    float tmin = -INFINITY, tmax = INFINITY;
    if (!slab_axis(mn.x, mx.x, r.o.x, r.d.x, tmin, tmax)) return false;
    if (!slab_axis(mn.y, mx.y, r.o.y, r.d.y, tmin, tmax)) return false;
    return slab_axis(mn.z, mx.z, r.o.z, r.d.z, tmin, tmax);
}
RT_HD V3 box_center(const Box& b) { return 0.5f * (b.mn + b.mx); }

// z_order.cu:5-36 — 64-bit interleave of the raw float bits, x first, MSB first.
// The loop emits, MSB first, x bit 31-k at output bit 63-3k (k = 0..21), y bit 31-k at
// 62-3k and z bit 31-k at 61-3k (k = 0..20); with X = x >> 10, Y = y >> 11, Z = z >> 11
// that is bit j of X -> 3j, of Z -> 3j+1, of Y -> 3j+2: three magic-mask bit spreads.
RT_HD uint64_t spread3(uint64_t v) {                 // bit j (j < 21) -> bit 3j
    v &= 0x1fffffull;
    v = (v | v << 32) & 0x1f00000000ffffull;
    v = (v | v << 16) & 0x1f0000ff0000ffull;
    v = (v | v << 8) & 0x100f00f00f00f00full;
    v = (v | v << 4) & 0x10c30c30c30c30c3ull;
    v = (v | v << 2) & 0x1249249249249249ull;
    return v;
}
RT_HD uint64_t z_order(V3 vec) {
    V3 inv = neg(vec);
    union { float f; uint32_t u; } cx{inv.x}, cy{inv.y}, cz{inv.z};
    const uint32_t X = cx.u >> 10, Y = cy.u >> 11, Z = cz.u >> 11;   // 22, 21, 21 bits
    return spread3(X) | ((uint64_t)(X >> 21) << 63) | (spread3(Z) << 1) | (spread3(Y) << 2);
}

// ---- triangle test (geometry.h:229-290) with ray-independent factors precomputed ----
// pn = normalized(cross(b-a, c-a)) (Plane ctor), area = |cross(b-a, c-a)|.
RT_HD bool tri_hit(V3 a, V3 b, V3 c, V3 pn, float area, const Ray& r, float& time, float& u, float& v) {
    float denom = dot(r.d, pn);
    if (fabsf(denom) < THRESH) return false;
    float t = rcp_cr(denom) * dot(a - r.o, pn);
    V3 p = at(r, t);
    float b0 = len(cross(c - p, b - p)) / area;
    float b1 = len(cross(c - p, a - p)) / area;
    float b2 = len(cross(a - p, b - p)) / area;
    if (fabsf(b0 + b1 + b2 - 1.0f) <= THRESH) { time = t; u = b1; v = b2; return true; }
    time = t;
    return false;
}

// ---- exactness-preserving filtered tests (device) ----------------------------
// The reference's box and triangle tests are decided by comparisons of correctly
// rounded quotients and square roots.  The filtered forms evaluate cheap
// approximations with a rigorous error bound and return the reference's exact
// answer whenever the approximation is decisive; inside the (tiny) uncertainty
// band they run the exact reference arithmetic.  Derivation (u = 2^-24):
//  * q' = fl(e * r'), r' = v_rcp_f32(d) within 1 ulp of 1/d, vs q = fl(e / d):
//    |q' - q| <= 4.02 u |q'| in the normal range (ray_inv below); the bound used is
//    16 u max|q'| + 2^-120 (absolute floor for the subnormal range; non-finite values
//    always fall back).  min/max of
//    perturbed values move by at most the same bound, and the slab test's
//    early exits are monotone, so its outcome is (T_min <= T_max && T_max >= 1e-5)
//    evaluated once at the end.
//  * v_sqrt_f32 / v_rcp_f32 are within 1 ulp; a barycentric term b' =
//    fl(sqrt'(s) * fl(1/area)) is within 6u of fl(fl(sqrt(s)) / area); the sum
//    test uses a 32u margin.  The accepted (t, u, v) are always recomputed exactly.
// b* = +inf for a zero direction component (the reference skips that slab): the packed
// pair test forms q0 = fma(mn - o, inv, -b), q1 = fma(mx - o, inv, +b), i.e. (-inf, +inf)
// = no constraint for a skipped axis and exactly fl((mn - o) * inv) otherwise.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
#else
RT_HD float fast_sqrt(float x) { return sqrtf(x); }
RT_HD float fast_rcp(float x) { return 1.0f / x; }
#endif
// The reciprocals are v_rcp_f32 on the device (within 1 ulp, i.e. 2u relative, for
// 2^-64 <= |d| <= 2^64): a quotient q' = fl(e * r') is then within 4.02u |q'| of the
// reference's fl(e / d) (2u + 1u + 1u and second-order terms), and the box filters' margins
// are 16u per slab bound (min/max keep the relative bound; the sums below add < 1u each).
// Components outside that range (never the case for the normalised directions of the
// integrator, whose nonzero components are >= ~1e-7) take the exact reference test.
struct RayInv { float ix, iy, iz, bx, by, bz; int exact; };
RT_HD bool rcp_range(float d) { const float a = fabsf(d); return d == 0.0f || (a >= 0x1p-64f && a <= 0x1p64f); }
RT_HD RayInv ray_inv(const Ray& r) {
    RayInv v;
    v.ix = r.d.x != 0 ? fast_rcp(r.d.x) : 0.0f;
    v.iy = r.d.y != 0 ? fast_rcp(r.d.y) : 0.0f;
    v.iz = r.d.z != 0 ? fast_rcp(r.d.z) : 0.0f;
    v.bx = r.d.x != 0 ? 0.0f : INFINITY;
    v.by = r.d.y != 0 ? 0.0f : INFINITY;
    v.bz = r.d.z != 0 ? 0.0f : INFINITY;
    v.exact = !(rcp_range(r.d.x) && rcp_range(r.d.y) && rcp_range(r.d.z)) ||
              (r.d.x == 0.0f && r.d.y == 0.0f && r.d.z == 0.0f);    // no slab constrains t
    return v;
}
constexpr float FILT_BOX = 0x1p-20f;       // 16 u
constexpr float FILT_TRI = 0x1p-19f;       // 32 u
constexpr float FILT_ABS = 0x1p-120f;

RT_HD void slab_axis_f(float mn, float mx, float o, float d, float inv, float& tmin, float& tmax, float& m) {
    if (d == 0) return;
    float q0 = (mn - o) * inv, q1 = (mx - o) * inv;
    tmin = fmaxf(tmin, fminf(q0, q1));
    tmax = fminf(tmax, fmaxf(q0, q1));
    m = fmaxf(m, fmaxf(fabsf(q0), fabsf(q1)));
}
RT_HD bool box_hit_f(V3 mn, V3 mx, const Ray& r, const RayInv& ri) {
    if (ri.exact) return box_hit(mn, mx, r);
    float tmin = -INFINITY, tmax = INFINITY, m = 0.0f;
    slab_axis_f(mn.x, mx.x, r.o.x, r.d.x, ri.ix, tmin, tmax, m);
    slab_axis_f(mn.y, mx.y, r.o.y, r.d.y, ri.iy, tmin, tmax, m);
    slab_axis_f(mn.z, mx.z, r.o.z, r.d.z, ri.iz, tmin, tmax, m);
    const float E = m * FILT_BOX + FILT_ABS;
    if (tmin - tmax > 2.0f * E || tmax + E < THRESH) return false;     // certainly a miss
    if (tmin + 2.0f * E <= tmax && tmax - E >= THRESH) return true;      // certainly a hit
    return box_hit(mn, mx, r);                                           // near a tie: exact
}

// box_hit_f that also returns tlo, a lower bound of the exact slab entry distance
// (|tmin_f - tmin| <= E, see above); -inf when the exact test decided.
RT_HD bool box_hit_ft(V3 mn, V3 mx, const Ray& r, const RayInv& ri, float& tlo) {
    tlo = -INFINITY;
    if (ri.exact) return box_hit(mn, mx, r);
    float tmin = -INFINITY, tmax = INFINITY, m = 0.0f;
    slab_axis_f(mn.x, mx.x, r.o.x, r.d.x, ri.ix, tmin, tmax, m);
    slab_axis_f(mn.y, mx.y, r.o.y, r.d.y, ri.iy, tmin, tmax, m);
    slab_axis_f(mn.z, mx.z, r.o.z, r.d.z, ri.iz, tmin, tmax, m);
    const float E = m * FILT_BOX + FILT_ABS;
    if (tmin - tmax > 2.0f * E || tmax + E < THRESH) return false;
    if (tmin + 2.0f * E <= tmax && tmax - E >= THRESH) { tlo = tmin - 2.0f * E; return true; }
    return box_hit(mn, mx, r);
}


// tri_hit (above) + TriInner::tri_hit's acceptance (trimesh.cu:56), filtered.
// inv_area = fl(1 / area) (host-precomputed; only used by the filter).
// Split in two so the trace kernel can start the next triangle's loads between them:
// tri_plane_f needs only (pn, a) and rejects most triangles; tri_inside_f finishes.
// `lo` (<= 1e-5 when unused): a proven lower bound of any acceptable t (the leaf box's
// entry distance minus the pruning slack, see closest_hit in rt_kernels.hip).
RT_HD bool tri_plane_f(V3 a, V3 pn, const Ray& r, float best, float lo, float& denom, float& num) {
    denom = dot(r.d, pn);
    if (fabsf(denom) < THRESH) return false;
    num = dot(a - r.o, pn);
    float ta = num * fast_rcp(denom);                    // ~1 ulp of the exact fl(fl(1/denom) * num)
    float et = fabsf(ta) * FILT_TRI + FILT_ABS;
    return !(ta + et < fmaxf(THRESH, lo) || ta - et >= best);   // false: certainly rejected
}
// Inside test of a plane crossing at the exact reference time t (already known to satisfy
// 1e-5 <= t < best): geometry.h:280-286, filtered.
RT_HD bool tri_inside_t(V3 a, V3 b, V3 c, float area, float inv_area, const Ray& r, float t, float& time, float& u,
                        float& v) {
    V3 p = at(r, t);
    V3 x0 = cross(c - p, b - p), x1 = cross(c - p, a - p), x2 = cross(a - p, b - p);
    float s0 = dot(x0, x0), s1 = dot(x1, x1), s2 = dot(x2, x2);
    float sum = (fast_sqrt(s0) * inv_area + fast_sqrt(s1) * inv_area) + fast_sqrt(s2) * inv_area;
    float dev = fabsf(sum - 1.0f), eb = sum * FILT_TRI + FILT_ABS;
    if (!(dev <= THRESH + eb)) return false;             // certainly outside (also catches NaN)
    float b1 = sqrtf(s1) / area, b2 = sqrtf(s2) / area;  // exact barycentrics (geometry.h:281-283)
    if (dev < THRESH - eb) { time = t; u = b1; v = b2; return true; }   // certainly inside
    float b0 = sqrtf(s0) / area;
    if (fabsf(b0 + b1 + b2 - 1.0f) <= THRESH) { time = t; u = b1; v = b2; return true; }
    return false;
}
RT_HD bool tri_inside_f(V3 a, V3 b, V3 c, float area, float inv_area, const Ray& r, float best, float denom,
                        float num, float& time, float& u, float& v) {
    float t = rcp_cr(denom) * num;                        // exact (geometry.h:259)
    if (!(t >= THRESH && t < best)) return false;
    return tri_inside_t(a, b, c, area, inv_area, r, t, time, u, v);
}

// Axis-plane triangles (every cube face): the three vertices share coordinate `ax`
// exactly and the stored plane normal pn is exactly +-e_ax (two +-0 components).  Then
// the reference's plane arithmetic collapses without rounding: dot(r.d, pn) = +0 + ... =
// s * d_ax and dot(a - r.o, pn) = s * fl(a_ax - o_ax) with s = sign(pn_ax) (the +-0
// products add to +0, and x + 0 = x), and fl(1/(s d)) = s fl(1/d), so
//   t = fl(fl(1/denom) * num) = fl(fl(1/d_ax) * fl(a_ax - o_ax))     (geometry.h:255-259)
// bit for bit, and |denom| < 1e-5 <=> |d_ax| < 1e-5.  `inv_ax` carries fl(1/d_ax), or NaN
// when |d_ax| < 1e-5 (the reference rejects: every comparison with NaN fails).
RT_HD float axis_plane_t(float a_ax, float o_ax, float inv_ax) { return inv_ax * (a_ax - o_ax); }

// x^y for float x > 0 and y with |y ln x| <= 700, in double and rounded once to float: the
// same value as (float)pow((double)x, (double)y) except when x^y lies within ~2^-45 (relative)
// of a float rounding midpoint, and in every case one of the two floats around x^y, so within
// 1 ulp of glibc powf (which is within 0.82 ulp).  Returns false outside that domain.
//   log x = e ln2 + 2 atanh(s), s = (m - 1)/(m + 1), m in [sqrt(1/2), sqrt(2)): m - 1 and m + 1
//   are exact (m carries x's 24 bits), the division is correctly rounded, |s| <= 0.1716 and the
//   series to s^19 leaves < 2^-60; e ln2 = e LN2_HI (exact, |e| <= 149) + e LN2_LO.
//   exp z = 2^k exp r, k = rint(z / ln2), |r| <= 0.3466 + 2^-40: Taylor to r^12 leaves < 2^-52.
// Rounding: |error of z| <= 2^-52 (|z| + 1), so the relative error of the double is < 2^-44
// for the float range (|z| < 104) and below 2^-51 on the shading's |z| < 2.
constexpr double POW_LN2_HI = 6.93147180369123816490e-01;   // 0x3fe62e42fee00000 (32 bits)
constexpr double POW_LN2_LO = 1.90821492927058770002e-10;   // ln2 - POW_LN2_HI
RT_HD bool pow_pos(float xf, float yf, float& out) {
    if (!(xf > 0.0f) || !(fabsf(xf) <= 3.4028235e38f) || !(fabsf(yf) <= 3.4028235e38f)) return false;
    int e;
    double m = frexp((double)xf, &e);                   // [0.5, 1)
    if (m < 0.70710678118654752440) { m = 2.0 * m; e -= 1; }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double p = 2.0 / 19;
    p = fma(p, s2, 2.0 / 17); p = fma(p, s2, 2.0 / 15); p = fma(p, s2, 2.0 / 13);
    p = fma(p, s2, 2.0 / 11); p = fma(p, s2, 2.0 / 9);  p = fma(p, s2, 2.0 / 7);
    p = fma(p, s2, 2.0 / 5);  p = fma(p, s2, 2.0 / 3);
    const double lm = fma(s * s2, p, 2.0 * s);          // log m
    const double lx = (double)e * POW_LN2_HI + (lm + (double)e * POW_LN2_LO);
    const double z = (double)yf * lx;
    if (!(fabs(z) <= 700.0)) return false;
    const double k = rint(z * 1.44269504088896340736);
    const double r = fma(-k, POW_LN2_LO, fma(-k, POW_LN2_HI, z));
    double q = 1.0 / 479001600;                         // 1/12!
    q = fma(q, r, 1.0 / 39916800); q = fma(q, r, 1.0 / 3628800); q = fma(q, r, 1.0 / 362880);
    q = fma(q, r, 1.0 / 40320);    q = fma(q, r, 1.0 / 5040);    q = fma(q, r, 1.0 / 720);
    q = fma(q, r, 1.0 / 120);      q = fma(q, r, 1.0 / 24);      q = fma(q, r, 1.0 / 6);
    q = fma(q, r, 0.5);            q = fma(q, r, 1.0);           q = fma(q, r, 1.0);
    out = (float)ldexp(q, (int)k);
    return true;
}

// Host-built record of a triangle for the axis-plane path (rt_kernels.hip, cast_local).
// code: bits 0-1 axis (3 = general triangle), bit 2 = the next triangle of the mesh has the
// same axis and plane coordinate (identical t: when no lane accepts this plane crossing, the
// next one is rejected too), bit 3 = the in-plane reject below is valid for this triangle.
// [ulo, uhi] x [vlo, vhi]: the triangle's extent along the two in-plane axes (u = ax+1,
// v = ax+2 mod 3) grown by m = 1e-4 D (D = longest edge); win = 1e3 D; off = m.
// In-plane reject (exact): the point p = at(r, t) fails the reference's inside test when its
// in-plane excess e = max(ulo - p_u, p_u - uhi, vlo - p_v, p_v - vhi) has 0 < e <= win and
// |p_ax - a_ax| <= off.  Proof: the exact barycentric weights of p's projection satisfy
// sum|l_i| - 1 >= e / D (the set sum|l_i| - 1 <= k is the triangle grown about itself by at
// most k D per side); lifting p off the plane only enlarges the three areas; the reference's
// float evaluation (differences, cross products, squared norm, sqrt, division by the stored
// area A~ = A (1 + eta), two additions) differs from the exact sum S by at most
// 41.8 u M^2 / A + (5.6 u + eta) S with M <= D + e + off.  The host checks
// (e/D)(1 - 5.6u - eta) - (5.6u + eta) - 41.8 u (D + e + off)^2 / A > 1.01e-5 at e = m and
// e = win; the left side is concave in e, so it holds on the whole range.
struct TriAx { int code; float a_ax, ulo, uhi, vlo, vhi, win, off; };
RT_HD bool tri_accept_f(V3 a, V3 b, V3 c, V3 pn, float area, float inv_area, const Ray& r, float best,
                        float& time, float& u, float& v) {
    float denom, num;
    return tri_plane_f(a, pn, r, best, -INFINITY, denom, num) &&
           tri_inside_f(a, b, c, area, inv_area, r, best, denom, num, time, u, v);
}

// ---- quaternion <-> basis (geometry.h:36-41, 183-198) ----
inline Q axis_angle_gxx(V3 axis, float theta) {   // g++ TU (cube_world.cc): double cos/sin
    float hc = (float)cos((double)(0.5f * theta));
    float hs = (float)sin((double)(0.5f * theta));
    return Q{axis.x * hs, axis.y * hs, axis.z * hs, hc};
}
RT_HD void to_mat3(Q q, float m[3][3]) {
    float length = sqrtf(dot4(qv(q), qv(q)));
    float ni = q.i / length, nj = q.j / length, nk = q.k / length, nr = q.r / length;
    float ii = 2.0f * ni * ni, jj = 2.0f * nj * nj, kk = 2.0f * nk * nk;
    float ri = 2.0f * nr * ni, rj = 2.0f * nr * nj, rk = 2.0f * nr * nk;
    float ij = 2.0f * ni * nj, ik = 2.0f * ni * nk, jk = 2.0f * nj * nk;
    m[0][0] = 1 - (jj + kk); m[0][1] = ij - rk;       m[0][2] = ik + rj;
    m[1][0] = ij + rk;       m[1][1] = 1 - (ii + kk); m[1][2] = jk - ri;
    m[2][0] = ik - rj;       m[2][1] = jk + ri;       m[2][2] = 1 - (ii + jj);
}

}  // namespace rtm
