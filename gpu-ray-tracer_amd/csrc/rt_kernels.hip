// rt_kernels.hip — gfx950 kernels of the ray-tracing core + the C ABI (rt_amd.h).
//
// Hot path (BASELINE.json north_star): rtracer::gpu::update_scene
// (src/raytracer.cu:102-120) = per-frame BVH build + the per-pixel `trace`
// megakernel running renv::gpu::propagate_ray (src/rayenv/scene.cu:92-188).
//
// MI355X design:
//  * bvh_build_kernel: ONE workgroup of 1024 threads per frame builds the reference's Morton
//    BVH (boxes -> 64-bit z-order keys -> an LDS rank sort equal to thrust's stable
//    sort_by_key -> pairwise level merges, bvh.cu:11-91) in the reference's heap layout (child
//    pairs as three float4) and, from the same sorted leaves, an ordered LBVH for the fast
//    kernels (64-B records, leaves met in the heap's DFS order).  Above 8192 padded leaves the
//    grid-wide build of rt_bvh_large.hip takes over.
//  * sky_kernel: a pre-pass over pixel groups (8 pixels x 8 samples at 8 spp): a group none of
//    whose primary rays enters the tree's root is written here (zeros, -1 hit ids) and the
//    live groups go onto per-queue lists (and, hist = 2, the previous frame's heavy groups onto
//    a heavy list run first).
//  * trace_kernel: persistent 1024-thread blocks, one per CU, with the scene (ordered tree,
//    instances, shading records) staged in LDS.  A wave takes live groups from work queues;
//    lane = (pixel, sample).  Each lane runs propagate_ray (scene.cu:92-188) as a state machine
//    whose only wave-collective step is the closest-hit query: a packet traversal with the node
//    index wave-uniform (SGPR), 16-B broadcast LDS record reads, a filtered slab test with the
//    exact reference test as fallback, and ballots for descend / push / pop.  Integrator state
//    the traversal does not read is parked in LDS during the query.  Every filter and pruning
//    is exact: hit ids equal the reference's single-ray semantics and
//    radiance its float32 operations.
#include <dlfcn.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types only: RCCL is opened at run time (MultiDev), never linked

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <fstream>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rt_bvh.h"
#include "rt_math.h"
#include "rt_scene.h"
#include "../../include/rt_amd.h"

using namespace rtm;
using namespace rtb;
using rt::DCamera;
using rt::DInst;
using rt::DLight;
using rt::DMat;
using rt::DMesh;
using rt::DNode;
using rt::DTri;

namespace {

constexpr int MAX_FRAMES = 10;           // renv::gpu::MAX_DEPTH (scene.cu:25)
constexpr int BVH_WG_LEAVES = 8192;      // single-workgroup BVH build (LDS keys); above: bvh_build_large
constexpr int BVH_MAX_LEAVES = 1 << 24;  // padded leaves (int indexing of the 12n-float pair records)
#ifndef RT_BLOCK
#define RT_BLOCK 1024
#endif
constexpr int TRACE_BLOCK_P = RT_BLOCK;  // persistent block: 16 waves (4 per SIMD, 128-VGPR budget) sharing one LDS BVH copy
constexpr int LDS_LIMIT = 150 * 1024;    // above this the BVH is read from global memory
constexpr int PARK_LDS_LIMIT = 158 * 1024;   // BVH image + parking area (160 KB per CU)
#ifndef RT_NQ
#define RT_NQ 8
#endif
constexpr int NQ = RT_NQ;                    // work queues (one per XCD dispatch slot), 64-B apart
// work counters: [16 q] queue q's tickets, [16 NQ] the heavy list's, [16 (NQ + 1 + q)] the
// length of live-group list q (sky_kernel), [16 (2 NQ + 1)] the length of this frame's heavy
// live list (hist = 2)
constexpr int WORK_INTS = 16 * (2 * NQ + 2);
constexpr int WORK_HEAVY_LEN = 16 * (2 * NQ + 1);
// Statistics / profiling counters (d_stats): [0, 22) rt_stats and the PROF step counts and
// cycle split (rt_experiment), [22, 24) spare, [24, 64) the PROF variant's query-occupancy
// counters (PROF_* below, rt_frame_work).
constexpr int STATS_N = 64;
enum : int {
    PROF_LANES_PRIMARY = 24, PROF_LANES_SECONDARY = 25, PROF_LANES_SHADOW = 26, PROF_LANES_UNLIT = 27,
    PROF_LIVE_WQ = 28, PROF_LIVE_LANES = 29,
    PROF_HIST_WQ = 30,      // [8] live wave queries by active lanes, buckets of 8 (1-8, 9-16, ..., 57-64)
    PROF_HIST_PAIR = 38,    // [8] their child-pair steps
    PROF_HIST_LEAF = 46,    // [8] their leaf visits
    PROF_END = 54
};
// PROF kernels keep the occupancy counters [24, PROF_END) per wave in LDS (a global atomic per wave
// query on a few shared addresses serialised and perturbed the profile 30x) and add them to d_stats
// once per wave at the end
constexpr int PROF_WAVE_SLOTS = 32;
static_assert(PROF_END - PROF_LANES_PRIMARY <= PROF_WAVE_SLOTS, "per-wave PROF counter slots");
constexpr size_t PROF_LDS_BYTES = 16 * PROF_WAVE_SLOTS * sizeof(unsigned long long);   // 16 waves per block

enum : int { F_NORMAL = 0, F_REFLECT = 1, F_REFRACT = 2 };
enum : int { PH_NORMAL = 1, PH_SHADOW = 2, PH_DONE = 3 };

__device__ __forceinline__ float max_std(float a, float b) { return (a < b) ? b : a; }   // std::max
// powf of the reference (nvcc pow(float,float)); evaluated in double and rounded:
// agrees with glibc powf except for 1-ulp cases.  pow_pos (rt_math.h)
// answers x > 0 with |y ln x| <= 700 in about 40 double operations; the rest (x <= 0, inf,
// nan, overflow and underflow far outside float range) take the library's double pow.
__device__ __forceinline__ float pow_lib(float x, float y) { return (float)pow((double)x, (double)y); }
__device__ __noinline__ float pow_ref(float x, float y) {   // rare: kept out of line
    float o;
    return pow_pos(x, y, o) ? o : pow_lib(x, y);
}
// pow_ref with the C99 / IEEE special cases that dominate the shading calls answered
// inline (every powf and pow agree on them bit for bit, F.9.4.4): pow(x, +-0) = 1 (the
// materials without "alpha"), pow(1, y) = 1, pow(+-0, y > 0) = +0 except -0 for odd integer
// y (lights behind the surface give max(dot, 0) = +-0).  A wave skips the double-precision
// call when none of its lanes needs it.
__device__ __forceinline__ float pow_fast(float x, float y) {
    if (y == 0.0f || x == 1.0f) return 1.0f;
    if (x == 0.0f && y > 0.0f) {
        const bool odd = y == rintf(y) && rintf(0.5f * y) != 0.5f * y;
        return (odd && signbit(x)) ? -0.0f : 0.0f;
    }
    return pow_ref(x, y);
}



// Unsigned division by a launch constant d with host-computed magic numbers (round-up
// method: l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1, q = (t + ((n - t) >> 1)) >> (l - 1),
// t = mulhi(n, m); exact for every 32-bit n; d = 1 passes through).  Wave-uniform operands stay
// on the scalar unit (the compiler's own sequence keeps a VGPR reciprocal live across the
// group loop, which was spilled and reloaded from scratch at every group).
struct UDiv { unsigned m, d; int s; };
__host__ inline UDiv udiv_make(unsigned d) {
    UDiv r{0u, d, 0};
    if (d <= 1) return r;
    int l = 0;
    while ((1ull << l) < d) l++;
    r.m = (unsigned)((((1ull << l) - d) << 32) / d + 1);
    r.s = l - 1;
    return r;
}
__device__ __forceinline__ unsigned udiv(unsigned n, const UDiv& D) {
    if (D.d <= 1) return n;
    const unsigned t = __umulhi(n, D.m);
    return (t + ((n - t) >> 1)) >> D.s;
}

struct SceneView {           // read-only scene data (HBM, L2-resident)
    const DTri* __restrict__ tris;
    const DMesh* __restrict__ meshes;
    const DInst* __restrict__ insts;
    const DMat* __restrict__ mats;
    const DLight* __restrict__ lights;
    const float4* node_pair;  // BVH child pairs, heap order (written by bvh_build_kernel), see BvhRefs
    const float4* fnode;      // ordered LBVH of the fast kernel (bvh_build_kernel)
    int n_real, ftree;        // its leaf count; 1 if usable (>= 2 leaves, depth <= 31)
    const int* leaf_inst;
    const float4* inst4;      // compact instance records
    int n_leaf, n_inst, n_lights, use_bvh;
    int n_mats, n_tris, n_meshes;   // record counts (LDS shading cache, M_SHADE)
    int ident_all;            // every instance and mesh rotation is the identity (cube worlds)
    float prune_abs;          // distance-pruning slack M0 (< 0: pruning off), see closest_hit
    const TriAx* tri_ax;      // axis-plane triangle records (fast kernel; null unless ident_all)
};

// Parts of a DTri (rt_scene.h): the plane filter's 32-B head and the rest of the test.
struct TriHot { V3 pn, a; float b_x, b_y; };
struct TriRest { V3 b, c; float area, inv_area; };
static_assert(sizeof(TriHot) == 32 && offsetof(DTri, b) == 24 && offsetof(DTri, inv_area) == 52, "DTri layout");

// Wave-uniform read-only records in global memory are read through the
// constant address space so that uniform indices compile to scalar (SMEM) loads.
template <class T> __device__ __forceinline__ T ldc(const T* p, int i) {
    static_assert(sizeof(T) % 4 == 0, "4-byte granular records");
    T r;
    uint32_t* d = reinterpret_cast<uint32_t*>(&r);
#if defined(__HIP_DEVICE_COMPILE__)
    const __attribute__((address_space(4))) uint32_t* s = (const __attribute__((address_space(4))) uint32_t*)(p + i);
#else
    const uint32_t* s = reinterpret_cast<const uint32_t*>(p + i);
#endif
#pragma unroll
    for (int w = 0; w < (int)(sizeof(T) / 4); w++) d[w] = s[w];
    return r;
}

__device__ __forceinline__ TriHot ld_hot(const DTri* T, int t) { return ldc(reinterpret_cast<const TriHot*>(T + t), 0); }
__device__ __forceinline__ TriRest ld_rest(const DTri* T, int t) {
    return ldc(reinterpret_cast<const TriRest*>(reinterpret_cast<const char*>(T + t) + 24), 0);
}

// BVH nodes and instance records as the trace kernel reads them: from LDS (staged
// once per persistent block) or, for scenes too large for LDS, from global memory.
// Nodes are stored by child pair: pair k holds heap nodes 2k (.x lanes) and 2k+1 (.y
// lanes) as three float4 = (mnx, mnx' , mny, mny'), (mnz, mnz', mxx, mxx'),
// (mxy, mxy', mxz, mxz'), so one pair test is three 16-B broadcast reads and packed
// (v_pk_*) slab arithmetic.  Pair 0 = (unused node 0, root).  Degenerate boxes are
// stored as min=+inf, max=-inf.
struct BvhRefs {
    const float4* fnode;    // ordered LBVH records (fast kernel): [4 (n_real - 1)]
    const float4* pair;     // [3n]
    const int* leaf;        // [n]  instance of leaf node n+i (bvh.cu ordering[])
    const float4* inst;     // [n_inst] (px, py, pz, mesh | 0x80000000 if the pose is not identity)
    // shading-side records (materials, lights, triangles, meshes): the scene's arrays, or
    // their LDS copies in M_SHADE kernels (hit normal, lighting and frame transitions read
    // them per lane after every query)
    const DMat* mats;
    const DLight* lights;
    const DTri* tris;
    const DMesh* meshes;
};

// Tuning parameters (build switches; the A/B logs under profiles/ record the values tried).
#ifndef RT_HIST_GROUPS_PER_WAVE
#define RT_HIST_GROUPS_PER_WAVE 12  // longest-first history only at <= this many groups per wave
#endif
#ifndef RT_SMALL_FRAME_GPW
#define RT_SMALL_FRAME_GPW 48       // groups per wave (half grid) below which overlapping frames take a quarter of the CUs
#endif
#ifndef RT_HEAVY_Q_DEFAULT
#define RT_HEAVY_Q_DEFAULT 6        // hist = 2: a group of >= this many wave queries is heavy
#endif
#ifndef RT_HEAVY_STATIC
#define RT_HEAVY_STATIC 1    // frames issued alone: heavy-list tickets assigned statically (trace_kernel)
#endif
#ifndef RT_TPC_WIDE
#define RT_TPC_WIDE 16       // live-list tickets of one-pixel groups (spp >= 64, M_PART): 16 consecutive pixels
#endif
#ifndef RT_LDS_SUM
#define RT_LDS_SUM 1         // spp >= 16 in parked kernels: per-channel in-order sample sums through LDS
#endif
#ifndef RT_TPC
#define RT_TPC 3             // work indices claimed per ticket (trace_kernel's group loop) over all
                             // groups; 3 vs 2: -0.8% world8_stress, -1.3% world8 (profiles/r01/ab_tpc_v33.log)
#endif
#ifndef RT_TPC_LIVE
#define RT_TPC_LIVE 1        // the same over live-group lists (sky pre-pass): ~8x fewer groups per
                             // wave, one per ticket balances them (profiles/r02/sky_live_tpc.log)
#endif
constexpr int TPC = RT_TPC;

// One child box's slab interval [lo, hi] against a ray through its reciprocals (ray_inv):
// fma(m - o, 1/d, -+bias) per face, the bias carrying the zero-direction skip (ray_inv).
__device__ __forceinline__ void slab(const Ray& r, const RayInv& ri, float mnx, float mny, float mnz, float mxx,
                                     float mxy, float mxz, float& lo, float& hi) {
    const float qx0 = fmaf(mnx - r.o.x, ri.ix, -ri.bx), qx1 = fmaf(mxx - r.o.x, ri.ix, ri.bx);
    const float qy0 = fmaf(mny - r.o.y, ri.iy, -ri.by), qy1 = fmaf(mxy - r.o.y, ri.iy, ri.by);
    const float qz0 = fmaf(mnz - r.o.z, ri.iz, -ri.bz), qz1 = fmaf(mxz - r.o.z, ri.iz, ri.bz);
    lo = fmaxf(fmaxf(fminf(qx0, qx1), fminf(qy0, qy1)), fminf(qz0, qz1));
    hi = fminf(fminf(fmaxf(qx0, qx1), fmaxf(qy0, qy1)), fmaxf(qz0, qz1));
}

// BoundingBox::intersects (bounding_box.cu:62-104) for both children of pair k.
// Filtered like box_hit_f (rt_math.h), with the bound taken from the slab results
// themselves: every quotient q' = fl(e * r'), r' = v_rcp_f32(d) (ray_inv), is within
// 4.02u |q'| of the reference's fl(e / d), min and max keep a relative bound (|max a' -
// max a| <= 4.05u max(|a|, |a'|)), so |lo' - lo| <= 8.2u |lo'| and the same for hi; the
// test uses 16u plus an absolute floor.  Zero direction components are skipped through
// the RayInv bias (see ray_inv); rays with a non-finite reciprocal (ri.exact) and
// boxes near a tie take the exact reference test.
// tlo (pruning) is a lower bound of the exact entry distance, -inf if undecided.
__device__ __forceinline__ void pair_hit_at(const float4* rec, const Ray& r, const RayInv& ri, bool active,
                                            bool& h0, bool& h1, float& t0, float& t1) {
    const float4 A = rec[0], B = rec[1], C = rec[2];
    const bool nd0 = A.x <= B.z, nd1 = A.y <= B.w;            // nondegenerate (bounding_box.cu:63-65)
    float lo0, hi0, lo1, hi1;
    slab(r, ri, A.x, A.z, B.x, B.z, C.x, C.z, lo0, hi0);
    slab(r, ri, A.y, A.w, B.y, B.w, C.y, C.w, lo1, hi1);
    // Certain outcomes (the exact reference result known): with el, eh the error margins of
    // lo, hi, c = lo + el and a = hi - eh bound the reference's tmin from above and its tmax
    // from below, so max(c, 1e-5) <= a is certainly a hit; with d = lo - el, b = hi + eh,
    // max(d, 1e-5) > b is certainly a miss (bounding_box.cu:98: tmin > tmax || tmax < 1e-5).
    // For filtered rays lo and hi are finite (ray_inv sends a direction without a nonzero
    // component to the exact test), so the max forms equal the pairs of comparisons.
    // Lanes in between run the exact reference test; one uniform branch for both children.
    const float el0 = fmaf(fabsf(lo0), FILT_BOX, FILT_ABS), el1 = fmaf(fabsf(lo1), FILT_BOX, FILT_ABS);
    const float eh0 = fmaf(fabsf(hi0), FILT_BOX, FILT_ABS), eh1 = fmaf(fabsf(hi1), FILT_BOX, FILT_ABS);
    const float d0 = lo0 - el0, d1 = lo1 - el1;
    const bool fx = active && !ri.exact;
    const bool c0 = fx && nd0 && fmaxf(lo0 + el0, THRESH) <= hi0 - eh0;
    const bool c1 = fx && nd1 && fmaxf(lo1 + el1, THRESH) <= hi1 - eh1;
    const bool m0 = !nd0 || (fx && fmaxf(d0, THRESH) > hi0 + eh0);
    const bool m1 = !nd1 || (fx && fmaxf(d1, THRESH) > hi1 + eh1);
    h0 = c0; h1 = c1;
    t0 = c0 ? d0 : -INFINITY;
    t1 = c1 ? d1 : -INFINITY;
    const bool x0 = active && !m0 && !c0, x1 = active && !m1 && !c1;
    if (__builtin_expect(__ballot(x0 || x1) != 0, 0)) {
        if (x0) h0 = box_hit(v3(A.x, A.z, B.x), v3(B.z, C.x, C.z), r);
        if (x1) h1 = box_hit(v3(A.y, A.w, B.y), v3(B.w, C.y, C.w), r);
    }
}
// 0/1 in an SGPR from a wave mask, opaque to the optimizer (a boolean taken from a ballot is
// otherwise rebuilt through a VGPR: v_cndmask + v_cmp per use)
__device__ __forceinline__ unsigned any_lane(unsigned long long m) {
    unsigned h;
    asm("s_cmp_lg_u64 %1, 0\n\ts_cselect_b32 %0, 1, 0" : "=s"(h) : "s"(m) : "scc");
    return h;
}
// pair_hit_at for the fast traversal step, with each child's result as one float: the entry
// lower bound (lo - el, or -inf after the exact test) for a hit, NaN for a miss.  Every record
// of the ordered tree is a proper finite box (the host leaves a frame with a degenerate or
// non-finite real box to the heap kernels: ordered_tree_shape), so there is no per-child
// degenerate test; a ray that needs the exact test everywhere (ri.exact) enters with NaN
// reciprocals (closest_hit), so both its slab results are NaN and both outcome tests are
// false: it takes the exact test with no filtered-ray mask.  ta/tb carry no activity mask: an
// inactive lane's cut is NaN, so t <= cut is false for it.
__device__ __forceinline__ void pair_hit_tt2(const float4* rec, const Ray& r, const RayInv& ri, bool active,
                                             float& ta, float& tb) {
    const float4 A = rec[0], B = rec[1], C = rec[2];
    float lo0, hi0, lo1, hi1;
    slab(r, ri, A.x, A.z, B.x, B.z, C.x, C.z, lo0, hi0);
    slab(r, ri, A.y, A.w, B.y, B.w, C.y, C.w, lo1, hi1);
    const float el0 = fmaf(fabsf(lo0), FILT_BOX, FILT_ABS), eh0 = fmaf(fabsf(hi0), FILT_BOX, FILT_ABS);
    const float el1 = fmaf(fabsf(lo1), FILT_BOX, FILT_ABS), eh1 = fmaf(fabsf(hi1), FILT_BOX, FILT_ABS);
    const float d0 = lo0 - el0, d1 = lo1 - el1;
    const bool hc0 = fmaxf(lo0 + el0, THRESH) <= hi0 - eh0, hc1 = fmaxf(lo1 + el1, THRESH) <= hi1 - eh1;
    const bool mc0 = fmaxf(d0, THRESH) > hi0 + eh0, mc1 = fmaxf(d1, THRESH) > hi1 + eh1;
    const float QNAN = __builtin_nanf("");
    ta = hc0 ? d0 : QNAN;
    tb = hc1 ? d1 : QNAN;
    const bool k0 = hc0 || mc0, k1 = hc1 || mc1;               // outcome certain
    if (__builtin_expect(any_lane(__ballot(active && !(k0 && k1))), 0)) {
        if (active && !k0) ta = box_hit(v3(A.x, A.z, B.x), v3(B.z, C.x, C.z), r) ? -INFINITY : QNAN;
        if (active && !k1) tb = box_hit(v3(A.y, A.w, B.y), v3(B.w, C.y, C.w), r) ? -INFINITY : QNAN;
    }
}
// pair_hit_tt2 with the lane's activity as its cut ct (active: ct == ct) and the outcome tests
// issued as four v_cmp into SGPR masks, combined on the scalar unit: the compiler's form of
// `__ballot(active && !(k0 && k1))` rebuilt the combined mask through a VGPR (v_cndmask 0/1 +
// v_cmp_ne) before the branch, two VALU and a dependent hand-off per traversal step.
#ifndef RT_ASM_OUTCOME
#define RT_ASM_OUTCOME 1
#endif
__device__ __forceinline__ void pair_hit_tt2c(const float4* rec, const Ray& r, const RayInv& ri, float ct,
                                              float& ta, float& tb) {
#if RT_ASM_OUTCOME
    const float4 A = rec[0], B = rec[1], C = rec[2];
    float lo0, hi0, lo1, hi1;
    slab(r, ri, A.x, A.z, B.x, B.z, C.x, C.z, lo0, hi0);
    slab(r, ri, A.y, A.w, B.y, B.w, C.y, C.w, lo1, hi1);
    const float el0 = fmaf(fabsf(lo0), FILT_BOX, FILT_ABS), eh0 = fmaf(fabsf(hi0), FILT_BOX, FILT_ABS);
    const float el1 = fmaf(fabsf(lo1), FILT_BOX, FILT_ABS), eh1 = fmaf(fabsf(hi1), FILT_BOX, FILT_ABS);
    const float d0 = lo0 - el0, d1 = lo1 - el1;
    // certain hit: a <= b; certain miss: c > e (pair_hit_at)
    const float a0 = fmaxf(lo0 + el0, THRESH), b0 = hi0 - eh0, a1 = fmaxf(lo1 + el1, THRESH), b1 = hi1 - eh1;
    const float c0 = fmaxf(d0, THRESH), e0 = hi0 + eh0, c1 = fmaxf(d1, THRESH), e1 = hi1 + eh1;
    const float QNAN = __builtin_nanf("");
    unsigned long long h0, h1, m0, m1;
    asm("v_cmp_le_f32 %[h0], %[a0], %[b0]\n\t"
        "v_cmp_le_f32 %[h1], %[a1], %[b1]\n\t"
        "v_cmp_gt_f32 %[m0], %[c0], %[e0]\n\t"
        "v_cmp_gt_f32 %[m1], %[c1], %[e1]\n\t"
        "v_cndmask_b32 %[ta], %[nan], %[d0], %[h0]\n\t"
        "v_cndmask_b32 %[tb], %[nan], %[d1], %[h1]\n\t"
        "s_or_b64 %[m0], %[m0], %[h0]\n\t"                  // outcome of child A certain
        "s_or_b64 %[m1], %[m1], %[h1]\n\t"                  // ... of child B
        "s_and_b64 %[m0], %[m0], %[m1]\n\t"
        "v_cmp_o_f32 %[m1], %[ct], %[ct]\n\t"               // active lanes
        "s_andn2_b64 %[m0], %[m1], %[m0]"                   // active, some outcome uncertain
        : [h0] "=&s"(h0), [h1] "=&s"(h1), [m0] "=&s"(m0), [m1] "=&s"(m1), [ta] "=&v"(ta), [tb] "=&v"(tb)
        : [a0] "v"(a0), [b0] "v"(b0), [a1] "v"(a1), [b1] "v"(b1), [c0] "v"(c0), [e0] "v"(e0), [c1] "v"(c1),
          [e1] "v"(e1), [d0] "v"(d0), [d1] "v"(d1), [nan] "v"(QNAN), [ct] "v"(ct));
    if (__builtin_expect(m0 != 0, 0)) {
        const bool active = ct == ct;
        const bool k0 = a0 <= b0 || c0 > e0, k1 = a1 <= b1 || c1 > e1;
        if (active && !k0) ta = box_hit(v3(A.x, A.z, B.x), v3(B.z, C.x, C.z), r) ? -INFINITY : QNAN;
        if (active && !k1) tb = box_hit(v3(A.y, A.w, B.y), v3(B.w, C.y, C.w), r) ? -INFINITY : QNAN;
    }
#else
    pair_hit_tt2(rec, r, ri, ct == ct, ta, tb);
#endif
}
__device__ __forceinline__ void pair_hit(const float4* np, int k, const Ray& r, const RayInv& ri, bool active,
                                         bool& h0, bool& h1, float& t0, float& t1) {
    pair_hit_at(np + 3 * k, r, ri, active, h0, h1, t0, t1);
}

struct Best { float time; int inst, tri; float u, v; };     // closest accepted triangle so far
// Per-lane work counters (rays/nodes/leaves/triangle tests, the reference's units) plus
// wave-level step counts for the profiling experiment (query iterations, child-pair
// steps, leaf visits, triangle-loop iterations -- SIMD work regardless of active lanes).
struct WaveCounters { unsigned long long rays, nodes, leaves, tris, wq, wpair, wleaf, wtri, cyc_q, cyc_leaf, cyc_all, cyc_sample, cyc_post, wbary, lbary, live,
                      cyc_light, cyc_normal, cyc_park;      // PROF: light step, hit normal, parking
                      unsigned long long* pc; };            // PROF: this wave's occupancy counters in LDS

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }   // value known wave-uniform
__device__ __forceinline__ Pose inst_pose(const SceneView& S, const BvhRefs& bv, int ti, int& mesh) {
    const float4 I = bv.inst[ti];
    const int w = __float_as_int(I.w);
    mesh = w & 0x7fffffff;
    if (w < 0) return ldc(S.insts, ti).pose;                  // general pose (precomputed quaternions)
    Pose e;
    e.p = v3(I.x, I.y, I.z); e.identity = 1;
    return e;
}

// Closest hit against one instance: renv::gpu::cast_local (scene.cu:27-40) ->
// Hitable::hit (hitable.cu:29-38) -> Trimesh::hit_local (trimesh.cu:11-19) with a
// wave-uniform instance; times are rescaled here exactly as in the reference
// (later comparisons depend on them); the normal is formed after traversal.
// With identity rotations everywhere (S.ident_all), the direction half of cast_local's
// two pose changes depends on the ray only: it is computed once per query by the same
// operations (qrot_identity, len, the Ray ctor's normalisation), so every leaf sees
// the same bits it would compute itself; only the origin chain is per leaf.
// `inv` (axis-plane triangles, axis_plane_t): fl(1/mrd_a), NaN where |mrd_a| < 1e-5.
struct DirPre { V3 mrd, inv; float scale, dir_len; };
__device__ __forceinline__ float axis_inv(float d) { return fabsf(d) < THRESH ? __builtin_nanf("") : rcp_cr(d); }
template <bool AXIS = false>
__device__ __forceinline__ DirPre dir_pre(V3 d) {
    DirPre p;
    const V3 ld = qrot_identity(d);                          // Entity::vec_to_local, identity pose
    p.dir_len = len(ld);
    const V3 lrd = normalized(ld);                           // Ray ctor (geometry.h:216)
    const V3 md = qrot_identity(lrd);                        // HitHandle::get_local_ray, identity mesh pose
    p.scale = len(md);
    p.mrd = normalized(md);
    if (AXIS) p.inv = v3(axis_inv(p.mrd.x), axis_inv(p.mrd.y), axis_inv(p.mrd.z));
    return p;
}

// Component `a` of a vector (a wave-uniform axis index: the selects fold into branches).
__device__ __forceinline__ float comp(V3 v, int a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; }

// t_lo: lower bound of any acceptable local time (-inf if none): the leaf box's entry
// distance minus the pruning slack M (closest_hit).  A triangle whose plane crossing is
// certainly below it lies outside the box, so its inside test is skipped.
// AXIS: the axis-plane triangle path (S.tri_ax, pre.inv set; identity rotations only).
template <bool STATS, bool AXIS = false, bool PROF = false>
__device__ __forceinline__ bool cast_local(const SceneView& S, const BvhRefs& bv, int ti, const Ray& r, Best& b,
                                           const DirPre& pre, WaveCounters& wc, float t_lo) {
    int mesh_id;
    const Pose ip = inst_pose(S, bv, ti, mesh_id);
    mesh_id = uni(mesh_id);
    const DMesh mesh = ldc(S.meshes, mesh_id);
    float dir_len, scale;
    Ray mr;
    if (S.ident_all) {
        dir_len = pre.dir_len; scale = pre.scale;
        mr.o = qrot_identity(qrot_identity(r.o - ip.p) - mesh.pose.p);
        mr.d = pre.mrd;
    } else {
        V3 ld = vec_to_local(ip, r.d);
        dir_len = len(ld);
        Ray lr = make_ray(point_to_local(ip, r.o), ld);
        V3 md = vec_to_local(mesh.pose, lr.d);               // HitHandle::get_local_ray
        scale = len(md);
        mr = make_ray(point_to_local(mesh.pose, lr.o), md);
    }
    int best = -1;
    float bu = 0.0f, bv_ = 0.0f, t_best = b.time;
    if (AXIS) {
        // Axis-plane path (fast kernel, identity rotations): exact plane time from the
        // per-query reciprocal (axis_plane_t), then the exact in-plane reject (TriAx);
        // general triangles take the filtered test below.  Same decisions, same order.
        const float lo = fmaxf(THRESH, t_lo);
        for (int t = mesh.tri_begin; t < mesh.tri_begin + mesh.tri_count; t++) {
            const TriAx x = ldc(S.tri_ax, t);
            const int ax = x.code & 3;
            float time, u, v;
            if (PROF) wc.wtri++;
            if (ax == 3) {                                    // general triangle
                const TriHot h = ld_hot(S.tris, t);
                float denom, num;
                const bool pass = tri_plane_f(h.a, h.pn, mr, t_best, t_lo, denom, num);
                if (!__ballot(pass)) continue;
                const TriRest q = ld_rest(S.tris, t);
                if (pass && tri_inside_f(h.a, q.b, q.c, q.area, q.inv_area, mr, t_best, denom, num, time, u, v)) {
                    t_best = time; best = t; bu = u; bv_ = v;
                }
                continue;
            }
            const int au = ax == 2 ? 0 : ax + 1, av = ax == 0 ? 2 : ax - 1;
            const float tt = axis_plane_t(x.a_ax, comp(mr.o, ax), comp(pre.inv, ax));
            bool pass = tt >= lo && tt < t_best;
            if (!__ballot(pass)) {
                if (x.code & 4) t++;                          // same plane, same t, same best: rejected too
                continue;
            }
            if (x.code & 8) {                                 // in-plane reject (TriAx)
                const float pu = comp(mr.o, au) + tt * comp(mr.d, au), pv = comp(mr.o, av) + tt * comp(mr.d, av);
                const float pa = comp(mr.o, ax) + tt * comp(mr.d, ax);
                const float e = fmaxf(fmaxf(x.ulo - pu, pu - x.uhi), fmaxf(x.vlo - pv, pv - x.vhi));
                pass = pass && !(e > 0.0f && e <= x.win && fabsf(pa - x.a_ax) <= x.off);
                if (!__ballot(pass)) continue;
            }
            if (PROF) { wc.wbary++; wc.lbary += __popcll(__ballot(pass)); }
            const TriHot h = ld_hot(S.tris, t);
            const TriRest q = ld_rest(S.tris, t);
            if (pass && tri_inside_t(h.a, q.b, q.c, q.area, q.inv_area, mr, tt, time, u, v)) {
                t_best = time; best = t; bu = u; bv_ = v;
            }
        }
    } else
    // The plane filter needs only the 32-B head (pn, a) of each record (one batch of
    // scalar loads); the rest is read only for triangles that pass it.
    for (int t = mesh.tri_begin; t < mesh.tri_begin + mesh.tri_count; t++) {
        const TriHot h = ld_hot(S.tris, t);
        float denom, num, time, u, v;
        const bool pass = tri_plane_f(h.a, h.pn, mr, t_best, t_lo, denom, num);
        if (STATS) {
            const unsigned long long pm = __ballot(pass);
            wc.wbary += pm != 0;
            wc.lbary += __popcll(pm);
        }
        if (!pass) continue;
        const TriRest q = ld_rest(S.tris, t);
        if (tri_inside_f(h.a, q.b, q.c, q.area, q.inv_area, mr, t_best, denom, num, time, u, v)) {
            t_best = time; best = t; bu = u; bv_ = v;
        }
    }
    if (best < 0) return false;
    b.time = (t_best * scale) * dir_len;                      // fix_isect, then cast_local
    b.inst = ti; b.tri = best; b.u = bu; b.v = bv_;
    return true;
}

// World-space normal of the accepted hit (trimesh.cu:58-65, hitable.cu:20-23, scene.cu:35-37).
__device__ __forceinline__ V3 hit_normal(const SceneView& S, const BvhRefs& bv, const Best& b, int& mat) {
    int mesh_id;
    const Pose ip = inst_pose(S, bv, b.inst, mesh_id);
    const Pose mp = bv.meshes[mesh_id].pose;
    const DTri& T = bv.tris[b.tri];
    mat = T.mat;
    float b0 = 1.0f - b.u - b.v;
    V3 n = normalized((b0 * T.n0 + b.u * T.n1) + b.v * T.n2);
    n = normalized(vec_from_local(mp, n));
    return vec_from_local(ip, n);
}

// Zero direction components (box bound, see closest_hit).  The reference's slab test
// skips an axis with d_a == 0 (bounding_box.cu:62-104), so such a ray "hits" every
// box its other coordinates cross, whatever o_a: the shadow rays of the directional
// light (0, -1, 1) and the primary rays of the centre column/row sweep whole rows
// of leaves.  Along the ray the coordinate stays o_a exactly (world and local:
// d_a and the local direction's component are 0), so an accepted hit lies within
// the slack of the leaf box on that axis: a node whose a-range excludes o_a by more
// than prune_abs has no acceptable hit below it (node boxes contain their leaves').
// The slab then becomes [K (mn - o - M), K (mx - o + M)] through the same fma and
// bias as a nonzero axis (pair_hit_at): both ends > 0 or < 0 exactly when o_a is
// outside [mn - M, mx + M] (a certain miss), else lo_a <= 0 < 1e-5 <= hi_a never
// binds (every nonzero axis bounds t by ~1e3; lo <= 0 is below any acceptable
// time, so entry bounds stay valid).  closest_hit's `im` keeps the nonzero axes only.
// Fast (ordered-LBVH) kernels only.
__device__ __forceinline__ void zero_axis_cut(const SceneView& S, const Ray& r, RayInv& ri) {
    if (!(S.prune_abs >= 0.0f)) return;
    constexpr float K = 0x1p32f;
    if (r.d.x == 0.0f) { ri.ix = K; ri.bx = K * S.prune_abs; }
    if (r.d.y == 0.0f) { ri.iy = K; ri.by = K * S.prune_abs; }
    if (r.d.z == 0.0f) { ri.iz = K; ri.bz = K * S.prune_abs; }
}

// First step of the fast traversal for a ray (closest_hit, FT path, node 0 with an empty
// closest hit): whether it hits either child of the ordered LBVH's root.  A lane for which
// this is false visits nothing, and its query returns no hit.
__device__ __forceinline__ bool ft_root_hit(const SceneView& S, const BvhRefs& bv, bool active, const Ray& r) {
    RayInv ri = ray_inv(r);
    zero_axis_cut(S, r, ri);
    bool h0, h1;
    float t0, t1;
    pair_hit_at(bv.fnode, r, ri, active, h0, h1, t0, t1);     // the root record
    return h0 || h1;
}

// renv::gpu::cast_ray (scene.cu:42-73) for the whole wave.  Packet traversal of
// the reference's implicit heap: at an internal node hit by some lane, both
// children (2k, 2k+1: adjacent records) are tested; the wave descends into 2k
// first and keeps 2k+1 pending in a per-depth bit trail (wave-uniform, SGPR).
// Each lane processes exactly the leaves its own ray hits, in the reference's
// DFS order, so results equal the single-ray semantics; counters are the
// single-ray node tests (1 + 2 per internal node hit).
// `occl_t` >= 0 enables the occlusion early exit (shadow rays, all-opaque scenes): a
// lane stops once it has accepted a hit with time <= occl_t = max_t * (1 - 8u).
// The reference's closest hit is then also <= max_t and opaque (every later accept
// is < that time up to the instance/mesh rescaling, |scale - 1| <= 4u), so
// Light::attenuate returns 0 either way (light.cu:39-45).  Counters then count
// the work done, so it is only used when statistics are not requested.
//
// Box bound on acceptable times (S.prune_abs >= 0).  Claim: a triangle of a leaf can
// only be accepted at a local time t >= tmin(box) - M(t).  The accepted point lies
// within eps of its triangle (the barycentric-sum tolerance 1e-5 of geometry.h:
// 281-286 allows ~1e-5 x triangle size in its plane), the triangle lies in the leaf
// box when every pose is a pure translation and mesh offsets are zero (the host
// checks; the boxes ignore the mesh pose, raytracer.cu:54-89), and the local ray
// differs from the world ray by O(u (|coords| + t)).  So the world ray is within
// eps + delta of the box at time t, i.e. inside the box grown by that distance,
// whose slab entry is >= tmin - (eps + delta) * max_a |1/d_a| (a zero component is
// no constraint, a subnormal one gives an infinite bound).  The slack used is
// M(t) = (prune_abs + 2^-14 |t|) * im + 2^-14 |t|, im = max_a |1/d_a|, prune_abs =
// 4e-4 x max vertex coordinate + 2^-14 x scene radius: >= 20x the tolerance terms.
// Uses (both exact):
//  * distance pruning (frames without statistics): a lane skips a subtree whose box
//    entry bound tlo exceeds c + M(c), c = min(b.time, lim).  Its leaves would be
//    processed with b.time <= c and nothing in them can be accepted (a nested box is
//    entered no earlier).  `lim` = max_t for shadow segments: hits beyond it never
//    change Light::attenuate (light.cu:35-58).
//  * triangle skip (cast_local's t_lo): a triangle whose plane crossing is certainly
//    before tlo(leaf) - M cannot be accepted, so its inside test is not run.
template <bool NOLEAF, bool STATS, bool FT = false, bool AXIS = false, bool PROF = false, bool BRUTE = false>
__device__ __forceinline__ bool closest_hit(const SceneView& S, const BvhRefs& bv, bool active_in, const Ray& r,
                                            Best& b, WaveCounters& wc, float occl_t = -1.0f,
                                            float lim = INFINITY) {
    const bool prune = !STATS && S.prune_abs >= 0.0f;
    float im = 0.0f;                                           // max_a |1/d_a| (set below)
    auto slack = [&](float t) { return (S.prune_abs + 0x1p-14f * fabsf(t)) * im + 0x1p-14f * fabsf(t); };
    auto cut = [&]() {
        const float c = fminf(b.time, lim);
        return c + slack(c);
    };
    bool active = active_in;
    const unsigned long long am = __ballot(active);
    if (STATS || PROF) { wc.rays += __popcll(am); wc.wq++; }
    bool hit = false;
    if (BRUTE) {
        // Brute-force kernels (M_BRUTE; the reference's -r, scene.cu:48-52): every instance in
        // ascending order, strict < on time, with no tree code compiled in (the traversal's
        // registers and its second copy of the leaf code made config 2's kernel spill).  The
        // triangles take the axis-plane path (AXIS: identity rotations) with no entry bound;
        // a lane that found an occluding hit (occl_t, all-opaque scenes) stops.
        DirPre pre{};
        if (AXIS) pre = dir_pre<true>(r.d);
        else if (S.ident_all) pre = dir_pre(r.d);
        bool live = active;
        for (int i = 0; i < S.n_inst; i++) {
            if (!__ballot(live)) break;
            if (live && cast_local<false, AXIS, PROF>(S, bv, i, r, b, pre, wc, -INFINITY)) {
                hit = true;
                if (b.time <= occl_t) live = false;
            }
        }
        return hit;
    }
    if (!FT && (!S.use_bvh || S.n_leaf == 0)) {               // brute force (scene.cu:48-52)
        DirPre pre{};
        if (S.ident_all) pre = dir_pre(r.d);
        for (int i = 0; i < S.n_inst; i++) {
            if (STATS) {
                wc.leaves += __popcll(am);
                wc.tris += (unsigned long long)__popcll(am) * ldc(S.meshes, uni(__float_as_int(bv.inst[i].w) & 0x7fffffff)).tri_count;
            }
            if (active && cast_local<STATS>(S, bv, i, r, b, pre, wc, -INFINITY)) hit = true;
        }
        return hit;
    }
    const int n = S.n_leaf;
    RayInv ri = ray_inv(r);
    im = ri.exact ? INFINITY : fmaxf(fabsf(ri.ix), fmaxf(fabsf(ri.iy), fabsf(ri.iz)));
    if (FT) zero_axis_cut(S, r, ri);
    if (FT) {
        // Ordered LBVH (fast kernel, S.ftree): same leaves and leaf order as the heap, so
        // each lane meets exactly the leaves its ray hits, in the heap's DFS order (a
        // hit leaf's ancestors contain it and are hit: the slab test is monotone in the
        // box).  Wave-uniform stack of pending B children in lanes 0..31 of one VGPR
        // (tree depth <= 31 is checked on the host): an internal node as its index, a
        // leaf B as -2 - parent, whose pair test is re-run when it is popped (fresh hit
        // and entry bound under the current cut).  Pruning and triangle skip as above.
        // The per-query direction chain (dir_pre) is formed at the wave's first leaf visit:
        // most queries (sky rays) reach no leaf, and it depends on the ray only.
        DirPre pre{};
        bool pre_ok = false;                                   // wave-uniform
        const bool box_bound = S.prune_abs >= 0.0f;
        auto t_low = [&](float tl) { return box_bound ? tl - slack(tl) : -INFINITY; };
        // One pair-test site and one leaf site (the leaf code is the bulk of the kernel):
        // an iteration tests a node's pair -- or, for a popped pending leaf B, re-tests its
        // parent's pair for child B only -- then runs at most one leaf; when both children
        // are leaves, B waits in registers (h2, t2, inst2) for the next iteration.
        // Per-lane state as floats, not booleans (a boolean live across the loop's blocks
        // costs scalar mask updates on every edge): a child's test result is its entry bound
        // t, or NaN for a miss; the lane's cut ct (the pruning bound, +inf without pruning)
        // is NaN once the lane is inactive (no query, or occluded), so "hit and not pruned"
        // is the one comparison t <= ct, false for every NaN.  The cut changes only when a
        // leaf improves the closest hit: recomputed after each leaf visit, not every step.
        const float QNAN = __builtin_nanf("");
        float ct = !active_in ? QNAN : prune ? cut() : INFINITY;
        // Compact step (same visits, same order), one loop latch: a step either descends into
        // A (B pushed when hit) or runs up to two leaves at the single leaf site (A then B) and
        // continues at an internal B or pops.  A popped "leaf B of node X" re-runs X's pair test
        // and goes straight to the leaf site.  A leaf A before an internal B no longer pushes B
        // (the stack holds no more than before).  Pushes are v_writelane into the stack VGPR.
        // Same-box A/B (profiles/r02/ab_trav2.log): frame 0.833 -> 0.810 ms, trace 0.973 -> 0.952.
        if (ri.exact) ri.ix = ri.iy = ri.iz = QNAN;           // every box: the exact test (pair_hit_tt2)
        int node = 0, sp = 0, stk = 0, bonly = 0;
        auto push = [&](int e) { asm("v_writelane_b32 %0, %1, m0" : "+v"(stk) : "s"(e), "{m0}"(sp)); sp++; };
        for (;;) {
            const float4* rec = bv.fnode + 4 * node;
            if (PROF) wc.wpair++;
            const float2 rf = *reinterpret_cast<const float2*>(rec + 3);
            const int ra = uni(__float_as_int(rf.x)), rb = uni(__float_as_int(rf.y));
            float ta, tb;
            pair_hit_tt2c(rec, r, ri, ct, ta, tb);
            float lt = QNAN, t2 = QNAN;                        // leaf entry bounds (NaN: missed)
            int linst = -1, inst2 = -1, next = -1;             // their instances, the next node (uniform; -1: pop)
            if (bonly) {                                       // popped: leaf B of this node
                bonly = 0;
                lt = tb; linst = -1 - rb;
            } else {
                const unsigned hA = any_lane(__ballot(ta <= ct)), hB = any_lane(__ballot(tb <= ct));
                if (ra >= 0 && hA) {                           // descend into A, B after A's subtree
                    next = ra;
                    if (hB) push(rb >= 0 ? rb : -2 - node);
                } else {
                    if (hA) { lt = ta; linst = -1 - ra; }      // leaf A (ra < 0 here)
                    if (hB) {
                        if (rb >= 0) next = rb;                // after leaf A, if any
                        else if (linst >= 0) { t2 = tb; inst2 = -1 - rb; }
                        else { lt = tb; linst = -1 - rb; }
                    }
                }
            }
            if (linst >= 0) {
                for (;;) {                                     // the leaf site: one or two leaves
                    const bool lh = lt <= ct;                  // (ct only decreases: fresh for the second leaf)
                    if (__ballot(lh)) {
                        if (!pre_ok) {
                            if (AXIS) pre = dir_pre<true>(r.d);    // S.tri_ax set: identity rotations
                            else if (S.ident_all) pre = dir_pre(r.d);
                            pre_ok = true;
                        }
                        const unsigned long long cl0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
                        if (PROF) { wc.wleaf++; wc.leaves += __popcll(__ballot(lh)); }
                        if (lh && cast_local<false, AXIS, PROF>(S, bv, linst, r, b, pre, wc, t_low(lt)))
                            if (b.time <= occl_t) ct = QNAN;   // occluded: this lane is done
                        if (prune && ct == ct) ct = cut();
                        if (PROF) wc.cyc_leaf += __builtin_amdgcn_s_memtime() - cl0;
                        if (!__ballot(ct == ct)) { next = -1; sp = 0; break; }   // every lane occluded: done
                    }
                    if (inst2 < 0) break;
                    lt = t2; linst = inst2; inst2 = -1;
                }
            }
            if (next >= 0) { node = next; continue; }
            if (sp == 0) break;
            sp--;                                              // an internal node, or leaf B of node -2 - e
            const int e = __builtin_amdgcn_readlane(stk, sp);
            if (e < 0) { node = -2 - e; bonly = 1; }
            else node = e;
        }
        return active_in && b.time < INFINITY;                 // an accepted triangle has a finite time
    }
    if (STATS) wc.nodes += __popcll(am);                       // root test
    bool hr, hdummy;
    float tdummy, troot;
    pair_hit(bv.pair, 0, r, ri, active, hdummy, hr, tdummy, troot);   // pair 0 = (unused, root)
    const unsigned long long br = __ballot(hr);
    if (!br) return false;
    DirPre pre{};
    if (S.ident_all) pre = dir_pre(r.d);
    // lower bound of acceptable local times in a leaf entered at >= tl (see distance pruning)
    const bool box_bound = !STATS && S.prune_abs >= 0.0f;   // counted kernel: plain reference path
    auto t_low = [&](float tl) { return box_bound ? tl - slack(tl) : -INFINITY; };
    auto leaf = [&](bool h, int li, float tl) {
        const unsigned long long m = __ballot(h);
        if (!m) return;
        const int ti = uni(bv.leaf[li]);                       // leaf instance: wave-uniform
        if (STATS) {
            const int tc = ldc(S.meshes, uni(__float_as_int(bv.inst[ti].w) & 0x7fffffff)).tri_count;
            wc.leaves += __popcll(m);
            wc.tris += (unsigned long long)__popcll(m) * tc;
            wc.wleaf++;
            wc.wtri += tc;
        }
        const unsigned long long c0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
        if (NOLEAF) { if (h) { hit = true; b.inst = ti; } }
        else if (h && cast_local<STATS>(S, bv, ti, r, b, pre, wc, t_low(tl))) {
            hit = true;
            if (b.time <= occl_t) active = false;             // occluded: this lane is done
        }
        if (STATS) wc.cyc_leaf += __builtin_amdgcn_s_memtime() - c0;
    };
    if (n == 1) { leaf(hr, 0, troot); return hit; }
    // one copy of the leaf code for both children (keeps the kernel small)
    if (STATS) wc.nodes += 2ull * __popcll(br);
    int k = 1;
    unsigned pending = 0;
    for (;;) {
        const int c0 = 2 * k;
        bool h0, h1;
        float t0, t1;
        pair_hit(bv.pair, k, r, ri, active, h0, h1, t0, t1);  // children 2k, 2k+1
        if (prune) {
            const float ct = cut();
            h0 = h0 && !(t0 > ct);
            h1 = h1 && !(t1 > ct);
        }
        if (STATS) wc.wpair++;
        if (c0 >= n) {                                         // children are leaves: DFS order 2k, 2k+1
#pragma nounroll
            for (int c = 0; c < 2; c++) leaf(c == 0 ? h0 : (h1 && !(prune && t1 > cut())), c0 + c - n, c == 0 ? t0 : t1);
            if (!__ballot(active)) break;                      // every lane occluded
        } else {
            const unsigned long long b0 = __ballot(h0), b1 = __ballot(h1);
            if (STATS) wc.nodes += 2ull * (__popcll(b0) + __popcll(b1));
            if (b0) {
                if (b1) pending |= 1u << (31 - __clz(c0));
                k = c0;
                continue;
            }
            if (b1) { k = c0 + 1; continue; }
        }
        if (!pending) break;
        const int d = 31 - __clz(pending);                     // deepest pending right sibling
        pending &= ~(1u << d);
        k = (k >> ((31 - __clz(k)) - d)) + 1;
    }
    return hit;
}

// ---------------------------------------------------------------------------
// Shading: phong.cu:14-53, light.cu:11-77, scene.cu:14-22
// ---------------------------------------------------------------------------
// kd: the material's Kd (the reference), or the atlas texel in the textured mode
// diffuse + specular: phong's factor of the incoming light
// tl_len = len(to_light), tl_neg_unit = normalized(neg(to_light)) (the shadow ray's direction
// negated: the light step has them)
__device__ __forceinline__ V4 phong_factor(const DMat& m, V4 kd, V3 nrm, V3 nrm_unit, V3 ray_dir, V3 to_light,
                                           float tl_len, V3 tl_neg_unit) {
    float nd = max_std(dot(to_light, nrm), 0.0f);
    V4 diffuse = nd * kd;
    V3 reflected = reflect_pre(tl_len, tl_neg_unit, nrm_unit);         // reflect(neg(to_light), nrm)
    float rd = dot(neg(reflected), ray_dir);
    V4 specular = pow_fast(max_std(rd, 0.0f), m.alpha) * m.Ks;
    return diffuse + specular;
}
// phong(m, kd, nrm, incoming, ...) = phong_factor(m, kd, nrm, normalized(nrm), ...) * incoming (trace_sample's
// light step)

// RayFrame (scene.cu:81-90).  The top frame's hit point and normal are not kept in
// registers: while the frame is being lit they equal at(ray, is_time) and is_norm
// (the reference assigns them from exactly those, scene.cu:117-120), and a frame
// resumed from the stack reads them from its saved copy.
struct Frame {
    Ray ray;
    V4 atten;
    int last_mat, type, depth, in_obj;
};
struct SavedFrame { Frame f; V3 hit_pt, norm; };   // suspended under its reflection child

struct TraceParams {
    DCamera cam;
    V3 dist_atten;
    V4 ambience;
    int W, H, row0, row_step, n_rows, compact, spp, depth;
    float spp_recip;          // 2^-k when spp = 2^k (exact reciprocal), else 0
    int lanes_per_px, px_per_wave, gw, gh, n_gx, n_groups;   // sample-parallel lane mapping
    int l_shift, gw_shift;    // log2(lanes_per_px), log2(gw) when powers of two, else -1
    UDiv div_ngx, div_perq;   // g / n_gx and ticket permutation mod per-queue length
    int scramble;             // ticket -> group permutation factor (coprime with the queue length)
    int scramble_small;       // 1: ticket * scramble < 2^32 for every ticket (32-bit modulo)
    const float2* __restrict__ spp_off;
    uint32_t* rgba;
    float4* radiance;
    int* hit_inst;
    int* hit_tri;
    unsigned long long* stats;
    int* work;                // persistent-wave work counters (zeroed before each launch); work[16 NQ]: heavy list
    // Longest-first scheduling history (fast frames only, hist = 1): the previous frame's
    // heavy groups (hl_prev[0, *hc_prev)) run first and are skipped in the normal queues
    // (hf_prev); this frame records its own into the *_next buffers.  hs_* = summed group
    // durations (100 MHz ticks) for the threshold (4x the mean group).
    int hist, heavy_cap;      // heavy_cap: most heavy groups recorded per frame
    // hist = 2 (whole frames with the sky pre-pass): heavy = a group that took >= heavy_q wave
    // queries (counted, no clock); hf_next[g] = 1 records it, and the next frame's sky pre-pass
    // puts the groups flagged in hf_prev on a heavy live list the trace kernel drains first
    int heavy_q;
    const int* hl_prev; int* hl_next;
    const unsigned char* hf_prev; unsigned char* hf_next;
    const unsigned long long* hctl_prev; unsigned long long* hctl_next;   // {count, sum}
    int occl_exit;            // shadow-ray occlusion early exit (all-opaque scene, no statistics)
    const float4* atlas;      // textured mode: atlas texels, byte / 255 (rt_scene_set_atlas)
    int atlas_w, atlas_h;
    int* dbg_log;             // debug_cast event log (NULL in normal frames)
    int dbg_x, dbg_y;
    unsigned* gdur;           // profiling (rt_profile_groups): per-group duration, 100 MHz ticks; NULL normally
    // Sky pre-pass (sky_kernel, fast frames): gsky[g] = 1 when no primary of group g enters
    // the tree's root -- its outputs are written already and the trace kernel skips it.
    // NULL: no pre-pass (the trace kernel runs the same test itself).
    const unsigned char* gsky;
    // Live-group lists (sky_kernel): queue q's groups are live[q * live_cap + i] for i below
    // work[16 (NQ + 1 + q)], in arrival order.  NULL: queue q's groups are q + NQ j.
    const int* live; int live_cap;
    int tpc;                  // work indices per ticket (normal queues)
    int grid_waves;           // waves of this launch (the heavy list's static rounds)
    int heavy_static;         // 1: heavy-list tickets assigned statically (frames issued alone)
    int unlit_skip;           // fast frames: no shadow segments for a light whose phong factor is zero (1),
                              // and no phong term for it either (2)
};

// The launch's TraceParams read in place from the kernel-argument segment (constant address
// space: scalar loads) through a pointer made fresh at each use site.  Passed by value and
// used directly, its ~80 dwords were loaded once and held in SGPRs for the whole persistent
// kernel; the scalar register file overflowed into VGPR lanes, and every group and every
// state-machine step re-read them with v_readlane (VALU issue slots).  Fresh per scope, a
// field is loaded (s_load) where it is needed and its SGPRs are free elsewhere.
typedef __attribute__((address_space(4))) const TraceParams KTP;
// a struct field of the in-place parameters, copied to registers word by word (scalar loads)
template <class T> __device__ __forceinline__ T kld(const __attribute__((address_space(4))) T& x) {
    static_assert(sizeof(T) % 4 == 0, "4-byte granular");
    T r;
    const __attribute__((address_space(4))) uint32_t* src = (const __attribute__((address_space(4))) uint32_t*)&x;
    uint32_t* d = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
    for (int w = 0; w < (int)(sizeof(T) / 4); w++) d[w] = src[w];
    return r;
}
__device__ __forceinline__ KTP& kparams() {
    KTP* p = (KTP*)__builtin_amdgcn_kernarg_segment_ptr();     // the first kernel argument
    asm volatile("" : "+s"(p));
    return *p;
}
// The trace kernel's SceneView (its second argument, right after TraceParams) read the same way:
// a fresh copy per scope (the state loop's iteration, the group) is loaded where it is used
// instead of being held in SGPRs across the persistent loops.  RT_FRESH_SCENE=0: the by-value
// argument throughout (the A/B arm).
#ifndef RT_FRESH_SCENE
#define RT_FRESH_SCENE 1
#endif
typedef __attribute__((address_space(4))) const SceneView KSV;
static_assert(sizeof(TraceParams) % alignof(SceneView) == 0, "SceneView follows TraceParams in the kernarg segment");
__device__ __forceinline__ SceneView kscene() {
    const __attribute__((address_space(4))) char* p =
        (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return kld(*(KSV*)(p + sizeof(TraceParams)));
}
#if RT_FRESH_SCENE
#define SV() kscene()
#else
#define SV() S
#endif

// Textured mode (build-defined; phong.cu:18-23 leaves texture mapping a TODO): the
// diffuse colour of a hit on a triangle with TextureCoords is the atlas texel at
// (tx, ty) + u (ux, uy) + v (vx, vy), clamped to the atlas and truncated to a texel
// index (point sampling, clamp addressing: the reference's texture setup); other hits
// keep the material's Kd.  gfx950 has no image/sampler instructions (HIP marks tex2D
// unavailable there), so the atlas is a plain float4 array in HBM.
template <class PT>
__device__ __forceinline__ V4 hit_kd(const PT& P, const BvhRefs& bv, const Best& b, int mat) {
    const DTri& T = bv.tris[b.tri];
    if (!T.tex) return bv.mats[mat].Kd;
    const float x = (T.tx + b.u * T.ux) + b.v * T.vx;
    const float y = (T.ty + b.u * T.uy) + b.v * T.vy;
    const int ix = (int)fminf(fmaxf(x, 0.0f), (float)(P.atlas_w - 1));
    const int iy = (int)fminf(fmaxf(y, 0.0f), (float)(P.atlas_h - 1));
    const float4 c = P.atlas[(size_t)iy * P.atlas_w + ix];
    return v4(c.x, c.y, c.z, c.w);
}

// Opaque to the optimiser: values derived from x (64-bit output addresses) are formed
// here instead of being hoisted to the group start and spilled across the trace.
__device__ __forceinline__ void opaque(int& x) { asm volatile("" : "+v"(x)); }
// Build-defined sample offset k (rt_scene.cpp spp_offset: R2 sequence in double), computed
// with the same correctly rounded double operations as the host table (no memory access in
// the group loop: a vector load there waits, in order, for the previous group's stores and
// for the work-ticket atomic in flight).
__device__ __forceinline__ float2 spp_offset_dev(int k) {
    const double u = (double)k * 0.7548776662466927, v = (double)k * 0.5698402909980532;
    return make_float2((float)(u - floor(u)), (float)(v - floor(v)));
}

// A wave-uniform value made loop-variant where it is used: per-group constants derived from
// it (camera terms of the kernel arguments) are recomputed there instead of being hoisted out
// of the persistent group loop, held in VGPRs across the trace and spilled (the spill reloads
// were long-latency scratch misses at every group start).
template <class T> __device__ __forceinline__ T fresh_s(T x) { asm volatile("" : "+s"(x)); return x; }
// This lane's index, recomputed where it is used (two VALU) rather than held across the
// persistent loop (it was spilled and reloaded from scratch at every group).
__device__ __forceinline__ int lane_id_fresh() {
    const unsigned m = fresh_s(~0u);
    return (int)__builtin_amdgcn_mbcnt_hi(m, __builtin_amdgcn_mbcnt_lo(m, 0u));
}

// Lane -> (pixel, sample) of pixel group g, from the launch parameters (shifts for powers of
// two).  Recomputed where each term is used (camera ray, hit-id and output stores) rather than
// held in registers across the trace: the output pixel's index held across it was spilled to
// scratch (a store per group and lane; brute-force frames at spp = 1 wrote ~12 B per pixel).
struct GroupLane { int px, py, sub, base, pix; bool valid; };
__device__ __forceinline__ GroupLane group_lane(int g) {
    KTP& P = kparams();
    const int L = P.lanes_per_px;
    const int gy = (int)udiv((unsigned)g, kld(P.div_ngx)), gx = g - gy * P.n_gx;
    const int ln = lane_id_fresh();
    const int pix_g = P.l_shift >= 0 ? ln >> P.l_shift : ln / L;
    const int pxo = P.gw_shift >= 0 ? pix_g & (P.gw - 1) : pix_g % P.gw;
    const int pyo = P.gw_shift >= 0 ? pix_g >> P.gw_shift : pix_g / P.gw;
    GroupLane o;
    o.sub = P.l_shift >= 0 ? ln & (L - 1) : ln - pix_g * L;
    o.base = ln - o.sub;
    o.px = gx * P.gw + pxo;
    const int pr = gy * P.gh + pyo;
    o.valid = pix_g < P.px_per_wave && o.px < P.W && pr < P.n_rows;
    o.py = P.row0 + pr * P.row_step;
    o.pix = P.compact ? pr * P.W + o.px : o.py * P.W + o.px;   // < 2^31 (checked on the host)
    return o;
}



template <class PT>
__device__ __forceinline__ void dbg(const PT& P, bool me, int ev) {
    if (P.dbg_log && me) {
        int i = atomicAdd(P.dbg_log, 1);
        if (i < 4094) P.dbg_log[2 + i] = ev;
    }
}

// Camera::at (camera.cu:33-42), basis hoisted (bitwise identical, computed on the host)
__device__ __forceinline__ Ray camera_at(const DCamera& c, float cx, float cy) {
    float gx = (cx - (0.5f * c.W)) / c.unit;
    float gy = (0.5f * c.H - cy) / c.unit;
    V3 dir = (c.near_ * c.f + gx * c.r) + gy * c.u;
    return make_ray(c.pos, dir);
}

// One camera sample per lane through renv::gpu::propagate_ray (scene.cu:92-188),
// run as an explicit state machine whose only wave-collective step is the
// closest-hit query.  Each piece of the reference's control flow appears once:
//   ST_ADVANCE     REFLECT / REFRACT frame transitions until a NORMAL frame needs a ray
//   ST_WAIT_NORMAL waiting for the frame's closest hit (scene.cu:101-127)
//   ST_LIGHT       illuminate(): set up the shadow ray of light `li` (phong.cu:42-53)
//   ST_WAIT_SHADOW waiting for a shadow segment (Light::attenuate, light.cu:29-61)
// The top frame lives in registers; frames suspended under a reflection child (at
// most `depth`) in the private array `stk`.  rec_ids: this lane carries the pixel's
// sample 0 and records the primary hit ids of its pixel in group g.
enum : int { ST_DONE = 0, ST_ADVANCE = 1, ST_WAIT_NORMAL = 2, ST_LIGHT = 3, ST_WAIT_SHADOW = 4 };

// Parking (PARK): integrator state the traversal never reads is written to this lane's
// LDS column before each query and read back after it, so the query runs with those
// registers free (instead of the allocator spilling to scratch, whose working set is
// larger than L2: measured ~0.9 GB of write-back per frame).  The memory clobbers
// stop the compiler from forwarding the stored values and keeping them live.
// The light's phong factor (phong.cu:14-53 without the incoming light) is formed once, when the
// shadow query is set up, and parked: the light's term after the query is factor x incoming,
// the same operations in the same order as the reference's phong.  NS = 0 kernels run only scenes without a
// refractive material (launch_trace): there a shadow ray's light is never attenuated (rv = the
// light's colour, reloaded after the query), so they park 4 fields fewer.
// Parked kernels also park normalized(hit normal), formed once per hit for phong's reflect
// (every light) and the reflection ray, instead of once per use (same value: frame -1.8%,
// profiles/r04/ab_nn.log).
constexpr int PARK_FIELDS = 29;
__host__ __device__ constexpr int park_fields(int ns) { return ns == 0 ? 25 : PARK_FIELDS; }
// Partial parking (M_PART): scenes whose ordered tree fills most of the LDS (world16: 93 KB)
// park the first PART_FIELDS fields only (the ray, its attenuation and the accumulated
// radiance); the rest stay in registers.  The instance records are then read from global
// memory (L2-resident; as scalar loads they measured +1%) to leave the LDS to the tree.
constexpr int PART_FIELDS = 14;
template <int NS, bool STATS, bool PARK, bool TEX, bool FT, bool AXIS, bool PROF = false, bool BRUTE = false,
          bool PART = false>
__device__ __forceinline__ V4 trace_sample(const SceneView& S, const BvhRefs& bv, bool valid,
                                           Ray r0, bool me, bool rec_ids, int g, WaveCounters& wc, float* park, int& nq) {
    constexpr bool OPQ = NS == 0;                               // no refractive material in the scene
    constexpr bool NN = PARK;                                   // is_nn parked across the queries
    KTP& P0 = kparams();
    Frame cur;
    SavedFrame stk[NS > 0 ? NS : 1];
    int top = -1, st = ST_DONE;
    // bit 0: primary ray not yet answered; bit 1: pop after illumination (depth 0);
    // bit 2: `cur` was resumed from stk[top] (hit point / normal live there);
    // bit 3: this lane records the pixel's primary hit ids (sample 0)
    int fl = rec_ids ? 9 : 1;
    V4 acc = v4(0, 0, 0, 0);
    float is_time = INFINITY;                                   // the sample's shared Isect
    V3 is_norm = v3(0, 0, 0);
    V3 is_nn = v3(0, 0, 0);                                     // normalized(is_norm) (parked kernels)
    int is_mat = 0;
    V4 is_kd = v4(0, 0, 0, 0);                                  // textured mode: the hit's diffuse colour
    int li = 0;
    V4 summed = v4(0, 0, 0, 0), rv = v4(0, 0, 0, 0);
    V4 fct = v4(0, 0, 0, 0);                                    // the light's phong factor
    float da = 1.0f, max_t = 0.0f;
    Ray q = r0;
    if (valid) {
        cur.ray = r0;
        cur.atten = v4(1.0f, 1.0f, 1.0f, 1.0f); cur.last_mat = -1;
        cur.type = F_NORMAL; cur.depth = P0.depth; cur.in_obj = 0;
        top = 0; st = ST_ADVANCE;
    }
    auto pop = [&]() {
        top--;
        if (NS > 0 && top >= 0) { cur = stk[top].f; fl |= 4; }
    };
    unsigned long long c_post = 0;
    for (;;) {
        KTP& P = kparams();
        if ((STATS || PROF) && c_post) { wc.cyc_post += __builtin_amdgcn_s_memtime() - c_post; c_post = 0; }
        // ---- local transitions until this lane waits for a query or is done ----
        while (st == ST_ADVANCE || st == ST_LIGHT) {
            const unsigned long long cl = PROF ? __builtin_amdgcn_s_memtime() : 0;
            if (st == ST_LIGHT) {
                if (li < SV().n_lights) {
                    const DLight L = bv.lights[li];
                    const V3 hpos = at(cur.ray, is_time);          // org_ray.at(isect.time) (phong.cu:48)
                    V3 dtl;
                    if (L.type == 0) {                             // PointLight::shine (light.cu:63-70)
                        V3 disp = L.v - hpos;
                        float dist = len(disp);
                        float quad = P.dist_atten.x + P.dist_atten.y * dist + P.dist_atten.z * dist * dist;
                        da = quad < 1.0f ? 1.0f : 1.0f / quad;
                        dtl = normalized(disp);
                        max_t = dist;
                    } else {                                       // DirLight::shine (light.cu:72-77)
                        dtl = neg(L.v);
                        max_t = INFINITY;
                    }
                    // to = make_ray(hpos, dtl): normalized(dtl) formed here once; phong's
                    // reflect(neg(dtl), n) takes |neg(dtl)| = |dtl| (the same squares) and
                    // normalized(neg(dtl)) = neg(normalized(dtl)) (the same magnitudes, RNE is
                    // sign-symmetric; +0s below THRESH in both)
                    const float tl = len(dtl);
                    const bool tl_ok = tl > THRESH;
                    const float tr = rcp_cr(tl);
                    const Ray to{hpos, tl_ok ? tr * dtl : v3(0.0f, 0.0f, 0.0f)};
                    const V3 tn = tl_ok ? tr * neg(dtl) : v3(0.0f, 0.0f, 0.0f);
                    rv = L.col;                                    // Light::attenuate (light.cu:30-31)
                    // Unlit skip: when phong's factor (diffuse + specular) is zero in every
                    // channel -- the light behind the surface, no specular lobe -- the light's
                    // term (factor x incoming) is that signed zero for every incoming light
                    // >= +0, which the host guarantees (unlit_skip: light colours >= +0 and
                    // finite, transmission Kt in [+0, 1], so every attenuation is >= +0 and
                    // finite).  The shadow segments cannot change the sum: none is traced.
                    // The lane still takes the wait-for-shadow step, with no query (max_t = -inf
                    // marks it): no hit, so the light's term is phong's with the unshadowed
                    // light, the same signed zeros.
                    const DMat& mm = bv.mats[is_mat];
                    fct = phong_factor(mm, TEX ? is_kd : mm.Kd, is_norm, NN ? is_nn : normalized(is_norm), cur.ray.d,
                                       dtl, tl, tn);
                    if (P.unlit_skip && fct.x == 0.0f && fct.y == 0.0f && fct.z == 0.0f && fct.w == 0.0f)
                        max_t = -INFINITY;
                    q = make_ray(at(to, THRESH), to.d);
                    dbg(P, me, 4);
                    st = ST_WAIT_SHADOW;
                } else {
                    acc = acc + cur.atten * summed;                 // scene.cu:127
                    if (fl & 2) { fl &= ~2; pop(); }
                    st = top < 0 ? ST_DONE : ST_ADVANCE;
                }
                if (PROF) wc.cyc_light += __builtin_amdgcn_s_memtime() - cl;
                continue;
            }
            // ST_ADVANCE
            if (cur.type == F_NORMAL) {                            // scene.cu:100-103
                is_time = INFINITY;
                dbg(P, me, 1);
                q = cur.ray;
                st = ST_WAIT_NORMAL;
                continue;
            }
            const DMat& m = bv.mats[is_mat];
            bool do_pop = false;
            if (cur.type == F_REFLECT) {                           // scene.cu:129-148 (frame's own hit)
                cur.type = F_REFRACT;
                if (m.reflective) {
                    dbg(P, me, 2);
                    const V3 hp = at(cur.ray, is_time);
                    // NS = 0 with depth > 0: the host picks it only when no material is refractive.
                    // The suspended frame would then only be popped when resumed (its REFRACT step
                    // pops: the material of the shared Isect is never refractive, scene.cu:149-184),
                    // and so would every frame under it, so the child replaces it (a tail call):
                    // no stack, no scratch writes.
                    if (NS > 0) {
                        stk[top].f = cur; stk[top].hit_pt = hp; stk[top].norm = is_norm;
                        top++;
                    }
                    cur.type = F_NORMAL;                           // the child: last_mat, in_obj inherited
                    cur.atten = cur.atten * m.Kr;
                    cur.depth = cur.depth - 1;
                    cur.ray = make_ray(hp, reflect(cur.ray.d, NN ? is_nn : normalized(is_norm)));
                }
            } else if (!OPQ && m.refractive) {                    // F_REFRACT (scene.cu:149-184)
                dbg(P, me, 3);
                cur.type = F_NORMAL;
                float n1, n2;
                if (cur.in_obj) { n1 = bv.mats[cur.last_mat].eta; n2 = 1.0f; }
                else { n1 = 1.0f; n2 = bv.mats[cur.last_mat].eta; }
                V3 hp, nn;
                if (fl & 4) { hp = stk[top].hit_pt; nn = stk[top].norm; }
                else { hp = at(cur.ray, is_time); nn = is_norm; }
                bool tir;
                V3 rd = refract(cur.ray.d, normalized(nn), n1, n2, tir);
                if (tir) do_pop = true;
                else { cur.ray = make_ray(hp, rd); cur.in_obj = !cur.in_obj; cur.depth--; }
            } else {
                do_pop = true;
            }
            if (do_pop) { pop(); if (top < 0) st = ST_DONE; }
        }
        // ---- the wave-collective closest-hit query ----
        const bool need = (st == ST_WAIT_NORMAL || st == ST_WAIT_SHADOW);
        if (!__ballot(need)) break;
        nq++;                                                  // a wave query (uniform)
        Best b;
        b.time = INFINITY; b.inst = -1; b.tri = -1; b.u = 0.0f; b.v = 0.0f;
        float occl = -1.0f;
        if (P.occl_exit && st == ST_WAIT_SHADOW) occl = max_t * (1.0f - 0x1p-21f);
        const float lim = st == ST_WAIT_SHADOW ? max_t : INFINITY;
        const unsigned long long cpk0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
        if (PARK) {
            float* pk = park;
            int f = 0;
            auto put = [&](float v) { if (!PART || f < PART_FIELDS) pk[f * TRACE_BLOCK_P] = v; f++; };
            put(cur.ray.o.x); put(cur.ray.o.y); put(cur.ray.o.z); put(cur.ray.d.x); put(cur.ray.d.y); put(cur.ray.d.z);
            put(cur.atten.x); put(cur.atten.y); put(cur.atten.z); put(cur.atten.w);
            put(acc.x); put(acc.y); put(acc.z); put(acc.w);
            put(summed.x); put(summed.y); put(summed.z); put(summed.w);
            put(fct.x); put(fct.y); put(fct.z); put(fct.w);
            if (NN) { put(is_nn.x); put(is_nn.y); put(is_nn.z); }
            if (!OPQ) { put(rv.x); put(rv.y); put(rv.z); put(rv.w); }
            asm volatile("" ::: "memory");
        }
        const unsigned long long c0 = (STATS || PROF) ? __builtin_amdgcn_s_memtime() : 0;
        if (PROF) wc.cyc_park += c0 - cpk0;
        // (an unlit-skipped shadow step, max_t = -inf, takes no query)
        const bool qa = st == ST_WAIT_NORMAL || (st == ST_WAIT_SHADOW && max_t >= 0.0f);
        const unsigned long long prof_p0 = wc.wpair, prof_l0 = wc.wleaf;
        const bool hit = closest_hit<false, STATS, FT, AXIS, PROF, BRUTE>(SV(), bv, qa, q, b, wc, occl, lim);
        if (PROF && P.stats) {                                 // query occupancy (rt_frame_work)
            const unsigned long long mp = __ballot(st == ST_WAIT_NORMAL && (fl & 1));
            const unsigned long long mn = __ballot(st == ST_WAIT_NORMAL);
            const unsigned long long ms = __ballot(st == ST_WAIT_SHADOW && qa);
            const unsigned long long mu = __ballot(st == ST_WAIT_SHADOW && !qa);
            const int na = __popcll(mn | ms);
            if (lane_id_fresh() == 0) {
                unsigned long long* pc = wc.pc - PROF_LANES_PRIMARY;     // index by the d_stats slot
                pc[PROF_LANES_PRIMARY] += (unsigned long long)__popcll(mp);
                pc[PROF_LANES_SECONDARY] += (unsigned long long)__popcll(mn & ~mp);
                pc[PROF_LANES_SHADOW] += (unsigned long long)__popcll(ms);
                pc[PROF_LANES_UNLIT] += (unsigned long long)__popcll(mu);
                if (wc.live && na > 0) {
                    const int bk = (na - 1) >> 3;
                    pc[PROF_LIVE_WQ] += 1ull;
                    pc[PROF_LIVE_LANES] += (unsigned long long)na;
                    pc[PROF_HIST_WQ + bk] += 1ull;
                    pc[PROF_HIST_PAIR + bk] += wc.wpair - prof_p0;
                    pc[PROF_HIST_LEAF + bk] += wc.wleaf - prof_l0;
                }
            }
        }
        const unsigned long long cq1 = PROF ? __builtin_amdgcn_s_memtime() : 0;
        if (PARK) {
            asm volatile("" ::: "memory");
            const float* pk = park;
            int f = 0;
            auto get = [&](float& x) { if (!PART || f < PART_FIELDS) x = pk[f * TRACE_BLOCK_P]; f++; };
            get(cur.ray.o.x); get(cur.ray.o.y); get(cur.ray.o.z);
            get(cur.ray.d.x); get(cur.ray.d.y); get(cur.ray.d.z);
            get(cur.atten.x); get(cur.atten.y); get(cur.atten.z); get(cur.atten.w);
            get(acc.x); get(acc.y); get(acc.z); get(acc.w);
            get(summed.x); get(summed.y); get(summed.z); get(summed.w);
            get(fct.x); get(fct.y); get(fct.z); get(fct.w);
            if (NN) { get(is_nn.x); get(is_nn.y); get(is_nn.z); }
            if (!OPQ) { get(rv.x); get(rv.y); get(rv.z); get(rv.w); }
            if (PROF) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); wc.cyc_park += __builtin_amdgcn_s_memtime() - cq1; }
        }
        unsigned long long c1 = 0;
        if (STATS || PROF) { c1 = __builtin_amdgcn_s_memtime(); wc.cyc_q += c1 - c0; c_post = c1; }
        if (!need) continue;
        int hmat = 0;
        V3 hn = v3(0, 0, 0);
        // (opaque scenes: a shadow segment needs neither the normal nor the material -- any hit
        // before the light is opaque, light.cu:44-46)
        const unsigned long long cn0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
        if (hit && (!OPQ || st == ST_WAIT_NORMAL)) hn = hit_normal(SV(), bv, b, hmat);
        if (PROF) wc.cyc_normal += __builtin_amdgcn_s_memtime() - cn0;
        if (st == ST_WAIT_NORMAL) {
            if (fl & 1) {
                fl &= ~1;
                if (fl & 8) {                                  // the pixel of group g, recomputed here
                    const int op = group_lane(g).pix;
                    if (P.hit_inst) P.hit_inst[op] = hit ? b.inst : -1;
                    if (P.hit_tri) P.hit_tri[op] = hit ? b.tri : -1;
                }
            }
            if (!hit) {                                            // scene.cu:124-126
                is_time = INFINITY;
                pop();
                st = top >= 0 ? ST_ADVANCE : ST_DONE;
                continue;
            }
            is_time = b.time; is_norm = hn; is_mat = hmat;
            if (NN) is_nn = normalized(hn);
            if (TEX) is_kd = hit_kd(P, bv, b, hmat);
            fl &= ~4;                                              // hit point / normal = at(ray, is_time), is_norm
            if (cur.depth > 0) {                                   // scene.cu:109-121
                if (!OPQ && cur.in_obj) {
                    const V4 kt = bv.mats[is_mat].Kt;               // trans_atten (scene.cu:14-22): time^Kt
                    cur.atten = cur.atten * v4(pow_fast(is_time, kt.x), pow_fast(is_time, kt.y),
                                               pow_fast(is_time, kt.z), pow_fast(is_time, kt.w));
                }
                cur.type = F_REFLECT;
                cur.last_mat = is_mat;
            } else {
                fl |= 2;                                           // popped after illumination (frame still needed)
            }
            const DMat& m = bv.mats[is_mat];                       // org_light (phong.cu:36-39)
            summed = m.Ke + m.Ka * kld(P.ambience);
            li = 0;
            st = ST_LIGHT;
            continue;
        }
        // ST_WAIT_SHADOW: one shadow segment (light.cu:35-58)
        bool light_done = true;
        if (OPQ && PARK) {                                     // not parked: the light's own colour
            rv = bv.lights[li].col;
        }
        V4 att = rv;
        if (hit && !(b.time > max_t)) {
            const DMat& m = bv.mats[hmat];
            if (OPQ || !m.refractive) {
                att = v4(0, 0, 0, 0);
            } else {
                if (dot(hn, q.d) > 0) {                            // calc_shadow_atten (light.cu:18-25)
                    rv = rv * v4(pow_fast(m.Kt.x, b.time), pow_fast(m.Kt.y, b.time), pow_fast(m.Kt.z, b.time),
                                 pow_fast(m.Kt.w, b.time));
                }
                q = make_ray(at(q, b.time), q.d);
                max_t -= b.time;
                dbg(P, me, 4);
                light_done = false;
            }
        }
        if (light_done) {
            // An unlit light's term is its factor's signed zeros times the light: adding it leaves
            // `summed` as it is unless `summed` is -0, which the host rules out (unlit_skip = 2:
            // no material's Ke + Ka * ambience has a -0 channel, and x + y is -0 only for two -0).
            if (!(max_t == -INFINITY && kparams().unlit_skip == 2)) {
                const V4 inc = (bv.lights[li].type == 0) ? da * att : att;  // PointLight: dist_atten * attenuate()
                summed = summed + fct * inc;                   // phong(): factor x incoming (phong.cu:50-52)
            }
            li++;
            st = ST_LIGHT;
        }
    }
    return acc;
}

// stage_bvh's LDS image size (16-B multiple)
__host__ __device__ inline size_t a16(size_t b) { return (b + 15) & ~(size_t)15; }
// LDS shading cache (M_SHADE): mats | lights | tris | meshes, each 16-B aligned
__host__ __device__ inline size_t shade_bytes(const SceneView& S) {
    return a16(sizeof(DMat) * (size_t)S.n_mats) + a16(sizeof(DLight) * (size_t)S.n_lights) +
           a16(sizeof(DTri) * (size_t)S.n_tris) + a16(sizeof(DMesh) * (size_t)S.n_meshes);
}
__host__ __device__ inline size_t lds_bytes(const SceneView& S, bool ft = false, bool shade = false, bool brute = false,
                                            bool part = false) {
    const size_t sh = shade ? shade_bytes(S) : 0;
    if (brute) return a16(16 * (size_t)S.n_inst) + sh;        // inst4 only (M_BRUTE)
    if (ft && part) return 64 * (size_t)(S.n_real - 1) + sh;   // the ordered tree only (M_PART)
    if (ft) return 64 * (size_t)(S.n_real - 1) + 16 * (size_t)S.n_inst + sh;
    return a16(48 * (size_t)S.n_leaf + 4 * (size_t)S.n_leaf) + a16(16 * (size_t)S.n_inst) + sh;
}
// word copy of n records of T into LDS at `dst` (block-cooperative)
template <class T> __device__ __forceinline__ const T* stage_words(unsigned char* dst, const T* src, int n) {
    static_assert(sizeof(T) % 4 == 0 && alignof(T) <= 16, "word-granular records");
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
    const int w = (int)(sizeof(T) / 4) * n;
    for (int i = threadIdx.x; i < w; i += blockDim.x) d32[i] = s32[i];
    return reinterpret_cast<const T*>(dst);
}

// LDS image of a persistent block: node pairs [3n float4] | leaf_inst [n] | inst4 [n_inst]
// (16-B aligned); lds_bytes() on the host must match.
template <bool LDS, bool FT = false, bool SHADE = false, bool BRUTE = false, bool PART = false>
__device__ __forceinline__ BvhRefs stage_bvh(const SceneView& S, unsigned char* smem) {
    BvhRefs bv;
    bv.fnode = S.fnode;
    bv.pair = S.node_pair; bv.leaf = S.leaf_inst; bv.inst = S.inst4;
    bv.mats = S.mats; bv.lights = S.lights; bv.tris = S.tris; bv.meshes = S.meshes;
    if (LDS && SHADE) {                                    // after the BVH image (lds_bytes without the cache)
        unsigned char* p = smem + lds_bytes(S, FT, false, BRUTE, PART);
        bv.mats = stage_words(p, S.mats, S.n_mats);       p += a16(sizeof(DMat) * (size_t)S.n_mats);
        bv.lights = stage_words(p, S.lights, S.n_lights); p += a16(sizeof(DLight) * (size_t)S.n_lights);
        bv.tris = stage_words(p, S.tris, S.n_tris);       p += a16(sizeof(DTri) * (size_t)S.n_tris);
        bv.meshes = stage_words(p, S.meshes, S.n_meshes);
    }
    if (LDS && BRUTE) {                                    // inst4 (no tree)
        float4* in = reinterpret_cast<float4*>(smem);
        for (int i = threadIdx.x; i < S.n_inst; i += blockDim.x) in[i] = S.inst4[i];
        __syncthreads();
        bv.inst = in;
    } else if (LDS && FT && PART) {                        // ordered LBVH (inst4 stays in global memory)
        const int nf = 4 * (S.n_real - 1);
        const float4* src = S.fnode;
        float4* fn = reinterpret_cast<float4*>(smem);
        for (int i = threadIdx.x; i < nf; i += blockDim.x) fn[i] = src[i];
        __syncthreads();
        bv.fnode = fn;
    } else if (LDS && FT) {                                // ordered LBVH | inst4
        const int nf = 4 * (S.n_real - 1);
        const float4* src = S.fnode;
        float4* fn = reinterpret_cast<float4*>(smem);
        float4* in = fn + nf;
        for (int i = threadIdx.x; i < nf; i += blockDim.x) fn[i] = src[i];
        for (int i = threadIdx.x; i < S.n_inst; i += blockDim.x) in[i] = S.inst4[i];
        __syncthreads();
        bv.fnode = fn; bv.inst = in;
    } else if (LDS) {
        const int n3 = 3 * S.n_leaf;
        float4* np = reinterpret_cast<float4*>(smem);
        int* lf = reinterpret_cast<int*>(smem + 16 * (size_t)n3);
        float4* in = reinterpret_cast<float4*>(smem + ((16 * (size_t)n3 + 4 * (size_t)S.n_leaf + 15) & ~(size_t)15));
        for (int i = threadIdx.x; i < n3; i += blockDim.x) np[i] = S.node_pair[i];
        for (int i = threadIdx.x; i < S.n_leaf; i += blockDim.x) lf[i] = S.leaf_inst[i];
        for (int i = threadIdx.x; i < S.n_inst; i += blockDim.x) in[i] = S.inst4[i];
        __syncthreads();
        bv.pair = np; bv.leaf = lf; bv.inst = in;
    }
    return bv;
}

__device__ __forceinline__ V4 shfl4(V4 v, int src) {
    return v4(__shfl(v.x, src), __shfl(v.y, src), __shfl(v.z, src), __shfl(v.w, src));
}

// Persistent blocks (one per CU): the BVH and the instance records are staged in
// LDS once, then every wave repeatedly takes a pixel group from the work counter.
// A group = `px_per_wave` pixels x `lanes_per_px` samples; lane (pixel p, sub s)
// traces samples k = round*L + s and the group leader sums the clamped sample
// radiance in k order (build-defined spp extension).
// MODE bit 0 (MULTI): spp > 64 -- several rounds of samples per lane (the per-pixel sums
// then stay live across rounds, which the common single-round kernel avoids).
// MODE bit 1 (STATS): exact work counters.  The divergent state machine keeps 64-bit
// counters in VGPRs, so frames without statistics use a kernel without them.
// MODE bit 2 (PARK): park integrator state in LDS during queries (trace_sample); needs
// PARK_FIELDS x 4 B x TRACE_BLOCK_P of LDS beside the BVH image.
// MODE bit 3 (TEX): textured shading (hit_kd), generic frame depth only.
// MODE bit 4 (FT): traverse the ordered LBVH (closest_hit) instead of the reference heap.
// MODE bit 5 (AXIS): FT with the axis-plane triangle path (S.tri_ax, cast_local).
// MODE bit 6 (PROF): profiling variant of the fast kernel -- wave-level step counts and
// s_memtime cycle accounting (rt_experiment 6); results identical, timing perturbed.
// MODE bit 8 (BRUTE): brute-force frames (use_bvh = 0) with only the instance loop compiled
// (closest_hit); LDS image = inst4 (+ the shading cache, parking area).
// MODE bit 9 (PART): partial parking (PART_FIELDS) with the tree alone in LDS (see PART_FIELDS).
constexpr int M_MULTI = 1, M_STATS = 2, M_PARK = 4, M_TEX = 8, M_FT = 16, M_AXIS = 32, M_PROF = 64, M_SHADE = 128,
              M_BRUTE = 256, M_PART = 512;
template <int NS, bool LDS, int MODE>
__global__ __launch_bounds__(TRACE_BLOCK_P) void trace_kernel(TraceParams P_arg, SceneView S) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    (void)P_arg;                                               // read in place: kparams()
    KTP& P = kparams();
    constexpr bool FT = (MODE & M_FT) != 0, AXIS = (MODE & M_AXIS) != 0;
    constexpr bool SHADE = (MODE & M_SHADE) != 0, BRUTE = (MODE & M_BRUTE) != 0, PART = (MODE & M_PART) != 0;
    static_assert(!(BRUTE && FT), "a brute-force kernel has no tree");
    static_assert(!PART || (FT && (MODE & M_PARK)), "partial parking is a parked ordered-tree kernel");
    const BvhRefs bv = stage_bvh<LDS, FT, SHADE, BRUTE, PART>(S, smem);
    // LDS-staged sample sums (spp >= 16) in the partially parked kernels (config 5's world16 at
    // 64 spp); compiled out of the fully parked headline kernel, whose registers it would crowd
    constexpr bool LSUM = RT_LDS_SUM && PART;
    const int lane = threadIdx.x & 63;
    const int L = P.lanes_per_px;
    constexpr bool MULTI = (MODE & M_MULTI) != 0, STATS = (MODE & M_STATS) != 0, PARK = (MODE & M_PARK) != 0;
    constexpr bool PROF = (MODE & M_PROF) != 0, CYC = STATS || PROF;
    constexpr bool TEX = (MODE & M_TEX) != 0;
    float* park = PARK ? reinterpret_cast<float*>(smem + lds_bytes(S, FT, SHADE, BRUTE, PART)) + threadIdx.x : nullptr;
    const int rounds = MULTI ? (P.spp + L - 1) / L : 1;
    WaveCounters wc{0, 0, 0, 0};
    if (PROF) {                                                // this wave's occupancy counters (zeroed)
        wc.pc = reinterpret_cast<unsigned long long*>(smem + lds_bytes(S, FT, SHADE, BRUTE, PART) +
                                                       (PARK ? (size_t)park_fields(NS) * 4 * TRACE_BLOCK_P : 0)) +
                (threadIdx.x >> 6) * PROF_WAVE_SLOTS;
        if (lane < PROF_WAVE_SLOTS) wc.pc[lane] = 0;
    }
    // Dynamic group assignment over NQ interleaved queues (queue c owns groups g = c + NQ*j):
    // a wave drains its own queue (c = block % NQ, i.e. one per XCD dispatch slot) then the
    // others.  The next ticket is requested one group ahead so the atomic's latency hides
    // behind the current group; a single global counter serialised ~260k atomics (~2.5 ms,
    // measured) and a static split left a 1.5x load-imbalance tail (measured).
    const int q0 = blockIdx.x % NQ;
    const int per_q = (P.n_groups + NQ - 1) / NQ;
    int n_heavy = 0;
    unsigned long long thr = ~0ull, wave_sum = 0;
    if (P.hist == 2) {
        n_heavy = ldc(P.work, WORK_HEAVY_LEN);                 // this frame's heavy live list (sky_kernel)
    } else if (P.hist) {
        n_heavy = (int)min(P.hctl_prev[0], (unsigned long long)P.heavy_cap);
        // heavy: over 4x the previous frame's mean group and over 20 us (2000 ticks of the 100 MHz
        // clock) -- in a frame of uniformly cheap groups the mean-relative test alone flags
        // timing noise, and a long heavy list (one atomic per group) is slower than none
        if (P.hctl_prev[1]) thr = max(4 * P.hctl_prev[1] / (unsigned long long)P.n_groups, 2000ull);
    }
    int qi = n_heavy > 0 ? -1 : 0;                           // -1: the previous frame's heavy groups first
    // Lane 0 holds the raw result of the pending ticket request.  A ticket claims TPC
    // consecutive work indices of its queue (one index in the heavy list); the next one is
    // requested when the batch's last group starts, after that group's own global loads
    // (vmcnt retires in order, so an earlier atomic would hold them up), and read when the
    // batch is used up.  Fewer, batched device-scope atomics: the counters sustain ~100 M
    // atomics/s each, which alone bounded a TPC = 1 frame at 0.75 ms (measured, group
    // loop without tracing).
    int pend = 0, inflight = 0;
    auto step_of = [&](int q) { return q < 0 ? 1 : kparams().tpc; };
#if RT_HEAVY_STATIC
    // A frame issued alone (heavy_static: every block starts at once) deals the heavy list out
    // statically, wave w taking tickets w, w + W, w + 2W, ... with no atomic: otherwise the
    // grid's 4096 waves all queue on the one heavy counter before their first group (~100 M
    // atomics/s: ~40 us).  Lone trace 0.768 -> 0.702 ms (profiles/r04/ab_hs2.log).  Frames that
    // overlap others keep the counter: their blocks start as CUs free up, and a late block's
    // static share became the tail (pipelined frame +1.9% with it; profiles/r04/ab_hs.log).
    int hnext = (int)blockIdx.x * (TRACE_BLOCK_P / 64) + (int)(threadIdx.x >> 6);   // this wave's next heavy ticket
#endif
    // live lists: tickets [0, 2^k) of a list of n <= 2^k groups visit (t * odd) mod 2^k, a
    // bijection that spreads consecutive tickets over the list (arrival order is roughly
    // raster order, where expensive regions cluster); indices >= n are skipped
    auto live_n = [&](int q) { return ldc(kparams().work, 16 * (NQ + 1 + (q0 + q) % NQ)); };
    auto live_span = [&](int q) { const int n = live_n(q); return n <= 1 ? n : 1 << (32 - __builtin_clz((unsigned)n - 1)); };
    auto pow2_span = [](int n) { return n <= 1 ? n : 1 << (32 - __builtin_clz((unsigned)n - 1)); };
    auto request = [&](int q) {
        KTP& Pq = kparams();
        // The address goes through a VGPR so the atomic optimizer leaves the atomic alone:
        // its rewrite waits for the returned value right after issuing it, while the value is
        // needed only when the batch is used up (resolve), groups later.
        unsigned long long a = (unsigned long long)(q < 0 ? &Pq.work[16 * NQ] : &Pq.work[16 * ((q0 + q) % NQ)]);
        asm volatile("" : "+v"(a));
        typedef __attribute__((address_space(1))) int gint;   // keep the global (not flat) atomic
#if RT_HEAVY_STATIC
        if (q < 0 && kparams().heavy_static) { pend = hnext; hnext += kparams().grid_waves; inflight = 1; return; }
#endif
        if (lane == 0) pend = __hip_atomic_fetch_add((gint*)a, step_of(q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        inflight = 1;
    };
    auto resolve = [&]() { inflight = 0; return __builtin_amdgcn_readfirstlane(pend); };   // all lanes active here
    // one-pixel groups (LSUM kernels, spp >= 64): RGBA results of consecutive pixels buffered one
    // per lane (wbuf), stored as one piece when the run breaks: a 4-B store per pixel-wave left
    // as its own memory-side write (config 5 wrote 20x its frame)
    unsigned wbuf = 0;
    int wbase = 0, wn = 0;                                     // (uniform) first pixel, count
    auto wflush = [&]() {
        if (wn > 0) {
            if (lane_id_fresh() < wn) kparams().rgba[wbase + lane_id_fresh()] = wbuf;
            wn = 0;
        }
    };
    request(qi);
    int tbase = resolve(), j = 0;
    const unsigned long long c_start = CYC ? __builtin_amdgcn_s_memtime() : 0;
    const unsigned long long rt_start = CYC ? __builtin_amdgcn_s_memrealtime() : 0;   // global 100 MHz clock
    for (;;) {
        KTP& P = kparams();                                    // this group's reads of the launch parameters
        for (;;) {                                             // next work index tbase + j of queue qi
            if (qi >= NQ) break;
            const int lim = qi < 0 ? (kparams().hist == 2 ? pow2_span(n_heavy) : n_heavy) : kparams().live ? live_span(qi) : per_q;
            if (tbase + j >= lim) {                             // queue drained (a pending batch is past it too)
                if (inflight) (void)resolve();
                qi++; j = 0;
                if (qi < NQ) { request(qi); tbase = resolve(); }
                continue;
            }
            if (j < step_of(qi)) break;
            if (!inflight) request(qi);                        // batch used up
            tbase = resolve(); j = 0;
        }
        if (qi >= NQ) break;
        const int ticket = tbase + j++;
        const bool last_of_batch = j == step_of(qi);
        // tickets visit the queue's groups in a scrambled order (t * scramble mod per_q, a
        // bijection): expensive image regions are spread over the frame instead of all
        // starting last and leaving a long tail of idle CUs (measured: first wave done at
        // 69% of the kernel span with row order)
        // The scheduling history is read with scalar loads: a vector load here would wait
        // (vmcnt is in order) for the previous group's output stores to be acknowledged.
        auto umod = [&](unsigned n) { return n - udiv(n, kld(P.div_perq)) * (unsigned)per_q; };
        auto live_g = [&]() {
            const int n = live_n(qi);
            int i;
            if (LSUM && kparams().tpc > 1) {
                // a ticket's tpc (a power of two) consecutive indices stay consecutive list entries
                // -- neighbouring pixels of one sky block -- and the runs are scrambled, so that a
                // wave stores their results as one wide piece (wstore below)
                const int rl = 31 - __builtin_clz((unsigned)kparams().tpc), span = live_span(qi);
                if (span <= (1 << rl)) i = ticket;
                else i = (int)((((((unsigned)ticket >> rl) * 0x9E3779B1u) & (unsigned)((span >> rl) - 1)) << rl) |
                               ((unsigned)ticket & ((1u << rl) - 1u)));
            } else {
                i = (int)(((unsigned)ticket * 0x9E3779B1u) & (unsigned)(live_span(qi) - 1));
            }
            return i < n ? ldc(P.live, ((q0 + qi) % NQ) * P.live_cap + i) : P.n_groups;
        };
        auto heavy_g = [&]() {                                 // hist = 2: the heavy live list, scrambled
            const int i = (int)(((unsigned)ticket * 0x9E3779B1u) & (unsigned)(pow2_span(n_heavy) - 1));
            return i < n_heavy ? ldc(P.live, NQ * P.live_cap + i) : P.n_groups;
        };
        const int g = qi < 0 ? (P.hist == 2 ? heavy_g() : ldc(P.hl_prev, ticket))
                             : P.live ? live_g()
                             : ((q0 + qi) % NQ) + NQ * (P.scramble_small ? (int)umod((unsigned)ticket * (unsigned)P.scramble)
                                                                         : (int)(((long long)ticket * P.scramble) % per_q));
        auto flag = [&](const unsigned char* f) { return (ldc(reinterpret_cast<const uint32_t*>(f), g >> 2) >> (8 * (g & 3))) & 0xffu; };
        if (g >= P.n_groups || (qi < 0 && P.hist == 1 && P.gsky && flag(P.gsky)) ||    // sky group: done by sky_kernel
            (qi >= 0 && P.hist == 1 && flag(P.hf_prev)))
            continue;
        const unsigned long long g_start = P.hist == 1 ? __builtin_amdgcn_s_memrealtime() : 0;
        int nq = 0;                                            // wave queries of this group (hist = 2)
        const GroupLane gl = group_lane(g);
        const int sub_g = gl.sub, px = gl.px, py = gl.py;
        const bool valid = gl.valid;
        const bool me = valid && sub_g == 0 && px == P.dbg_x && py == P.dbg_y;
        V4 sum_c = v4(0, 0, 0, 0), sum_r = v4(0, 0, 0, 0);
        float acc = 0.0f;                                      // RT_LDS_SUM: this lane's (pixel, channel) sum
        const unsigned long long g_t0 = CYC ? __builtin_amdgcn_s_memrealtime() : 0, g_q0 = wc.wq;
        const unsigned long long g_p0 = wc.wpair, g_l0 = wc.wleaf, g_r0 = wc.wtri;
        const unsigned long long g_c0 = wc.cyc_q, g_c1 = wc.cyc_leaf, g_c2 = wc.cyc_sample, g_c3 = wc.cyc_post;
        const unsigned long long g_c4 = wc.cyc_light, g_c5 = wc.cyc_normal, g_c6 = wc.cyc_park;
        const unsigned long long g_m0 = CYC ? __builtin_amdgcn_s_memtime() : 0;
        for (int rd = 0; rd < rounds; rd++) {
            const int k = rd * L + sub_g;
            const bool act = valid && k < P.spp;
            Ray r0{v3(0, 0, 0), v3(0, 0, 1)};
            if (act) {
                const float2 o = spp_offset_dev(k);
                DCamera cam = kld(P.cam);
                cam.W = fresh_s(cam.W); cam.H = fresh_s(cam.H); cam.near_ = fresh_s(cam.near_);
                r0 = camera_at(cam, (float)px + o.x, (float)py + o.y);
            }
            if (rd == 0 && last_of_batch) request(qi);         // next ticket, in flight during the trace
            // Whole-group miss (fast kernels): when no lane's primary ray hits a child of the
            // tree's root -- the traversal's first step, same test -- every sample misses, its
            // radiance is the integrator's initial zero (scene.cu:124-126) and the group's
            // outputs are zeros (and -1 hit ids).  Most groups of the reference scenes are sky.
            if (FT && !STATS && !PROF && !MULTI && SV().use_bvh && SV().n_leaf > 0 && !kparams().gsky && !__ballot(ft_root_hit(SV(), bv, act, r0))) {
                if (act && k == 0) {
                    const int op = gl.pix;
                    if (P.hit_inst) P.hit_inst[op] = -1;
                    if (P.hit_tri) P.hit_tri[op] = -1;
                }
                break;                                         // sum_c = sum_r = 0
            }
            // PROF: the group is live when some primary enters the tree's root (the sky pre-pass's
            // test); occupancy counters are taken over live groups' queries only
            if (PROF && FT) wc.live = __ballot(ft_root_hit(SV(), bv, act, r0)) != 0;
            const unsigned long long cs = CYC ? __builtin_amdgcn_s_memtime() : 0;
            V4 c = trace_sample<NS, STATS, PARK, TEX, FT, AXIS, PROF, BRUTE, PART>(S, bv, act, r0, me && rd == 0, act && k == 0, g, wc,
                                                 park, nq);
            if (CYC) wc.cyc_sample += __builtin_amdgcn_s_memtime() - cs;
            auto clamp1 = [](V4 v) {                           // raytracer.cu:37-40
                return v4(v.x > 1.0f ? 1.0f : v.x, v.y > 1.0f ? 1.0f : v.y, v.z > 1.0f ? 1.0f : v.z, v.w > 1.0f ? 1.0f : v.w);
            };
            // in-order reduction over samples (ds_bpermute: the LDS pipe has room, the VALU
            // does not -- a DPP row-shift form measured 4% slower).  Each lane clamps its own
            // sample before the exchange (the same bits the leader would compute), and the raw
            // sum is formed only when the radiance output is requested.
            // (lane addresses and sample bounds formed here, after the trace: hoisted above it,
            // they were held across the trace and spilled)
            KTP& Pr = kparams();
            const bool want_r = Pr.radiance != nullptr;
            const int spp_n = Pr.spp;
            const GroupLane ga = group_lane(g);                // after the trace (not held across it)
            const int bb = ga.base, sub_a = ga.sub;
            const V4 cc = clamp1(c);
            if (L == 8) {                               // spp = 8: all permutes in one LDS round trip
                V4 v[8];
#pragma unroll
                for (int s = 0; s < 8; s++) v[s] = shfl4(cc, bb + s);
                if (sub_a == 0)
#pragma unroll
                    for (int s = 0; s < 8; s++)
                        if (rd * L + s < spp_n) sum_c = sum_c + v[s];
                if (want_r) {
#pragma unroll
                    for (int s = 0; s < 8; s++) v[s] = shfl4(c, bb + s);
                    if (sub_a == 0)
#pragma unroll
                        for (int s = 0; s < 8; s++)
                            if (rd * L + s < spp_n) sum_r = sum_r + v[s];
                }
            } else if (LSUM && L >= 16) {
                // spp >= 16 (whole waves, or 16-32 lanes, per pixel): the in-order sums run one per
                // lane and channel through the wave's own parking columns (free between queries),
                // a ds_read and an add per sample, instead of four ds_bpermutes, four adds and the
                // leader's select per sample.  Lane j = (pixel p, channel f): channels 0-3 the
                // clamped colour, 4-7 the raw radiance when requested; the same adds in k order.
                const int ln = lane_id_fresh();                // (not held across the group loop)
                float* wcol = park - ln;                       // the wave's column 0, field 0
                float* mine = park;
                mine[0] = cc.x; mine[TRACE_BLOCK_P] = cc.y; mine[2 * TRACE_BLOCK_P] = cc.z; mine[3 * TRACE_BLOCK_P] = cc.w;
                if (want_r) {
                    mine[4 * TRACE_BLOCK_P] = c.x; mine[5 * TRACE_BLOCK_P] = c.y;
                    mine[6 * TRACE_BLOCK_P] = c.z; mine[7 * TRACE_BLOCK_P] = c.w;
                }
                __builtin_amdgcn_wave_barrier();
                const int nsh = want_r ? 3 : 2;                // log2 of the channels per pixel
                const int pj = ln >> nsh, fj = ln & ((1 << nsh) - 1);
                const int n_s = min(L, spp_n - rd * L);        // samples of this round (uniform)
                if (pj < kparams().px_per_wave) {
                    const float* src = wcol + fj * TRACE_BLOCK_P + pj * L;
                    int s = 0;
                    for (; s + 4 <= n_s; s += 4) {             // 16-B reads (pj * L: a multiple of 16 floats)
                        const float4 v = *reinterpret_cast<const float4*>(src + s);
                        acc = acc + v.x; acc = acc + v.y; acc = acc + v.z; acc = acc + v.w;
                    }
                    for (; s < n_s; s++) acc = acc + src[s];
                }
                __builtin_amdgcn_wave_barrier();
            } else {
                for (int s = 0; s < L; s++) {
                    const V4 v = shfl4(cc, bb + s);
                    if (sub_a == 0 && rd * L + s < spp_n) sum_c = sum_c + v;
                }
                if (want_r)
                    for (int s = 0; s < L; s++) {
                        const V4 v = shfl4(c, bb + s);
                        if (sub_a == 0 && rd * L + s < spp_n) sum_r = sum_r + v;
                    }
            }
        }
        if (LSUM && L >= 16) {                 // the channel sums to their pixel's leader
            const int ln = lane_id_fresh();
            float* wcol = park - ln;
            const int nsh = kparams().radiance != nullptr ? 3 : 2;
            const int pj = ln >> nsh, fj = ln & ((1 << nsh) - 1);
            if (pj < kparams().px_per_wave) wcol[fj * TRACE_BLOCK_P + pj * L] = acc;
            __builtin_amdgcn_wave_barrier();
            const float* mine = park;
            sum_c = v4(mine[0], mine[TRACE_BLOCK_P], mine[2 * TRACE_BLOCK_P], mine[3 * TRACE_BLOCK_P]);
            if (nsh == 3) sum_r = v4(mine[4 * TRACE_BLOCK_P], mine[5 * TRACE_BLOCK_P], mine[6 * TRACE_BLOCK_P], mine[7 * TRACE_BLOCK_P]);
            __builtin_amdgcn_wave_barrier();
        }
        const GroupLane go = group_lane(g);                    // the output pixel, recomputed here
        const bool wide = LSUM && L == 64 && kparams().rgba != nullptr;   // (uniform) buffered RGBA stores
        uint32_t w_enc = 0;
        int w_pix = -1;
        if (go.valid && go.sub == 0) {
            KTP& P = kparams();
            const int p = go.pix;
            const float inv = (float)P.spp;
            // mean = sum / spp (raytracer.cu's per-sample colour, build-defined spp average);
            // for spp = 2^k, x * 2^-k is the same correctly rounded value as x / 2^k
            auto mean = [&](float x) { return P.spp_recip != 0.0f ? x * P.spp_recip : x / inv; };
            const float mr = mean(sum_c.x), mg = mean(sum_c.y), mb = mean(sum_c.z), ma = mean(sum_c.w);
            // Color(float r, g, b, a) truncation to uint8 and to_encoding (color.h:41-42, color.cu:23-26)
            const uint32_t enc = ((uint32_t)(uint8_t)((float)255 * mr) << 24) + ((uint32_t)(uint8_t)((float)255 * mg) << 16) +
                                 ((uint32_t)(uint8_t)((float)255 * mb) << 8) + (uint32_t)(uint8_t)((float)255 * ma);
            if (wide) { w_enc = enc; w_pix = p; }
            else if (P.rgba) P.rgba[p] = enc;
            if (P.radiance) P.radiance[p] = make_float4(mean(sum_r.x), mean(sum_r.y), mean(sum_r.z), mean(sum_r.w));
        }
        if (wide) {                                            // lane 0 is the pixel's leader (L = 64)
            const int pu = __builtin_amdgcn_readlane(w_pix, 0);
            const unsigned eu = (unsigned)__builtin_amdgcn_readlane((int)w_enc, 0);
            if (pu >= 0) {
                if (wn > 0 && (pu != wbase + wn || wn == 64)) wflush();
                if (wn == 0) wbase = pu;
                asm("v_writelane_b32 %0, %1, m0" : "+v"(wbuf) : "s"(eu), "{m0}"(wn));
                wn++;
            }
        }
        if (STATS && P.stats && lane == 0) {                 // profiling: heaviest group (PROF: rt_profile_groups)
            atomicMax(&P.stats[20], __builtin_amdgcn_s_memrealtime() - g_t0);
            atomicMax(&P.stats[21], wc.wq - g_q0);
        }
        if (kparams().hist == 2) {            // heavy by work: the next frame's pre-pass runs it first
            KTP& P = kparams();
            if (nq >= P.heavy_q && lane_id_fresh() == 0) P.hf_next[g] = 1;
        } else if (kparams().hist) {          // record for the next frame's order
            KTP& P = kparams();
            const unsigned long long dur = __builtin_amdgcn_s_memrealtime() - g_start;   // wave-uniform (scalar)
            const bool heavy = dur > thr;
            wave_sum += dur;
            if (lane_id_fresh() == 0) {
            // at most heavy_cap recorded (a few per wave: the list is there to start the frame's
            // longest groups first); a group flagged in hf_next is always in hl_next
            int slot = -1;
            if (heavy) slot = atomicAdd(reinterpret_cast<int*>(P.hctl_next), 1);
            const bool rec = heavy && slot < P.heavy_cap;
            P.hf_next[g] = rec ? 1 : 0;
            if (rec) P.hl_next[slot] = g;
            if (P.gdur) {
                P.gdur[g] = (unsigned)dur;
                if (PROF) {                                    // wave step counts and cycle split of the group
                    unsigned* c = P.gdur + P.n_groups + 12 * (size_t)g;
                    c[0] = (unsigned)(wc.wq - g_q0); c[1] = (unsigned)(wc.wpair - g_p0);
                    c[2] = (unsigned)(wc.wleaf - g_l0); c[3] = (unsigned)(wc.wtri - g_r0);
                    c[4] = (unsigned)(wc.cyc_q - g_c0); c[5] = (unsigned)(wc.cyc_leaf - g_c1);
                    c[6] = (unsigned)(wc.cyc_sample - g_c2); c[7] = (unsigned)(wc.cyc_post - g_c3);
                    c[9] = (unsigned)(wc.cyc_light - g_c4); c[10] = (unsigned)(wc.cyc_normal - g_c5);
                    c[11] = (unsigned)(wc.cyc_park - g_c6);
                    c[8] = (unsigned)(__builtin_amdgcn_s_memtime() - g_m0);
                }
            }
            }
        }
    }
    if (LSUM) wflush();
    if (P.hist == 1 && lane == 0 && wave_sum) atomicAdd(&P.hctl_next[1], wave_sum);
    if (CYC && P.stats && lane == 0) {
        if (wc.rays) atomicAdd(&P.stats[0], wc.rays);
        if (wc.nodes) atomicAdd(&P.stats[1], wc.nodes);
        if (wc.leaves) atomicAdd(&P.stats[2], wc.leaves);
        if (wc.tris) atomicAdd(&P.stats[3], wc.tris);
        atomicAdd(&P.stats[4], wc.wq); atomicAdd(&P.stats[5], wc.wpair);
        atomicAdd(&P.stats[6], wc.wleaf); atomicAdd(&P.stats[7], wc.wtri);
        atomicAdd(&P.stats[8], wc.cyc_q); atomicAdd(&P.stats[9], wc.cyc_leaf);
        atomicAdd(&P.stats[10], __builtin_amdgcn_s_memtime() - c_start);
        atomicAdd(&P.stats[11], wc.cyc_sample); atomicAdd(&P.stats[12], wc.cyc_post);
        atomicAdd(&P.stats[13], wc.wbary); atomicAdd(&P.stats[14], wc.lbary);
        const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
        atomicMin(&P.stats[15], rt_start);                      // kernel span (earliest start, latest end)
        atomicMax(&P.stats[16], rt_end);
        atomicAdd(&P.stats[17], rt_end - rt_start);             // summed wave lifetimes (same clock)
        atomicMax(&P.stats[18], rt_start);                      // latest start / earliest end
        atomicMin(&P.stats[19], rt_end);
        if (PROF)
            for (int i = 0; i < PROF_END - PROF_LANES_PRIMARY; i++)
                if (wc.pc[i]) atomicAdd(&P.stats[PROF_LANES_PRIMARY + i], wc.pc[i]);
    }
}


// Sky pre-pass of the fast frames: one wave per pixel group, the trace kernel's lane mapping
// (lane = pixel x sample), the primary ray of each lane (camera_at, camera.cu:33-42) and the
// traversal's first step on it (ft_root_hit: the same ray_inv, zero-axis cut and pair test on
// the root's children as closest_hit's first iteration).  A group none of whose primaries
// enters the root is a sky group: every sample's query returns no hit, its radiance is the
// integrator's initial zero (scene.cu:124-126), so the group's outputs are written here --
// rgba = the encoding of a zero mean (0), radiance 0, hit ids -1 -- exactly what the trace
// kernel's own whole-group miss test writes, and gsky[g] = 1 tells the trace kernel to skip
// the group.  84% of world8_stress's 1080p groups are sky: in the persistent trace kernel
// each one cost the group loop's whole prologue (ticket, parameter loads, register spills
// and restores around the integrator) -- a lean, high-occupancy kernel does the test
// instead.  The root records are read from global memory (all lanes the same address).
// Group-level sky test: the rays of a group leave the camera position through its pixel
// rectangle [x0, x1] x [y0, y1] (pixels and sample offsets in [0, 1); rows row_step apart
// are covered by their hull), i.e. they lie in the convex cone spanned by the four corner
// directions D(cx, cy) = near f + ((cx - W/2) / unit) r + ((H/2 - cy) / unit) u.  A box
// outside one of the cone's four side half-spaces {x : n . (x - pos) >= 0} meets no ray of
// the group.  Conservative margins: the rectangle grown by 1/64 pixel (the computed rays'
// direction rounding is ~1e-6 rad, 1/64 pixel ~1e-5 rad), the box grown by 1e-4 of its
// coordinate scale, a separation required beyond 1e-5 relative; and the test is only
// trusted when no direction component comes near zero over the rectangle (|D_a| >= 2^-40
// |D|), so every ray of the group takes the geometric slab test (no zero-axis skip and
// no exact-path fallback for tiny components: ray_inv).  A group it does not decide gets
// the exact per-ray root test.
// Brute-force sky test.  In frames without a tree (the reference's -r,
// scene.cu:48-52) every primary ray runs cast_local on every instance, and no box is tested.
// With pure translations and zero mesh offsets (S.prune_abs >= 0) the distance-pruning claim
// (closest_hit) bounds where an accepted hit can lie: a triangle of instance k is accepted at
// world time t only at a point within prune_abs + 2^-13 t of its box (the claim's spatial
// slack plus its time slack).  So when no t >= 0 puts the ray inside the box grown by A + B t
// with A = 2 prune_abs, B = 2^-12 (twice that), no triangle of the instance is accepted.  The
// interval of such t is formed in float: each bound's rounding (a few ulps of the scene radius
// R and of t) is far below what the doubling adds (prune_abs >= 2^-14 R, and 2^-13 t), so an
// interval found empty here is empty under the claim's slack.  Answers "maybe" unless empty.
__device__ __forceinline__ bool grown_box_maybe(float4 lo, float4 hi, float A, float B, const Ray& r) {
    float tl = 0.0f, th = INFINITY;
    auto axis = [&](float l, float h, float o, float d) {
        const float c1 = (l - A) - o, k1 = d + B;            // (d + B) t >= l - A - o
        if (k1 > 0.0f) tl = fmaxf(tl, c1 / k1);
        else if (k1 < 0.0f) th = fminf(th, c1 / k1);
        else if (c1 > 0.0f) tl = INFINITY;
        const float c2 = (h + A) - o, k2 = d - B;            // (d - B) t <= h + A - o
        if (k2 > 0.0f) th = fminf(th, c2 / k2);
        else if (k2 < 0.0f) tl = fmaxf(tl, c2 / k2);
        else if (c2 < 0.0f) tl = INFINITY;
    };
    axis(lo.x, hi.x, r.o.x, r.d.x);
    axis(lo.y, hi.y, r.o.y, r.d.y);
    axis(lo.z, hi.z, r.o.z, r.d.z);
    return !(tl > th);
}

// Brute-force frames (item 30): cone_misses_root's group cone and box test, factored so that
// one cone can be tested against several boxes (cone_misses_root keeps its own inline form: the
// headline's sky kernel measured 1.8% slower in a pipelined frame with this one).  GroupCone:
// the four corner directions, the side planes' normals (pointing inward), the largest
// direction component; ok = 0 when a direction component may come near zero (nothing decided).
struct GroupCone { V3 k[4], n[4]; float dmax; int ok; };
__device__ __forceinline__ GroupCone group_cone(const TraceParams& P, int g) {
    GroupCone gc;
    gc.ok = 0;
    const DCamera& c = P.cam;
    if (!(c.near_ > 0.0f)) return gc;
    const int gy = (int)udiv((unsigned)g, P.div_ngx), gx = g - gy * P.n_gx;
    const int pr0 = gy * P.gh;
    const float e = 1.0f / 64.0f;
    const float x0 = (float)(gx * P.gw) - e, x1 = (float)(gx * P.gw + P.gw) + e;
    const float y0 = (float)(P.row0 + pr0 * P.row_step) - e;
    const float y1 = (float)(P.row0 + (pr0 + P.gh - 1) * P.row_step + 1) + e;
    auto D = [&](float cx, float cy) {
        const float a = (cx - 0.5f * c.W) / c.unit, b = (0.5f * c.H - cy) / c.unit;
        return (c.near_ * c.f + a * c.r) + b * c.u;
    };
    gc.k[0] = D(x0, y0); gc.k[1] = D(x1, y0); gc.k[2] = D(x1, y1); gc.k[3] = D(x0, y1);
    const V3 mid = D(0.5f * (x0 + x1), 0.5f * (y0 + y1));
    auto amax = [](V3 v) { return fmaxf(fabsf(v.x), fmaxf(fabsf(v.y), fabsf(v.z))); };
    gc.dmax = fmaxf(fmaxf(amax(gc.k[0]), amax(gc.k[1])), fmaxf(amax(gc.k[2]), amax(gc.k[3])));
    const float tiny = 0x1p-40f * gc.dmax;
    auto near0 = [&](float a, float b, float cc, float d) {
        return fminf(fminf(a, b), fminf(cc, d)) <= tiny && fmaxf(fmaxf(a, b), fmaxf(cc, d)) >= -tiny;
    };
    const V3* k = gc.k;
    if (near0(k[0].x, k[1].x, k[2].x, k[3].x) || near0(k[0].y, k[1].y, k[2].y, k[3].y) || near0(k[0].z, k[1].z, k[2].z, k[3].z))
        return gc;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        gc.n[i] = cross(k[i], k[(i + 1) & 3]);
        if (dot(gc.n[i], mid) < 0.0f) gc.n[i] = neg(gc.n[i]);
    }
    gc.ok = 1;
    return gc;
}
// Whether no ray of the cone meets box [mn, mx] (nd = 0: a degenerate box, never hit), with
// conservative margins: the box grown by 1e-4 of its coordinate scale, separations beyond the
// rays' rounding (1e-5 relative).
__device__ __forceinline__ bool cone_outside(const GroupCone& gc, V3 pos, V3 mn, V3 mx, bool nd) {
    if (!nd) return true;
    auto amax = [](V3 v) { return fmaxf(fabsf(v.x), fmaxf(fabsf(v.y), fabsf(v.z))); };
    const float m = 1e-4f * (fmaxf(amax(mn), amax(mx)) + amax(pos)) + 1e-30f;
    mn = mn - v3(m, m, m); mx = mx + v3(m, m, m);
    // a box face plane: the apex beyond it and every direction pointing away from it by
    // more than the rounding of the computed rays (1e-5 relative)
    const float away = 1e-5f * gc.dmax;
    const V3* k = gc.k;
    auto face = [&](float o, float lo, float hi, float a0, float a1, float a2, float a3) {
        return (o > hi && fminf(fminf(a0, a1), fminf(a2, a3)) >= away) || (o < lo && fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)) <= -away);
    };
    bool sep = face(pos.x, mn.x, mx.x, k[0].x, k[1].x, k[2].x, k[3].x) || face(pos.y, mn.y, mx.y, k[0].y, k[1].y, k[2].y, k[3].y) ||
               face(pos.z, mn.z, mx.z, k[0].z, k[1].z, k[2].z, k[3].z);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const V3 nn = gc.n[i];
        const V3 q = v3(nn.x >= 0.0f ? mx.x : mn.x, nn.y >= 0.0f ? mx.y : mn.y, nn.z >= 0.0f ? mx.z : mn.z) - pos;
        const float sv = dot(nn, q);
        const float tol = 1e-5f * (fabsf(nn.x) + fabsf(nn.y) + fabsf(nn.z)) * (fabsf(q.x) + fabsf(q.y) + fabsf(q.z));
        sep = sep || sv < -tol;
    }
    return sep;
}
__device__ __forceinline__ bool cone_misses_root(const TraceParams& P, const SceneView& S, int g) {
    const DCamera& c = P.cam;
    if (!(c.near_ > 0.0f) || S.n_real < 2) return false;
    const int gy = (int)udiv((unsigned)g, P.div_ngx), gx = g - gy * P.n_gx;
    const int pr0 = gy * P.gh;
    const float e = 1.0f / 64.0f;
    const float x0 = (float)(gx * P.gw) - e, x1 = (float)(gx * P.gw + P.gw) + e;
    const float y0 = (float)(P.row0 + pr0 * P.row_step) - e;
    const float y1 = (float)(P.row0 + (pr0 + P.gh - 1) * P.row_step + 1) + e;
    auto D = [&](float cx, float cy) {
        const float a = (cx - 0.5f * c.W) / c.unit, b = (0.5f * c.H - cy) / c.unit;
        return (c.near_ * c.f + a * c.r) + b * c.u;
    };
    const V3 k0 = D(x0, y0), k1 = D(x1, y0), k2 = D(x1, y1), k3 = D(x0, y1);
    const V3 mid = D(0.5f * (x0 + x1), 0.5f * (y0 + y1));
    auto amax = [](V3 v) { return fmaxf(fabsf(v.x), fmaxf(fabsf(v.y), fabsf(v.z))); };
    const float dmax = fmaxf(fmaxf(amax(k0), amax(k1)), fmaxf(amax(k2), amax(k3)));
    const float tiny = 0x1p-40f * dmax;
    auto near0 = [&](float a, float b, float cc, float d) {
        return fminf(fminf(a, b), fminf(cc, d)) <= tiny && fmaxf(fmaxf(a, b), fmaxf(cc, d)) >= -tiny;
    };
    if (near0(k0.x, k1.x, k2.x, k3.x) || near0(k0.y, k1.y, k2.y, k3.y) || near0(k0.z, k1.z, k2.z, k3.z)) return false;
    V3 n[4] = {cross(k0, k1), cross(k1, k2), cross(k2, k3), cross(k3, k0)};
#pragma unroll
    for (int i = 0; i < 4; i++) if (dot(n[i], mid) < 0.0f) n[i] = neg(n[i]);
    const float4* rec = S.fnode;                               // the root's two children (pair_hit_at)
    const float4 A = rec[0], B = rec[1], C = rec[2];
    auto outside = [&](V3 mn, V3 mx, bool nd) {
        if (!nd) return true;                                  // degenerate: never hit
        const float m = 1e-4f * (fmaxf(amax(mn), amax(mx)) + amax(c.pos)) + 1e-30f;
        mn = mn - v3(m, m, m); mx = mx + v3(m, m, m);
        // a box face plane: the apex beyond it and every direction pointing away from it by
        // more than the rounding of the computed rays (1e-5 relative)
        const float away = 1e-5f * dmax;
        auto face = [&](float o, float lo, float hi, float a0, float a1, float a2, float a3) {
            return (o > hi && fminf(fminf(a0, a1), fminf(a2, a3)) >= away) || (o < lo && fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)) <= -away);
        };
        bool sep = face(c.pos.x, mn.x, mx.x, k0.x, k1.x, k2.x, k3.x) || face(c.pos.y, mn.y, mx.y, k0.y, k1.y, k2.y, k3.y) ||
                   face(c.pos.z, mn.z, mx.z, k0.z, k1.z, k2.z, k3.z);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const V3 q = v3(n[i].x >= 0.0f ? mx.x : mn.x, n[i].y >= 0.0f ? mx.y : mn.y, n[i].z >= 0.0f ? mx.z : mn.z) - c.pos;
            const float sv = dot(n[i], q);
            const float tol = 1e-5f * (fabsf(n[i].x) + fabsf(n[i].y) + fabsf(n[i].z)) * (fabsf(q.x) + fabsf(q.y) + fabsf(q.z));
            sep = sep || sv < -tol;
        }
        return sep;
    };
    return outside(v3(A.x, A.z, B.x), v3(B.z, C.x, C.z), A.x <= B.z) && outside(v3(A.y, A.w, B.y), v3(B.w, C.y, C.w), A.y <= B.w);
}
// Brute-force frames (item 30): whether no ray of the cone comes within the grown slack of
// any instance box.  A ray meets box k grown by A + B t only at times t <= (F + A) / (1 - B), F the
// distance from the camera to the box's farthest corner, so growing the box by
// G = A + B (F + A) / (1 - B), doubled for rounding, covers every such t.
__device__ __forceinline__ bool cone_misses_boxes(const TraceParams& P, int g, const float4* lo, const float4* hi, int nb,
                                                  float A, float B) {
    const GroupCone gc = group_cone(P, g);
    if (!gc.ok) return false;
    const V3 pos = P.cam.pos;
    for (int k = 0; k < nb; k++) {
        const float4 l = lo[k], h = hi[k];
        if (!(l.x <= h.x)) continue;                           // an empty mesh: never hit
        const V3 far = v3(fmaxf(fabsf(l.x - pos.x), fabsf(h.x - pos.x)), fmaxf(fabsf(l.y - pos.y), fabsf(h.y - pos.y)),
                          fmaxf(fabsf(l.z - pos.z), fabsf(h.z - pos.z)));
        const float F = (far.x + far.y) + far.z;               // >= the farthest corner's distance
        const float G = 2.0f * (A + B * (F + A) / (1.0f - B));
        if (!cone_outside(gc, pos, v3(l.x - G, l.y - G, l.z - G), v3(h.x + G, h.y + G, h.z + G), true)) return false;
    }
    return true;
}

// One block of 4 waves per 64 consecutive groups: wave 0 runs the cone test, one group per
// lane; the block writes the outputs of the groups it decided; the 4 waves share the groups it
// left undecided (exact per-ray test, one group per wave step); the block's live groups are
// appended to list (block % NQ) with one atomic.  Small blocks keep ~8 per CU resident: the
// per-ray tests are latency-bound chains (measured: 1024-group blocks, 102 -> 71 us per
// 1080p frame; per-ray tests of every group, 108 us).
#ifndef RT_SKY_WAVES
#define RT_SKY_WAVES 4       // waves per sky_kernel block (64 groups per block)
#endif
constexpr int SKY_THREADS = 64 * RT_SKY_WAVES;
// the heavy-list append runs on threads 64..127 beside the live list's 0..63 (one wave: after it)
constexpr int SKY_HOFF = SKY_THREADS >= 128 ? 64 : 0;
template <bool BRUTE>
// BRUTE: brute-force frames test the instance boxes (mesh box `mbox` + position) grown by
// sky_A + sky_B t instead of a tree's root (grown_box_maybe, cone_misses_boxes)
__global__ __launch_bounds__(SKY_THREADS) void sky_kernel(TraceParams P, SceneView S, unsigned char* gsky, int* live,
                                                          const Box* mbox, float sky_A, float sky_B) {
    __shared__ unsigned long long s_sky, s_todo;
    __shared__ int s_cnt, s_base, s_list[64];
    __shared__ int s_hcnt, s_hbase, s_hlist[64];               // hist = 2: last frame's heavy groups
    // sky_brute: the instance boxes (2 KB); the tree's pass keeps its LDS footprint without them
    struct Boxes { float4 lo[BRUTE ? 64 : 1], hi[BRUTE ? 64 : 1]; };
    __shared__ Boxes s_bx;
    float4* const s_blo = s_bx.lo;
    float4* const s_bhi = s_bx.hi;
    const bool h2 = P.hist == 2;
    constexpr bool brute = BRUTE;
    int nb = 0;
    if (brute) {                                               // (uniform) instance k's box: mesh box + position
        nb = S.n_inst;
        if ((int)threadIdx.x < nb) {
            const float4 I = S.inst4[threadIdx.x];
            const Box mb = mbox[__float_as_int(I.w) & 0x7fffffff];
            s_blo[threadIdx.x] = mb.nd ? make_float4(mb.mn.x + I.x, mb.mn.y + I.y, mb.mn.z + I.z, 0.0f)
                                       : make_float4(INFINITY, INFINITY, INFINITY, 0.0f);   // empty mesh: no hit
            s_bhi[threadIdx.x] = mb.nd ? make_float4(mb.mx.x + I.x, mb.mx.y + I.y, mb.mx.z + I.z, 0.0f)
                                       : make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
        }
        __syncthreads();
    }
    // does ray r (when act) possibly hit anything: the tree's root (the traversal's first step)
    // or, in brute-force frames, some instance's grown box
    auto root_hit = [&](bool act, const Ray& r) {
        if constexpr (!BRUTE) {
            BvhRefs bv{};
            bv.fnode = S.fnode;
            return ft_root_hit(S, bv, act, r);
        }
        if (!act) return false;
        const float A = 2.0f * sky_A, B = sky_B;
        for (int k = 0; k < nb; k++)
            if (s_blo[k].x <= s_bhi[k].x && grown_box_maybe(s_blo[k], s_bhi[k], A, B, r)) return true;
        return false;
    };
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, L = P.lanes_per_px;
    const int base = blockIdx.x * 64;
    const int n_in = min(64, P.n_groups - base);
    if (wv == 0) {
        const int gl = base + lane;
        const bool in = lane < n_in;
        const bool csky = in && (brute ? cone_misses_boxes(P, gl, s_blo, s_bhi, nb, 2.0f * sky_A, sky_B)
                                       : cone_misses_root(P, S, gl));
        // Representative ray: a group the cone test leaves undecided is live as
        // soon as one of its primaries enters the root -- lane 0's (pixel 0, sample 0), the
        // trace kernel's own ray and test -- so only the groups whose representative misses
        // need the 64-ray test below.  One group per lane here.
        bool rlive = false;
        if (in && !csky) {
            const int gy = (int)udiv((unsigned)gl, P.div_ngx), gx = gl - gy * P.n_gx;
            const float2 o = spp_offset_dev(0);
            const Ray rr = camera_at(P.cam, (float)(gx * P.gw) + o.x, (float)(P.row0 + gy * P.gh * P.row_step) + o.y);
            rlive = root_hit(true, rr);
        }
        const unsigned long long m = __ballot(csky), t = __ballot(in && !csky && !rlive);
        if (csky) {
            gsky[gl] = 1;
            // the trace kernel records (hf_next) only the groups it runs: a sky group's entry
            // must not keep a heavy flag from the frame that last wrote this buffer
            if (P.hist == 1) P.hf_next[gl] = 0;
        }
        if (lane == 0) { s_sky = m; s_todo = t; s_cnt = 0; s_hcnt = 0; }
        if (rlive) gsky[gl] = 0;
        // hist = 2: a live group the previous frame found heavy goes on the heavy list instead
        const bool hv = rlive && h2 && P.hf_prev[gl];
        const unsigned long long rl = __ballot(rlive && !hv), hl = __ballot(hv);
        if (rl) {                                              // live already: into the block's list
            const int pos = __popcll(rl & ((1ull << lane) - 1ull));
            if (rlive && !hv) s_list[pos] = gl;
            if (lane == 0) s_cnt = __popcll(rl);
        }
        if (hl) {
            const int pos = __popcll(hl & ((1ull << lane) - 1ull));
            if (hv) s_hlist[pos] = gl;
            if (lane == 0) s_hcnt = __popcll(hl);
        }
    }
    __syncthreads();
    if (h2 && (int)threadIdx.x < n_in) P.hf_next[base + threadIdx.x] = 0;   // this frame records afresh
    auto sky_pixel = [&](int g, int pix) {                     // pixel pix of sky group g: zeros, -1 hit ids
        const int gy = (int)udiv((unsigned)g, P.div_ngx), gx = g - gy * P.n_gx;
        const int qx = P.gw_shift >= 0 ? pix & (P.gw - 1) : pix % P.gw;
        const int qy = P.gw_shift >= 0 ? pix >> P.gw_shift : pix / P.gw;
        const int px = gx * P.gw + qx, pr = gy * P.gh + qy;
        if (!(px < P.W && pr < P.n_rows)) return;
        const int pix_index = P.compact ? pr * P.W + px : (P.row0 + pr * P.row_step) * P.W + px;
        if (P.hit_inst) P.hit_inst[pix_index] = -1;
        if (P.hit_tri) P.hit_tri[pix_index] = -1;
        if (P.rgba) P.rgba[pix_index] = 0u;                   // to_encoding of Color(0, 0, 0, 0)
        if (P.radiance) P.radiance[pix_index] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    };
    const unsigned long long skym = s_sky;
    if (skym)
        for (int i = threadIdx.x; i < 64 * P.px_per_wave; i += SKY_THREADS) {
            const int gi = i / P.px_per_wave;
            if ((skym >> gi) & 1) sky_pixel(base + gi, i - gi * P.px_per_wave);
        }
    // undecided groups: the exact per-ray root test, waves taking every 4th
    const int pix_g = P.l_shift >= 0 ? lane >> P.l_shift : lane / L;
    const int sub_g = lane - pix_g * L;
    const int pxo = P.gw_shift >= 0 ? pix_g & (P.gw - 1) : pix_g % P.gw;
    const int pyo = P.gw_shift >= 0 ? pix_g >> P.gw_shift : pix_g / P.gw;
    const bool lane_ok = pix_g < P.px_per_wave && sub_g < P.spp;   // k = sub_g (spp <= 64: one round)
    unsigned long long todo = s_todo;
    for (int k = 0; todo; k++) {
        const int bit = __builtin_ctzll(todo);
        todo &= todo - 1;
        if ((k % RT_SKY_WAVES) != wv) continue;
        const int g = base + bit;
        const int gy = (int)udiv((unsigned)g, P.div_ngx), gx = g - gy * P.n_gx;
        const int px = gx * P.gw + pxo, pr = gy * P.gh + pyo;
        const bool valid = pix_g < P.px_per_wave && px < P.W && pr < P.n_rows;
        const int py = P.row0 + pr * P.row_step;
        const bool act = valid && lane_ok;
        Ray r0{v3(0, 0, 0), v3(0, 0, 1)};
        if (act) {
            const float2 o = spp_offset_dev(sub_g);            // the trace kernel's own offsets
            r0 = camera_at(P.cam, (float)px + o.x, (float)py + o.y);
        }
        const bool sky = __ballot(root_hit(act, r0)) == 0;
        if (lane == 0) {
            gsky[g] = sky ? 1 : 0;
            if (sky && P.hist == 1) P.hf_next[g] = 0;
            if (!sky) {
                if (h2 && P.hf_prev[g]) s_hlist[atomicAdd(&s_hcnt, 1)] = g;
                else s_list[atomicAdd(&s_cnt, 1)] = g;
            }
        }
        if (sky && valid && sub_g == 0) sky_pixel(g, pix_g);
    }
    __syncthreads();
    const int q = blockIdx.x % NQ, n = s_cnt, nh = s_hcnt;
    if (n == 0 && nh == 0) return;
    if (threadIdx.x == 0 && n) s_base = atomicAdd(&P.work[16 * (NQ + 1 + q)], n);
    if ((int)threadIdx.x == SKY_HOFF + (SKY_HOFF ? 0 : 1) && nh) s_hbase = atomicAdd(&P.work[WORK_HEAVY_LEN], nh);
    __syncthreads();
    if ((int)threadIdx.x < n) live[q * P.live_cap + s_base + threadIdx.x] = s_list[threadIdx.x];
    if ((int)threadIdx.x >= SKY_HOFF && (int)threadIdx.x < SKY_HOFF + nh)   // heavy list after the NQ lists
        live[NQ * P.live_cap + s_hbase + threadIdx.x - SKY_HOFF] = s_hlist[threadIdx.x - SKY_HOFF];
}

// ---------------------------------------------------------------------------
// BVH build: ropt::gpu::BVH::BVH (bvh.cu:74-91) + create_boxes (raytracer.cu:54-74)
// in one workgroup.  Output: heap-ordered nodes[1 .. 2n-1].
// ---------------------------------------------------------------------------
template <bool LDS_TREE>
__global__ __launch_bounds__(1024) void bvh_build_kernel(BvhArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);
    int* idx = reinterpret_cast<int*>(smem + sizeof(unsigned long long) * A.n);
    TreeStore<LDS_TREE> tree;
    if constexpr (LDS_TREE) { tree.f = reinterpret_cast<float*>(smem + 12 * (size_t)A.n); tree.cap = 2 * A.n - 1; }
    else tree.t = A.tree;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int n = A.n;
    for (int i = tid; i < A.n_work; i += nt) A.work[i] = 0;
    if (A.hctl && tid < 2) A.hctl[tid] = 0;

    // instance boxes (create_boxes, raytracer.cu:54-74: from_local of the mesh box) and
    // Morton keys (gen_morton, bvh.cu:20-32); padding is degenerate -> ULONG_MAX
    auto inst_box = [&](int i) { return bvh_inst_box(A, i); };
    for (int i = tid; i < n; i += nt) {
        keys[i] = bvh_key(inst_box(i));
        idx[i] = i;
    }
    __syncthreads();
    // Sort on (key, index): identical order to a stable sort by key (thrust sort_by_key,
    // bvh.cu:86).  Entries [n_inst, n) are padding with key ~0 and the largest indices, so
    // they already sit at their rank; only [0, n_inst) moves.
    const int m = A.n_inst, nch = (m + 63) >> 6;
    bool sorted = false;
    if constexpr (LDS_TREE) {
        if (n >= 64 && nch * 64 <= nt) {
            // Chunked rank sort: wave w sorts entries [64w, 64w + 64) in registers (bitonic
            // network over lanes), then each entry's rank = its lane + its rank in every other
            // sorted chunk (branchless binary search in LDS).  Earlier chunks hold smaller
            // indices, so equal keys count there (<=) and not in later chunks (<).  Three
            // barriers instead of the bitonic network's 20 LDS phases.  The sorted chunks are
            // staged in the tree's LDS region (8 * 64 * nch <= 8n < 28 (2n - 1) bytes).
            unsigned long long* S = reinterpret_cast<unsigned long long*>(smem + 12 * (size_t)n);
            const int lane = tid & 63, c = tid >> 6;
            unsigned long long k = ~0ull;
            int x = tid;
            if (tid < nch * 64) {                                  // whole waves
                if (tid < m) k = keys[tid];
                for (int size = 2; size <= 64; size <<= 1) {
                    const bool up = (lane & size) == 0;
                    for (int st = size >> 1; st > 0; st >>= 1) {
                        const unsigned lo = __shfl_xor((unsigned)k, st), hi = __shfl_xor((unsigned)(k >> 32), st);
                        const unsigned long long pk = ((unsigned long long)hi << 32) | lo;
                        const int px = __shfl_xor(x, st);
                        const bool mine_less = k < pk || (k == pk && x < px);
                        if (mine_less != (((lane & st) == 0) == up)) { k = pk; x = px; }
                    }
                }
                S[tid] = k;
            }
            __syncthreads();
            int pos = lane;
            if (tid < m) {
                for (int cb = 0; cb < nch; cb += 4) {              // four independent searches in flight
                    int p4[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int sp = 32; sp >= 1; sp >>= 1) {
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const int cc = cb + u;
                            if (cc < nch && cc != c) {
                                const unsigned long long v = S[(cc << 6) + p4[u] + sp - 1];
                                if (cc < c ? v <= k : v < k) p4[u] += sp;
                            }
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int cc = cb + u;
                        if (cc < nch && cc != c) {
                            const unsigned long long v = S[(cc << 6) + 63];
                            pos += p4[u] + (p4[u] == 63 && (cc < c ? v <= k : v < k));
                        }
                    }
                }
            }
            __syncthreads();
            if (tid < m) { keys[pos] = k; idx[pos] = x; }
            __syncthreads();
            sorted = true;
        }
    }
    // bitonic sort on (key, index) otherwise.  Strides >= 64 exchange through the LDS; the
    // strides below 64 of each merge run in registers within the wave (lane ^ stride), one
    // LDS round trip and barrier per merge instead of per stride.
    for (int size = 2; size <= n && !sorted; size <<= 1) {
        int stride = size >> 1;
        for (; stride >= 64 || (n < 64 && stride > 0); stride >>= 1) {
            for (int i = tid; i < n; i += nt) {
                int j = i ^ stride;
                if (j > i) {
                    bool up = (i & size) == 0;
                    unsigned long long ki = keys[i], kj = keys[j];
                    int ii = idx[i], ij = idx[j];
                    bool gt = (ki > kj) || (ki == kj && ii > ij);
                    if (gt == up) { keys[i] = kj; keys[j] = ki; idx[i] = ij; idx[j] = ii; }
                }
            }
            __syncthreads();
        }
        if (stride > 0) {                                      // n >= 64: whole waves in range
            for (int i = tid; i < n; i += nt) {
                unsigned long long k = keys[i];
                int x = idx[i];
                const bool up = (i & size) == 0;
                for (int st = stride; st > 0; st >>= 1) {
                    const unsigned lo = __shfl_xor((unsigned)k, st), hi = __shfl_xor((unsigned)(k >> 32), st);
                    const unsigned long long pk = ((unsigned long long)hi << 32) | lo;
                    const int px = __shfl_xor(x, st);
                    const bool mine_less = k < pk || (k == pk && x < px);
                    if (mine_less != (((i & st) == 0) == up)) { k = pk; x = px; }   // lower lane keeps min iff up
                }
                keys[i] = k; idx[i] = x;
            }
            __syncthreads();
        }
    }
    // reorder (bvh.cu:34-41: the box is recomputed, same arithmetic) and pairwise level
    // merges (bvh.cu:43-61)
    for (int i = tid; i < n; i += nt) tree.put(i, inst_box(idx[i]));
    __syncthreads();
    {
        int lvl = 0, size = n, out = n;
        while (size >= 2) {
            for (int i = tid; i < size / 2; i += nt) tree.put(out + i, merge(tree.get(lvl + 2 * i), tree.get(lvl + 2 * i + 1)));
            __syncthreads();
            lvl += size; out += size / 2; size >>= 1;
        }
    }
    for (int k = tid; k < 2 * n; k += nt) bvh_heap_node(A, idx, tree, k);
    for (int i = tid; i < A.n_real - 1; i += nt) bvh_fnode(A, keys, idx, tree, i);
}

// ---------------------------------------------------------------------------
// Device KAT kernel (test hook): the same inline functions the trace kernel uses.
// ---------------------------------------------------------------------------
__global__ void kat_kernel(int op, int n, const float* a, const float* b, const float* c, float* of, int* oi,
                           unsigned long long* ou) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    auto L3 = [](const float* p) { return v3(p[0], p[1], p[2]); };
    auto S3 = [](float* p, V3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; };
    switch (op) {
        case 0: S3(of + 3 * i, normalized(L3(a + 3 * i))); break;
        case 1: S3(of + 3 * i, cross(L3(a + 3 * i), L3(b + 3 * i))); break;
        case 2: S3(of + 3 * i, reflect(L3(a + 3 * i), L3(b + 3 * i))); break;
        case 3: { bool t; S3(of + 3 * i, refract(L3(a + 3 * i), L3(b + 3 * i), c[2 * i], c[2 * i + 1], t)); oi[i] = t; break; }
        case 4: {
            Q q{a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]};
            Pose e{};  // exercise the same Pose path the kernels use (incl. the identity specialisation)
            e.identity = (__float_as_uint(q.i) == 0u && __float_as_uint(q.j) == 0u && __float_as_uint(q.k) == 0u &&
                          __float_as_uint(q.r) == 0x3f800000u);
            e.tn = qnormalized(q); e.ti = qinverse(q);
            S3(of + 3 * i, vec_to_local(e, L3(b + 3 * i)));
            break;
        }
        case 5: { Q r = qinverse(Q{a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]}); of[4 * i] = r.i; of[4 * i + 1] = r.j; of[4 * i + 2] = r.k; of[4 * i + 3] = r.r; break; }
        case 6: {
            Q r = qmul(Q{a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]}, Q{b[4 * i], b[4 * i + 1], b[4 * i + 2], b[4 * i + 3]});
            of[4 * i] = r.i; of[4 * i + 1] = r.j; of[4 * i + 2] = r.k; of[4 * i + 3] = r.r; break;
        }
        case 7: {
            const float* t = a + 9 * i;
            V3 A = L3(t), B = L3(t + 3), C = L3(t + 6);
            V3 pn = cross(B - A, C - A);
            Ray r = make_ray(L3(b + 6 * i), L3(b + 6 * i + 3));
            float tm = NAN, u = NAN, v = NAN;
            bool h = tri_hit(A, B, C, normalized(pn), len(pn), r, tm, u, v);
            oi[i] = h; of[3 * i] = h ? tm : NAN; of[3 * i + 1] = h ? u : NAN; of[3 * i + 2] = h ? v : NAN;
            break;
        }
        case 8: { Ray r = make_ray(L3(a + 6 * i), L3(a + 6 * i + 3)); S3(of + 6 * i, r.o); S3(of + 6 * i + 3, r.d); break; }
        case 9: ou[i] = z_order(L3(a + 3 * i)); break;
        case 10: { float m[3][3]; to_mat3(Q{a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]}, m);
                   for (int x = 0; x < 9; x++) of[9 * i + x] = m[x / 3][x % 3]; break; }
        case 11: {
            const float* bx = a + 7 * i;
            Ray r = make_ray(L3(b + 6 * i), L3(b + 6 * i + 3));
            oi[i] = bx[6] != 0 && box_hit(L3(bx), L3(bx + 3), r);
            break;
        }
        case 12: of[i] = pow_ref(a[i], b[i]); break;
        case 13: {   // filtered triangle test (best = +inf): must equal the exact test bit for bit
            const float* t = a + 9 * i;
            V3 A = L3(t), B = L3(t + 3), C = L3(t + 6);
            V3 pn = cross(B - A, C - A);
            float area = len(pn);
            Ray r = make_ray(L3(b + 6 * i), L3(b + 6 * i + 3));
            float tm = NAN, u = NAN, v = NAN;
            bool h = tri_accept_f(A, B, C, normalized(pn), area, 1.0f / area, r, INFINITY, tm, u, v);
            oi[i] = h; of[3 * i] = h ? tm : NAN; of[3 * i + 1] = h ? u : NAN; of[3 * i + 2] = h ? v : NAN;
            break;
        }
        case 14: {   // filtered box test
            const float* bx = a + 7 * i;
            Ray r = make_ray(L3(b + 6 * i), L3(b + 6 * i + 3));
            oi[i] = bx[6] != 0 && box_hit_f(L3(bx), L3(bx + 3), r, ray_inv(r));
            break;
        }
        case 18: case 19: {   // box_from_local (create_boxes' from_local) / box_merge (the level merges)
            const float* x = a + 7 * i;
            const float* y = b + 7 * i;
            Box bx; bx.mn = L3(x); bx.mx = L3(x + 3); bx.nd = x[6] != 0;
            Box r;
            if (op == 18) {
                const Q o{y[0], y[1], y[2], y[3]};
                Pose e;
                e.p = L3(y + 4);
                e.identity = __float_as_uint(o.i) == 0u && __float_as_uint(o.j) == 0u && __float_as_uint(o.k) == 0u &&
                             __float_as_uint(o.r) == 0x3f800000u;
                e.tn = qnormalized(o); e.ti = qinverse(o);
                const Q inv = qinverse(o);
                e.fn = qnormalized(inv); e.fi = qinverse(inv);
                r = from_local(bx, e);
            } else {
                Box by; by.mn = L3(y); by.mx = L3(y + 3); by.nd = y[6] != 0;
                r = merge(bx, by);
            }
            S3(of + 6 * i, r.mn); S3(of + 6 * i + 3, r.mx); oi[i] = r.nd ? 1 : 0;
            break;
        }
        case 20: {   // entity pose transforms (cast_local / Hitable::hit pose chain)
            const float* y = a + 7 * i;
            const Q o{y[0], y[1], y[2], y[3]};
            Pose e;
            e.p = L3(y + 4);
            e.identity = __float_as_uint(o.i) == 0u && __float_as_uint(o.j) == 0u && __float_as_uint(o.k) == 0u &&
                         __float_as_uint(o.r) == 0x3f800000u;
            e.tn = qnormalized(o); e.ti = qinverse(o);
            const Q inv = qinverse(o);
            e.fn = qnormalized(inv); e.fi = qinverse(inv);
            const V3 v = L3(b + 3 * i);
            S3(of + 12 * i, point_to_local(e, v)); S3(of + 12 * i + 3, vec_to_local(e, v));
            S3(of + 12 * i + 6, point_from_local(e, v)); S3(of + 12 * i + 9, vec_from_local(e, v));
            break;
        }
        case 16: of[i] = rcp_cr(a[i]); break;                   // device CR reciprocal (rt_math.h)
        case 17: of[i] = sqrt_cr(a[i]); break;                  // device CR sqrt
        case 15: {   // packed child-pair box test (pair_hit): two boxes (mn, mx, nd) x 2 vs one ray
            const float* bx = a + 14 * i;
            float q[12];
            for (int c = 0; c < 2; c++) {
                const float* x = bx + 7 * c;
                const bool nd = x[6] != 0;
                for (int j = 0; j < 3; j++) {
                    q[2 * j + c] = nd ? x[j] : INFINITY;
                    q[6 + 2 * j + c] = nd ? x[3 + j] : -INFINITY;
                }
            }
            const float4 np[3] = {make_float4(q[0], q[1], q[2], q[3]), make_float4(q[4], q[5], q[6], q[7]),
                                  make_float4(q[8], q[9], q[10], q[11])};
            Ray r = make_ray(L3(b + 6 * i), L3(b + 6 * i + 3));
            bool h0, h1;
            float t0, t1;
            pair_hit(np, 0, r, ray_inv(r), true, h0, h1, t0, t1);
            oi[2 * i] = h0; oi[2 * i + 1] = h1;
            break;
        }
        default: break;
    }
}

}  // namespace

// ===========================================================================
// Host side: scene object and the C ABI
// ===========================================================================
struct MultiDev;
// Host framebuffer in pinned memory: rt_update_scene's device-to-host copy of the frame (the
// reference's post-condition, raytracer.cu:102-120) is then one direct transfer; into pageable
// memory HIP stages it in chunks through a bounce buffer.  Pageable fallback when pinning fails
// (no HIP device: the scene is still built and exported, nothing is rendered).
struct HostCanvas {
    uint32_t* p = nullptr;
    size_t n = 0;
    bool pinned = false;
    HostCanvas() = default;
    HostCanvas(const HostCanvas&) = delete;
    HostCanvas& operator=(const HostCanvas&) = delete;
    ~HostCanvas() { release(); }
    void release() {
        if (p) { if (pinned) (void)hipHostFree(p); else free(p); }
        p = nullptr; n = 0; pinned = false;
    }
    void assign(size_t m, uint32_t v) {
        release();
        if (!m) return;
        if (hipHostMalloc((void**)&p, m * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess) {
            pinned = true;
        } else {
            (void)hipGetLastError();
            p = static_cast<uint32_t*>(malloc(m * sizeof(uint32_t)));
            if (!p) return;
        }
        n = m;
        std::fill(p, p + m, v);
    }
    uint32_t* data() { return p; }
    const uint32_t* data() const { return p; }
    size_t size() const { return n; }
    uint32_t operator[](size_t i) const { return p[i]; }
};

struct rt_scene {
    rt::Scene h;
    MultiDev* multi = nullptr;                   // rt_scene_set_devices: frames split over several GPUs
    bool finished = false;
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // device buffers
    DTri* d_tris = nullptr; DMesh* d_meshes = nullptr; DInst* d_insts = nullptr; DMat* d_mats = nullptr;
    DLight* d_lights = nullptr; Box* d_mesh_box = nullptr; Box* d_tree = nullptr;
    float4* d_node_pair = nullptr; int* d_leaf = nullptr;
    float4* d_fnode = nullptr; int n_real = 0, fdepth = 0;   // ordered LBVH (fast kernel)
    void* d_bscratch = nullptr;                  // bvh_build_large's sort buffers (scenes above BVH_WG_LEAVES)
    float4* d_inst4 = nullptr;
    TriAx* d_tri_ax = nullptr;                   // axis-plane triangle records (tri_axis_records)
    int* d_work = nullptr; int n_cu = 0;
    bool work_zeroed = false;                    // bvh_build_kernel zeroed d_work for the next trace launch
    // longest-first scheduling history (TraceParams::hist): double-buffered by frame parity
    int* d_hlist[2] = {nullptr, nullptr};
    unsigned char* d_hflag[2] = {nullptr, nullptr};
    unsigned long long* d_hctl = nullptr;        // [2][count, sum]
    int hist_cap = 0, hist_parity = 0;
    int hctl_zeroed = -1;                        // heavy-list slot the pending bvh_build_kernel zeroes (-1: none)
    long long hist_key[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    unsigned char* d_gsky = nullptr; int gsky_cap = 0;   // sky pre-pass flags (TraceParams::gsky)
    int* d_live = nullptr; int live_cap = 0;             // sky pre-pass live-group lists [NQ][live_cap]
    float2* d_spp = nullptr; int spp_cap = 0;
    unsigned long long* d_stats = nullptr;
    uint32_t* d_canvas = nullptr;
    int* d_dbg = nullptr;
    float4* d_atlas = nullptr;                   // atlas texels (float4, byte / 255)
    bool atlas_dirty = false;
    void* d_out[4] = {nullptr, nullptr, nullptr, nullptr};   // staging for host_outputs
    std::vector<hipEvent_t> tev;      // timing=1 events, 4 per frame: bvh start/stop, trace start/stop (pool)
    size_t tev_used = 0;
    size_t d_out_px = 0;
    int n_leaf = 0;
    bool uploaded = false, bvh_valid = false;
    HostCanvas canvas;               // host framebuffer (Canvas buffer, canvas.cu:7), pinned
    // Frame slots (rt_scene_set_frame_slots): with n > 1 slots, consecutive frames rotate
    // through n copies of the per-frame state (BVH, work counters, scheduling history), so a
    // frame on another stream can start on CUs freed by the previous frames' tails.  The
    // fields above always hold the current slot; store[i] the others (store[cur] is stale).
    // Instance arrays are per-slot state too (rt_builder_set_trans after finish): a frame in
    // flight keeps the poses its BVH was built from, and the next frame of a slot receives the
    // current poses by a stream-ordered copy (sync_slot_insts) from the slot's pinned staging.
    DInst* h_insts_pin = nullptr; float4* h_inst4_pin = nullptr;   // current slot's staging (pinned)
#ifndef RT_OVERLAP_DEFAULT
#define RT_OVERLAP_DEFAULT RT_OVERLAP_HALF   // (RT_OVERLAP_FULL: the A/B arm of round 3's policy)
#endif
    int overlap = RT_OVERLAP_DEFAULT;                                // rt_scene_set_overlap
    int ranks_per_device = 1;                    // > 1: virtual ranks of rt_scene_set_devices share this device
    unsigned slot_inst_gen = 0;                  // instance generation the current slot's arrays hold
    unsigned inst_gen = 1;                       // generation of the host instance array (set_trans bumps it)
    unsigned shape_gen = 0;                      // generation n_real / fdepth were computed for
#ifndef RT_MAX_SLOTS
#define RT_MAX_SLOTS 8
#endif
    static constexpr int MAX_SLOTS = RT_MAX_SLOTS;
    struct Slot {
        Box* d_tree = nullptr; float4* d_node_pair = nullptr; int* d_leaf = nullptr; float4* d_fnode = nullptr;
        void* d_bscratch = nullptr;
        int* d_work = nullptr; bool work_zeroed = false, bvh_valid = false;
        int* d_hlist[2] = {nullptr, nullptr}; unsigned char* d_hflag[2] = {nullptr, nullptr};
        unsigned long long* d_hctl = nullptr;
        int hist_cap = 0, hist_parity = 0, hctl_zeroed = -1;
        long long hist_key[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
        unsigned char* d_gsky = nullptr; int gsky_cap = 0;
        int* d_live = nullptr; int live_cap = 0;
        DInst* d_insts = nullptr; float4* d_inst4 = nullptr;
        DInst* h_insts_pin = nullptr; float4* h_inst4_pin = nullptr;
        unsigned slot_inst_gen = 0;
    } store[MAX_SLOTS];
    int n_slots = 1, cur_slot = 0;
    // Last frame of each slot (recorded on its stream, also with one slot): the next frame of
    // the slot, and side entries (debug_cast, experiments), wait for it stream-ordered.
    hipEvent_t slot_done[MAX_SLOTS] = {};
    bool slot_pending[MAX_SLOTS] = {};
    ~rt_scene();
};

// Move the current per-frame state into store[cur_slot] and load slot i's.
void select_slot(rt_scene* s, int i) {
    if (i == s->cur_slot) return;
    auto xfer = [](auto& a, auto& b) { a = b; };
    auto move = [&](rt_scene::Slot& o, bool save) {
        auto f = [&](auto& field, auto& slot) { if (save) xfer(slot, field); else xfer(field, slot); };
        f(s->d_tree, o.d_tree); f(s->d_node_pair, o.d_node_pair); f(s->d_leaf, o.d_leaf); f(s->d_fnode, o.d_fnode);
        f(s->d_bscratch, o.d_bscratch);
        f(s->d_work, o.d_work); f(s->work_zeroed, o.work_zeroed); f(s->bvh_valid, o.bvh_valid);
        for (int p = 0; p < 2; p++) { f(s->d_hlist[p], o.d_hlist[p]); f(s->d_hflag[p], o.d_hflag[p]); }
        f(s->d_hctl, o.d_hctl); f(s->hist_cap, o.hist_cap); f(s->hist_parity, o.hist_parity);
        f(s->hctl_zeroed, o.hctl_zeroed);
        for (int k = 0; k < 8; k++) f(s->hist_key[k], o.hist_key[k]);
        f(s->d_gsky, o.d_gsky); f(s->gsky_cap, o.gsky_cap); f(s->d_live, o.d_live); f(s->live_cap, o.live_cap);
        f(s->d_insts, o.d_insts); f(s->d_inst4, o.d_inst4);
        f(s->h_insts_pin, o.h_insts_pin); f(s->h_inst4_pin, o.h_inst4_pin);
        f(s->slot_inst_gen, o.slot_inst_gen);
    };
    move(s->store[s->cur_slot], true);
    move(s->store[i], false);
    s->cur_slot = i;
}

namespace {
thread_local std::string g_err;
thread_local int g_device = 0;

int fail(int code, const std::string& msg) { g_err = msg; return code; }
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return fail(RT_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); } while (0)

template <class T> void dfree(T*& p) { if (p) { (void)hipFree(p); p = nullptr; } }

int padded(int n_t) {   // raytracer.cu:79: 1 << ceil(log2(n))
    if (n_t <= 0) return 0;
    int n = 1;
    while (n < n_t) n <<= 1;
    return n;
}

int upload_inst4(rt_scene* s);
int ensure_other_slot(rt_scene* s);
int mirror_slot_caps(rt_scene* s);

// TriAx records (rt_math.h) of the axis-plane triangle path: axis, plane coordinate,
// shared-plane flag and the in-plane reject box with its host-checked error bound.
std::vector<TriAx> tri_axis_records(const rt::Scene& h) {
    const double u = 0x1p-24;
    std::vector<TriAx> out(h.d_tris.size());
    auto c3 = [](V3 v, int a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; };
    for (size_t i = 0; i < h.d_tris.size(); i++) {
        const DTri& T = h.d_tris[i];
        TriAx x{};
        x.code = 3;
        int ax = -1, zeros = 0;
        for (int a = 0; a < 3; a++) {
            const float c = c3(T.pn, a);
            if (c == 0.0f) zeros++;                          // +0 or -0
            else if (c == 1.0f || c == -1.0f) ax = a;
        }
        if (zeros == 2 && ax >= 0 && c3(T.b, ax) == c3(T.a, ax) && c3(T.c, ax) == c3(T.a, ax)) {
            x.code = ax;
            x.a_ax = c3(T.a, ax);
            const int au = (ax + 1) % 3, av = (ax + 2) % 3;
            const V3 P[3] = {T.a, T.b, T.c};
            double D = 0, lo[2] = {INFINITY, INFINITY}, hi[2] = {-INFINITY, -INFINITY};
            for (int k = 0; k < 3; k++) {
                const V3 p = P[k], q = P[(k + 1) % 3];
                const double dx = (double)p.x - q.x, dy = (double)p.y - q.y, dz = (double)p.z - q.z;
                D = std::max(D, std::sqrt(dx * dx + dy * dy + dz * dz));
                const double pc[2] = {c3(p, au), c3(p, av)};
                for (int j = 0; j < 2; j++) { lo[j] = std::min(lo[j], pc[j]); hi[j] = std::max(hi[j], pc[j]); }
            }
            // exact (double) doubled area vs the stored float area
            const double e1[3] = {(double)T.b.x - T.a.x, (double)T.b.y - T.a.y, (double)T.b.z - T.a.z};
            const double e2[3] = {(double)T.c.x - T.a.x, (double)T.c.y - T.a.y, (double)T.c.z - T.a.z};
            const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
            const double A = std::sqrt(cx * cx + cy * cy + cz * cz);
            const double m = 1e-4 * D, win = 1e3 * D, off = m;
            bool ok = A > 0 && D > 0 && std::isfinite(A) && std::isfinite(D) && std::isfinite(win);
            if (ok) {
                const double eta = std::fabs((double)T.area - A) / A + 1e-12;
                auto margin = [&](double e) {
                    return (e / D) * (1 - 5.6 * u - eta) - (5.6 * u + eta) - 41.8 * u * (D + e + off) * (D + e + off) / A - 1.01e-5;
                };
                ok = margin(m) > 0 && margin(win) > 0;
            }
            if (ok) {
                // bounds rounded outwards to float
                x.ulo = std::nextafter((float)(lo[0] - m), -INFINITY); x.uhi = std::nextafter((float)(hi[0] + m), INFINITY);
                x.vlo = std::nextafter((float)(lo[1] - m), -INFINITY); x.vhi = std::nextafter((float)(hi[1] + m), INFINITY);
                x.win = std::nextafter((float)win, 0.0f);
                x.off = std::nextafter((float)off, 0.0f);
                x.code |= 8;
            }
        }
        out[i] = x;
    }
    // shared plane with the next triangle of the same mesh
    for (const DMesh& M : h.d_meshes)
        for (int t = M.tri_begin; t + 1 < M.tri_begin + M.tri_count; t++) {
            const TriAx &x = out[t], &y = out[t + 1];
            if ((x.code & 3) != 3 && (x.code & 3) == (y.code & 3)) {
                uint32_t bx, by;
                memcpy(&bx, &x.a_ax, 4); memcpy(&by, &y.a_ax, 4);
                if (bx == by) out[t].code |= 4;
            }
        }
    return out;
}

// Leaf count and depth (internal nodes on the longest root-leaf path) of the ordered
// LBVH bvh_build_kernel will build: the same box, Morton and sort arithmetic on the
// host (RT_HD functions).  The fast traversal's stack holds <= FT_MAX_DEPTH entries.
constexpr int FT_MAX_DEPTH = 31;
// Mesh boxes: Trimesh::compute_bounding_box (trimesh.cu:21-32, sequential fit order) and
// the mesh pose.  They depend only on the immutable mesh data, so they are computed once
// here; the per-frame build (bvh_build_kernel) redoes everything per instance.
std::vector<Box> mesh_boxes(const rt::Scene& h) {
    std::vector<Box> mbox(h.d_meshes.size());
    for (size_t m = 0; m < h.d_meshes.size(); m++) {
        Box b; b.nd = 0; b.mn = b.mx = v3(0, 0, 0);
        const DMesh& mesh = h.d_meshes[m];
        for (int t = mesh.tri_begin; t < mesh.tri_begin + mesh.tri_count; t++) {
            fit_vertex(b, h.d_tris[t].a); fit_vertex(b, h.d_tris[t].b); fit_vertex(b, h.d_tris[t].c);
        }
        mbox[m] = from_local(b, mesh.pose);
    }
    return mbox;
}
// n_real and the deepest internal node's depth (root = 1).
void ordered_tree_shape(const rt::Scene& h, int* n_real, int* depth) {
    const std::vector<Box> mbox = mesh_boxes(h);
    std::vector<std::pair<unsigned long long, int>> kv;
    bool ordered = true;                                      // every real box finite with mn <= mx
    for (size_t i = 0; i < h.d_insts.size(); i++) {
        const Box b = from_local(mbox[h.d_insts[i].mesh], h.d_insts[i].pose);
        if (b.nd) {
            kv.push_back({z_order(neg(box_center(b))), (int)i});
            const float c[6] = {b.mn.x, b.mn.y, b.mn.z, b.mx.x, b.mx.y, b.mx.z};
            for (float x : c) ordered = ordered && std::isfinite(x);
            ordered = ordered && b.mn.x <= b.mx.x && b.mn.y <= b.mx.y && b.mn.z <= b.mx.z;
        }
    }
    std::stable_sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    const int nr = (int)kv.size();
    *n_real = nr;
    *depth = 0;
    // The fast traversal takes every record of the ordered tree as a proper box (no
    // degenerate / NaN test per child, pair_hit_tt): a pose that makes a box non-finite
    // leaves the frame to the heap kernels.
    if (!ordered) { *depth = 1 << 20; return; }
    if (nr < 2) return;
    std::vector<unsigned long long> keys(nr);
    for (int i = 0; i < nr; i++) keys[i] = kv[i].first;
    std::vector<int> child(2 * (nr - 1));                   // internal children (-1: leaf)
    for (int i = 0; i < nr - 1; i++) {
        int first, last, gamma;
        fnode_split(keys.data(), nr, i, first, last, gamma);
        child[2 * i] = gamma + 1 == last ? -1 : gamma + 1;
        child[2 * i + 1] = gamma == first ? -1 : gamma;
    }
    std::vector<std::pair<int, int>> todo{{0, 1}};
    while (!todo.empty()) {
        const auto [node, d] = todo.back();
        todo.pop_back();
        *depth = std::max(*depth, d);
        if (d > nr) { *depth = 1 << 20; return; }          // malformed: disable the fast tree
        for (int c = 0; c < 2; c++) if (child[2 * node + c] >= 0) todo.push_back({child[2 * node + c], d + 1});
    }
}
void free_atlas(rt_scene* s);
int ensure_atlas(rt_scene* s);

// The scene's own stream, created on first use: a caller passing its own streams (frame
// pipelining) keeps every HIP stream of the process on a hardware queue of its own
// (GPU_MAX_HW_QUEUES = 4; streams beyond that share queues and serialise).
hipStream_t sstream(rt_scene* s) {
    if (!s->stream) (void)hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    return s->stream;
}

int upload(rt_scene* s) {
    if (s->uploaded) return RT_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RT_ERR_NODEV, "no HIP device available");
    s->device = g_device;
    HIPCHK(hipSetDevice(s->device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, s->device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return fail(RT_ERR_NODEV, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
    for (auto& e : s->ev) HIPCHK(hipEventCreate(&e));
    const rt::Scene& h = s->h;
    auto up = [&](auto*& dst, const auto& vec) -> int {
        using T = typename std::remove_reference<decltype(vec)>::type::value_type;
        size_t bytes = std::max<size_t>(1, vec.size()) * sizeof(T);
        HIPCHK(hipMalloc((void**)&dst, bytes));
        if (!vec.empty()) HIPCHK(hipMemcpy(dst, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice));
        return RT_OK;
    };
    int r;
    if ((r = up(s->d_tris, h.d_tris)) || (r = up(s->d_meshes, h.d_meshes)) || (r = up(s->d_insts, h.d_insts)) ||
        (r = up(s->d_mats, h.d_mats)) || (r = up(s->d_lights, h.d_lights)))
        return r;
    s->n_leaf = padded((int)h.d_insts.size());
    if (s->n_leaf > BVH_MAX_LEAVES) return fail(RT_ERR_LIMIT, "more than 2^24 padded instances");
    s->n_cu = prop.multiProcessorCount;
    size_t nl = std::max(1, s->n_leaf);
    HIPCHK(hipMalloc((void**)&s->d_node_pair, 3 * nl * sizeof(float4)));
    ordered_tree_shape(h, &s->n_real, &s->fdepth);
    s->shape_gen = s->inst_gen;
    HIPCHK(hipMalloc((void**)&s->d_fnode, 4 * (size_t)std::max(1, s->n_real - 1) * sizeof(float4)));
    HIPCHK(hipMalloc((void**)&s->d_leaf, nl * sizeof(int)));
    HIPCHK(hipMalloc((void**)&s->d_inst4, std::max<size_t>(1, h.d_insts.size()) * sizeof(float4)));
    HIPCHK(hipMalloc((void**)&s->d_work, WORK_INTS * sizeof(int)));
    if ((r = upload_inst4(s)) != RT_OK) return r;
    if ((r = up(s->d_tri_ax, tri_axis_records(h))) != RT_OK) return r;
    if ((r = up(s->d_mesh_box, mesh_boxes(h))) != RT_OK) return r;
    HIPCHK(hipMalloc((void**)&s->d_tree, 2 * nl * sizeof(Box)));
    if (s->n_leaf > BVH_WG_LEAVES) HIPCHK(hipMalloc(&s->d_bscratch, bvh_large_scratch_bytes(s->n_leaf)));
    HIPCHK(hipMalloc((void**)&s->d_stats, STATS_N * sizeof(unsigned long long)));
    HIPCHK(hipMalloc((void**)&s->d_canvas, (size_t)h.cam.W * h.cam.H * sizeof(uint32_t)));
    HIPCHK(hipMalloc((void**)&s->d_dbg, 4096 * sizeof(int)));
    for (auto& e : s->slot_done) if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    s->slot_inst_gen = s->inst_gen;
    s->uploaded = true;
    if (s->n_slots > 1) return ensure_other_slot(s);
    return RT_OK;
}

// compact instance records for the trace kernel: (p, mesh | 0x80000000 when the pose is not identity)
void fill_inst4(const rt::Scene& h, float4* v) {
    for (size_t i = 0; i < h.d_insts.size(); i++) {
        const DInst& d = h.d_insts[i];
        uint32_t w = (uint32_t)d.mesh | (d.pose.identity ? 0u : 0x80000000u);
        float fw; memcpy(&fw, &w, 4);
        v[i] = make_float4(d.pose.p.x, d.pose.p.y, d.pose.p.z, fw);
    }
}
int upload_inst4(rt_scene* s) {
    std::vector<float4> v(s->h.d_insts.size());
    fill_inst4(s->h, v.data());
    if (!v.empty()) HIPCHK(hipMemcpy(s->d_inst4, v.data(), v.size() * sizeof(float4), hipMemcpyHostToDevice));
    return RT_OK;
}

// Bring the current slot's instance arrays to the host's generation, stream-ordered on `st`
// (after the slot's previous frame, which the caller has made `st` wait for).  The pinned
// staging is rewritten only once the copy that last read it has run (the slot's last frame,
// recorded after that copy).
int sync_slot_insts(rt_scene* s, hipStream_t st) {
    if (s->slot_inst_gen == s->inst_gen) return RT_OK;
    const size_t n = s->h.d_insts.size();
    if (n) {
        if (!s->h_insts_pin) {
            HIPCHK(hipHostMalloc((void**)&s->h_insts_pin, n * sizeof(DInst), hipHostMallocDefault));
            HIPCHK(hipHostMalloc((void**)&s->h_inst4_pin, n * sizeof(float4), hipHostMallocDefault));
            int r;
            if (s->n_slots > 1 && (r = mirror_slot_caps(s)) != RT_OK) return r;
        } else if (s->slot_pending[s->cur_slot]) {
            HIPCHK(hipEventSynchronize(s->slot_done[s->cur_slot]));
        }
        memcpy(s->h_insts_pin, s->h.d_insts.data(), n * sizeof(DInst));
        fill_inst4(s->h, s->h_inst4_pin);
        HIPCHK(hipMemcpyAsync(s->d_insts, s->h_insts_pin, n * sizeof(DInst), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(s->d_inst4, s->h_inst4_pin, n * sizeof(float4), hipMemcpyHostToDevice, st));
        HIPCHK(hipEventRecord(s->slot_done[s->cur_slot], st));   // covers the staging until the frame records it again
        s->slot_pending[s->cur_slot] = true;
    }
    s->slot_inst_gen = s->inst_gen;
    return RT_OK;
}

// Ordered-LBVH shape (leaf count, depth) for the current host poses: instances that moved
// change the Morton order and with it the tree depth the fast traversal's stack must hold.
void refresh_shape(rt_scene* s) {
    if (s->shape_gen == s->inst_gen) return;
    int nr = 0;
    ordered_tree_shape(s->h, &nr, &s->fdepth);
    s->shape_gen = s->inst_gen;
}

// Begin a frame on the current slot: `st` waits for the slot's previous frame (all slots'
// last frames for side entries that do not rotate slots), then the slot's instances are
// brought up to date.  end_frame records the slot's completion.
int begin_frame(rt_scene* s, hipStream_t st, bool all_slots) {
    for (int i = 0; i < rt_scene::MAX_SLOTS; i++)
        if (s->slot_pending[i] && (all_slots || i == s->cur_slot)) HIPCHK(hipStreamWaitEvent(st, s->slot_done[i], 0));
    refresh_shape(s);
    return sync_slot_insts(s, st);
}
int end_frame(rt_scene* s, hipStream_t st) {
    HIPCHK(hipEventRecord(s->slot_done[s->cur_slot], st));
    s->slot_pending[s->cur_slot] = true;
    return RT_OK;
}

// Buffers of the frame slots other than the current one (sizes as in upload), slot events.
int ensure_other_slot(rt_scene* s) {
    const size_t nl = std::max(1, s->n_leaf);
    for (int i = 0; i < s->n_slots; i++) {
        rt_scene::Slot& o = s->store[i];
        if (i == s->cur_slot || o.d_work) continue;
        HIPCHK(hipMalloc((void**)&o.d_node_pair, 3 * nl * sizeof(float4)));
        HIPCHK(hipMalloc((void**)&o.d_fnode, 4 * (size_t)std::max(1, s->n_real - 1) * sizeof(float4)));
        HIPCHK(hipMalloc((void**)&o.d_leaf, nl * sizeof(int)));
        HIPCHK(hipMalloc((void**)&o.d_tree, 2 * nl * sizeof(Box)));
        HIPCHK(hipMalloc((void**)&o.d_work, WORK_INTS * sizeof(int)));
        HIPCHK(hipMalloc((void**)&o.d_insts, std::max<size_t>(1, s->h.d_insts.size()) * sizeof(DInst)));
        HIPCHK(hipMalloc((void**)&o.d_inst4, std::max<size_t>(1, s->h.d_insts.size()) * sizeof(float4)));
        // the grid-wide build's sort buffers now, not at the slot's first frame inside a pipeline
        if (s->n_leaf > BVH_WG_LEAVES && !o.d_bscratch) HIPCHK(hipMalloc(&o.d_bscratch, bvh_large_scratch_bytes(s->n_leaf)));
        // the current poses now (blocking copies, here rather than at the slot's first frame: an
        // asynchronous copy on a frame's stream may start a new SDMA engine, ~7 ms of host time
        // the first time, profiles/r06/rblog/); later pose changes reach the slot through
        // sync_slot_insts, stream-ordered
        const size_t n = s->h.d_insts.size();
        if (n) {
            std::vector<float4> v4(n);
            fill_inst4(s->h, v4.data());
            HIPCHK(hipMemcpy(o.d_insts, s->h.d_insts.data(), n * sizeof(DInst), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(o.d_inst4, v4.data(), n * sizeof(float4), hipMemcpyHostToDevice));
        }
        o.slot_inst_gen = s->inst_gen;
        o.work_zeroed = false; o.bvh_valid = false;
    }
    return mirror_slot_caps(s);                              // the current slot's grown buffers too
}

// The current slot grew a per-frame buffer (sky flags, live lists, history, pinned instance
// staging) at its first frame of a new layout: give every other allocated slot the same
// capacity now, so that their first frames -- possibly inside a steady pipeline -- allocate
// nothing (an allocation there cost the first 8 frames of a run up to ~1 ms: hipFree waits for
// the device, pinned allocations take milliseconds).  The slots' contents are reset on first
// use as before (history key, instance generation).  Only growth reaches here: waiting for the
// device before freeing a smaller buffer is a one-time cost per layout.
int mirror_slot_caps(rt_scene* s) {
    bool synced = false;
    auto sync_once = [&]() -> hipError_t { if (synced) return hipSuccess; synced = true; return hipDeviceSynchronize(); };
    for (int i = 0; i < s->n_slots; i++) {
        if (i == s->cur_slot) continue;
        rt_scene::Slot& o = s->store[i];
        if (!o.d_work) continue;                              // not allocated (ensure_other_slot)
        if (s->d_gsky && o.gsky_cap < s->gsky_cap) {
            if (o.d_gsky) { HIPCHK(sync_once()); dfree(o.d_gsky); }
            HIPCHK(hipMalloc((void**)&o.d_gsky, s->gsky_cap));
            o.gsky_cap = s->gsky_cap;
        }
        if (s->d_live && o.live_cap < s->live_cap) {
            if (o.d_live) { HIPCHK(sync_once()); dfree(o.d_live); }
            HIPCHK(hipMalloc((void**)&o.d_live, (size_t)s->live_cap * sizeof(int)));
            o.live_cap = s->live_cap;
        }
        if (s->d_hctl && o.hist_cap < s->hist_cap) {
            if (o.d_hctl) {
                HIPCHK(sync_once());
                for (int q = 0; q < 2; q++) { dfree(o.d_hlist[q]); dfree(o.d_hflag[q]); }
                dfree(o.d_hctl);
            }
            for (int q = 0; q < 2; q++) {
                HIPCHK(hipMalloc((void**)&o.d_hlist[q], (size_t)s->hist_cap * sizeof(int)));
                HIPCHK(hipMalloc((void**)&o.d_hflag[q], s->hist_cap));
            }
            HIPCHK(hipMalloc((void**)&o.d_hctl, 4 * sizeof(unsigned long long)));
            o.hist_cap = s->hist_cap;
            o.hist_key[0] = -1;                               // reset at the slot's first use
        }
        const size_t n = s->h.d_insts.size();
        if (s->h_insts_pin && !o.h_insts_pin && n) {
            HIPCHK(hipHostMalloc((void**)&o.h_insts_pin, n * sizeof(DInst), hipHostMallocDefault));
            HIPCHK(hipHostMalloc((void**)&o.h_inst4_pin, n * sizeof(float4), hipHostMallocDefault));
        }
    }
    return RT_OK;
}

// Atlas -> float4 texels (byte / 255, as assets.cc:61-81) in HBM; the reference's CUDA
// texture (gputils TextureBuffer4D, alloc.h:24-80: point sampling, clamp) is sampled
// explicitly by hit_kd, since gfx950 has no texture units.
void free_atlas(rt_scene* s) {
    if (s->d_atlas) (void)hipFree(s->d_atlas);
    s->d_atlas = nullptr;
}
int ensure_atlas(rt_scene* s) {
    const rt::Scene& h = s->h;
    if (h.atlas_rgba.empty()) return fail(RT_ERR_STATE, "textured rendering needs an atlas: rt_scene_load_atlas / rt_scene_set_atlas");
    if (!s->atlas_dirty && s->d_atlas) return RT_OK;
    free_atlas(s);
    const size_t n = (size_t)h.atlas_w * h.atlas_h;
    std::vector<float4> texels(n);
    for (size_t i = 0; i < n; i++)
        texels[i] = make_float4((float)h.atlas_rgba[4 * i] / 255, (float)h.atlas_rgba[4 * i + 1] / 255,
                                (float)h.atlas_rgba[4 * i + 2] / 255, (float)h.atlas_rgba[4 * i + 3] / 255);
    HIPCHK(hipMalloc((void**)&s->d_atlas, n * sizeof(float4)));
    HIPCHK(hipMemcpy(s->d_atlas, texels.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    s->atlas_dirty = false;
    return RT_OK;
}

// A factor coprime with the queue length, so t -> t * f mod len is a permutation
// (checked with gcd; f near len * 0.618 spreads consecutive tickets across the image).
int ticket_scramble(int len) {
    if (len <= 2) return 1;
    int f = (int)(len * 0.6180339887) | 1;
    while (std::gcd(f % len, len) != 1) f++;
    return f % len;
}

// (Re)allocate / reset the scheduling history when the launch layout changes.
int ensure_history(rt_scene* s, int n_groups, const long long* key, hipStream_t st) {
    if (n_groups > s->hist_cap) {
        for (int p = 0; p < 2; p++) { dfree(s->d_hlist[p]); dfree(s->d_hflag[p]); }
        dfree(s->d_hctl);
        const int cap = (std::max(n_groups, 1024) + 3) & ~3;   // whole dwords (flag() reads scalar dwords)
        for (int p = 0; p < 2; p++) {
            HIPCHK(hipMalloc((void**)&s->d_hlist[p], cap * sizeof(int)));
            HIPCHK(hipMalloc((void**)&s->d_hflag[p], cap));
        }
        HIPCHK(hipMalloc((void**)&s->d_hctl, 4 * sizeof(unsigned long long)));
        s->hist_cap = cap;
        s->hist_key[0] = -1;
    }
    if (memcmp(key, s->hist_key, sizeof s->hist_key) != 0) {
        for (int p = 0; p < 2; p++) HIPCHK(hipMemsetAsync(s->d_hflag[p], 0, s->hist_cap, st));
        HIPCHK(hipMemsetAsync(s->d_hctl, 0, 4 * sizeof(unsigned long long), st));
        memcpy(s->hist_key, key, sizeof s->hist_key);
        s->hist_parity = 0;
    }
    return RT_OK;
}

// Per-frame buffers (sky flags, live lists, scheduling history) sized for a layout of n_groups
// pixel groups in the current slot and every allocated one, ahead of the first frame that needs
// them (warm_scene: the whole frame at 2-8 pixels per wave, the layouts of spp 8-32).  Contents
// are reset at first use as before (the history key); only capacity is reserved here.
int reserve_layout(rt_scene* s, int n_groups) {
    const int cap = (std::max(n_groups, 1024) + 3) & ~3;
    bool grew = false;
    if (cap > s->gsky_cap) {
        dfree(s->d_gsky);
        HIPCHK(hipMalloc((void**)&s->d_gsky, cap));
        s->gsky_cap = cap; grew = true;
    }
    const int sblocks = (n_groups + 63) / 64;
    const int need = (sblocks + NQ - 1) / NQ * 64 * NQ + n_groups;
    if (need > s->live_cap) {
        dfree(s->d_live);
        HIPCHK(hipMalloc((void**)&s->d_live, (size_t)need * sizeof(int)));
        s->live_cap = need; grew = true;
    }
    if (cap > s->hist_cap) {
        for (int p = 0; p < 2; p++) { dfree(s->d_hlist[p]); dfree(s->d_hflag[p]); }
        dfree(s->d_hctl);
        for (int p = 0; p < 2; p++) {
            HIPCHK(hipMalloc((void**)&s->d_hlist[p], cap * sizeof(int)));
            HIPCHK(hipMalloc((void**)&s->d_hflag[p], cap));
        }
        HIPCHK(hipMalloc((void**)&s->d_hctl, 4 * sizeof(unsigned long long)));
        s->hist_cap = cap;
        s->hist_key[0] = -1;
        grew = true;
    }
    return (grew && s->n_slots > 1) ? mirror_slot_caps(s) : RT_OK;
}

int ensure_spp(rt_scene* s, int spp) {
    if (spp <= s->spp_cap) return RT_OK;
    int cap = std::max(spp, 64);
    std::vector<float2> tab(cap);
    for (int k = 0; k < cap; k++) rt::spp_offset(k, &tab[k].x, &tab[k].y);
    dfree(s->d_spp);
    HIPCHK(hipMalloc((void**)&s->d_spp, cap * sizeof(float2)));
    HIPCHK(hipMemcpy(s->d_spp, tab.data(), cap * sizeof(float2), hipMemcpyHostToDevice));
    s->spp_cap = cap;
    return RT_OK;
}

int build_bvh(rt_scene* s, hipStream_t st, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
    if (s->n_leaf == 0) {
        if (e0) { HIPCHK(hipEventRecord(e0, st)); HIPCHK(hipEventRecord(e1, st)); }
        s->bvh_valid = true;
        return RT_OK;
    }
    BvhArgs A;
    A.insts = s->d_insts; A.n_inst = (int)s->h.d_insts.size();
    A.mesh_box = s->d_mesh_box; A.n = s->n_leaf;
    A.tree = s->d_tree;
    A.node_pair = reinterpret_cast<float*>(s->d_node_pair); A.leaf_inst = s->d_leaf;
    A.fnode = s->d_fnode; A.n_real = s->n_real;
    A.work = s->d_work; A.n_work = WORK_INTS;
    // the slot the next fast frame records its heavy list into (launch_trace skips its memset)
    A.hctl = s->d_hctl ? s->d_hctl + 2 * (1 - s->hist_parity) : nullptr;
    s->hctl_zeroed = s->d_hctl ? 1 - s->hist_parity : -1;
    if (A.n > BVH_WG_LEAVES) {                                // above one workgroup's LDS: the grid-wide build
        if (!s->d_bscratch) HIPCHK(hipMalloc(&s->d_bscratch, bvh_large_scratch_bytes(A.n)));
        HIPCHK(bvh_build_large(A, s->d_bscratch, st, e0, e1));
        s->bvh_valid = true;
        s->work_zeroed = true;
        return RT_OK;
    }
    const bool lds_tree = bvh_lds_bytes(A.n, true) <= 160 * 1024;       // n <= 2048
    const size_t lds = bvh_lds_bytes(A.n, lds_tree);
    if (lds > 160 * 1024) return fail(RT_ERR_LIMIT, "BVH build needs more LDS than one CU has");
    const void* fn = lds_tree ? (const void*)bvh_build_kernel<true> : (const void*)bvh_build_kernel<false>;
    if (lds > 64 * 1024) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    void* args[] = {&A};
    // e0/e1 (timing=1): timestamps taken by the dispatch itself, no marker packets
    HIPCHK(hipExtLaunchKernel(fn, dim3(1), dim3(1024), args, lds, st, e0, e1, 0));
    HIPCHK(hipGetLastError());
    s->bvh_valid = true;
    s->work_zeroed = true;
    return RT_OK;
}

SceneView view_of(const rt_scene* s, bool use_bvh) {
    SceneView v;
    v.tris = s->d_tris; v.meshes = s->d_meshes; v.insts = s->d_insts; v.mats = s->d_mats; v.lights = s->d_lights;
    v.node_pair = s->d_node_pair; v.leaf_inst = s->d_leaf;
    v.fnode = s->d_fnode; v.n_real = s->n_real;
    v.ftree = (s->n_real >= 2 && s->fdepth <= FT_MAX_DEPTH) ? 1 : 0; v.inst4 = s->d_inst4;
    v.n_leaf = s->n_leaf; v.n_inst = (int)s->h.d_insts.size();
    v.n_lights = (int)s->h.d_lights.size(); v.use_bvh = use_bvh ? 1 : 0;
    v.n_mats = (int)s->h.d_mats.size(); v.n_tris = (int)s->h.d_tris.size(); v.n_meshes = (int)s->h.d_meshes.size();
    v.ident_all = 1;
    for (const auto& i : s->h.d_insts) v.ident_all &= i.pose.identity ? 1 : 0;
    for (const auto& m : s->h.d_meshes) v.ident_all &= m.pose.identity ? 1 : 0;
    // Distance pruning (closest_hit): boxes provably contain their triangles only for
    // pure translations with zero mesh offsets (the BVH boxes ignore the mesh pose,
    // raytracer.cu:54-89).  Slack: 1e-4 x mesh size + 2^-14 x scene radius.
    bool prune_ok = v.ident_all != 0;
    float vmax = 0.0f, pmax = 0.0f;
    for (const auto& m : s->h.d_meshes) prune_ok = prune_ok && m.pose.p.x == 0 && m.pose.p.y == 0 && m.pose.p.z == 0;
    auto amax = [](rtm::V3 a) { return std::max(std::fabs(a.x), std::max(std::fabs(a.y), std::fabs(a.z))); };
    for (const auto& t : s->h.d_tris) vmax = std::max(vmax, std::max(amax(t.a), std::max(amax(t.b), amax(t.c))));
    for (const auto& i : s->h.d_insts) pmax = std::max(pmax, amax(i.pose.p));
    const float radius = pmax + vmax + amax(s->h.d_cam.pos) + 1.0f;
    prune_ok = prune_ok && std::isfinite(radius);
    v.prune_abs = prune_ok ? 4e-4f * vmax + 0x1p-14f * radius : -1.0f;
    v.tri_ax = (v.ident_all && !s->h.d_tris.empty()) ? s->d_tri_ax : nullptr;
    return v;
}

bool opaque_scene(const rt_scene* s) {
    for (const DMat& m : s->h.d_mats) if (m.refractive) return false;
    return true;
}

int launch_trace(rt_scene* s, const rt_render_opts& o, hipStream_t st, uint32_t* rgba, int* dbg, int dbg_x, int dbg_y,
                 bool want_stats, int occl_force = -1, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr,
                 bool prof = false, unsigned* gdur = nullptr, int* geo = nullptr) {
    TraceParams P{};
    P.gdur = gdur;
    const rt::Scene& h = s->h;
    P.cam = h.d_cam; P.dist_atten = h.dist_atten; P.ambience = h.ambience;
    P.W = h.cam.W; P.H = h.cam.H; P.row0 = o.row0; P.row_step = o.row_step;
    P.n_rows = (P.H - o.row0 + o.row_step - 1) / o.row_step;
    if (P.n_rows <= 0) {
        if (e0) { HIPCHK(hipEventRecord(e0, st)); HIPCHK(hipEventRecord(e1, st)); }
        return RT_OK;
    }
    P.compact = o.compact; P.spp = o.spp; P.depth = h.depth;
    P.spp_recip = (o.spp & (o.spp - 1)) == 0 ? 1.0f / (float)o.spp : 0.0f;
    P.spp_off = s->d_spp;
    P.rgba = rgba; P.radiance = reinterpret_cast<float4*>(o.radiance); P.hit_inst = o.hit_inst; P.hit_tri = o.hit_tri;
    P.stats = (want_stats || prof) ? s->d_stats : nullptr; P.dbg_log = dbg; P.dbg_x = dbg_x; P.dbg_y = dbg_y;
    if (o.textures) {
        int r;
        if ((r = ensure_atlas(s)) != RT_OK) return r;
        P.atlas = s->d_atlas; P.atlas_w = s->h.atlas_w; P.atlas_h = s->h.atlas_h;
    }
    SceneView S = view_of(s, o.use_bvh != 0);
    // sample-parallel mapping: L lanes per pixel (one sample each per round), 64/L pixels per wave
    P.lanes_per_px = std::min(o.spp, 64);
    P.px_per_wave = 64 / P.lanes_per_px;
    int gw = 1;
    if ((P.px_per_wave & (P.px_per_wave - 1)) == 0) { while (gw * gw < P.px_per_wave) gw <<= 1; }
    else gw = P.px_per_wave;
    // Row slices with rows >= 8 frame rows apart (N >= 8 ranks): a 2-row group would pair
    // rows that far apart, so groups are one row (8 x 1 at 8 spp).  Measured with four frames
    // in flight: 8-way slice 0.234 -> 0.229 ms; whole frames and 2-way slices keep 4 x 2
    // (8 x 1 there: +3.4% / +2%; profiles/r01/ab_group_shape_v31.log).
    if (o.row_step >= 8) gw = P.px_per_wave;
    P.gw = gw; P.gh = P.px_per_wave / gw;
    auto log2_exact = [](int v) { int k = 0; while ((1 << k) < v) k++; return (1 << k) == v ? k : -1; };
    P.l_shift = log2_exact(P.lanes_per_px); P.gw_shift = log2_exact(P.gw);
    P.n_gx = (P.W + P.gw - 1) / P.gw;
    P.n_groups = P.n_gx * ((P.n_rows + P.gh - 1) / P.gh);
    if (geo) { geo[0] = P.n_groups; geo[1] = P.gw; geo[2] = P.gh; geo[3] = P.n_gx; }
    P.scramble = ticket_scramble((P.n_groups + NQ - 1) / NQ);
    P.scramble_small = (unsigned long long)((P.n_groups + NQ - 1) / NQ + TPC) * (unsigned long long)P.scramble < (1ull << 32);
    P.div_ngx = udiv_make((unsigned)P.n_gx);
    P.div_perq = udiv_make((unsigned)((P.n_groups + NQ - 1) / NQ));
    P.work = s->d_work; P.tpc = TPC;
    {   // unlit skip (trace_sample, ST_LIGHT): every incoming light must be >= +0 and finite
        bool ok = !want_stats && !dbg;                        // (the PROF variant profiles the fast frame: on)
        auto pos0 = [](float v) { return std::isfinite(v) && !std::signbit(v); };
        for (const DLight& l : h.d_lights) ok = ok && pos0(l.col.x) && pos0(l.col.y) && pos0(l.col.z) && pos0(l.col.w);
        for (const DMat& m : h.d_mats)
            ok = ok && pos0(m.Kt.x) && pos0(m.Kt.y) && pos0(m.Kt.z) && pos0(m.Kt.w) && m.Kt.x <= 1.0f && m.Kt.y <= 1.0f &&
                 m.Kt.z <= 1.0f && m.Kt.w <= 1.0f;
        bool start_ok = true;                                  // no -0 channel in Ke + Ka * ambience (org_light)
        for (const DMat& m : h.d_mats) {
            const V4 o = m.Ke + m.Ka * h.ambience;
            for (float v : {o.x, o.y, o.z, o.w}) start_ok = start_ok && !(v == 0.0f && std::signbit(v));
        }
        P.unlit_skip = ok ? (start_ok ? 2 : 1) : 0;
    }
    P.occl_exit = (opaque_scene(s) && (occl_force == 1 || (occl_force < 0 && !want_stats))) ? 1 : 0;
    if (!s->work_zeroed) HIPCHK(hipMemsetAsync(s->d_work, 0, WORK_INTS * sizeof(int), st));
    const bool tex = o.textures != 0;
    const int mode0 = (o.spp > 64 ? M_MULTI : 0) | (want_stats ? M_STATS : 0);
    // brute force (the reference's -r): no tree kernel (closest_hit's FT path assumes a tree)
    const bool brute = !S.use_bvh || S.n_leaf == 0;
    const bool ft = !brute && mode0 == 0 && S.ftree && lds_bytes(S, true) <= (size_t)LDS_LIMIT;
    const size_t lds = lds_bytes(S, ft);
    const bool use_lds = lds <= (size_t)LDS_LIMIT;
    // suspended frames needed (<= MAX_FRAMES - 1); none without a refractive material, where a
    // reflection child replaces its parent (trace_sample, F_REFLECT)
    // (NS = 0 kernels assume that: a depth-0 scene with refraction takes the NS = 2 bucket)
    const int ns = opaque_scene(s) ? 0 : std::max(h.depth, 1);
    const void* fn;
    const int mode = (o.spp > 64 ? M_MULTI : 0) | (want_stats ? M_STATS : 0);
    constexpr int NG = MAX_FRAMES - 1;                     // generic frame-stack depth
    static const void* const generic[2][4] = {
        {(const void*)trace_kernel<NG, false, 0>, (const void*)trace_kernel<NG, false, 1>,
         (const void*)trace_kernel<NG, false, 2>, (const void*)trace_kernel<NG, false, 3>},
        {(const void*)trace_kernel<NG, true, 0>, (const void*)trace_kernel<NG, true, 1>,
         (const void*)trace_kernel<NG, true, 2>, (const void*)trace_kernel<NG, true, 3>}};
    static const void* const textured[2][4] = {
        {(const void*)trace_kernel<NG, false, 8>, (const void*)trace_kernel<NG, false, 9>,
         (const void*)trace_kernel<NG, false, 10>, (const void*)trace_kernel<NG, false, 11>},
        {(const void*)trace_kernel<NG, true, 8>, (const void*)trace_kernel<NG, true, 9>,
         (const void*)trace_kernel<NG, true, 10>, (const void*)trace_kernel<NG, true, 11>}};
    const size_t park_bytes = (size_t)park_fields(ns <= 0 ? 0 : 2) * 4 * TRACE_BLOCK_P;
    const bool park = !tex && mode == 0 && use_lds && lds + park_bytes + (prof ? PROF_LDS_BYTES : 0) <= (size_t)PARK_LDS_LIMIT;
    // LDS shading cache beside the parked main kernel (not with the profiling variant)
    const bool shade = park && ft && S.tri_ax && !prof &&
                       lds + shade_bytes(S) + park_bytes <= (size_t)PARK_LDS_LIMIT;
    // brute-force fast frames: the instance loop only (M_BRUTE), axis-plane triangles, parked
    // state and the LDS shading cache beside the instance records
    const size_t lds_br = lds_bytes(S, false, true, true);
    const bool brute_k = brute && !tex && mode == 0 && !prof && S.tri_ax && lds_br + park_bytes <= (size_t)PARK_LDS_LIMIT;
    // ordered tree in LDS but no room for the whole parking area beside the instance records
    // (world16: 93 KB tree + 23 KB instances): partial parking, instances from global memory
    const size_t lds_pt = lds_bytes(S, true, true, false, true);
    const size_t part_bytes = (size_t)PART_FIELDS * 4 * TRACE_BLOCK_P;
    // (textured frames too: the hit's atlas colour stays in registers)
    const bool part_k = !brute_k && ft && (!park || tex) && mode == 0 && !prof && S.tri_ax && ns <= 0 &&
                        lds_pt + part_bytes <= (size_t)PARK_LDS_LIMIT && !getenv("RT_NO_PART");
    if (part_k) {
        constexpr int PT = M_PARK | M_FT | M_AXIS | M_SHADE | M_PART;
        fn = tex ? (const void*)trace_kernel<0, true, PT | M_TEX> : (const void*)trace_kernel<0, true, PT>;
    } else if (brute_k) {
        constexpr int BR = M_BRUTE | M_PARK | M_SHADE | M_AXIS;
        fn = ns <= 0 ? (const void*)trace_kernel<0, true, BR> : ns <= 2 ? (const void*)trace_kernel<2, true, BR>
                                                               : (const void*)trace_kernel<NG, true, BR>;
    } else if (tex && ft) {                                    // textured fast frames: ordered LBVH, unparked
        constexpr int TF = M_TEX | M_FT, TA = M_TEX | M_FT | M_AXIS;
        fn = S.tri_ax ? (ns <= 2 ? (const void*)trace_kernel<2, true, TA> : (const void*)trace_kernel<NG, true, TA>)
                      : (ns <= 2 ? (const void*)trace_kernel<2, true, TF> : (const void*)trace_kernel<NG, true, TF>);
    } else if (tex) {
        fn = textured[use_lds ? 1 : 0][mode];
    } else if (ft && park && S.tri_ax && prof) {
        constexpr int PP = M_PARK | M_FT | M_AXIS | M_PROF;
        fn = ns <= 0 ? (const void*)trace_kernel<0, true, PP> : ns <= 2 ? (const void*)trace_kernel<2, true, PP>
                                                                 : (const void*)trace_kernel<NG, true, PP>;
    } else if (ft && park && S.tri_ax && shade) {
        constexpr int PS = M_PARK | M_FT | M_AXIS | M_SHADE;
        fn = ns <= 0 ? (const void*)trace_kernel<0, true, PS> : ns <= 2 ? (const void*)trace_kernel<2, true, PS>
                                                                 : (const void*)trace_kernel<NG, true, PS>;
    } else if (ft && park && S.tri_ax) {
        constexpr int PA = M_PARK | M_FT | M_AXIS;
        fn = ns <= 0 ? (const void*)trace_kernel<0, true, PA> : ns <= 2 ? (const void*)trace_kernel<2, true, PA>
                                                                 : (const void*)trace_kernel<NG, true, PA>;
    } else if (ft) {
        constexpr int PF = M_PARK | M_FT;
        fn = park ? (ns <= 0 ? (const void*)trace_kernel<0, true, PF> : ns <= 2 ? (const void*)trace_kernel<2, true, PF>
                                                                         : (const void*)trace_kernel<NG, true, PF>)
                  : (ns <= 0 ? (const void*)trace_kernel<0, true, M_FT> : ns <= 2 ? (const void*)trace_kernel<2, true, M_FT>
                                                                           : (const void*)trace_kernel<NG, true, M_FT>);
    } else if (park) {
        fn = ns <= 0 ? (const void*)trace_kernel<0, true, M_PARK> : ns <= 2 ? (const void*)trace_kernel<2, true, M_PARK>
                     : (const void*)trace_kernel<NG, true, M_PARK>;
    } else if (mode != 0 || ns > 2) fn = generic[use_lds ? 1 : 0][mode];
    else if (use_lds) fn = ns <= 0 ? (const void*)trace_kernel<0, true, 0> : (const void*)trace_kernel<2, true, 0>;
    else fn = ns <= 0 ? (const void*)trace_kernel<0, false, 0> : (const void*)trace_kernel<2, false, 0>;
    const size_t shm = part_k ? lds_pt + part_bytes : brute_k ? lds_br + park_bytes
                               : (park ? lds + park_bytes : use_lds ? lds : 0) + (shade ? shade_bytes(S) : 0) +
                                     (prof ? PROF_LDS_BYTES : 0);
    if (shm > 64 * 1024) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    int per_cu = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, TRACE_BLOCK_P, shm) != hipSuccess || per_cu < 1) per_cu = 1;
    const int waves_needed = P.n_groups;
    // Frames in flight: a launch issued while the scene's previous frame is still running takes
    // half the CUs.  A persistent block holds its CU (the LDS image) until its slowest wave
    // ends; fewer blocks, each running twice the groups, leave fewer CUs held by one wave's last
    // group, and two frames' blocks still cover the GPU.  Measured with four in flight
    // (tools/pipe_slices.py, per-rank ms per frame at N = 1/2/4/8, same box): 0.655-0.665 /
    // 0.374 / 0.226 / 0.156-0.157 with every CU, 0.646-0.654 / 0.347-0.354 / 0.200-0.205 /
    // 0.137-0.140 with half; 3/8, 5/8 and 3/4 of the CUs in between (profiles/r03/ab_grid/).
    // A frame issued alone (no other frame running) keeps every CU.  Requiring two or three
    // running frames instead of one measured the same (profiles/r03/ab_grid/grid2.log).  A
    // pipeline that copies every frame to the host measured 12% slower this way, with the copy
    // anywhere (render stream, copy stream, high priority, fewer blit workgroups) and with the
    // optional second half of the grid gated on later frames being queued
    // (profiles/r03/ab_grid/readback.log): such callers set RT_OVERLAP_FULL.
    int cap = s->n_cu * per_cu;
    // another frame of the scene still in flight (any slot count, any overlap policy): the heavy
    // list's static dealing below is for frames whose blocks all start at once
    bool other_running = false;
    for (int i = 1; i < s->n_slots && !other_running; i++) {
        const int sl = (s->cur_slot + s->n_slots - i) % s->n_slots;
        other_running = s->slot_pending[sl] && hipEventQuery(s->slot_done[sl]) == hipErrorNotReady;
    }
    if (s->n_slots >= 4 && s->overlap != RT_OVERLAP_FULL) {
        const bool running = s->overlap == RT_OVERLAP_STREAM || other_running;   // or a stream
        // Small frames (row slices of N >= 4 ranks: under ~48 groups per wave on half the CUs)
        // take a quarter: four frames' blocks share the GPU, each block runs twice the groups,
        // so its LDS staging and its slowest wave's tail weigh half as much.  Measured per-rank
        // ms per frame, 60-frame streams, same box (profiles/r04/grid_div.log): N = 8 0.112 ->
        // 0.101, N = 4 0.175 -> 0.171; whole frames unchanged by it (0.597 / 0.599), kept at half.
        const long long half_waves = (long long)(cap / 2) * (TRACE_BLOCK_P / 64);
        // (Not with virtual ranks, several slices of one frame per device from one scene: those
        // slices share frame slots, and a quarter measured slower there: --gpus 1 --ranks 8 per
        // slice 0.153 -> 0.173 ms, profiles/r04/grid_div.log.)
        const int div = ((long long)P.n_groups < RT_SMALL_FRAME_GPW * half_waves && s->ranks_per_device == 1) ? 4 : 2;
        if (running) cap = std::max(1, cap / div);
    }
    int blocks = std::min(cap, (waves_needed + TRACE_BLOCK_P / 64 - 1) / (TRACE_BLOCK_P / 64));
    blocks = std::max(blocks, 1);
    P.grid_waves = blocks * (TRACE_BLOCK_P / 64);              // the launch below: dim3(blocks)
    // every block starts at once: a full grid and no other frame of the scene running (RT_OVERLAP_FULL
    // and 2-3 frame slots keep the full grid for overlapping frames; those frames keep the counter)
    P.heavy_static = (blocks == s->n_cu * per_cu && !other_running) ? 1 : 0;
    P.heavy_cap = std::max(2 * blocks * (TRACE_BLOCK_P / 64), P.n_groups / 4);   // a bound, not a target
    // longest-first history (fast frames): valid while the launch layout is unchanged
    // Only where a wave runs few groups (1080p 8-way row slices: ~8 per wave): with more (63
    // for a whole 1080p frame, 16 for a 4-way slice) the dynamic queues already balance the
    // frame and the two clock reads per group cost as much as the shorter tail saves or more
    // (measured, four frames in flight, ms per frame with / without: whole frame 0.919 / 0.914,
    // 4-way 0.360 / 0.360, 8-way 0.179-0.186 / 0.200-0.204; profiles/r02/hist_policy.log).
    P.hist = 0;
    const long long waves = (long long)blocks * (TRACE_BLOCK_P / 64);
    // sky pre-pass: the fast (ordered-LBVH) kernels, one round of samples, a tree to test
    // (brute-force frames: the instances' grown boxes instead, when the pruning claim holds)
    const bool sky_brute = brute_k && !prof && !want_stats && o.spp <= 64 && S.prune_abs >= 0.0f && S.n_inst >= 1 &&
                           S.n_inst <= 64 && !getenv("RT_NO_BRUTE_SKY");
    const bool sky = (ft && !prof && o.spp <= 64 && S.use_bvh && S.n_leaf > 0) || sky_brute;
    // Heavy-first by work (hist = 2) where groups per wave are many: a group whose samples took
    // >= heavy_q wave queries (mirror pixels: primary, shadow and reflection chains) is flagged,
    // and the next frame of the slot runs the flagged groups first off a heavy live list the sky
    // pre-pass builds.  No clock reads (the timed history's cost, item 17), one byte store per
    // heavy group.  RT_HEAVY_Q (environment) sets heavy_q; 0 turns it off.
    // The mode must not depend on the grid (half or whole, frames in flight or alone): the two
    // modes' flags mean different things (hist = 1 flags only the groups on its heavy list and
    // skips them in the normal queues; hist = 2 flags by work and lists nothing), so the history
    // key includes the mode and a change of mode resets the flags.
    static const int heavy_q = [] { const char* e = getenv("RT_HEAVY_Q"); return e ? atoi(e) : RT_HEAVY_Q_DEFAULT; }();
    const long long full_waves = (long long)s->n_cu * per_cu * (TRACE_BLOCK_P / 64);
    const bool hist2 = !want_stats && !dbg && sky && heavy_q > 0;
    const bool hist1 = !hist2 && !want_stats && !dbg && (prof || (long long)P.n_groups <= RT_HIST_GROUPS_PER_WAVE * full_waves);
    (void)waves;
    if (hist1 || hist2) {
        const long long key[8] = {P.W, P.H, P.row0, P.row_step, P.n_rows, P.spp, P.n_groups,
                                  (long long)o.textures | (hist2 ? 2 : 1) << 8};
        int r;
        const int cap0 = s->hist_cap;
        if ((r = ensure_history(s, P.n_groups, key, st)) != RT_OK) return r;
        if (s->n_slots > 1 && s->hist_cap > cap0 && (r = mirror_slot_caps(s)) != RT_OK) return r;
        const int prev = s->hist_parity, next = 1 - prev;
        P.hist = hist1 ? 1 : 2;
        P.heavy_q = heavy_q;
        P.hl_prev = s->d_hlist[prev]; P.hl_next = s->d_hlist[next];
        P.hf_prev = s->d_hflag[prev]; P.hf_next = s->d_hflag[next];
        P.hctl_prev = s->d_hctl + 2 * prev; P.hctl_next = s->d_hctl + 2 * next;
        if (hist1 && s->hctl_zeroed != next) HIPCHK(hipMemsetAsync(s->d_hctl + 2 * next, 0, 2 * sizeof(unsigned long long), st));
        s->hist_parity = next;
    }
    s->work_zeroed = false;                                   // this launch consumes the counters
    s->hctl_zeroed = -1;
    if (sky) {
        bool grew = false;
        if (P.n_groups > s->gsky_cap) {
            grew = true;
            dfree(s->d_gsky);
            const int cap = (std::max(P.n_groups, 1024) + 3) & ~3;   // whole dwords (scalar loads)
            HIPCHK(hipMalloc((void**)&s->d_gsky, cap));
            s->gsky_cap = cap;
        }
        const int sblocks = (P.n_groups + 63) / 64;
        const int lcap = (sblocks + NQ - 1) / NQ * 64;          // most groups of the blocks b = q mod NQ
        const int need = lcap * NQ + P.n_groups;                // + the heavy live list (hist = 2)
        if (need > s->live_cap) {
            grew = true;
            dfree(s->d_live);
            HIPCHK(hipMalloc((void**)&s->d_live, (size_t)need * sizeof(int)));
            s->live_cap = need;
        }
        P.gsky = s->d_gsky;
        P.live = s->d_live; P.live_cap = lcap;
        if (s->n_slots > 1 && grew) { int r; if ((r = mirror_slot_caps(s)) != RT_OK) return r; }
        P.tpc = (part_k && P.lanes_per_px == 64) ? RT_TPC_WIDE : RT_TPC_LIVE;
        const Box* mbox = s->d_mesh_box;
        float sky_A = S.prune_abs, sky_B = 0x1p-12f;          // brute-force frames: the grown boxes' slack
        void* sargs[] = {&P, &S, &s->d_gsky, &s->d_live, &mbox, &sky_A, &sky_B};
        HIPCHK(hipExtLaunchKernel(sky_brute ? (const void*)sky_kernel<true> : (const void*)sky_kernel<false>, dim3(sblocks), dim3(SKY_THREADS), sargs, 0, st, e0, nullptr, 0));
    }
    void* args[] = {&P, &S};
    HIPCHK(hipExtLaunchKernel(fn, dim3(blocks), dim3(TRACE_BLOCK_P), args, shm, st, sky ? nullptr : e0, e1, 0));
    HIPCHK(hipGetLastError());
    return RT_OK;
}

#define CHECK_SCENE(s) do { if (!(s)) return fail(RT_ERR_ARG, "null scene"); } while (0)
#define CHECK_BUILDING(s) do { CHECK_SCENE(s); if ((s)->finished) return fail(RT_ERR_STATE, "scene already finished"); } while (0)
#define CHECK_FINISHED(s) do { CHECK_SCENE(s); if (!(s)->finished) return fail(RT_ERR_STATE, "scene not finished (call rt_builder_finish)"); } while (0)

rt::Material mat_from(const float* m) {
    rt::Material r;
    r.Ke = v4(m[0], m[1], m[2], m[3]); r.Ka = v4(m[4], m[5], m[6], m[7]); r.Kd = v4(m[8], m[9], m[10], m[11]);
    r.Ks = v4(m[12], m[13], m[14], m[15]); r.Kt = v4(m[16], m[17], m[18], m[19]); r.Kr = v4(m[20], m[21], m[22], m[23]);
    r.alpha = m[24]; r.eta = m[25];
    return r;
}

void invalidate(rt_scene* s) {
    s->bvh_valid = false;
    for (auto& o : s->store) o.bvh_valid = false;
}

}  // namespace

void free_multi(rt_scene* s);
rt_scene::~rt_scene() {
    free_multi(this);
    if (uploaded) (void)hipSetDevice(device);
    free_atlas(this);
    dfree(d_fnode);
    if (d_bscratch) (void)hipFree(d_bscratch);
    for (int p = 0; p < 2; p++) { dfree(d_hlist[p]); dfree(d_hflag[p]); }
    dfree(d_hctl);
    dfree(d_gsky); dfree(d_live);
    dfree(d_tris); dfree(d_meshes); dfree(d_insts); dfree(d_mats); dfree(d_lights); dfree(d_tri_ax);
    dfree(d_node_pair); dfree(d_leaf); dfree(d_inst4); dfree(d_work);
    dfree(d_mesh_box); dfree(d_tree); dfree(d_spp); dfree(d_stats); dfree(d_canvas); dfree(d_dbg);
    for (auto& p : d_out) dfree(p);
    for (auto& e : ev) if (e) (void)hipEventDestroy(e);
    for (auto& e : tev) (void)hipEventDestroy(e);
    auto hfree = [](auto*& p) { if (p) { (void)hipHostFree(p); p = nullptr; } };
    hfree(h_insts_pin); hfree(h_inst4_pin);
    for (int i = 0; i < MAX_SLOTS; i++) {                      // store[cur_slot] is the (freed) current state
        if (i == cur_slot) continue;
        Slot& o = store[i];
        dfree(o.d_tree); dfree(o.d_node_pair); dfree(o.d_leaf); dfree(o.d_fnode); dfree(o.d_work);
        if (o.d_bscratch) (void)hipFree(o.d_bscratch);
        for (int p = 0; p < 2; p++) { dfree(o.d_hlist[p]); dfree(o.d_hflag[p]); }
        dfree(o.d_hctl); dfree(o.d_gsky); dfree(o.d_live);
        dfree(o.d_insts); dfree(o.d_inst4);
        hfree(o.h_insts_pin); hfree(o.h_inst4_pin);
    }
    for (auto& e : slot_done) if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
}

// ---------------------------------------------------------------------------
// Multi-GPU frames from one host process (rt_scene_set_devices).  The frame is
// split row-cyclically into n_ranks slices (slice r = rows r, r + N, ...), the BVH and scene
// replicated on every device (each replica rebuilds the same tree from the same instance
// array, raytracer.cu:103-119), so the one exchange is the gather of the RGBA8 slices:
//   1. device i renders ranks [i k, (i+1) k) (k = n_ranks / n_devices) into its slice buffer
//      sbuf[i] = k slices of rows_max x W (compact rows; rows_max = ceil(H / N)), on its stream;
//   2. ncclGroupStart; per device ncclGather(sbuf[i], gbuf on device 0, k rows_max W uint32,
//      root 0, comm[i], stream[i]); ncclGroupEnd -- one communicator per device from
//      ncclCommInitAll, so rank order = device order = slice order;
//   3. device 0 un-permutes gbuf into the frame (unpermute_kernel).
// Several ranks per device ("virtual" ranks: n_ranks > n_devices) keep the same sequence, so a
// one-GPU box runs the whole call sequence with a one-rank communicator.  RCCL is opened
// with dlopen at the first multi-device frame (the copy torch loaded, if any): the library
// has no link-time RCCL dependency.
// ---------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(256) void unpermute_kernel(const uint32_t* __restrict__ g, uint32_t* __restrict__ out, int W,
                                                        int H, int N, int rows_max) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)W * H) return;
    const int y = (int)(i / W), x = (int)(i - (long long)y * W);
    out[i] = g[((size_t)(y % N) * rows_max + y / N) * W + x];         // frame row y = slice y % N, row y / N
}

struct Rccl {
    void* lib = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*err)(ncclResult_t) = nullptr;
};
Rccl* rccl(std::string* why) {
    static Rccl R;
    static std::string reason;
    static bool tried = false;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (!tried) {
        tried = true;
        for (const char* n : {"librccl.so", "librccl.so.1"})                 // the copy already loaded (torch's)
            if (!R.lib) R.lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
        for (const char* n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
            if (!R.lib) R.lib = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        if (!R.lib) { reason = std::string("cannot load RCCL: ") + dlerror(); }
        else {
            auto sym = [&](const char* n) { void* f = dlsym(R.lib, n); if (!f && reason.empty()) reason = std::string("RCCL lacks ") + n; return f; };
            R.comm_init_all = (decltype(R.comm_init_all))sym("ncclCommInitAll");
            R.comm_destroy = (decltype(R.comm_destroy))sym("ncclCommDestroy");
            R.gather = (decltype(R.gather))sym("ncclGather");
            R.group_start = (decltype(R.group_start))sym("ncclGroupStart");
            R.group_end = (decltype(R.group_end))sym("ncclGroupEnd");
            R.err = (decltype(R.err))sym("ncclGetErrorString");
        }
    }
    if (!reason.empty()) { if (why) *why = reason; return nullptr; }
    return &R;
}
}  // namespace

struct MultiDev {
    std::vector<int> devices;
    int n_ranks = 1, per_dev = 1, rows_max = 0, W = 0, H = 0;
    std::vector<rt_scene*> reps;                 // reps[0] = the scene itself; reps[i > 0] owned replicas
    std::vector<unsigned> inst_gen;              // host instance generation each replica holds
    std::vector<ncclComm_t> comms;               // one per device (ncclCommInitAll: rank = device order)
    // Frames in flight: the scene's frame slots (rt_scene_set_frame_slots) give `depth`; frame f
    // uses slot k = f % depth -- its own stream per device, slice buffers and gather buffer -- so
    // frame f + 1 renders while frame f gathers and un-permutes.  A slot's stream orders frame f
    // after frame f - depth, the last user of the slot's buffers.
    int depth = 0;
    long long frame = 0;
    std::vector<std::vector<hipStream_t>> streams;   // [device][slot]
    std::vector<std::vector<uint32_t*>> sbuf;        // [device][slot]: per_dev slices of rows_max x W
    std::vector<uint32_t*> gbuf;                     // [slot], device 0: n_ranks slices
    hipEvent_t ev_in = nullptr, ev_out = nullptr;    // device 0: caller's stream -> frame -> caller's stream
    // per device: the last frame's gather; the next frame's gather (another slot's stream) waits
    // for it, so operations on a communicator run in issue order whatever RCCL does across streams
    std::vector<hipEvent_t> gdone;
    bool gdone_pending = false;
};

namespace {
// The per-slot streams and buffers (and their device work) released; the replicas and the
// communicators stay.
void free_multi_slots(MultiDev* m) {
    for (size_t i = 0; i < m->streams.size(); i++) {
        (void)hipSetDevice(m->devices[i]);
        for (hipStream_t st : m->streams[i]) if (st) { (void)hipStreamSynchronize(st); (void)hipStreamDestroy(st); }
        if (i < m->sbuf.size()) for (uint32_t* b : m->sbuf[i]) if (b) (void)hipFree(b);
    }
    (void)hipSetDevice(m->devices[0]);
    for (uint32_t* b : m->gbuf) if (b) (void)hipFree(b);
    m->streams.clear(); m->sbuf.clear(); m->gbuf.clear();
    m->depth = 0;
}
}  // namespace

void free_multi(rt_scene* s) {
    MultiDev* m = s->multi;
    if (!m) return;
    s->multi = nullptr;
    s->ranks_per_device = 1;
    free_multi_slots(m);
    Rccl* R = rccl(nullptr);
    for (size_t i = 0; i < m->comms.size(); i++) {
        (void)hipSetDevice(m->devices[i]);
        if (R && m->comms[i]) (void)R->comm_destroy(m->comms[i]);
    }
    for (size_t i = 0; i < m->gdone.size(); i++) {
        (void)hipSetDevice(m->devices[i]);
        if (m->gdone[i]) (void)hipEventDestroy(m->gdone[i]);
    }
    (void)hipSetDevice(m->devices[0]);
    if (m->ev_in) (void)hipEventDestroy(m->ev_in);
    if (m->ev_out) (void)hipEventDestroy(m->ev_out);
    for (size_t i = 1; i < m->reps.size(); i++) delete m->reps[i];
    if (s->uploaded) (void)hipSetDevice(s->device);
    delete m;
}

namespace {
// Replica i's host scene brought up to the primary's: camera, environment, instance poses,
// atlas (the device copies follow at its next frame, as for any scene).
void sync_replica(rt_scene* s, MultiDev* m, size_t i) {
    rt_scene* r = m->reps[i];
    r->h.cam = s->h.cam; r->h.d_cam = s->h.d_cam;
    r->h.dist_atten = s->h.dist_atten; r->h.ambience = s->h.ambience; r->h.depth = s->h.depth;
    r->overlap = s->overlap;
    if (m->inst_gen[i] != s->inst_gen) {
        r->h.insts = s->h.insts; r->h.d_insts = s->h.d_insts;
        r->inst_gen++;
        invalidate(r);
        m->inst_gen[i] = s->inst_gen;
    }
    if (r->h.atlas_rgba.size() != s->h.atlas_rgba.size() || (s->atlas_dirty && !s->h.atlas_rgba.empty())) {
        r->h.atlas_rgba = s->h.atlas_rgba; r->h.atlas_w = s->h.atlas_w; r->h.atlas_h = s->h.atlas_h;
        r->atlas_dirty = true;
    }
}

// Replicas and communicators on first use; per-slot streams and buffers whenever the frame
// slots changed (the work in flight is waited for first).
int setup_multi(rt_scene* s, MultiDev* m, Rccl* R) {
    const int nd = (int)m->devices.size(), W = m->W;
    int r;
    for (int i = (int)m->reps.size(); i < nd; i++) {
        HIPCHK(hipSetDevice(m->devices[i]));
        rt_scene* rp = new rt_scene;
        rp->h = s->h; rp->finished = true;
        rp->h.atlas_rgba.clear();
        rp->overlap = s->overlap;
        rp->ranks_per_device = m->per_dev;
        m->reps.push_back(rp);
        m->inst_gen.push_back(0);
        const int saved = g_device;
        g_device = m->devices[i];
        r = upload(rp);
        g_device = saved;
        if (r != RT_OK) return r;
    }
    if (m->gdone.empty()) {
        m->gdone.assign(nd, nullptr);
        for (int i = 0; i < nd; i++) {
            HIPCHK(hipSetDevice(m->devices[i]));
            HIPCHK(hipEventCreateWithFlags(&m->gdone[i], hipEventDisableTiming));
        }
    }
    if (m->comms.empty()) {
        m->comms.assign(nd, nullptr);
        ncclResult_t e = R->comm_init_all(m->comms.data(), nd, m->devices.data());
        if (e != ncclSuccess) { m->comms.clear(); return fail(RT_ERR_HIP, std::string("ncclCommInitAll: ") + R->err(e)); }
    }
    HIPCHK(hipSetDevice(m->devices[0]));
    if (!m->ev_in) HIPCHK(hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming));
    if (!m->ev_out) HIPCHK(hipEventCreateWithFlags(&m->ev_out, hipEventDisableTiming));
    const int D = s->n_slots;
    if (m->depth == D) return RT_OK;
    free_multi_slots(m);
    for (int i = 1; i < nd; i++) {                             // replicas rotate as many frame slots
        m->reps[i]->overlap = s->overlap;
        if ((r = rt_scene_set_frame_slots(m->reps[i], D)) != RT_OK) return r;
    }
    m->streams.assign(nd, std::vector<hipStream_t>(D, nullptr));
    m->sbuf.assign(nd, std::vector<uint32_t*>(D, nullptr));
    m->gbuf.assign(D, nullptr);
    for (int i = 0; i < nd; i++) {
        HIPCHK(hipSetDevice(m->devices[i]));
        for (int k = 0; k < D; k++) {
            HIPCHK(hipStreamCreateWithFlags(&m->streams[i][k], hipStreamNonBlocking));
            HIPCHK(hipMalloc((void**)&m->sbuf[i][k], (size_t)m->per_dev * m->rows_max * W * 4));
        }
    }
    HIPCHK(hipSetDevice(m->devices[0]));
    for (int k = 0; k < D; k++) HIPCHK(hipMalloc((void**)&m->gbuf[k], (size_t)m->n_ranks * m->rows_max * W * 4));
    m->depth = D;
    m->frame = 0;
    m->gdone_pending = false;
    return RT_OK;
}

int render_multi(rt_scene* s, const rt_render_opts* o, rt_stats* stats) {
    MultiDev* m = s->multi;
    if (o->radiance || o->hit_inst || o->hit_tri) return fail(RT_ERR_ARG, "multi-device frames write RGBA8 only");
    std::string why;
    Rccl* R = rccl(&why);
    if (!R) return fail(RT_ERR_STATE, why);
    const int nd = (int)m->devices.size(), N = m->n_ranks, W = s->h.cam.W, H = s->h.cam.H;
    int r;
    if (m->W != W || m->H != H) return fail(RT_ERR_STATE, "canvas size changed after rt_scene_set_devices");
    if ((r = setup_multi(s, m, R)) != RT_OK) return r;
    for (int i = 1; i < nd; i++) sync_replica(s, m, i);
    const int k = (int)(m->frame % m->depth);
    hipStream_t caller = o->stream ? (hipStream_t)o->stream : nullptr;
    if (caller) {                                          // the caller's work before this frame (its output buffer)
        HIPCHK(hipSetDevice(m->devices[0]));
        HIPCHK(hipEventRecord(m->ev_in, caller));
    }
    unsigned long long tot[4] = {0, 0, 0, 0};
    double bvh_ms = 0, trace_ms = 0;
    // 1. every rank's slice, on its device's stream of this slot.  Event timing (o->timing)
    // covers the first device's ranks (the scene's own rt_timing_collect); replicas untimed.
    for (int i = 0; i < nd; i++) {
        double dev_bvh = 0, dev_trace = 0;
        for (int j = 0; j < m->per_dev; j++) {
            rt_render_opts so = *o;
            so.row0 = i * m->per_dev + j; so.row_step = N; so.compact = 1;
            so.rgba = m->sbuf[i][k] + (size_t)j * m->rows_max * W;
            so.stream = m->streams[i][k]; so.host_outputs = 0; so.sync = 0;
            if (i > 0) so.timing = 0;
            rt_stats st{};
            if ((r = rt_render(m->reps[i], &so, stats ? &st : nullptr)) != RT_OK) return r;
            if (stats) {
                tot[0] += st.rays; tot[1] += st.nodes; tot[2] += st.leaves; tot[3] += st.tri_tests;
                dev_bvh += st.bvh_ms; dev_trace += st.trace_ms;
            }
        }
        bvh_ms = std::max(bvh_ms, dev_bvh); trace_ms = std::max(trace_ms, dev_trace);
    }
    // 2. the gather to device 0 (one communicator per device, grouped)
    const size_t cnt = (size_t)m->per_dev * m->rows_max * W;
    if (m->gdone_pending)                                  // after the previous frame's gather (issue order)
        for (int i = 0; i < nd; i++) {
            HIPCHK(hipSetDevice(m->devices[i]));
            HIPCHK(hipStreamWaitEvent(m->streams[i][k], m->gdone[i], 0));
        }
    ncclResult_t e = R->group_start();
    for (int i = 0; i < nd && e == ncclSuccess; i++) {
        HIPCHK(hipSetDevice(m->devices[i]));
        e = R->gather(m->sbuf[i][k], i == 0 ? m->gbuf[k] : nullptr, cnt, ncclUint32, 0, m->comms[i], m->streams[i][k]);
    }
    ncclResult_t e2 = R->group_end();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) return fail(RT_ERR_HIP, std::string("ncclGather: ") + R->err(e));
    for (int i = 0; i < nd; i++) {
        HIPCHK(hipSetDevice(m->devices[i]));
        HIPCHK(hipEventRecord(m->gdone[i], m->streams[i][k]));
    }
    m->gdone_pending = true;
    // 3. un-permute on device 0 into the caller's buffer (after the caller's earlier work on it)
    // or the canvas
    HIPCHK(hipSetDevice(m->devices[0]));
    hipStream_t s0 = m->streams[0][k];
    if (caller) HIPCHK(hipStreamWaitEvent(s0, m->ev_in, 0));
    uint32_t* out = (o->rgba && !o->host_outputs) ? o->rgba : s->d_canvas;
    const long long px = (long long)W * H;
    hipLaunchKernelGGL(unpermute_kernel, dim3((unsigned)((px + 255) / 256)), dim3(256), 0, s0, m->gbuf[k], out, W, H, N,
                       m->rows_max);
    HIPCHK(hipGetLastError());
    if (caller) {                                          // the caller's stream continues after the frame
        HIPCHK(hipEventRecord(m->ev_out, s0));
        HIPCHK(hipStreamWaitEvent(caller, m->ev_out, 0));
    }
    m->frame++;
    if (o->sync || o->host_outputs || stats)               // this frame only: the other slots keep running
        for (int i = 0; i < nd; i++) { HIPCHK(hipSetDevice(m->devices[i])); HIPCHK(hipStreamSynchronize(m->streams[i][k])); }
    HIPCHK(hipSetDevice(m->devices[0]));
    if (o->host_outputs && o->rgba) HIPCHK(hipMemcpy(o->rgba, out, (size_t)px * 4, hipMemcpyDeviceToHost));
    if (stats) {
        // counters summed over ranks; bvh_ms / trace_ms: the slowest device's summed kernel times
        // (its ranks run one after another on its stream), the frame's parallel kernel time
        stats->rays = tot[0]; stats->nodes = tot[1]; stats->leaves = tot[2]; stats->tri_tests = tot[3];
        stats->bvh_ms = bvh_ms; stats->trace_ms = trace_ms;
    }
    return RT_OK;
}
}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_err.c_str(); }

int rt_device_count(int* count) {
    if (!count) return fail(RT_ERR_ARG, "null count");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RT_OK;
}

int rt_set_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RT_ERR_NODEV, "no HIP device available");
    if (device < 0 || device >= n) return fail(RT_ERR_ARG, "device index out of range");
    g_device = device;
    HIPCHK(hipSetDevice(device));
    return RT_OK;
}

// Profile marker (rt_profile_marker): an empty kernel whose grid (64 x tag threads) tells a
// rocprofv3 trace where a caller's timed region begins and ends (tools/pmc_step.py).
namespace {
__global__ __launch_bounds__(64) void profile_marker_kernel(int tag) { (void)tag; }

// rt_copy_engines_warm's gate: one wave that holds the copies queued behind it pending until the
// host opens the gate (a flag in coherent host memory) or `max_ticks` of the wall clock pass, so
// that every queued copy finds the engines of the copies before it busy.  Vector loads only.
__global__ __launch_bounds__(64) void copy_gate_kernel(const unsigned* flag, unsigned long long max_ticks) {
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u && wall_clock64() - t0 < max_ticks)
        __builtin_amdgcn_s_sleep(32);
}
}  // namespace

int rt_profile_marker(int tag, void* stream) {
    if (tag < 1 || tag > 64) return fail(RT_ERR_ARG, "marker tag must be 1..64");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RT_ERR_NODEV, "no HIP device available");
    hipLaunchKernelGGL(profile_marker_kernel, dim3(tag), dim3(64), 0, (hipStream_t)stream, tag);
    HIPCHK(hipGetLastError());
    return RT_OK;
}

int rt_spp_offset(int k, float* dx, float* dy) {
    if (k < 0 || !dx || !dy) return fail(RT_ERR_ARG, "bad arguments");
    rt::spp_offset(k, dx, dy);
    return RT_OK;
}

int rt_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes <= 0) return fail(RT_ERR_ARG, "bytes > 0 and an output pointer required");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RT_ERR_NODEV, "no HIP device available");
    HIPCHK(hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault));
    return RT_OK;
}
int rt_host_free(void* p) {
    if (p) HIPCHK(hipHostFree(p));
    return RT_OK;
}
// A device -> pinned-host copy on a DMA copy engine.  hipMemcpyDeviceToDeviceNoCU asks the
// runtime for the SDMA path explicitly (the copy still goes where the pointers live: with a
// hipHostMalloc destination it writes host memory over PCIe).  Measured on this image
// (tools/copy_probe.hip, profiles/r06/copy/): 8.29 MB in 0.157 ms (53 GB/s), finished 0.66 ms
// into a grid that held every CU for 3 ms, and no dispatch in the kernel trace; the torch
// pinned-tensor copy the round-5 bench used ran as 320-us `__amd_rocclr_copyBuffer` blit kernels
// that competed with the persistent trace blocks for CUs.
int rt_copy_to_host_async(void* host_dst, const void* dev_src, int64_t bytes, void* stream) {
    if (!host_dst || !dev_src || bytes < 0) return fail(RT_ERR_ARG, "null pointer or negative size");
    if (bytes == 0) return RT_OK;
    HIPCHK(hipMemcpyAsync(host_dst, dev_src, (size_t)bytes, hipMemcpyDeviceToDeviceNoCU, (hipStream_t)stream));
    return RT_OK;
}

// The runtime gives a stream's first copy (and a copy after the stream's last one has drained)
// an idle SDMA engine, and keeps the stream on that engine otherwise; a pipeline's copies queue
// behind frames still rendering, so as they pile up they land on engines 1, 2, 4, ... and the
// first copy on an engine in a direction creates that engine's queue: ~7 ms of host time inside
// hipMemcpyAsync (profiles/r06/rblog/).  Here each of the n streams queues one copy behind a
// gate kernel (on a stream of its own), so every copy finds the engines before it busy and the
// n copies start n engines; then the gate opens.  The streams should be the ones the pipeline
// will use.  Once per process and device for up to the largest n asked for.
int rt_copy_engines_warm(void* const* streams, int n) {
    if (!streams || n < 1 || n > 64) return fail(RT_ERR_ARG, "1 to 64 streams");
    int ndev = 0, dev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RT_ERR_NODEV, "no HIP device available");
    HIPCHK(hipGetDevice(&dev));
    static std::mutex mu;
    static int warmed[64] = {};
    std::lock_guard<std::mutex> lock(mu);
    if (dev < 0 || dev >= 64 || warmed[dev] >= n) return RT_OK;
    unsigned* flag = nullptr; uint8_t* h = nullptr; uint8_t* d = nullptr;
    hipStream_t gate = nullptr;
    hipEvent_t ev = nullptr;
    int clk_khz = 0;
    // (copies below the runtime's SDMA threshold run elsewhere: 1 MB each, all into one buffer)
    constexpr size_t B = 1 << 20;
    HIPCHK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, dev));
    HIPCHK(hipHostMalloc((void**)&flag, 4, hipHostMallocCoherent));
    HIPCHK(hipHostMalloc((void**)&h, B, hipHostMallocDefault));
    HIPCHK(hipMalloc((void**)&d, B));
    HIPCHK(hipMemset(d, 0, B));
    HIPCHK(hipStreamCreateWithFlags(&gate, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(copy_gate_kernel, dim3(1), dim3(64), 0, gate, (const unsigned*)flag,
                       (unsigned long long)clk_khz * 2000ull);                     // at most 2 s
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev, gate));
    hipError_t e = hipSuccess;
    for (int i = 0; i < n && e == hipSuccess; i++) {
        e = hipStreamWaitEvent((hipStream_t)streams[i], ev, 0);
        if (e == hipSuccess) e = hipMemcpyAsync(h, d, B, hipMemcpyDeviceToDeviceNoCU, (hipStream_t)streams[i]);
    }
    __atomic_store_n(flag, 1u, __ATOMIC_RELEASE);                              // open the gate
    HIPCHK(hipStreamSynchronize(gate));
    for (int i = 0; i < n; i++) HIPCHK(hipStreamSynchronize((hipStream_t)streams[i]));
    HIPCHK(e);
    (void)hipEventDestroy(ev);
    (void)hipStreamDestroy(gate);
    (void)hipFree(d); (void)hipHostFree(h); (void)hipHostFree(flag);
    warmed[dev] = n;
    return RT_OK;
}

// procedural::gpu::generate / SceneBuilder::build_gpu_scene put the scene on the device when it
// is made (cube_world.cc:195-207, scene_builder.cu:29-81); the first update_scene then only
// renders.  Here the upload is lazy (host-only scenes must load without a GPU), so a finished
// scene on a machine with a gfx950 device is uploaded at once and one untimed 1-spp frame is
// rendered into the device canvas: the code object, the scene's stream and the frame layout's
// buffers (sky flags, live lists, scheduling history) are then in place before the caller's
// first frame.  Without a usable device nothing happens (render calls report RT_ERR_NODEV as
// before); a failure here is left for the first render to report.  RT_NO_WARM=1 turns it off.
static int warm_scene(rt_scene* s);

int rt_scene_load_json(const char* path, int width, int height, rt_scene** out) {
    if (!path || !out) return fail(RT_ERR_ARG, "null argument");
    std::unique_ptr<rt_scene> s(new rt_scene);
    std::string err;
    int r = rt::load_cube_world(path, width, height, &s->h, &err);
    if (r == -2) return fail(RT_ERR_IO, err);
    if (r != 0) return fail(RT_ERR_PARSE, err);
    s->finished = true;
    s->canvas.assign((size_t)s->h.cam.W * s->h.cam.H, 0u);
    (void)warm_scene(s.get());
    *out = s.release();
    return RT_OK;
}

int rt_scene_create(const char* atlas, rt_scene** out) {
    if (!out) return fail(RT_ERR_ARG, "null argument");
    rt_scene* s = new rt_scene;
    s->h.atlas = atlas ? atlas : "";
    *out = s;
    return RT_OK;
}

int rt_scene_free(rt_scene* s) { delete s; return RT_OK; }

int rt_builder_add_vertex(rt_scene* s, float x, float y, float z, int* idx) {
    CHECK_BUILDING(s);
    int i = s->h.add_vertex(v3(x, y, z));
    if (idx) *idx = i;
    return RT_OK;
}
int rt_builder_create_mesh(rt_scene* s, const float* pos, const float* q, int* mesh) {
    CHECK_BUILDING(s);
    int m = s->h.create_mesh(pos ? v3(pos[0], pos[1], pos[2]) : v3(0, 0, 0), q ? Q{q[0], q[1], q[2], q[3]} : Q{0, 0, 0, 1});
    if (mesh) *mesh = m;
    return RT_OK;
}
int rt_builder_add_triangle(rt_scene* s, int mesh, int i0, int i1, int i2, const float* mat) {
    CHECK_BUILDING(s);
    if (!mat) return fail(RT_ERR_ARG, "null material");
    if (mesh < 0 || mesh >= (int)s->h.meshes.size()) return fail(RT_ERR_ARG, "mesh index out of range");
    int nv = (int)s->h.verts.size();
    if (i0 < 0 || i1 < 0 || i2 < 0 || i0 >= nv || i1 >= nv || i2 >= nv) return fail(RT_ERR_ARG, "vertex index out of range");
    s->h.add_triangle(mesh, i0, i1, i2, s->h.add_material(mat_from(mat)));
    return RT_OK;
}
int rt_builder_add_triangle_tex(rt_scene* s, int mesh, int i0, int i1, int i2, const float* mat, const float* tex) {
    CHECK_BUILDING(s);
    if (!mat || !tex) return fail(RT_ERR_ARG, "null argument");
    if (mesh < 0 || mesh >= (int)s->h.meshes.size()) return fail(RT_ERR_ARG, "mesh index out of range");
    int nv = (int)s->h.verts.size();
    if (i0 < 0 || i1 < 0 || i2 < 0 || i0 >= nv || i1 >= nv || i2 >= nv) return fail(RT_ERR_ARG, "vertex index out of range");
    rt::TexDesc t;
    t.has = 1; t.tx = tex[0]; t.ty = tex[1]; t.ux = tex[2]; t.uy = tex[3]; t.vx = tex[4]; t.vy = tex[5];
    s->h.add_triangle(mesh, i0, i1, i2, s->h.add_material(mat_from(mat)), t);
    return RT_OK;
}
int rt_builder_add_trans(rt_scene* s, int mesh, int* trans) {
    CHECK_BUILDING(s);
    if (mesh < 0 || mesh >= (int)s->h.meshes.size()) return fail(RT_ERR_ARG, "mesh index out of range");
    int t = s->h.add_trans(mesh);
    if (trans) *trans = t;
    return RT_OK;
}
int rt_builder_set_trans(rt_scene* s, int t, const float* pos, const float* q) {
    CHECK_SCENE(s);
    if (t < 0 || t >= (int)s->h.insts.size()) return fail(RT_ERR_ARG, "transformation index out of range");
    if (pos) s->h.insts[t].pos = v3(pos[0], pos[1], pos[2]);
    if (q) s->h.insts[t].rot = Q{q[0], q[1], q[2], q[3]};
    if (s->finished) {   // instances moved after finishing: refresh the flat copy
        // Device copies are per frame slot and are refreshed, stream-ordered, by the next frame
        // of each slot (sync_slot_insts): frames in flight keep the poses they were built from.
        s->h.d_insts[t].pose = make_pose(s->h.insts[t].rot, s->h.insts[t].pos);
        s->inst_gen++;
        invalidate(s);
    }
    return RT_OK;
}
int rt_builder_build_cube(rt_scene* s, float scale, const float* mat, int* mesh) {
    CHECK_BUILDING(s);
    if (!mat) return fail(RT_ERR_ARG, "null material");
    int m = s->h.build_cube(scale, mat_from(mat));
    if (mesh) *mesh = m;
    return RT_OK;
}
int rt_builder_build_cube_tex(rt_scene* s, float scale, const float* mat, const float* tile, int* mesh) {
    CHECK_BUILDING(s);
    if (!mat || !tile) return fail(RT_ERR_ARG, "null argument");
    int m = s->h.build_cube(scale, mat_from(mat), tile);
    if (mesh) *mesh = m;
    return RT_OK;
}
int rt_builder_add_point_light(rt_scene* s, const float* pos, const float* col) {
    CHECK_BUILDING(s);
    if (!pos || !col) return fail(RT_ERR_ARG, "null argument");
    s->h.add_point_light(v3(pos[0], pos[1], pos[2]), v4(col[0], col[1], col[2], col[3]));
    return RT_OK;
}
int rt_builder_add_directional_light(rt_scene* s, const float* dir, const float* col) {
    CHECK_BUILDING(s);
    if (!dir || !col) return fail(RT_ERR_ARG, "null argument");
    s->h.add_directional_light(v3(dir[0], dir[1], dir[2]), v4(col[0], col[1], col[2], col[3]));
    return RT_OK;
}
int rt_builder_finish(rt_scene* s, int W, int H, float fov, float unit, const float* cpos, const float* cq,
                      const float* da, const float* amb, int depth) {
    CHECK_BUILDING(s);
    if (W <= 0 || H <= 0 || !(unit > 0)) return fail(RT_ERR_ARG, "bad canvas/camera parameters");
    s->h.set_camera(W, H, fov, unit);
    if (cpos) s->h.cam.pos = v3(cpos[0], cpos[1], cpos[2]);
    if (cq) s->h.cam.rot = Q{cq[0], cq[1], cq[2], cq[3]};
    if (da) s->h.dist_atten = v3(da[0], da[1], da[2]);
    if (amb) s->h.ambience = v4(amb[0], amb[1], amb[2], amb[3]);
    s->h.depth = depth;
    std::string err;
    if (s->h.flatten(&err) != 0) return fail(RT_ERR_PARSE, err);
    s->finished = true;
    s->canvas.assign((size_t)W * H, 0u);
    (void)warm_scene(s);
    return RT_OK;
}

int rt_scene_info(const rt_scene* s, int32_t* c) {
    CHECK_FINISHED(s);
    if (!c) return fail(RT_ERR_ARG, "null argument");
    const rt::Scene& h = s->h;
    c[0] = h.cam.W; c[1] = h.cam.H; c[2] = (int)h.verts.size(); c[3] = (int)h.tris.size(); c[4] = (int)h.meshes.size();
    c[5] = (int)h.insts.size(); c[6] = (int)h.d_lights.size(); c[7] = (int)h.points.size(); c[8] = h.depth;
    c[9] = (int)h.mats.size();
    return RT_OK;
}

// (ABI 3) hit_tri indexes the triangles in flattened mesh order, so the meshes must list every
// triangle exactly once: a bitmap of the triangles seen, failing on a repeat or on one left out
// (a count alone would pass a list that repeats one triangle and omits another).
static bool meshes_cover_tris_once(const rt::Scene& h) {
    std::vector<unsigned char> seen(h.tris.size(), 0);
    size_t n = 0;
    for (auto& m : h.meshes)
        for (int i : m.tris) {
            if (i < 0 || (size_t)i >= seen.size() || seen[i]) return false;
            seen[i] = 1;
            n++;
        }
    return n == h.tris.size();
}

int rt_scene_export(const rt_scene* s, int what, void* dst, int64_t cap) {
    CHECK_FINISHED(s);
    const rt::Scene& h = s->h;
    if ((what == RT_EXPORT_TRIS || what == RT_EXPORT_TEXCOORDS) && !meshes_cover_tris_once(h))
        return fail(RT_ERR_STATE, "meshes do not cover every triangle once");
    std::vector<float> f;
    std::vector<int32_t> iv;
    switch (what) {
        case RT_EXPORT_VERTICES: for (auto& v : h.verts) { f.push_back(v.x); f.push_back(v.y); f.push_back(v.z); } break;
        case RT_EXPORT_NORMALS: f = h.verts_norm; break;
        case RT_EXPORT_TRIS:                                   // flattened (mesh) order: hit_tri indexes it
            for (auto& m : h.meshes)
                for (int i : m.tris) { const auto& t = h.tris[i]; iv.insert(iv.end(), {t.i0, t.i1, t.i2, t.mat}); }
            break;
        case RT_EXPORT_MATERIALS:
            for (auto& m : h.mats) {
                for (const V4* v : {&m.Ke, &m.Ka, &m.Kd, &m.Ks, &m.Kt, &m.Kr}) { f.push_back(v->x); f.push_back(v->y); f.push_back(v->z); f.push_back(v->w); }
                f.push_back(m.alpha); f.push_back(m.eta);
            }
            break;
        case RT_EXPORT_INSTANCES:
            for (auto& t : h.insts) { f.insert(f.end(), {t.rot.i, t.rot.j, t.rot.k, t.rot.r, t.pos.x, t.pos.y, t.pos.z}); }
            break;
        case RT_EXPORT_INST_MESH: for (auto& t : h.insts) iv.push_back(t.mesh); break;
        case RT_EXPORT_LIGHTS:
            for (auto& l : h.d_lights) f.insert(f.end(), {l.v.x, l.v.y, l.v.z, (float)l.type, l.col.x, l.col.y, l.col.z, l.col.w});
            break;
        case RT_EXPORT_CAMERA: {
            const DCamera& c = h.d_cam;
            f = {c.pos.x, c.pos.y, c.pos.z, h.cam.rot.i, h.cam.rot.j, h.cam.rot.k, h.cam.rot.r, c.near_, c.unit, c.W, c.H,
                 c.r.x, c.r.y, c.r.z, c.u.x, c.u.y, c.u.z, c.f.x, c.f.y, c.f.z, 0.0f};
            break;
        }
        case RT_EXPORT_ENV:
            f = {h.dist_atten.x, h.dist_atten.y, h.dist_atten.z, h.ambience.x, h.ambience.y, h.ambience.z, h.ambience.w};
            break;
        case RT_EXPORT_TEXCOORDS:
            for (auto& m : h.meshes)
                for (int i : m.tris) {
                    const auto& t = h.tris[i];
                    f.insert(f.end(), {(float)t.tex.has, t.tex.tx, t.tex.ty, t.tex.ux, t.tex.uy, t.tex.vx, t.tex.vy});
                }
            break;
        case RT_EXPORT_ATLAS: {
            const size_t n = h.atlas_rgba.size();
            if (!dst || cap < (int64_t)n) return fail(RT_ERR_ARG, "destination too small");
            if (n) memcpy(dst, h.atlas_rgba.data(), n);
            return RT_OK;
        }
        default: return fail(RT_ERR_ARG, "unknown export");
    }
    size_t bytes = f.size() * 4 + iv.size() * 4;
    if (!dst || cap < (int64_t)bytes) return fail(RT_ERR_ARG, "destination too small");
    if (!f.empty()) memcpy(dst, f.data(), f.size() * 4);
    if (!iv.empty()) memcpy(dst, iv.data(), iv.size() * 4);
    return RT_OK;
}

int rt_camera_get(const rt_scene* s, float* pos, float* q) {
    CHECK_SCENE(s);
    if (pos) { pos[0] = s->h.cam.pos.x; pos[1] = s->h.cam.pos.y; pos[2] = s->h.cam.pos.z; }
    if (q) { q[0] = s->h.cam.rot.i; q[1] = s->h.cam.rot.j; q[2] = s->h.cam.rot.k; q[3] = s->h.cam.rot.r; }
    return RT_OK;
}
int rt_camera_set(rt_scene* s, const float* pos, const float* q) {
    CHECK_FINISHED(s);
    if (pos) s->h.cam.pos = v3(pos[0], pos[1], pos[2]);
    if (q) s->h.cam.rot = Q{q[0], q[1], q[2], q[3]};
    s->h.update_camera_basis();
    return RT_OK;
}
int rt_camera_translate(rt_scene* s, const float* d) {           // entity.h:53-56: translate_global(vec_to_local(dp))
    CHECK_FINISHED(s);
    if (!d) return fail(RT_ERR_ARG, "null argument");
    s->h.cam.pos = s->h.cam.pos + qrot(s->h.cam.rot, v3(d[0], d[1], d[2]));
    s->h.update_camera_basis();
    return RT_OK;
}
int rt_camera_rotate(rt_scene* s, const float* dq) {             // entity.h:63-65: o = dr * o
    CHECK_FINISHED(s);
    if (!dq) return fail(RT_ERR_ARG, "null argument");
    s->h.cam.rot = qmul(Q{dq[0], dq[1], dq[2], dq[3]}, s->h.cam.rot);
    s->h.update_camera_basis();
    return RT_OK;
}
int rt_camera_axes(const rt_scene* s, float* r, float* u, float* f) {
    CHECK_FINISHED(s);
    const DCamera& c = s->h.d_cam;
    if (r) { r[0] = c.r.x; r[1] = c.r.y; r[2] = c.r.z; }
    if (u) { u[0] = c.u.x; u[1] = c.u.y; u[2] = c.u.z; }
    if (f) { f[0] = c.f.x; f[1] = c.f.y; f[2] = c.f.z; }
    return RT_OK;
}
int rt_env_set(rt_scene* s, const float* amb, const float* da, int depth) {
    CHECK_FINISHED(s);
    if (depth < 0 || depth >= MAX_FRAMES) return fail(RT_ERR_ARG, "depth must be in [0, 9]");
    if (amb) s->h.ambience = v4(amb[0], amb[1], amb[2], amb[3]);
    if (da) s->h.dist_atten = v3(da[0], da[1], da[2]);
    s->h.depth = depth;
    return RT_OK;
}

int rt_scene_set_atlas(rt_scene* s, const uint8_t* rgba8, int w, int h) {
    if (!s) return fail(RT_ERR_ARG, "null scene");
    if (!rgba8 || w <= 0 || h <= 0 || w > 16384 || h > 16384) return fail(RT_ERR_ARG, "bad atlas image");
    s->h.atlas_rgba.assign(rgba8, rgba8 + (size_t)w * h * 4);
    s->h.atlas_w = w; s->h.atlas_h = h;
    s->atlas_dirty = true;
    return RT_OK;
}
int rt_scene_load_atlas(rt_scene* s, const char* path) {
    if (!s) return fail(RT_ERR_ARG, "null scene");
    std::vector<std::string> tries;
    if (path) tries.push_back(path);
    else {
        if (s->h.atlas.empty()) return fail(RT_ERR_STATE, "the scene names no atlas");
        if (s->h.atlas[0] != '/' && !s->h.base_dir.empty()) tries.push_back(s->h.base_dir + "/" + s->h.atlas);
        tries.push_back(s->h.atlas);
    }
    std::string err;
    for (const std::string& p : tries) {
        std::ifstream probe(p, std::ios::binary);
        if (!probe) { err = p + ": cannot open"; continue; }
        std::vector<uint8_t> px;
        int w = 0, h = 0;
        if (rt::load_png_rgba8(p, &px, &w, &h, &err) != 0) return fail(RT_ERR_PARSE, err);
        return rt_scene_set_atlas(s, px.data(), w, h);
    }
    return fail(RT_ERR_IO, err);
}
int rt_scene_atlas_info(const rt_scene* s, int32_t* a) {
    if (!s || !a) return fail(RT_ERR_ARG, "null argument");
    a[0] = s->h.atlas_w; a[1] = s->h.atlas_h; a[2] = s->h.atlas_rgba.empty() ? 0 : 1;
    return RT_OK;
}

void rt_render_opts_default(rt_render_opts* o) {
    if (!o) return;
    memset(o, 0, sizeof *o);
    o->spp = 1; o->use_bvh = 1; o->rebuild_bvh = 1; o->row0 = 0; o->row_step = 1; o->kernel_dim = 16; o->sync = 1;
}

int rt_render(rt_scene* s, const rt_render_opts* o, rt_stats* stats) {
    CHECK_FINISHED(s);
    if (!o) return fail(RT_ERR_ARG, "null options");
    if (o->spp < 1 || o->row_step < 1 || o->row0 < 0) return fail(RT_ERR_ARG, "spp >= 1, row_step >= 1, row0 >= 0 required");
    int r;
    if ((r = upload(s)) != RT_OK) return r;
    HIPCHK(hipSetDevice(s->device));
    if ((size_t)s->h.cam.W * s->h.cam.H > (size_t)INT32_MAX) return fail(RT_ERR_LIMIT, "frame larger than 2^31 pixels");
    if (s->multi && o->row0 == 0 && o->row_step == 1) return render_multi(s, o, stats);   // whole frames: split
    if ((r = ensure_spp(s, o->spp)) != RT_OK) return r;
    hipStream_t st = o->stream ? (hipStream_t)o->stream : sstream(s);
    const bool timed = stats != nullptr;
    hipEvent_t* te = nullptr;
    if (o->timing) {
        if (s->tev_used + 4 > s->tev.size()) {
            if (s->tev.size() >= 4 * 4096) return fail(RT_ERR_STATE, "too many timed frames pending: call rt_timing_collect");
            for (int i = 0; i < 4 * 64; i++) { hipEvent_t e; HIPCHK(hipEventCreate(&e)); s->tev.push_back(e); }
        }
        te = &s->tev[s->tev_used];
        s->tev_used += 4;
    }
    if (s->n_slots > 1) {                                    // rotate frame slots (rt_scene_set_frame_slots)
        if ((r = ensure_other_slot(s)) != RT_OK) return r;
        select_slot(s, (s->cur_slot + 1) % s->n_slots);
    }
    if ((r = begin_frame(s, st, false)) != RT_OK) return r;  // after the slot's previous frame, current poses
    if (timed) { HIPCHK(hipMemsetAsync(s->d_stats, 0, STATS_N * sizeof(unsigned long long), st)); HIPCHK(hipEventRecord(s->ev[0], st)); }
    if (o->use_bvh && (o->rebuild_bvh || !s->bvh_valid)) {
        if ((r = build_bvh(s, st, te ? te[0] : nullptr, te ? te[1] : nullptr)) != RT_OK) {
            if (te) s->tev_used -= 4;                            // the frame's events stay unrecorded
            return r;
        }
    } else if (te) {
        HIPCHK(hipEventRecord(te[0], st)); HIPCHK(hipEventRecord(te[1], st));
    }
    if (timed) HIPCHK(hipEventRecord(s->ev[1], st));
    rt_render_opts oo = *o;
    const size_t W = s->h.cam.W, H = s->h.cam.H;
    const size_t n_rows = (H > (size_t)o->row0) ? (H - o->row0 + o->row_step - 1) / o->row_step : 0;
    const size_t out_px = o->compact ? n_rows * W : W * H;
    if (o->host_outputs) {                                   // stage through device buffers
        if (s->d_out_px < W * H) {
            for (auto& p : s->d_out) dfree(p);
            HIPCHK(hipMalloc(&s->d_out[0], W * H * 4)); HIPCHK(hipMalloc(&s->d_out[1], W * H * 16));
            HIPCHK(hipMalloc(&s->d_out[2], W * H * 4)); HIPCHK(hipMalloc(&s->d_out[3], W * H * 4));
            s->d_out_px = W * H;
        }
        oo.rgba = o->rgba ? (uint32_t*)s->d_out[0] : nullptr;
        oo.radiance = o->radiance ? (float*)s->d_out[1] : nullptr;
        oo.hit_inst = o->hit_inst ? (int32_t*)s->d_out[2] : nullptr;
        oo.hit_tri = o->hit_tri ? (int32_t*)s->d_out[3] : nullptr;
    }
    uint32_t* rgba = oo.rgba ? oo.rgba : s->d_canvas;
    if ((r = launch_trace(s, oo, st, rgba, nullptr, -1, -1, timed, -1, te ? te[2] : nullptr, te ? te[3] : nullptr)) != RT_OK) {
        if (te) s->tev_used -= 4;
        return r;
    }
    if (timed) HIPCHK(hipEventRecord(s->ev[2], st));
    if ((r = end_frame(s, st)) != RT_OK) return r;           // the slot is free again once this frame is done
    if (o->sync || timed || o->host_outputs) HIPCHK(hipStreamSynchronize(st));
    if (o->host_outputs) {
        if (o->rgba) HIPCHK(hipMemcpy(o->rgba, oo.rgba, out_px * 4, hipMemcpyDeviceToHost));
        if (o->radiance) HIPCHK(hipMemcpy(o->radiance, oo.radiance, out_px * 16, hipMemcpyDeviceToHost));
        if (o->hit_inst) HIPCHK(hipMemcpy(o->hit_inst, oo.hit_inst, out_px * 4, hipMemcpyDeviceToHost));
        if (o->hit_tri) HIPCHK(hipMemcpy(o->hit_tri, oo.hit_tri, out_px * 4, hipMemcpyDeviceToHost));
    }
    if (timed) {
        unsigned long long v[4];
        HIPCHK(hipMemcpy(v, s->d_stats, sizeof v, hipMemcpyDeviceToHost));
        stats->rays = v[0]; stats->nodes = v[1]; stats->leaves = v[2]; stats->tri_tests = v[3];
        float a = 0, b = 0;
        HIPCHK(hipEventElapsedTime(&a, s->ev[0], s->ev[1]));
        HIPCHK(hipEventElapsedTime(&b, s->ev[1], s->ev[2]));
        stats->bvh_ms = a; stats->trace_ms = b;
    }
    return RT_OK;
}


int rt_scene_set_frame_slots(rt_scene* s, int n) {
    CHECK_FINISHED(s);
    if (n < 1 || n > rt_scene::MAX_SLOTS) return fail(RT_ERR_ARG, "frame slots: 1 to " + std::to_string(rt_scene::MAX_SLOTS));
    if (n == s->n_slots) return RT_OK;
    if (s->uploaded) { HIPCHK(hipSetDevice(s->device)); HIPCHK(hipDeviceSynchronize()); }   // nothing in flight
    select_slot(s, 0);
    for (auto& p : s->slot_pending) p = false;
    s->n_slots = n;
    return (n > 1 && s->uploaded) ? ensure_other_slot(s) : RT_OK;
}

int rt_scene_set_overlap(rt_scene* s, int policy) {
    CHECK_SCENE(s);
    if (policy != RT_OVERLAP_HALF && policy != RT_OVERLAP_FULL && policy != RT_OVERLAP_STREAM)
        return fail(RT_ERR_ARG, "overlap policy: RT_OVERLAP_HALF, RT_OVERLAP_FULL or RT_OVERLAP_STREAM");
    s->overlap = policy;
    if (s->multi)                                              // the replicas of rt_scene_set_devices too
        for (rt_scene* rp : s->multi->reps) rp->overlap = policy;
    return RT_OK;
}

int rt_scene_set_devices(rt_scene* s, const int* devices, int n_devices, int n_ranks) {
    CHECK_FINISHED(s);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RT_ERR_NODEV, "no HIP device available");
    if (!devices || n_devices < 1 || n_ranks < n_devices || n_ranks % n_devices != 0)
        return fail(RT_ERR_ARG, "n_devices >= 1 device indices, n_ranks a multiple of n_devices");
    for (int i = 0; i < n_devices; i++) {
        if (devices[i] < 0 || devices[i] >= ndev) return fail(RT_ERR_ARG, "device index out of range");
        for (int j = 0; j < i; j++) if (devices[j] == devices[i]) return fail(RT_ERR_ARG, "a device listed twice");
    }
    if (n_ranks > s->h.cam.H) return fail(RT_ERR_ARG, "more ranks than canvas rows");
    int r;
    if (s->uploaded && s->device != devices[0]) return fail(RT_ERR_STATE, "devices[0] must be the scene's device");
    if (!s->uploaded) {
        const int saved = g_device;
        g_device = devices[0];
        r = upload(s);
        g_device = saved;
        if (r != RT_OK) return r;
    }
    HIPCHK(hipSetDevice(s->device));
    HIPCHK(hipDeviceSynchronize());
    free_multi(s);
    if (n_devices == 1 && n_ranks == 1) return RT_OK;       // back to single-device frames
    MultiDev* m = new MultiDev;
    m->devices.assign(devices, devices + n_devices);
    m->n_ranks = n_ranks; m->per_dev = n_ranks / n_devices;
    m->W = s->h.cam.W; m->H = s->h.cam.H;
    m->rows_max = (m->H + n_ranks - 1) / n_ranks;
    m->reps.push_back(s);
    m->inst_gen.push_back(s->inst_gen);
    s->multi = m;
    s->ranks_per_device = m->per_dev;
    return RT_OK;
}

int rt_timing_collect(rt_scene* s, double* bvh_ms, double* trace_ms, int* n) {
    CHECK_FINISHED(s);
    double a = 0, b = 0;
    for (size_t i = 0; i + 4 <= s->tev_used; i += 4) {
        HIPCHK(hipEventSynchronize(s->tev[i + 3]));
        float x = 0, y = 0;
        HIPCHK(hipEventElapsedTime(&x, s->tev[i], s->tev[i + 1]));
        HIPCHK(hipEventElapsedTime(&y, s->tev[i + 2], s->tev[i + 3]));
        a += x; b += y;
    }
    if (bvh_ms) *bvh_ms = a;
    if (trace_ms) *trace_ms = b;
    if (n) *n = (int)(s->tev_used / 4);
    s->tev_used = 0;
    return RT_OK;
}

int rt_update_scene(rt_scene* s, int kernel_dim, int optimize) {    // raytracer.cu:102-120
    CHECK_FINISHED(s);
    if (kernel_dim <= 0) return fail(RT_ERR_ARG, "kernel_dim must be positive");
    rt_render_opts o;
    rt_render_opts_default(&o);
    o.use_bvh = optimize ? 1 : 0; o.rebuild_bvh = 1; o.kernel_dim = kernel_dim;
    o.sync = s->multi ? 1 : 0;                                // split frames end on the slot's streams
    int r = rt_render(s, &o, nullptr);
    if (r != RT_OK) return r;
    // the canvas is host-readable on return (canvas.cu:23-29): one copy-engine transfer into the
    // pinned host canvas on the frame's stream, then wait for that stream only
    hipStream_t st = sstream(s);
    if (s->canvas.pinned)
        HIPCHK(hipMemcpyAsync(s->canvas.data(), s->d_canvas, s->canvas.size() * sizeof(uint32_t), hipMemcpyDeviceToDeviceNoCU, st));
    else
        HIPCHK(hipMemcpyAsync(s->canvas.data(), s->d_canvas, s->canvas.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return RT_OK;
}

static int warm_scene(rt_scene* s) {
    static const bool off = [] { const char* e = getenv("RT_NO_WARM"); return e && atoi(e) != 0; }();
    int n = 0;
    if (off || hipGetDeviceCount(&n) != hipSuccess || n <= 0) { (void)hipGetLastError(); return RT_OK; }
    const std::string saved = g_err;
    // update_scene's own path: a 1-spp frame and its copy into the pinned canvas (the copy starts
    // the copy engine's queue for device-to-host transfers, ~7 ms the first time)
    if (s->h.cam.W > 0 && s->h.cam.H > 0 && rt_update_scene(s, 16, 1) != RT_OK) {
        g_err = saved;                                    // left for the caller's first render to report
        (void)hipGetLastError();
        return RT_OK;
    }
    // capacity for the whole frame at 8 pixels per wave (4 x 2 groups: 8-32 spp, the bench's layout)
    const long long groups = (long long)((s->h.cam.W + 3) / 4) * ((s->h.cam.H + 1) / 2);
    if (groups < (1ll << 26) && reserve_layout(s, (int)groups) != RT_OK) { g_err = saved; (void)hipGetLastError(); }
    return RT_OK;
}

int rt_canvas_read(const rt_scene* s, uint32_t* dst, int64_t n) {
    CHECK_FINISHED(s);
    if (!dst || n < (int64_t)s->canvas.size()) return fail(RT_ERR_ARG, "destination too small");
    memcpy(dst, s->canvas.data(), s->canvas.size() * sizeof(uint32_t));
    return RT_OK;
}
const uint32_t* rt_canvas_host_ptr(const rt_scene* s) { return s ? s->canvas.data() : nullptr; }
int rt_canvas_get_color(const rt_scene* s, int x, int y, uint8_t* c) {
    CHECK_FINISHED(s);
    if (!c || x < 0 || y < 0 || x >= s->h.cam.W || y >= s->h.cam.H) return fail(RT_ERR_ARG, "pixel out of range");
    uint32_t e = s->canvas[(size_t)y * s->h.cam.W + x];                  // Color::from_encoding (color.cu:28-34)
    c[0] = (uint8_t)(e >> 24); c[1] = (uint8_t)(e >> 16); c[2] = (uint8_t)(e >> 8); c[3] = (uint8_t)e;
    return RT_OK;
}

int rt_debug_cast(rt_scene* s, int x, int y, char* buf, int64_t cap) {   // raytracer.cu:91-100
    CHECK_FINISHED(s);
    if (x < 0 || y < 0 || x >= s->h.cam.W || y >= s->h.cam.H) return fail(RT_ERR_ARG, "pixel out of range");
    int r;
    if ((r = upload(s)) != RT_OK) return r;
    HIPCHK(hipSetDevice(s->device));
    if ((r = ensure_spp(s, 1)) != RT_OK) return r;
    // rebuilds the current slot's BVH: first wait for every frame in flight (any slot)
    if ((r = begin_frame(s, sstream(s), true)) != RT_OK) return r;
    if ((r = build_bvh(s, sstream(s))) != RT_OK) return r;
    HIPCHK(hipMemsetAsync(s->d_dbg, 0, 4096 * sizeof(int), sstream(s)));
    rt_render_opts o;
    rt_render_opts_default(&o);
    o.row0 = y; o.row_step = s->h.cam.H;                                  // just the row of (x, y)
    if ((r = launch_trace(s, o, sstream(s), s->d_canvas, s->d_dbg, x, y, true)) != RT_OK) return r;
    if ((r = end_frame(s, sstream(s))) != RT_OK) return r;
    std::vector<int> log(4096);
    HIPCHK(hipStreamSynchronize(sstream(s)));
    HIPCHK(hipMemcpy(log.data(), s->d_dbg, log.size() * sizeof(int), hipMemcpyDeviceToHost));
    static const char* names[] = {"", "shooting a ray", "preparing to shoot a reflection ray",
                                  "preparing to shoot a refraction ray", "shooting shadow ray"};
    std::string out;
    int n = std::min(log[0], 4094);
    for (int i = 0; i < n; i++) { int e = log[2 + i]; if (e >= 1 && e <= 4) { out += names[e]; out += '\n'; } }
    if (buf && cap > 0) { size_t m = std::min<size_t>(out.size(), (size_t)cap - 1); memcpy(buf, out.data(), m); buf[m] = 0; }
    return RT_OK;
}

// Profiling aid (not part of rt_amd.h's stable surface): run experiment `which` `reps`
// times -- 4: the counted kernel with the occlusion early exit, 5: the counted kernel,
// 6: the fast kernel's PROF variant (wave step counts, cycle split, and the queries the
// fast kernel issues) -- and return the mean kernel ms and the counters.
int rt_experiment(rt_scene* s, int which, int spp, int reps, double* ms, uint64_t* counters) {
    CHECK_FINISHED(s);
    int r;
    if (which == 4 || which == 5 || which == 6) {             // full frame: counted kernel (4: occlusion exit on),
                                                              // 6: the fast kernel's profiling variant (M_PROF)
        if ((r = upload(s)) != RT_OK) return r;
        HIPCHK(hipSetDevice(s->device));
        if ((r = ensure_spp(s, spp)) != RT_OK) return r;
        rt_render_opts o; rt_render_opts_default(&o); o.spp = spp;
        if ((r = begin_frame(s, sstream(s), true)) != RT_OK) return r;   // nothing else in flight on this slot
        if ((r = build_bvh(s, sstream(s))) != RT_OK) return r;
        float total = 0;
        for (int i = 0; i < reps; i++) {
            HIPCHK(hipMemsetAsync(s->d_stats, 0, STATS_N * sizeof(unsigned long long), sstream(s)));
            HIPCHK(hipMemsetAsync(s->d_stats + 15, 0xff, sizeof(unsigned long long), sstream(s)));
            HIPCHK(hipMemsetAsync(s->d_stats + 19, 0xff, sizeof(unsigned long long), sstream(s)));
            HIPCHK(hipEventRecord(s->ev[0], sstream(s)));
            if ((r = (which == 6 ? launch_trace(s, o, sstream(s), s->d_canvas, nullptr, -1, -1, false, -1, nullptr, nullptr, true)
                                 : launch_trace(s, o, sstream(s), s->d_canvas, nullptr, -1, -1, true, which == 4 ? 1 : 0))) != RT_OK)
                return r;
            HIPCHK(hipEventRecord(s->ev[1], sstream(s)));
            HIPCHK(hipEventSynchronize(s->ev[1]));
            float t = 0; HIPCHK(hipEventElapsedTime(&t, s->ev[0], s->ev[1]));
            if (i > 0 || reps == 1) total += t;
        }
        if ((r = end_frame(s, sstream(s))) != RT_OK) return r;
        unsigned long long v[22];
        HIPCHK(hipMemcpy(v, s->d_stats, sizeof v, hipMemcpyDeviceToHost));
        if (counters) for (int i = 0; i < 22; i++) counters[i] = v[i];
        if (ms) *ms = total / (reps > 1 ? reps - 1 : 1);
        return RT_OK;
    }
    return fail(RT_ERR_ARG, "experiment: 4 (counted, occlusion exit), 5 (counted), 6 (fast kernel, PROF counters)");
}

int rt_frame_work(rt_scene* s, const rt_render_opts* o, rt_work* w) {
    CHECK_FINISHED(s);
    if (!o || !w) return fail(RT_ERR_ARG, "null argument");
    if (o->spp < 1 || o->spp > 64 || o->row_step < 1 || o->row0 < 0 || !o->use_bvh || o->textures)
        return fail(RT_ERR_ARG, "rt_frame_work: BVH frames, 1 <= spp <= 64, untextured");
    int r;
    if ((r = upload(s)) != RT_OK) return r;
    HIPCHK(hipSetDevice(s->device));
    if ((r = ensure_spp(s, o->spp)) != RT_OK) return r;
    const size_t rows = (s->h.cam.H > o->row0) ? (size_t)(s->h.cam.H - o->row0 + o->row_step - 1) / o->row_step : 0;
    uint32_t* d_rgba = nullptr;
    HIPCHK(hipMalloc((void**)&d_rgba, std::max<size_t>(1, (o->compact ? rows : (size_t)s->h.cam.H) * s->h.cam.W) * 4));
    hipStream_t st = sstream(s);
    r = begin_frame(s, st, true);                             // nothing else in flight on this slot
    if (r == RT_OK) r = build_bvh(s, st);
    if (r == RT_OK) {
        HIPCHK(hipMemsetAsync(s->d_stats, 0, STATS_N * sizeof(unsigned long long), st));
        HIPCHK(hipMemsetAsync(s->d_stats + 15, 0xff, sizeof(unsigned long long), st));
        HIPCHK(hipMemsetAsync(s->d_stats + 19, 0xff, sizeof(unsigned long long), st));
        rt_render_opts oo = *o;
        oo.radiance = nullptr; oo.hit_inst = oo.hit_tri = nullptr;
        r = launch_trace(s, oo, st, d_rgba, nullptr, -1, -1, false, -1, nullptr, nullptr, true);
    }
    if (r == RT_OK) r = end_frame(s, st);
    unsigned long long v[STATS_N] = {};
    if (r == RT_OK) {
        HIPCHK(hipStreamSynchronize(st));
        HIPCHK(hipMemcpy(v, s->d_stats, sizeof v, hipMemcpyDeviceToHost));
        if (v[4] == 0 && rows > 0) r = fail(RT_ERR_STATE, "no profiling variant of the fast kernel for this scene");
    }
    (void)hipFree(d_rgba);
    if (r != RT_OK) return r;
    w->queries = v[0]; w->wave_queries = v[4]; w->pair_steps = v[5]; w->leaf_visits = v[6]; w->tri_iters = v[7];
    w->leaf_lanes = v[2];
    w->scene_bytes = lds_bytes(view_of(s, true), true, true);   // the scene image a block stages
    w->lanes_primary = v[PROF_LANES_PRIMARY]; w->lanes_secondary = v[PROF_LANES_SECONDARY];
    w->lanes_shadow = v[PROF_LANES_SHADOW]; w->lanes_unlit = v[PROF_LANES_UNLIT];
    w->live_wave_queries = v[PROF_LIVE_WQ]; w->live_lanes = v[PROF_LIVE_LANES];
    for (int i = 0; i < 8; i++) {
        w->hist_wave_queries[i] = v[PROF_HIST_WQ + i];
        w->hist_pair_steps[i] = v[PROF_HIST_PAIR + i];
        w->hist_leaf_visits[i] = v[PROF_HIST_LEAF + i];
    }
    return RT_OK;
}

// Profiling aid (tools/group_profile.py, not on the product path): per-group durations
// (100 MHz ticks) of the fast frame kernel over rows row0, row0 + row_step, ... (compact),
// as bench.py's rank row0 of row_step renders them.  `reps` frames, each with the per-frame
// BVH rebuild; the last one (scheduled from the previous frame's history) is recorded.
// geo = {n_groups, gw, gh, n_gx}; *ms = the last frame's kernel time.  prof = 1: the recorded
// frame runs the PROF variant (when the scene has one) and out[n_groups + 12 g ..] holds group
// g's wave queries, child-pair steps, leaf visits, triangle iterations, then shader cycles in
// queries, in leaf visits, in trace_sample, after queries (state machine), and in the group; then
// (slots 9-11) cycles in the light step (ST_LIGHT), in the hit normal of a query's step, and in
// parking (writes before the query, reads after it; the reads also count in the query's cycles).
int rt_profile_groups(rt_scene* s, int spp, int row0, int row_step, int reps, int prof, uint32_t* out, int64_t cap,
                      int* geo, double* ms) {
    CHECK_FINISHED(s);
    if (!out || !geo || cap <= 0 || reps < 1 || row_step < 1 || row0 < 0) return fail(RT_ERR_ARG, "bad arguments");
    int r;
    if ((r = upload(s)) != RT_OK) return r;
    HIPCHK(hipSetDevice(s->device));
    if ((r = ensure_spp(s, spp)) != RT_OK) return r;
    const int rows = (s->h.cam.H - row0 + row_step - 1) / row_step;
    if (rows <= 0) return fail(RT_ERR_ARG, "no rows in the slice");
    rt_render_opts o; rt_render_opts_default(&o);
    o.spp = spp; o.row0 = row0; o.row_step = row_step; o.compact = 1;
    uint32_t* d_rgba = nullptr;
    unsigned* d_g = nullptr;
    HIPCHK(hipMalloc((void**)&d_rgba, (size_t)s->h.cam.W * rows * sizeof(uint32_t)));
    geo[0] = geo[1] = geo[2] = geo[3] = 0;
    reps = std::max(reps, 2);                                 // frame 0 sizes the buffer and seeds the history
    const int nw = prof ? 13 : 1;                             // prof: + 12 counters per group (PROF kernel)
    if ((r = begin_frame(s, sstream(s), true)) != RT_OK) { (void)hipFree(d_rgba); return r; }
    for (int i = 0; i < reps && r == RT_OK; i++) {
        const bool rec = i == reps - 1;
        if (rec) {
            if (geo[0] <= 0 || (int64_t)geo[0] * nw > cap) { r = fail(RT_ERR_LIMIT, "group buffer too small"); break; }
            HIPCHK(hipMalloc((void**)&d_g, (size_t)geo[0] * nw * sizeof(unsigned)));
            HIPCHK(hipMemsetAsync(d_g, 0, (size_t)geo[0] * nw * sizeof(unsigned), sstream(s)));
        }
        if ((r = build_bvh(s, sstream(s))) != RT_OK) break;
        r = launch_trace(s, o, sstream(s), d_rgba, nullptr, -1, -1, false, -1, s->ev[0], s->ev[1], rec && prof,
                         rec ? d_g : nullptr, geo);
    }
    if (r == RT_OK) r = end_frame(s, sstream(s));
    if (r == RT_OK) {
        HIPCHK(hipEventSynchronize(s->ev[1]));
        float t = 0;
        HIPCHK(hipEventElapsedTime(&t, s->ev[0], s->ev[1]));
        if (ms) *ms = t;
        HIPCHK(hipMemcpy(out, d_g, (size_t)geo[0] * nw * sizeof(unsigned), hipMemcpyDeviceToHost));
    }
    (void)hipFree(d_rgba);
    (void)hipFree(d_g);
    return r;
}

int rt_kat_device(const char* op, int n, const float* in0, const float* in1, const float* in2, float* of, int32_t* oi,
                  uint64_t* ou) {
    static const char* ops[] = {"normalize3", "cross", "reflect", "refract", "quat_rotate", "quat_inverse", "quat_mul",
                                "tri_hit", "ray_ctor", "zorder", "to_mat3", "box_hit", "pow", "tri_hit_f", "box_hit_f",
                                "box_pair", "rcp_cr", "sqrt_cr", "box_from_local", "box_merge", "entity"};
    // per-op sizes (floats): in0, in1, in2, out_f, out_i, out_u per element
    static const int sz[][6] = {{3, 0, 0, 3, 0, 0}, {3, 3, 0, 3, 0, 0}, {3, 3, 0, 3, 0, 0}, {3, 3, 2, 3, 1, 0},
                                {4, 3, 0, 3, 0, 0}, {4, 0, 0, 4, 0, 0}, {4, 4, 0, 4, 0, 0}, {9, 6, 0, 3, 1, 0},
                                {6, 0, 0, 6, 0, 0}, {3, 0, 0, 0, 0, 1}, {4, 0, 0, 9, 0, 0}, {7, 6, 0, 0, 1, 0},
                                {1, 1, 0, 1, 0, 0}, {9, 6, 0, 3, 1, 0}, {7, 6, 0, 0, 1, 0}, {14, 6, 0, 0, 2, 0},
                                {1, 0, 0, 1, 0, 0}, {1, 0, 0, 1, 0, 0}, {7, 7, 0, 6, 1, 0}, {7, 7, 0, 6, 1, 0},
                                {7, 3, 0, 12, 0, 0}};
    if (!op || n <= 0) return fail(RT_ERR_ARG, "bad arguments");
    int k = -1;
    for (int i = 0; i < (int)(sizeof ops / sizeof *ops); i++) if (!strcmp(op, ops[i])) k = i;
    if (k < 0) return fail(RT_ERR_ARG, std::string("unknown op ") + op);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RT_ERR_NODEV, "no HIP device available");
    HIPCHK(hipSetDevice(g_device));
    const float* hin[3] = {in0, in1, in2};
    float* din[3] = {nullptr, nullptr, nullptr};
    float* dof = nullptr; int* doi = nullptr; unsigned long long* dou = nullptr;
    for (int i = 0; i < 3; i++)
        if (sz[k][i]) {
            if (!hin[i]) return fail(RT_ERR_ARG, "missing input");
            HIPCHK(hipMalloc((void**)&din[i], (size_t)n * sz[k][i] * 4));
            HIPCHK(hipMemcpy(din[i], hin[i], (size_t)n * sz[k][i] * 4, hipMemcpyHostToDevice));
        }
    if (sz[k][3]) HIPCHK(hipMalloc((void**)&dof, (size_t)n * sz[k][3] * 4));
    if (sz[k][4]) HIPCHK(hipMalloc((void**)&doi, (size_t)n * sz[k][4] * 4));
    if (sz[k][5]) HIPCHK(hipMalloc((void**)&dou, (size_t)n * 8));
    hipLaunchKernelGGL(kat_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, k, n, din[0], din[1], din[2], dof, doi, dou);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    if (sz[k][3] && of) HIPCHK(hipMemcpy(of, dof, (size_t)n * sz[k][3] * 4, hipMemcpyDeviceToHost));
    if (sz[k][4] && oi) HIPCHK(hipMemcpy(oi, doi, (size_t)n * sz[k][4] * 4, hipMemcpyDeviceToHost));
    if (sz[k][5] && ou) HIPCHK(hipMemcpy(ou, dou, (size_t)n * 8, hipMemcpyDeviceToHost));
    for (auto p : din) if (p) (void)hipFree(p);
    if (dof) (void)hipFree(dof);
    if (doi) (void)hipFree(doi);
    if (dou) (void)hipFree(dou);
    return RT_OK;
}

}  // extern "C"
