// rt_bvh.h — the per-frame BVH build shared by its two forms: the single-workgroup kernel
// (rt_kernels.hip, <= 8192 padded leaves) and the multi-kernel device build for larger
// scenes (rt_bvh_large.hip).  Both restate ropt::gpu::BVH::BVH (bvh.cu:11-91) and
// create_boxes (raytracer.cu:54-89) with the same per-element functions below, so they
// write identical trees.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_math.h"
#include "rt_scene.h"

namespace rtb {
using namespace rtm;
using rt::DInst;

struct BvhArgs {
    int* work; int n_work;   // the trace kernel's work counters, zeroed here (saves a memset launch)
    unsigned long long* hctl; // next frame's heavy-list counters (2 words), zeroed here too (may be null)
    const DInst* insts; int n_inst;
    const Box* mesh_box;     // per-mesh AABB, Trimesh::compute_bounding_box + the mesh pose (host, static)
    int n;                   // padded leaf count (power of two)
    Box* tree;               // 2n-1 boxes, reference storage order (global scratch when the LDS cannot hold it)
    float* node_pair;        // out: [12n] child-pair layout (BvhRefs); degenerate boxes: min=+inf, max=-inf
    float4* fnode;           // out: ordered LBVH of the fast kernel, [4 (n_real-1)] (see FNode below)
    int n_real;              // instances with a non-degenerate box (leaves of the ordered LBVH)
    int* leaf_inst;          // out: [n] instance of leaf node n+i
};

// Box storage of the build: the reference's level arrays (bvh.cu:43-61) as SoA columns
// (mn xyz, mx xyz, nd) in LDS -- conflict-free for consecutive boxes -- or the global
// Box array for trees too large for the LDS.
template <bool LDS_TREE> struct TreeStore;
template <> struct TreeStore<true> {
    float* f; int cap;
    __device__ Box get(int i) const {
        Box b;
        b.mn = v3(f[i], f[cap + i], f[2 * cap + i]); b.mx = v3(f[3 * cap + i], f[4 * cap + i], f[5 * cap + i]);
        b.nd = __float_as_int(f[6 * cap + i]);
        return b;
    }
    __device__ void put(int i, const Box& b) {
        f[i] = b.mn.x; f[cap + i] = b.mn.y; f[2 * cap + i] = b.mn.z;
        f[3 * cap + i] = b.mx.x; f[4 * cap + i] = b.mx.y; f[5 * cap + i] = b.mx.z;
        f[6 * cap + i] = __int_as_float(b.nd);
    }
};
template <> struct TreeStore<false> {
    Box* t;
    __device__ Box get(int i) const { return t[i]; }
    __device__ void put(int i, const Box& b) { t[i] = b; }
};
// LDS bytes of bvh_build_kernel<LDS_TREE>: keys u64[n] | idx int[n] | (tree 7 x f32 [2n-1])
__host__ __device__ inline size_t bvh_lds_bytes(int n, bool lds_tree) {
    return 12 * (size_t)n + (lds_tree ? 28 * (size_t)(2 * n - 1) : 0);
}

// Karras radix-tree node i over sorted 64-bit keys k[0, nr): range [first, last] and
// split gamma (left = [first, gamma], right = [gamma+1, last]); equal keys are told
// apart by their index (delta = 64 + clz(i ^ j)).
__host__ __device__ inline int fnode_delta(const unsigned long long* k, int nr, int i, int j) {
    if (j < 0 || j >= nr) return -1;
    const unsigned long long x = k[i] ^ k[j];
    if (x == 0) {
        const unsigned y = (unsigned)(i ^ j);
        return 64 + (y ? __builtin_clz(y) : 32);
    }
    return __builtin_clzll(x);
}
__host__ __device__ inline void fnode_split(const unsigned long long* k, int nr, int i, int& first, int& last, int& gamma) {
    const int d = fnode_delta(k, nr, i, i + 1) - fnode_delta(k, nr, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = fnode_delta(k, nr, i, i - d);
    int lmax = 2;
    while (fnode_delta(k, nr, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (fnode_delta(k, nr, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = fnode_delta(k, nr, i, j);
    int sp = 0;
    for (int div = 2;; div *= 2) {
        const int t = (l + div - 1) / div;
        if (fnode_delta(k, nr, i, i + (sp + t) * d) > dnode) sp += t;
        if (t <= 1) break;
    }
    gamma = i + sp * d + (d < 0 ? -1 : 0);
    first = i < j ? i : j;
    last = i < j ? j : i;
}

// Per-instance world box (create_boxes, raytracer.cu:54-74: from_local of the mesh box);
// padding [n_inst, n) is degenerate.
__device__ __forceinline__ Box bvh_inst_box(const BvhArgs& A, int i) {
    Box b; b.nd = 0; b.mn = b.mx = v3(0, 0, 0);
    if (i < A.n_inst) b = from_local(A.mesh_box[A.insts[i].mesh], A.insts[i].pose);
    return b;
}
// Morton key of a box (gen_morton, bvh.cu:20-32): ULONG_MAX for a degenerate box.
__device__ __forceinline__ unsigned long long bvh_key(const Box& b) { return b.nd ? z_order(neg(box_center(b))) : ~0ull; }

// Heap node k (1 <= k < 2n) lives at reference storage index 2n-1-k (bvh.h:51-53): its box
// into the child-pair records, and for a leaf its instance (the reference's ordering[]).
template <class TS>
__device__ __forceinline__ void bvh_heap_node(const BvhArgs& A, const int* idx, const TS& tree, int k) {
    const int n = A.n;
    Box b;
    b.nd = 0;
    if (k > 0) b = tree.get(2 * n - 1 - k);
    if (!b.nd) { b.mn = v3(INFINITY, INFINITY, INFINITY); b.mx = v3(-INFINITY, -INFINITY, -INFINITY); }
    float* q = A.node_pair + 12 * (k >> 1) + (k & 1);
    q[0] = b.mn.x; q[2] = b.mn.y; q[4] = b.mn.z; q[6] = b.mx.x; q[8] = b.mx.y; q[10] = b.mx.z;
    if (k >= n) A.leaf_inst[k - n] = idx[2 * n - 1 - k];
}

// Ordered LBVH (fast kernel): a radix tree (Karras 2012) over the same sorted leaves.
// Internal node i splits at the highest differing key bit; the child whose leaves are later
// in storage order is child A (visited first), so leaves are met in the heap's DFS order
// (heap leaf k <-> storage 2n-1-k).  Real leaves = storage [0, n_real) (padding sorts last).
template <class TS>
__device__ __forceinline__ void bvh_fnode(const BvhArgs& A, const unsigned long long* keys, const int* idx,
                                          const TS& tree, int i) {
    const int n = A.n, nr = A.n_real;
    int first, last, gamma;
    fnode_split(keys, nr, i, first, last, gamma);
    const int cl[2] = {gamma + 1, gamma}, lo[2] = {gamma + 1, first}, hi[2] = {last, gamma};
    float* q = reinterpret_cast<float*>(A.fnode + 4 * (size_t)i);
    int* refs = reinterpret_cast<int*>(A.fnode + 4 * (size_t)i + 3);
    for (int c = 0; c < 2; c++) {                   // c = 0: child A (later leaves), 1: child B
        // box of storage leaves [lo, hi]: the level arrays of A.tree are a segment
        // tree over storage order, so O(2 log n) aligned blocks cover the range
        // (min/max merges are exact, any grouping gives the same bounds)
        Box b;
        b.nd = 0; b.mn = b.mx = v3(0, 0, 0);
        for (int l = lo[c], r = hi[c] + 1, off = 0, size = n; l < r; l >>= 1, r >>= 1, off += size, size >>= 1) {
            if (l & 1) b = merge(b, tree.get(off + l++));
            if (r & 1) b = merge(b, tree.get(off + --r));
        }
        q[0 + c] = b.mn.x; q[2 + c] = b.mn.y; q[4 + c] = b.mn.z; q[6 + c] = b.mx.x; q[8 + c] = b.mx.y; q[10 + c] = b.mx.z;
        refs[c] = lo[c] == hi[c] ? -1 - idx[lo[c]] : cl[c];      // leaf: -1 - instance
    }
    refs[2] = refs[3] = 0;
}

// Device build for any padded leaf count (scenes above the single-workgroup limit): keys
// and boxes per instance, hipCUB's stable radix sort of (key, index) -- thrust's stable
// sort_by_key (bvh.cu:86) -- the reorder, one launch per level merge (bvh.cu:64-73 does the
// same for any n), the heap scatter and the ordered LBVH.  `scratch` holds
// bvh_large_scratch_bytes(n) bytes.  e0/e1 (optional) time the build on `st`.
size_t bvh_large_scratch_bytes(int n);
hipError_t bvh_build_large(const BvhArgs& A, void* scratch, hipStream_t st, hipEvent_t e0, hipEvent_t e1);

}  // namespace rtb
