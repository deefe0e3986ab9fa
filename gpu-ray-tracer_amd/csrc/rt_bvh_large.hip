// rt_bvh_large.hip — the per-frame BVH build for scenes above the single-workgroup limit
// (more than 8192 padded leaves): ropt::gpu::BVH::BVH (bvh.cu:11-91) and create_boxes
// (raytracer.cu:54-89) as a chain of grid-wide kernels on the frame's stream.
//
//   keys      per instance: world box, Morton key (gen_morton, bvh.cu:20-32), index
//   sort      hipCUB DeviceRadixSort::SortPairs over (key, index): LSD radix, stable, so
//             equal keys keep index order -- thrust::sort_by_key's order (bvh.cu:86)
//   level 0   reorder (bvh.cu:34-41): tree[i] = box of instance idx[i]
//   levels    one launch per pairwise merge level (build_bvh_layer, bvh.cu:43-61), the top
//             levels (<= 2048 boxes) in one single-block launch with barriers between them
//   heap      child-pair records + leaf instances (bvh_heap_node)
//   fnode     the ordered LBVH of the fast kernel (bvh_fnode)
// Every element is computed by the functions the single-workgroup kernel uses (rt_bvh.h),
// so both forms write the same tree.  The boxes live in HBM (Box[2n-1]); the sort's key
// and value buffers and hipCUB's temporary storage in the caller's scratch.
#include <hipcub/hipcub.hpp>

#include "rt_bvh.h"

namespace rtb {
namespace {

struct GlobalTree {
    Box* t;
    __device__ Box get(int i) const { return t[i]; }
};

constexpr int BT = 256;   // threads per block of the grid-wide phases

__global__ __launch_bounds__(BT) void large_keys_kernel(BvhArgs A, unsigned long long* keys, int* idx) {
    const int i = blockIdx.x * BT + threadIdx.x;
    if (blockIdx.x == 0) {                                     // the trace kernel's counters (as bvh_build_kernel)
        for (int w = threadIdx.x; w < A.n_work; w += BT) A.work[w] = 0;
        if (A.hctl && threadIdx.x < 2) A.hctl[threadIdx.x] = 0;
    }
    if (i >= A.n) return;
    keys[i] = bvh_key(bvh_inst_box(A, i));
    idx[i] = i;
}

__global__ __launch_bounds__(BT) void large_level0_kernel(BvhArgs A, const int* idx) {
    const int i = blockIdx.x * BT + threadIdx.x;
    if (i < A.n) A.tree[i] = bvh_inst_box(A, idx[i]);
}

// one level: tree[out + i] = merge(tree[lvl + 2i], tree[lvl + 2i + 1]), i < half
__global__ __launch_bounds__(BT) void large_level_kernel(Box* tree, int lvl, int out, int half) {
    const int i = blockIdx.x * BT + threadIdx.x;
    if (i < half) tree[out + i] = merge(tree[lvl + 2 * i], tree[lvl + 2 * i + 1]);
}

// the remaining levels, from `size` boxes at `lvl` up to the root, in one block
__global__ __launch_bounds__(1024) void large_top_kernel(Box* tree, int lvl, int out, int size) {
    while (size >= 2) {
        for (int i = threadIdx.x; i < size / 2; i += blockDim.x)
            tree[out + i] = merge(tree[lvl + 2 * i], tree[lvl + 2 * i + 1]);
        __syncthreads();
        lvl += size; out += size / 2; size >>= 1;
    }
}

__global__ __launch_bounds__(BT) void large_heap_kernel(BvhArgs A, const int* idx) {
    const int k = blockIdx.x * BT + threadIdx.x;
    if (k < 2 * A.n) bvh_heap_node(A, idx, GlobalTree{A.tree}, k);
}

__global__ __launch_bounds__(BT) void large_fnode_kernel(BvhArgs A, const unsigned long long* keys, const int* idx) {
    const int i = blockIdx.x * BT + threadIdx.x;
    if (i < A.n_real - 1) bvh_fnode(A, keys, idx, GlobalTree{A.tree}, i);
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t cub_temp_bytes(int n) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (int*)nullptr, (int*)nullptr, n, 0, 64);
    return tb;
}

}  // namespace

size_t bvh_large_scratch_bytes(int n) {
    return 2 * align256(8 * (size_t)n) + 2 * align256(4 * (size_t)n) + align256(cub_temp_bytes(n));
}

hipError_t bvh_build_large(const BvhArgs& A, void* scratch, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    const int n = A.n;
    char* p = static_cast<char*>(scratch);
    unsigned long long* k_in = reinterpret_cast<unsigned long long*>(p); p += align256(8 * (size_t)n);
    unsigned long long* k_out = reinterpret_cast<unsigned long long*>(p); p += align256(8 * (size_t)n);
    int* v_in = reinterpret_cast<int*>(p); p += align256(4 * (size_t)n);
    int* v_out = reinterpret_cast<int*>(p); p += align256(4 * (size_t)n);
    size_t tb = cub_temp_bytes(n);
    hipError_t e;
    auto blocks = [](long long m) { return dim3((unsigned)((m + BT - 1) / BT)); };
    if (e0 && (e = hipEventRecord(e0, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(large_keys_kernel, blocks(n), dim3(BT), 0, st, A, k_in, v_in);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(p, tb, k_in, k_out, v_in, v_out, n, 0, 64, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(large_level0_kernel, blocks(n), dim3(BT), 0, st, A, v_out);
    int lvl = 0, size = n, out = n;
    while (size > 2048) {
        hipLaunchKernelGGL(large_level_kernel, blocks(size / 2), dim3(BT), 0, st, A.tree, lvl, out, size / 2);
        lvl += size; out += size / 2; size >>= 1;
    }
    hipLaunchKernelGGL(large_top_kernel, dim3(1), dim3(1024), 0, st, A.tree, lvl, out, size);
    hipLaunchKernelGGL(large_heap_kernel, blocks(2LL * n), dim3(BT), 0, st, A, v_out);
    if (A.n_real >= 2) hipLaunchKernelGGL(large_fnode_kernel, blocks(A.n_real - 1), dim3(BT), 0, st, A, k_out, v_out);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (e1 && (e = hipEventRecord(e1, st)) != hipSuccess) return e;
    return hipSuccess;
}

}  // namespace rtb
