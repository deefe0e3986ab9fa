// Probe: does the NUMA node of a pinned host buffer set the device->host copy-engine rate?
// Prints the GPU's nearest host NUMA node, the node the default hipHostMalloc pages land on and
// the thread's CPU, then times 40 copies of one 1080p RGBA8 frame (copy engine) into buffers
// bound to each NUMA node in turn (set_mempolicy + hipHostMallocNumaUser).
// Build: hipcc -O2 -o tools/numa_probe tools/numa_probe.cpp
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static const int MPOL_DEFAULT_ = 0, MPOL_BIND_ = 2;

static int page_node(void* p) {
    void* pages[1] = {p};
    int status[1] = {-99};
    if (syscall(SYS_move_pages, 0, 1ul, pages, nullptr, status, 0) != 0) return -100;
    return status[0];
}

static int n_nodes() {
    int n = 0;
    for (int i = 0; i < 64; i++) {
        char path[96];
        snprintf(path, sizeof path, "/sys/devices/system/node/node%d", i);
        if (access(path, F_OK) == 0) n = i + 1;
    }
    return n;
}

static float time_copies(void* h, void* d, size_t n, hipStream_t st) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms = 0;
    for (int w = 0; w < 2; w++) {
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 40; i++) CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToDeviceNoCU, st));
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
    }
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 40;
}

int main() {
    const size_t n = 1920ull * 1080 * 4;
    int numa = -1;
    CK(hipDeviceGetAttribute(&numa, hipDeviceAttributeHostNumaId, 0));
    const int nn = n_nodes();
    printf("gpu nearest host numa node %d, %d nodes, thread on cpu %d\n", numa, nn, sched_getcpu());
    void* d;
    CK(hipMalloc(&d, n));
    CK(hipMemset(d, 7, n));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    void* h;
    CK(hipHostMalloc(&h, n, hipHostMallocDefault));
    float ms = time_copies(h, d, n, st);
    printf("default alloc: pages on node %d / %d, %.4f ms per copy, %.1f GB/s\n", page_node(h),
           page_node((char*)h + n - 4096), ms, n / (ms * 1e-3) / 1e9);
    CK(hipHostFree(h));
    for (int node = 0; node < nn && node < 8; node++) {
        unsigned long mask = 1ul << node;
        if (syscall(SYS_set_mempolicy, MPOL_BIND_, &mask, 64ul) != 0) { printf("node %d: set_mempolicy failed\n", node); continue; }
        hipError_t e = hipHostMalloc(&h, n, hipHostMallocNumaUser);
        syscall(SYS_set_mempolicy, MPOL_DEFAULT_, nullptr, 0ul);
        if (e != hipSuccess) { printf("node %d: hipHostMalloc %s\n", node, hipGetErrorString(e)); continue; }
        ms = time_copies(h, d, n, st);
        printf("bound to node %d: pages on node %d, %.4f ms per copy, %.1f GB/s\n", node, page_node(h), ms,
               n / (ms * 1e-3) / 1e9);
        CK(hipHostFree(h));
    }
    // a ramp: back-to-back 40-copy windows for about 2 s; a link whose speed follows its load
    // shows the rate step up part-way through
    CK(hipHostMalloc(&h, n, hipHostMallocDefault));
    for (int w = 0; w < 60; w++) {
        ms = time_copies(h, d, n, st);
        if (w % 4 == 0 || w == 59) printf("ramp window %2d: %.1f GB/s\n", w, n / (ms * 1e-3) / 1e9);
    }
    for (int idle_ms : {10, 100, 1000}) {                     // then idle, then one window again
        usleep(idle_ms * 1000);
        ms = time_copies(h, d, n, st);
        printf("after %4d ms idle: %.1f GB/s\n", idle_ms, n / (ms * 1e-3) / 1e9);
    }
    CK(hipHostFree(h));
    return 0;
}
