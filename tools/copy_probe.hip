// Probe: which device->pinned-host copy forms run on a copy engine (no CU) on this ROCm.
// Usage: copy_probe MODE [bytes [hipHostMalloc flags]]; MODE = d2h | default | nocu.
// Prints the mean copy time of 40 copies, then the completion time of one copy issued while a
// grid that holds every CU spins for 3 ms on another stream: a copy that needs a CU (a blit
// kernel) finishes after the spin, a copy-engine copy finishes long before it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void __launch_bounds__(1024) spin(unsigned long long ticks, int* out) {
    __shared__ int pad[40000];                         // 160 KB: one block per CU
    const unsigned long long t0 = wall_clock64();
    int acc = threadIdx.x;
    while (wall_clock64() - t0 < ticks) acc += 1;
    pad[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0 && acc == -1) out[blockIdx.x] = pad[1];
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "d2h";
    size_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1920ull * 1080 * 4;
    hipMemcpyKind kind = !strcmp(mode, "nocu") ? hipMemcpyDeviceToDeviceNoCU
                       : !strcmp(mode, "default") ? hipMemcpyDefault : hipMemcpyDeviceToHost;
    void *d, *h; int* dout;
    CK(hipMalloc(&d, n)); CK(hipMalloc(&dout, 4096 * 4));
    const unsigned hflags = argc > 3 ? (unsigned)strtoul(argv[3], nullptr, 0) : hipHostMallocDefault;
    CK(hipHostMalloc(&h, n, hflags));
    std::vector<unsigned> src(n / 4);
    for (size_t i = 0; i < src.size(); i++) src[i] = (unsigned)(i * 2654435761u);
    CK(hipMemcpy(d, src.data(), n, hipMemcpyHostToDevice));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    memset(h, 0, n);
    CK(hipMemcpyAsync(h, d, n, kind, a));                // warm-up + check
    CK(hipStreamSynchronize(a));
    if (memcmp(h, src.data(), n)) { printf("%s: DATA MISMATCH\n", mode); return 2; }
    CK(hipEventRecord(e0, a));
    for (int i = 0; i < 40; i++) CK(hipMemcpyAsync(h, d, n, kind, a));
    CK(hipEventRecord(e1, a));
    CK(hipStreamSynchronize(a));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s: %zu B, %.4f ms per copy, %.1f GB/s\n", mode, n, ms / 40, n / (ms / 40 * 1e-3) / 1e9);
    // the same 40 copies into further fresh host buffers, the first one still held
    for (int k = 0; k < 3; k++) {
        void* hk; CK(hipHostMalloc(&hk, n, hflags));
        for (int w = 0; w < 2; w++) {
            CK(hipEventRecord(e0, a));
            for (int i = 0; i < 40; i++) CK(hipMemcpyAsync(hk, d, n, kind, a));
            CK(hipEventRecord(e1, a));
            CK(hipStreamSynchronize(a));
        }
        float mk = 0;
        CK(hipEventElapsedTime(&mk, e0, e1));
        printf("%s: host buffer %d: %.4f ms per copy, %.1f GB/s\n", mode, k + 2, mk / 40, n / (mk / 40 * 1e-3) / 1e9);
        CK(hipHostFree(hk));
    }
    // the same 40 copies on each of 8 fresh streams in turn: a fresh stream may get another engine
    for (int k = 0; k < 8; k++) {
        hipStream_t sk; CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
        for (int w = 0; w < 2; w++) {
            CK(hipEventRecord(e0, sk));
            for (int i = 0; i < 40; i++) CK(hipMemcpyAsync(h, d, n, kind, sk));
            CK(hipEventRecord(e1, sk));
            CK(hipStreamSynchronize(sk));
        }
        float mk = 0;
        CK(hipEventElapsedTime(&mk, e0, e1));
        printf("%s: fresh stream %d: %.4f ms per copy, %.1f GB/s\n", mode, k, mk / 40, n / (mk / 40 * 1e-3) / 1e9);
    }
    // the same bytes as two halves on two streams at once (two copy engines)
    {
        hipStream_t c2; CK(hipStreamCreateWithFlags(&c2, hipStreamNonBlocking));
        hipEvent_t f0, f1; CK(hipEventCreate(&f0)); CK(hipEventCreate(&f1));
        const size_t h2 = (n / 2) & ~(size_t)255;
        for (int w = 0; w < 2; w++) {                                      // w = 0: warm both engines
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, a));
            CK(hipStreamWaitEvent(c2, e0, 0));
            for (int i = 0; i < 40; i++) {
                CK(hipMemcpyAsync(h, d, h2, kind, a));
                CK(hipMemcpyAsync((char*)h + h2, (const char*)d + h2, n - h2, kind, c2));
            }
            CK(hipEventRecord(f0, c2));
            CK(hipStreamWaitEvent(a, f0, 0));
            CK(hipEventRecord(e1, a));
            CK(hipStreamSynchronize(a));
        }
        float m2 = 0;
        CK(hipEventElapsedTime(&m2, e0, e1));
        if (memcmp(h, src.data(), n)) { printf("%s split: DATA MISMATCH\n", mode); return 2; }
        printf("%s split over two streams: %.4f ms per frame, %.1f GB/s\n", mode, m2 / 40, n / (m2 / 40 * 1e-3) / 1e9);
    }
    int dev = 0, freq = 0, ncu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&freq, hipDeviceAttributeWallClockRate, dev));     // kHz
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    unsigned long long ticks = (unsigned long long)freq * 3;                     // 3 ms
    CK(hipEventRecord(e0, b));
    hipLaunchKernelGGL(spin, dim3(ncu), dim3(1024), 0, b, ticks, dout);
    CK(hipEventRecord(e2, b));
    CK(hipStreamWaitEvent(a, e0, 0));
    CK(hipMemcpyAsync(h, d, n, kind, a));
    CK(hipEventRecord(e1, a));
    CK(hipDeviceSynchronize());
    float tc = 0, ts = 0;
    CK(hipEventElapsedTime(&tc, e0, e1));
    CK(hipEventElapsedTime(&ts, e0, e2));
    printf("%s: copy beside a 3 ms all-CU spin done at %.3f ms (spin done at %.3f ms): %s\n", mode, tc, ts,
           tc < 0.8 * ts ? "copy engine" : "needs CUs");
    return 0;
}
