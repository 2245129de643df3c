// PCIe copy rates from/to pinned host memory, one direction and both at once
// (diagnostic).  build: hipcc --offload-arch=gfx950 -O2 tools/diag/pcie.hip -o tools/diag/pcie
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>

// a kernel that keeps every CU busy for about `cycles` clocks
__global__ void spin(unsigned long long cycles, int* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    int x = threadIdx.x;
    while (__builtin_amdgcn_s_memtime() - t0 < cycles) x = x * 1664525 + 1013904223;
    if (x == 0x7fffffff) sink[0] = x;
}

// copy device -> mapped pinned host memory with vector stores (a D2H that is not a copy-engine transfer)
__global__ void kcopy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    const size_t n = 256u << 20, piece = 16u << 20;
    const int reps = 4;
    void *h1, *h2, *d1, *d2;
    CK(hipHostMalloc(&h1, n, hipHostMallocDefault));
    CK(hipHostMalloc(&h2, n, hipHostMallocDefault));
    CK(hipMalloc(&d1, n));
    CK(hipMalloc(&d2, n));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto gbs = [&](std::chrono::steady_clock::time_point a, size_t bytes) {
        return bytes / std::chrono::duration<double>(now() - a).count() / 1e9;
    };
    for (int mode = 0; mode < 4; mode++) {
        // 0: H2D alone, 1: D2H alone, 2: both at once (whole buffers), 3: both at once in 16 MiB pieces
        CK(hipDeviceSynchronize());
        auto t = now();
        for (int r = 0; r < reps; r++) {
            if (mode == 0 || mode == 2) CK(hipMemcpyAsync(d1, h1, n, hipMemcpyHostToDevice, s1));
            if (mode == 1 || mode == 2) CK(hipMemcpyAsync(h2, d2, n, hipMemcpyDeviceToHost, s2));
            if (mode == 3)
                for (size_t o = 0; o < n; o += piece) {
                    CK(hipMemcpyAsync((char*)d1 + o, (char*)h1 + o, piece, hipMemcpyHostToDevice, s1));
                    CK(hipMemcpyAsync((char*)h2 + o, (char*)d2 + o, piece, hipMemcpyDeviceToHost, s2));
                }
        }
        CK(hipDeviceSynchronize());
        const char* name[] = {"h2d alone", "d2h alone", "both, whole", "both, 16 MiB pieces"};
        printf("%-20s %.1f GB/s per direction\n", name[mode], gbs(t, n * reps));
    }
    // H2D while a kernel holds every CU (the pipeline's persistent k_zh does): is the copy an SDMA
    // transfer that runs beside it, or a blit kernel that waits for CUs?
    int* sink;
    CK(hipMalloc(&sink, 4));
    hipStream_t s3;
    CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
    for (int withk = 0; withk < 2; withk++) {
        CK(hipDeviceSynchronize());
        if (withk) hipLaunchKernelGGL(spin, dim3(256 * 8), dim3(256), 0, s3, 100000000ull, sink);  // ~45 ms
        auto t = now();
        for (int r = 0; r < reps; r++) CK(hipMemcpyAsync(d1, h1, n, hipMemcpyHostToDevice, s1));
        CK(hipStreamSynchronize(s1));
        printf("h2d %s: %.1f GB/s\n", withk ? "beside a kernel on every CU" : "alone", gbs(t, n * reps));
        CK(hipDeviceSynchronize());
    }
    // D2H by a kernel's stores into mapped pinned memory, alone and beside an SDMA H2D
    void* hm;
    uint4* dm;
    CK(hipHostMalloc(&hm, n, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&dm, hm, 0));
    for (int both = 0; both < 2; both++) {
        for (int grid : {64, 256, 1024}) {
            CK(hipDeviceSynchronize());
            auto t = now();
            for (int r = 0; r < reps; r++) {
                if (both) CK(hipMemcpyAsync(d1, h1, n, hipMemcpyHostToDevice, s1));
                hipLaunchKernelGGL(kcopy, dim3(grid), dim3(256), 0, s2, (const uint4*)d2, dm, n / 16);
            }
            CK(hipDeviceSynchronize());
            printf("kernel-store d2h, grid %d%s: %.1f GB/s per direction\n", grid, both ? ", beside SDMA h2d" : "",
                   gbs(t, n * reps));
        }
    }
    return 0;
}
