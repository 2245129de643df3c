// Diagnostic: which XCD (HW_REG_XCC_ID) each workgroup of a launch runs on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(unsigned* o) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    if (threadIdx.x == 0) o[blockIdx.x] = x;
}
int main() {
    for (int bs : {64, 256}) {
        const int n = 32768;
        unsigned* d;
        hipMalloc(&d, n * 4);
        hipLaunchKernelGGL(k, dim3(n), dim3(bs), 0, 0, d);
        std::vector<unsigned> h(n);
        hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
        int m[8][8] = {};
        for (int b = 0; b < n; b++) m[b % 8][h[b] & 7]++;
        printf("block size %d: rows b%%8, cols xcc\n", bs);
        for (int r = 0; r < 8; r++) {
            for (int c = 0; c < 8; c++) printf("%6d", m[r][c]);
            printf("\n");
        }
        hipFree(d);
    }
}
