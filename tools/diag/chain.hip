// chain.hip — what one wave pays per rune for k_long_dp's DP step (config 5b) when
// nothing waits on memory: every operand in registers, the step forms chosen by a
// wave-uniform pseudo-random class per rune with 5b's mix (55 % one item, 28 % two
// items L = 1, 2, 17 % up to four), cycles from s_memtime around the loop.
//   V0: one branch-free form for every rune (4 f64 adds, max, 2 compares, 2 selects)
//   V1: a scalar branch per rune: one item -> 1 add; (1, 2) -> 2 adds + max; else V0
//   V2: a pure dependent f64 add chain (the floor: one add per rune)
//   V3: V0 rewritten so that the chain is one add and one max per rune (the rest,
//       from best(s + 2 ..), off the chain: P = max(w1' + best(s + 1), q))
//   V4: every rune (1) or (1, 2): P = max(w1 + best(s + 1), w2 + best(s + 2))
//   V5: per group of four, a scalar branch: V4 for half the groups, V3 for the rest
//   V6: four independent add chains (the issue cost of v_add_f64)
//   V9 = V0 and V10 = V4 with the group loop unrolled 4 times (a back-edge per 16 runes)
//   (V1 and V5 came out as the sum of their forms: the compiler computes every form
//   and selects.  V7 = V1 and V8 = V5 with V0 for the rest, with real branches.)
// Diagnostic tool, not part of the product.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/diag/chain tools/diag/chain.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__device__ __forceinline__ double max_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int V>
__global__ __launch_bounds__(64) void k_chain(const double* __restrict__ wt, uint32_t n, double* __restrict__ out,
                                              unsigned long long* __restrict__ clk) {
    double W[4][4];
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
        for (int k = 0; k < 4; k++) W[u][k] = wt[u * 4 + k];
    double H0 = 0.0, H1 = 0.0, H2 = 0.0, H3 = 0.0;
    uint32_t x = 12345u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    constexpr int UNR = V >= 9 ? 4 : 1;
    for (uint32_t g = 0; g < n; g += 4 * UNR)
#pragma unroll
    for (int gg = 0; gg < UNR; gg++) {
        x = x * 1664525u + 1013904223u;
        const uint32_t cw = __builtin_amdgcn_readfirstlane(x);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t f = (cw >> (8 * u)) & 0xFFu;  // < 140: one item, < 213: (1, 2), else general
            double P;
            if (V == 2) {
                P = W[u][0] + H0;
            } else if (V == 4 || V == 10 || (V == 5 && (cw & 0x80000000u))) {  // every rune (1) or (1, 2)
                P = max_f64(W[u][0] + H0, W[u][1] + H1);
            } else if (V == 3 || V == 5) {  // the chain only adds and takes a max
                const double p2 = W[u][1] + H1, p3 = W[u][2] + H2, p4 = W[u][3] + H3;
                const bool k3 = p3 >= p2, k4 = p4 >= p3, X = k3 || k4;
                const double q = X ? (k4 ? p4 : p3) : p2;
                const double w1 = X ? -__builtin_inf() : W[u][0];
                P = max_f64(w1 + H0, q);
            } else if (V == 6) {  // independent adds: issue cost
                H1 = W[u][1] + H1;
                H2 = W[u][2] + H2;
                H3 = W[u][3] + H3;
                P = W[u][0] + H0;
                H0 = P;
                continue;
            } else if (V == 7 && f < 140u) {  // V1 with real branches (volatile asm: no if-conversion)
                asm volatile("; one item");
                P = W[u][0] + H0;
            } else if (V == 7 && f < 213u) {
                asm volatile("; two items");
                P = max_f64(W[u][0] + H0, W[u][1] + H1);
            } else if (V == 8 && (cw & 0x80000000u)) {  // per group: V4 or V0, real branches
                asm volatile("; group of (1) / (1, 2)");
                P = max_f64(W[u][0] + H0, W[u][1] + H1);
            } else if (V == 1 && f < 140u) {
                P = W[u][0] + H0;
            } else if (V == 1 && f < 213u) {
                P = max_f64(W[u][0] + H0, W[u][1] + H1);
            } else {
                const double p1 = W[u][0] + H0, p2 = W[u][1] + H1, p3 = W[u][2] + H2, p4 = W[u][3] + H3;
                const double R = max_f64(p1, p2);
                const bool k3 = p3 >= p2, k4 = p4 >= p3;
                const double p34 = k4 ? p4 : p3;
                P = (k3 || k4) ? p34 : R;
            }
            H3 = H2;
            H2 = H1;
            H1 = H0;
            H0 = P;
        }
        (void)0;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = H0 + H1 + H2 + H3;
        clk[0] = t1 - t0;
    }
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    double hw[16];
    for (int i = 0; i < 16; i++) hw[i] = -3.0 - 0.37 * i;  // (finite, distinct)
    hw[7] = __builtin_nan("");  // some absent items, as in the real descriptors
    hw[11] = __builtin_nan("");
    hw[15] = __builtin_nan("");
    double *dw, *dout;
    unsigned long long* dclk;
    CHK(hipMalloc(&dw, sizeof hw));
    CHK(hipMalloc(&dout, 8));
    CHK(hipMalloc(&dclk, 8));
    CHK(hipMemcpy(dw, hw, sizeof hw, hipMemcpyHostToDevice));
    for (int v = 0; v < 11; v++) {
        for (int rep = 0; rep < 2; rep++) {
            if (v == 0) k_chain<0><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 1) k_chain<1><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 2) k_chain<2><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 3) k_chain<3><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 4) k_chain<4><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 5) k_chain<5><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 6) k_chain<6><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 7) k_chain<7><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 8) k_chain<8><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 9) k_chain<9><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 10) k_chain<10><<<1, 64>>>(dw, n, dout, dclk);
            CHK(hipDeviceSynchronize());
        }
        unsigned long long c;
        double o;
        CHK(hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(&o, dout, 8, hipMemcpyDeviceToHost));
        printf("{\"variant\": %d, \"runes\": %u, \"cycles_per_rune\": %.2f, \"sink\": %g}\n", v, n, (double)c / n, o);
    }
    return 0;
}
