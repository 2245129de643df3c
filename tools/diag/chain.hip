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
//   V11: items with L <= 3 in any pattern, P = max(w1' + best(s+1), max(v2, v3)) with
//        w1' = -Inf when v3 >= v2 (8 VALU); V12: at most 3 items with L <= 4 (12 VALU)
//   V13: every subset of lengths 2..4 (P = max(k ? -Inf : p1, c34 ? v4 : max(v2, v3, v4))),
//        V14 the same unrolled 4 times, V15 = V11 unrolled 4 times; V16: per group a
//        branch (17 % of groups V13's form, the rest V11's), unrolled twice
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
    constexpr int UNR = (V == 9 || V == 10 || V == 14 || V == 15) ? 4 : (V == 16 ? 2 : 1);
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
            } else if (V == 13 || V == 14 || (V == 16 && (cw & 0xFFu) < 43u)) {  // universal (<= 4 items, L <= 4)
                const double v2 = W[u][1] + H1, v3 = W[u][2] + H2, v4 = W[u][3] + H3;
                const bool c34 = v4 >= v3, k = (v3 >= v2) || (v4 >= v2) || c34;
                const double Q = c34 ? v4 : max_f64(max_f64(v2, v3), v4);
                const double w1 = k ? -__builtin_inf() : W[u][0];
                P = max_f64(w1 + H0, Q);
            } else if (V == 11 || V == 15 || V == 16) {  // items L <= 3, any gaps
                const double v2 = W[u][1] + H1, v3 = W[u][2] + H2;
                const double q = max_f64(v2, v3);
                const double w1 = v3 >= v2 ? -__builtin_inf() : W[u][0];
                P = max_f64(w1 + H0, q);
            } else if (V == 12) {  // at most 3 items, L <= 4, any gaps
                const double v2 = W[u][1] + H1, v3 = W[u][2] + H2, v4 = W[u][3] + H3;
                const double q = max_f64(max_f64(v2, v3), v4);
                const bool k = (v3 >= v2) || (v4 >= v2) || (v4 >= v3);
                const double w1 = k ? -__builtin_inf() : W[u][0];
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

// V17+: the kernel's group structure (k_long_dp): weights of the next group loaded from
// LDS a group ahead into the other of two register sets, the class word a group ahead,
// the best value written to an LDS ring per rune, two groups per loop trip.
//   G = 0: every group class 0 (the short form)
//   G = 1: 17 % of groups (pseudo-random) take fold3i in an out-of-line branch
//   G = 2: every group fold3i, no branch
//   grp3: G = 0 with the best values stored in pairs (16-byte stores), grp4: G = 0 with
//   three weights per rune (six 16-byte reads per group), grp5: both
__device__ __forceinline__ double fold3i_(const double w[4], double H0, double H1, double H2, double H3) {
    const double v2 = w[1] + H1, v3 = w[2] + H2, v4 = w[3] + H3;
    const bool k = (v3 >= v2) || (v4 >= v2) || (v4 >= v3);
    const double w1 = k ? -__builtin_inf() : w[0];
    return max_f64(w1 + H0, max_f64(max_f64(v2, v3), v4));
}
template <int G, bool WR2 = false, bool W3 = false>
__global__ __launch_bounds__(64) void k_grp(const double* __restrict__ wt, uint32_t n, double* __restrict__ out,
                                            unsigned long long* __restrict__ clk) {
    __shared__ __attribute__((aligned(16))) double s_w[1024][6];  // 48-byte descriptors
    __shared__ uint32_t s_cls[256];
    __shared__ double s_ring[512];
    for (uint32_t i = threadIdx.x; i < 1024; i += 64)
        for (int k = 0; k < 4; k++) s_w[i][k] = wt[(i & 3) * 4 + k];
    for (uint32_t i = threadIdx.x; i < 256; i += 64) {
        uint32_t x = i * 2654435761u;
        x ^= x >> 13;
        s_cls[i] = (G == 1 && (x & 0xFFu) < 43u) ? 0x01000000u : 0u;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint32_t dz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(dz));
    struct WS {
        double w[4][4];
    } D0, D1;
    auto ld = [&](WS& D, uint32_t g) __attribute__((always_inline)) {
        if (W3) {  // three weights per rune, a group's twelve contiguous: six 16-byte reads
            const char* p = reinterpret_cast<const char*>(s_w) + (((g >> 2) & 255u) * 96u + dz);
#pragma unroll
            for (int q = 0; q < 6; q++) {
                const double2 x = *reinterpret_cast<const double2*>(p + 16 * q);
                D.w[(2 * q) / 3][(2 * q) % 3] = x.x;
                D.w[(2 * q + 1) / 3][(2 * q + 1) % 3] = x.y;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) D.w[r][3] = __builtin_nan("");
            return;
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const char* p = reinterpret_cast<const char*>(s_w) + (((g + r) & 1023u) * 48u + dz);
            const double2 x = *reinterpret_cast<const double2*>(p);
            const double2 y = *reinterpret_cast<const double2*>(p + 16);
            D.w[r][0] = x.x;
            D.w[r][1] = x.y;
            D.w[r][2] = y.x;
            D.w[r][3] = y.y;
        }
    };
    double H[4] = {0.0, 0.0, 0.0, 0.0};
    auto push = [&](double P) __attribute__((always_inline)) {
        H[3] = H[2];
        H[2] = H[1];
        H[1] = H[0];
        H[0] = P;
    };
    auto group = [&](uint32_t g, const WS& C, WS& N, uint32_t cw) __attribute__((always_inline)) {
        ld(N, g + 4u);
        double* rw = s_ring + (g & 511u);
        if (G != 2 && __builtin_expect(cw == 0u, 1)) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int r = 3 - u;
                const double v2 = C.w[r][1] + H[1], v3 = C.w[r][2] + H[2];
                const double w1 = v3 >= v2 ? -__builtin_inf() : C.w[r][0];
                const double P = max_f64(w1 + H[0], max_f64(v2, v3));
                if (!WR2) rw[r] = P;
                if (WR2 && (r & 1) == 0) {  // (best(s), best(s + 1)) in one store
                    typedef double d2 __attribute__((ext_vector_type(2)));
                    *reinterpret_cast<d2*>(rw + r) = d2{P, H[0]};
                }
                push(P);
            }
            return;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int r = 3 - u;
            const double P = fold3i_(C.w[r], H[0], H[1], H[2], H[3]);
            rw[r] = P;
            push(P);
        }
    };
    uint32_t cwn = s_cls[0];
    ld(D0, 0);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t g = 0; g < n; g += 8) {
        uint32_t cw = __builtin_amdgcn_readfirstlane(cwn);
        cwn = s_cls[((g + 4u) >> 2) & 255u];
        group(g, D0, D1, cw);
        cw = __builtin_amdgcn_readfirstlane(cwn);
        cwn = s_cls[((g + 8u) >> 2) & 255u];
        group(g + 4u, D1, D0, cw);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[0] = H[0] + H[1] + H[2] + H[3] + s_ring[5];
    clk[0] = t1 - t0;
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
    for (int v = 0; v < 17; v++) {
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
            if (v == 11) k_chain<11><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 12) k_chain<12><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 13) k_chain<13><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 14) k_chain<14><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 15) k_chain<15><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 16) k_chain<16><<<1, 64>>>(dw, n, dout, dclk);
            CHK(hipDeviceSynchronize());
        }
        unsigned long long c;
        double o;
        CHK(hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(&o, dout, 8, hipMemcpyDeviceToHost));
        printf("{\"variant\": %d, \"runes\": %u, \"cycles_per_rune\": %.2f, \"sink\": %g}\n", v, n, (double)c / n, o);
    }
    for (int v = 0; v < 6; v++) {
        for (int rep = 0; rep < 2; rep++) {
            if (v == 0) k_grp<0><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 1) k_grp<1><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 2) k_grp<2><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 3) k_grp<0, true, false><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 4) k_grp<0, false, true><<<1, 64>>>(dw, n, dout, dclk);
            if (v == 5) k_grp<0, true, true><<<1, 64>>>(dw, n, dout, dclk);
            CHK(hipDeviceSynchronize());
        }
        unsigned long long c;
        double o;
        CHK(hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(&o, dout, 8, hipMemcpyDeviceToHost));
        printf("{\"variant\": \"grp%d\", \"runes\": %u, \"cycles_per_rune\": %.2f, \"sink\": %g}\n", v, n,
               (double)c / n, o);
    }
    return 0;
}
