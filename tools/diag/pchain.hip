// pchain.hip — what k_long_dp's path chain (round 5) pays per path rune: one dependent
// f64 add, the values read from LDS 16 at a time a half ahead and the sums written back
// in 16-byte stores, on lane 0 of wave 0 of a 256-thread workgroup.  Cycles from s_memtime.
//   mode 0: the other three waves exit at once
//   mode 1: they spin on LDS reads and writes (fill's and verify's kind of work) until the
//           chain is done
//   mode 2: they spin on f64 VALU work
//   mode 3: mode 0 with the adds alone (no LDS traffic in the loop)
//   mode 4: the LDS reads only (the sums not stored)
//   mode 5: the LDS stores only (the values from registers)
//   mode 6: the reads as one-lane global loads (16-byte, a half ahead), no stores
//   mode 7: the reads as scalar loads (a read-only buffer), no stores
//   mode 8: the LDS reads, and one 8-byte store per 16 sums (a checkpoint)
// Diagnostic tool, not part of the product.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/diag/pchain tools/diag/pchain.hip
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

struct V16 {
    double v[16];
};

template <int MODE>
__global__ __launch_bounds__(256) void k_pc(const double* __restrict__ wt, uint32_t n, double* __restrict__ out,
                                            unsigned long long* __restrict__ clk) {
    __shared__ __attribute__((aligned(16))) double s_pw[512 + 32];
    __shared__ double s_junk[1024];
    __shared__ uint32_t s_done;
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    for (uint32_t i = tid; i < 512 + 32; i += 256) s_pw[i] = wt[i & 15];
    for (uint32_t i = tid; i < 1024; i += 256) s_junk[i] = wt[i & 15];
    if (tid == 0) s_done = 0;
    __syncthreads();
    if (wave != 0) {
        if (MODE != 1 && MODE != 2) return;
        double a = wt[tid & 15], b = 0.0;
        uint32_t k = tid;
        while (__atomic_load_n(&s_done, __ATOMIC_RELAXED) == 0u) {
            if (MODE == 1) {
                const double x = s_junk[(k * 7u) & 1023u];
                s_junk[(k * 13u + 5u) & 1023u] = x + a;
                k += 64u;
            } else {
#pragma unroll
                for (int r = 0; r < 16; r++) b = b * a + 1.0;
            }
        }
        out[1 + tid] = b + s_junk[tid];
        return;
    }
    if (tid != 0) return;
    double acc = 0.0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 3) {
        V16 A;
#pragma unroll
        for (int t = 0; t < 16; t++) A.v[t] = wt[t];
        for (uint32_t k = 0; k < n; k += 16u) {
#pragma unroll
            for (int t = 0; t < 16; t++) acc = A.v[t] + acc;
        }
    } else if (MODE == 7) {
        const double* __restrict__ g = wt + 16;  // (read-only in this kernel: scalar loads)
        for (uint32_t k = 0; k < n; k += 16u) {
            const uint32_t o = __builtin_amdgcn_readfirstlane(k & 4095u);
#pragma unroll
            for (int t = 0; t < 16; t++) acc = g[o + t] + acc;
        }
    } else if (MODE == 6) {
        const double* g = out + 512;
        V16 A, B;
        auto ld = [&](V16& X, uint32_t k) __attribute__((always_inline)) {
#pragma unroll
            for (int t = 0; t < 8; t++) {
                const double2 v = *reinterpret_cast<const double2*>(g + (k & 4095u) + 2u * t);
                X.v[2 * t] = v.x;
                X.v[2 * t + 1] = v.y;
            }
        };
        ld(A, 0u);
        for (uint32_t k = 0; k < n; k += 32u) {
            ld(B, k + 16u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 16; t++) acc = A.v[t] + acc;
            asm volatile("" ::"v"(B.v[0]), "v"(B.v[2]), "v"(B.v[4]), "v"(B.v[6]), "v"(B.v[8]), "v"(B.v[10]),
                         "v"(B.v[12]), "v"(B.v[14]));
            ld(A, k + 32u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 16; t++) acc = B.v[t] + acc;
            asm volatile("" ::"v"(A.v[0]), "v"(A.v[2]), "v"(A.v[4]), "v"(A.v[6]), "v"(A.v[8]), "v"(A.v[10]),
                         "v"(A.v[12]), "v"(A.v[14]));
        }
    } else if (MODE == 5) {
        double* const pw = s_pw;
        V16 A;
#pragma unroll
        for (int t = 0; t < 16; t++) A.v[t] = wt[t];
        for (uint32_t k = 0; k < n; k += 16u) {
            double a[16];
#pragma unroll
            for (int t = 0; t < 16; t++) {
                acc = A.v[t] + acc;
                a[t] = acc;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 8; t++)
                *reinterpret_cast<double2*>(pw + (k & 511u) + 2u * t) = make_double2(a[2 * t], a[2 * t + 1]);
        }
    } else {
        double* const pw = s_pw;
        V16 A, B;
        auto ld = [&](V16& X, uint32_t k) __attribute__((always_inline)) {
#pragma unroll
            for (int t = 0; t < 8; t++) {
                const double2 v = *reinterpret_cast<const double2*>(pw + (k & 511u) + 2u * t);
                X.v[2 * t] = v.x;
                X.v[2 * t + 1] = v.y;
            }
        };
        auto run = [&](const V16& X, uint32_t k) __attribute__((always_inline)) {
            double a[16];
#pragma unroll
            for (int t = 0; t < 16; t++) {
                acc = X.v[t] + acc;
                a[t] = acc;
            }
            __builtin_amdgcn_sched_barrier(0);
            if (MODE == 8) {
                s_pw[512 + (k & 31u)] = a[15];
            } else if (MODE != 4) {
#pragma unroll
                for (int t = 0; t < 8; t++)
                    *reinterpret_cast<double2*>(pw + (k & 511u) + 2u * t) = make_double2(a[2 * t], a[2 * t + 1]);
            }
        };
        ld(A, 0u);
        for (uint32_t k = 0; k < n; k += 32u) {
            ld(B, k + 16u);
            __builtin_amdgcn_sched_barrier(0);
            run(A, k);
            asm volatile("" ::"v"(B.v[0]), "v"(B.v[2]), "v"(B.v[4]), "v"(B.v[6]), "v"(B.v[8]), "v"(B.v[10]),
                         "v"(B.v[12]), "v"(B.v[14]));
            if (k + 16u >= n) break;
            ld(A, k + 32u);
            run(B, k + 16u);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __atomic_store_n(&s_done, 1u, __ATOMIC_RELAXED);
    out[0] = acc;
    clk[0] = t1 - t0;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    double *dw, *dout;
    unsigned long long* dclk;
    CHK(hipMalloc(&dw, 8 * (16 + 4096 + 16)));
    CHK(hipMalloc(&dout, 8 * (512 + 4096 + 16)));
    {
        double big[16 + 4096 + 16];
        for (int i = 0; i < 16 + 4096 + 16; i++) big[i] = -3.0 - 0.37 * (i & 15);
        CHK(hipMemcpy(dw, big, sizeof big, hipMemcpyHostToDevice));
        CHK(hipMemcpy(dout, big, sizeof big, hipMemcpyHostToDevice));
    }
    CHK(hipMalloc(&dclk, 8));
    for (int m = 0; m < 9; m++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEvent_t e0, e1;
            CHK(hipEventCreate(&e0));
            CHK(hipEventCreate(&e1));
            CHK(hipEventRecord(e0));
            if (m == 0) k_pc<0><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 1) k_pc<1><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 2) k_pc<2><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 3) k_pc<3><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 4) k_pc<4><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 5) k_pc<5><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 6) k_pc<6><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 7) k_pc<7><<<1, 256>>>(dw, n, dout, dclk);
            if (m == 8) k_pc<8><<<1, 256>>>(dw, n, dout, dclk);
            CHK(hipEventRecord(e1));
            CHK(hipDeviceSynchronize());
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (rep == 1) {
                unsigned long long c;
                double o;
                CHK(hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost));
                CHK(hipMemcpy(&o, dout, 8, hipMemcpyDeviceToHost));
                printf("{\"mode\": %d, \"adds\": %u, \"ticks_per_add\": %.2f, \"ns_per_add\": %.3f, \"sink\": %g}\n", m,
                       n, (double)c / n, ms * 1e6 / n, o);
            }
        }
    }
    return 0;
}
