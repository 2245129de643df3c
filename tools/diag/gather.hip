// gather.hip — what a vector-memory gather can sustain per CU on gfx950.
//
// k_mark_walk's trie probes and k_zh's weight gathers are
// wave instructions whose 64 lanes hit up to 64 different cache lines.  This
// program measures, for such instructions alone, the rate the vector L1 path
// (TA/TD/TCP) sustains: cache-line accesses per CU per cycle, by
//   W  bytes per lane (4, 8, 16),
//   D  distinct 128-byte lines per wave instruction (1 .. 64),
//   T  the table the lines come from (L1-, L2-, MALL- or HBM-sized),
//   O  waves per SIMD (1, 2, 4, 8).
// Each wave issues K independent loads per trip (the line of lane l is
// (base + (l % D) * 97) mod lines, base wave-uniform and pseudo-random per load,
// offset ((l / D) * W) mod 128 in the line), XORs the results into a sink and
// runs until every wave has done the same number of loads.  Cycles are the
// kernel's wall time times the in-kernel clock (s_memtime over s_memrealtime,
// 100 MHz), so "lines/CU/cyc" = D x wave-instructions / 256 CUs / cycles.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/diag/gather tools/diag/gather.hip
// Run:   tools/diag/gather [iters]     (one JSON line per configuration)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

constexpr int K = 8;  // independent loads in flight per trip

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int W>
struct Vec;
template <>
struct Vec<4> {
    typedef uint32_t T;
    static __device__ uint32_t fold(T x) { return x; }
};
template <>
struct Vec<8> {
    typedef uint2 T;
    static __device__ uint32_t fold(T x) { return x.x ^ x.y; }
};
template <>
struct Vec<16> {
    typedef uint4 T;
    static __device__ uint32_t fold(T x) { return x.x ^ x.y ^ x.z ^ x.w; }
};

template <int W>
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ table, uint32_t line_mask, uint32_t D,
                                               uint32_t iters, uint32_t* __restrict__ sink,
                                               unsigned long long* __restrict__ clk, uint32_t active, uint32_t bcast) {
    typedef typename Vec<W>::T T;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const uint32_t lpart = (lane % D) * 97u;
    const uint32_t off = bcast ? 0u : ((lane / D) * (uint32_t)W) & 127u;
    // only lanes (lane * 64 / active) hold an active load: "active" lanes spread over the wave
    if (active < 64u && (lane % (64u / active)) != 0u) return;
    uint32_t acc = 0;
    uint64_t t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    uint32_t s = mix(wave * 0x9E3779B9u + 1u);
    for (uint32_t it = 0; it < iters; it++) {
        T v[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            s = s * 1664525u + 1013904223u;  // wave-uniform (scalar) line base per load
            const uint32_t line = (s + lpart) & line_mask;
            v[k] = *reinterpret_cast<const T*>(table + ((size_t)line << 7) + off);
        }
#pragma unroll
        for (int k = 0; k < K; k++) acc ^= Vec<W>::fold(v[k]);
    }
    if (acc == 0x12345678u) sink[blockIdx.x * 256u + threadIdx.x] = acc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 512u;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const uint32_t ncu = (uint32_t)prop.multiProcessorCount;
    const size_t maxT = (size_t)1 << 30;
    uint8_t* table;
    CHK(hipMalloc(&table, maxT));
    CHK(hipMemset(table, 0x5A, maxT));
    uint32_t* sink;
    CHK(hipMalloc(&sink, (size_t)ncu * 8 * 256 * 4));
    unsigned long long* clk;
    CHK(hipMalloc(&clk, 16));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const size_t tables[] = {(size_t)16 << 10, (size_t)2 << 20, (size_t)8 << 20, (size_t)64 << 20, maxT};
    const int widths[] = {8, 4, 16};
    const uint32_t Ds[] = {1, 4, 16, 32, 64};
    const uint32_t occs[] = {8, 4, 2, 1};
    const bool extra = argc > 2 && argv[2][0] == 'x';  // masked and broadcast loads only
    uint32_t A = 64, B = 0;
    if (extra) {
        // (active lanes, broadcast) at D = 64 / D = 1, W = 8, 8 waves per SIMD, L1- and L2-sized tables
        const uint32_t As[] = {64, 16, 8, 4, 1};
        for (size_t T : {(size_t)16 << 10, (size_t)2 << 20})
            for (int bc = 0; bc < 2; bc++)
                for (uint32_t a : As) {
                    A = a;
                    B = (uint32_t)bc;
                    const uint32_t D = bc ? 1u : 64u, O = 8, nwg = ncu * O, lines = (uint32_t)(T >> 7);
                    auto launch = [&]() { k_gather<8><<<nwg, 256>>>(table, lines - 1u, D, iters, sink, clk, A, B); };
                    launch();
                    CHK(hipDeviceSynchronize());
                    CHK(hipEventRecord(e0));
                    for (int r = 0; r < 5; r++) launch();
                    CHK(hipEventRecord(e1));
                    CHK(hipEventSynchronize(e1));
                    float ms = 0;
                    CHK(hipEventElapsedTime(&ms, e0, e1));
                    unsigned long long c[2];
                    CHK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
                    const double ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 0.0;
                    const double sec = ms * 1e-3 / 5;
                    const double winst = (double)nwg * 4.0 * iters * K;
                    printf("{\"W\": 8, \"T_bytes\": %zu, \"D\": %u, \"active_lanes\": %u, \"broadcast\": %d, "
                           "\"ms\": %.4f, \"cyc_per_winst_per_cu\": %.2f}\n",
                           T, D, a, bc, sec * 1e3, ncu * sec * ghz * 1e9 / winst);
                    fflush(stdout);
                }
        return 0;
    }
    for (int W : widths)
        for (size_t T : tables)
            for (uint32_t D : Ds)
                for (uint32_t O : occs) {
                    if (W != 8 && (O != 8 || (T != ((size_t)8 << 20) && T != ((size_t)16 << 10)))) continue;
                    if (O != 8 && O != 4 && (D != 64 || T != ((size_t)8 << 20))) continue;
                    const uint32_t nwg = ncu * O;  // 4 waves per workgroup, O workgroups per CU = O waves per SIMD
                    const uint32_t lines = (uint32_t)(T >> 7);
                    auto launch = [&]() {
                        if (W == 4)
                            k_gather<4><<<nwg, 256>>>(table, lines - 1u, D, iters, sink, clk, A, B);
                        else if (W == 8)
                            k_gather<8><<<nwg, 256>>>(table, lines - 1u, D, iters, sink, clk, A, B);
                        else
                            k_gather<16><<<nwg, 256>>>(table, lines - 1u, D, iters, sink, clk, A, B);
                    };
                    launch();
                    launch();
                    CHK(hipDeviceSynchronize());
                    CHK(hipEventRecord(e0));
                    const int reps = 5;
                    for (int r = 0; r < reps; r++) launch();
                    CHK(hipEventRecord(e1));
                    CHK(hipEventSynchronize(e1));
                    float ms = 0;
                    CHK(hipEventElapsedTime(&ms, e0, e1));
                    unsigned long long c[2];
                    CHK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
                    const double ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 0.0;  // s_memrealtime: 100 MHz
                    const double sec = ms * 1e-3 / reps;
                    const double winst = (double)nwg * 4.0 * iters * K;  // wave instructions per launch
                    const double cyc = sec * ghz * 1e9;
                    printf("{\"W\": %d, \"T_bytes\": %zu, \"D\": %u, \"waves_per_simd\": %u, \"ms\": %.4f, "
                           "\"clock_ghz\": %.3f, \"winst_per_cu_cyc\": %.4f, \"lines_per_cu_cyc\": %.4f, "
                           "\"GBps\": %.1f}\n",
                           W, T, D, O, sec * 1e3, ghz, winst / ncu / cyc, winst * D / ncu / cyc,
                           winst * 64.0 * W / sec / 1e9);
                    fflush(stdout);
                }
    return 0;
}
