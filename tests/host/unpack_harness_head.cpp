// Test harness (tests/test_unpack.py): the library's packed-span decoder, compiled on the
// CPU with stand-ins for the few names it uses from jb_capi.cpp / jb_kernels.h.
#include <immintrin.h>
#include <stdint.h>
#include <algorithm>
#include <vector>
#include <thread>
#include <random>
#include <cstdio>
#include <cstdlib>
#include <cstring>
struct uint4 { uint32_t x, y, z, w; };
constexpr uint32_t kPackBlock = 4096, kPackGapBits = 6, kPackGapEsc = 63, kPackLenEsc = 1023;
constexpr unsigned kCopyThreads = 8;
static int env_int(const char* n, int d) { const char* v = getenv(n); return v && *v ? atoi(v) : d; }
template <class F> void run_threads(unsigned n, F& fn) { std::vector<std::thread> th; for (unsigned t = 1; t < n; t++) th.emplace_back([&, t] { fn(t); }); fn(0); for (auto& x : th) x.join(); }
