// jb_kernels.hip — gfx950 kernels of the jieba-go Cut path.
//
// Pipeline for one batch of documents (all in HBM, one stream):
//   k_docbits     document starts -> 1 bit per byte
//   k_mark_walk   per 4 KiB tile: UTF-8 decode at lead bytes (Go rules), \p{Han}
//                 runs -> block-start masks + counts (zh regex + splitText,
//                 tokenizer.go:21,154-155,165-210); then the trie walk (DAG
//                 edges) of every Han rune of the tile, one walk per lane at a
//                 time from an LDS entry list (buildDag, :462-497)
//   k_zh          per 6 KiB group (1 KiB in small batches): its Han blocks from the
//                 block-start masks, dealt to lanes by length; backward max-prob DP
//                 over the edges + forward path + BMES Viterbi on singleton runs
//                                               (cutZh/cutDAG/buildDag/calcDagProba/
//                                                findDagPath/maxIndexProba/viterbi/cutHMM,
//                                                tokenizer.go:221-285,462-578,668-756)
//   k_long_*      Han blocks of 8 KiB or more (one serial DP chain each)
//   k_nonzh       the non-Han blocks with an alnum byte, from the alnum16 bits and
//                 the masks: alnum runs, single runes, spaces dropped (cutNonZh,
//                 tokenizer.go:289-310; blocks without alnum have no tokens)
//   k_tok<0>/k_tok<1>  token start/end bitmaps -> counts (+ 256-tile sums, k_sup)
//                 -> (start, end) spans
//   k_doc_tok     per document first token (Cut per document)
//
// Output format on the device: two bitmaps, 1 bit per input byte each (token
// first byte, token last byte), compacted to u32 spans.  All float64
// arithmetic is IEEE add/compare in the reference's order; the library is
// built with -ffp-contract=off and without fast-math (±Inf must propagate).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "jb_kernels.h"

#include <algorithm>

#ifndef JB_STAMPS
#define JB_STAMPS 0
#endif

namespace jb {

const char* const kKernelNames[K_NUM] = {"k_docbits", "k_mark_walk", "k_zh", "k_nonzh", "k_tok_count", "k_scan_tok",
                                         "k_tok_write", "k_doc_tok", "k_long_spec", "k_long_dp", "k_long_seg", "k_long_path",
                                         "k_long_tail", "k_mask_merge", "k_long_pbits", "k_long", "k_tok1"};

// newJiebaHMM literals (tokenizer.go:629-652)
#define START_B (-0.26268660809250016)
#define START_S (-1.4652633398537678)
#define T_BE (-0.51082562376599)
#define T_BM (-0.916290731874155)
#define T_EB (-0.5897149736854513)
#define T_ES (-0.8085250474669937)
#define T_ME (-0.33344856811948514)
#define T_MM (-1.2603623820268226)
#define T_SB (-0.7211965654669841)
#define T_SS (-0.6658631448798212)

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
// 4 bytes at any offset: one 8-byte load at the dword below + v_alignbyte.  The
// text buffer is 4-byte aligned and readable 8 bytes past every offset used.
__device__ __forceinline__ uint32_t ld4(const uint8_t* __restrict__ t, uint64_t q) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2), aligned(4)));
    const u32x2 a = *reinterpret_cast<const u32x2*>(t + (q & ~3ull));
    return __builtin_amdgcn_alignbyte(a.y, a.x, (uint32_t)(q & 3));
}

// 4 bytes at window offset k of staged text (k + 8 readable).
__device__ __forceinline__ uint32_t lds4(const uint8_t* tx, uint32_t k) {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(tx + (k & ~3u));
    return __builtin_amdgcn_alignbyte(a[1], a[0], k & 3u);
}

// Token bitmaps: bits are accumulated per 32-byte word in registers and
// flushed with one atomicOr per word (neighbouring blocks may share a word).
struct Emitter {
    uint32_t* sb;
    uint32_t* eb;
    uint32_t word, s, e;
    uint32_t ties = 0;  // exact Viterbi route ties seen by this lane (Q12)
    bool off = false;   // drop the bits instead of flushing them (k_zh_long: only lane 0 writes)
    __device__ Emitter(uint32_t* s_, uint32_t* e_) : sb(s_), eb(e_), word(0xFFFFFFFFu), s(0), e(0) {}
    __device__ __forceinline__ void flush() {
        if (!off) {
            if (s) atomicOr(sb + word, s);
            if (e) atomicOr(eb + word, e);
        }
        s = e = 0;
    }
    __device__ __forceinline__ void at(uint32_t pos) {
        const uint32_t w = pos >> 5;
        if (w != word) {
            flush();
            word = w;
        }
    }
    // token = bytes [a, b)
    __device__ __forceinline__ void token(uint32_t a, uint32_t b) {
        at(a);
        s |= 1u << (a & 31u);
        at(b - 1u);
        e |= 1u << ((b - 1u) & 31u);
    }
    // start / end bits sm, em_ of bitmap word w
    __device__ __forceinline__ void bits(uint32_t w, uint32_t sm, uint32_t em_) {
        if (!(sm | em_)) return;
        if (w != word) {
            flush();
            word = w;
        }
        s |= sm;
        e |= em_;
    }
};

// The same for a wave's LDS token bitmaps: word index = global word - w0.
struct LdsEmitter {
    uint32_t* sb;
    uint32_t* eb;
    uint32_t w0;
    uint32_t word, s, e;
    uint32_t ties = 0;  // exact Viterbi route ties seen by this lane (Q12)
    __device__ LdsEmitter(uint32_t* s_, uint32_t* e_, uint32_t w0_)
        : sb(s_), eb(e_), w0(w0_), word(0xFFFFFFFFu), s(0), e(0) {}
    __device__ __forceinline__ void flush() {
        if (s) atomicOr(sb + (word - w0), s);
        if (e) atomicOr(eb + (word - w0), e);
        s = e = 0;
    }
    __device__ __forceinline__ void at(uint32_t pos) {
        const uint32_t w = pos >> 5;
        if (w != word) {
            flush();
            word = w;
        }
    }
    __device__ __forceinline__ void token(uint32_t a, uint32_t b) {
        at(a);
        s |= 1u << (a & 31u);
        at(b - 1u);
        e |= 1u << ((b - 1u) & 31u);
    }
};

// ---------------------------------------------------------------------------
// k_docbits
// ---------------------------------------------------------------------------
// The bitmap is all zeros between pipeline runs: k_nonzh clears the words a run
// set (one per document), after k_mark_walk (their only reader) is done with them.  The first
// launch also clears the run's counters (no kernel before it uses them).
__global__ void k_docbits(const uint64_t* __restrict__ doc_off, uint32_t ndocs, uint64_t nbytes,
                          uint32_t* __restrict__ bits, uint32_t* __restrict__ counters,
                          uint64_t* __restrict__ tstat, uint32_t ntt) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < CNT_ALL) counters[d] = 0u;
    if (d < ntt) tstat[d] = 0ull;  // (k_tok1's look-back: every token tile not ready)
    if (d >= ndocs) return;
    const uint64_t o = doc_off[d];
    if (o < nbytes) atomicOr(bits + (o >> 5), 1u << (o & 31u));
}

// ---------------------------------------------------------------------------
// k_blocks: classify 16 bytes per lane.  The lane sees the window
// [p0-4, p0+20); a byte belongs to the rune whose valid sequence (Go
// utf8.DecodeRune, bounded by the document end) covers it, else it starts a
// rune of its own.  Block starts: document starts and changes of Han-ness.
// ---------------------------------------------------------------------------
// Inclusive prefix sum over a wave's 64 lanes with DPP moves (VALU, no LDS round
// trips): row_shr 1/2/4/8 scans each row of 16 lanes, row_bcast15/31 carry the row
// totals into the rows above.  Lanes a move cannot source keep 0 (old = 0, bound_ctrl off).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t* lds, uint32_t* total) {
    // exclusive scan over a 256-thread workgroup
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t x = wave_incl_scan(v);
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    const uint32_t nw = blockDim.x >> 6;
    for (uint32_t k = 0; k < nw; k++) {
        const uint32_t t = lds[k];
        if (k < wid) base += t;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// Exclusive prefix of tile t's (x, y) counts, by a 256-thread workgroup: the
// 256-tile sums (k_sup) before t's group of 256, plus the counts of the tiles
// before t in its own group.  The loads are issued first (pf_load) and summed
// later (pf_sum), so their latency hides under the caller's own loads.
// Replaces a single-workgroup scan launch.
struct PrefixLoads {
    uint32_t x, y;
};
__device__ __forceinline__ PrefixLoads pf_load(const uint2* __restrict__ cnt, const uint2* __restrict__ sup,
                                               uint32_t t) {
    PrefixLoads p{0u, 0u};
    const uint32_t sn = t >> 8, r = t & 255u;
    for (uint32_t i = threadIdx.x; i < sn; i += 256u) {
        const uint2 v = sup[i];
        p.x += v.x;
        p.y += v.y;
    }
    if (threadIdx.x < r) {
        const uint2 c = cnt[(t & ~255u) + threadIdx.x];
        p.x += c.x;
        p.y += c.y;
    }
    return p;
}
__device__ uint2 pf_sum(PrefixLoads p, uint32_t* lds) {
    // wave sums by DPP scans (a shuffle reduction was twelve LDS round trips)
    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(p.x), 63);
    const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(p.y), 63);
    const uint32_t wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) {
        lds[wid] = x;
        lds[4u + wid] = y;
    }
    __syncthreads();
    const uint2 out = make_uint2(lds[0] + lds[1] + lds[2] + lds[3], lds[4] + lds[5] + lds[6] + lds[7]);
    __syncthreads();
    return out;
}

// k_sup: the (x, y) sums of each group of 256 consecutive tile counts.
__global__ __launch_bounds__(256) void k_sup(const uint2* __restrict__ cnt, uint32_t n, uint2* __restrict__ sup) {
    __shared__ uint32_t lds[8];
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    PrefixLoads p{0u, 0u};
    if (i < n) {
        const uint2 c = cnt[i];
        p.x = c.x;
        p.y = c.y;
    }
    const uint2 s = pf_sum(p, lds);
    if (threadIdx.x == 0) sup[blockIdx.x] = s;
}

// \p{Han} (unicode.Han, Unicode 13) with the common ranges first: the two
// big BMP blocks, a bitmask for U+3000-303F (CJK punctuation: only 3005,
// 3007, 3021-3029, 3038-303B are Han), and the full table only for the rare
// rest (radicals, compatibility ideographs, the supplementary planes).
__device__ __forceinline__ bool han_cp(uint32_t r) {
    constexpr uint64_t k3000 = (1ull << 5) | (1ull << 7) | (0x1FFull << 0x21) | (0xFull << 0x38);
    bool h = (r - 0x4E00u <= 0x9FFCu - 0x4E00u) | (r - 0x3400u <= 0x4DBFu - 0x3400u);
    const uint32_t o = r - 0x3000u;
    h |= o < 64u && ((k3000 >> (o & 63u)) & 1ull);
    const bool rare = (r - 0x2E80u < 0x180u) | (r - 0xF900u < 0x200u) | (r >= 0x16FF0u);
    if (rare) h = jb_is_han(r);
    return h;
}

constexpr uint32_t kEdgeMaxL = 8;     // edge lengths a record holds
constexpr uint32_t kEdgeIdxBits = 14;  // a record field: weight index + 1 (0: phantom edge)
constexpr uint32_t kRecIdxMax = (1u << kEdgeIdxBits) - 2u;  // the largest weight index a record holds
constexpr uint32_t kRecTop = 8u + 3u * kEdgeIdxBits;         // bit of the last field (a new edge enters there)
constexpr uint32_t kTileE = kTileBytes / 3 + 2;  // Han rune entries of a tile (>= 3 bytes each)
constexpr uint32_t kLA = 8;                      // lookahead entries: runes of the last run past the tile end
constexpr uint32_t kLABytes = 40;                // ... starting in the first 40 bytes after it
constexpr uint32_t kTileEX = kTileE + kLA;
constexpr uint32_t kMwStage = kTileBytes + 64u;  // staged text: bytes [t0-16, t0+4096+48)
// k_mark_walk's LDS carve-up (bytes)
constexpr uint32_t kMwOffE = kTileEX * 8u;                                // after s_c (u64 per entry)
constexpr uint32_t kMwOffDb = kMwOffE + kTileEX * 4u;                     // u32 per 32 bytes of the tile, +2
constexpr uint32_t kMwOffWl = kMwOffDb + (kTileBytes / 32u + 3u) * 4u;    // u16 per entry
constexpr uint32_t kMwOffScan = (kMwOffWl + kTileE * 2u + 3u) & ~3u;      // u32 x 8
#ifndef JB_MW_SORT
#define JB_MW_SORT 1  // the walk list grouped by the line of each walk's first probe
#endif
constexpr uint32_t kMwSortB = 64u;                   // buckets of the walk-list sort
constexpr uint32_t kMwOffHist = kMwOffScan + 8u * 4u;  // u32 per bucket
constexpr uint32_t kMwLds = kMwOffHist + (JB_MW_SORT ? kMwSortB * 4u : 0u);
constexpr uint32_t kMwOffHot = (kMwOffE + 15u) & ~15u;  // hot level-1 rows (phase 1 only), under the entries
static_assert(kMwOffHot % 16u == 0u && kMwOffHot + 10u * JB_HOT_SLOTS <= kMwOffDb && JB_HOT_SLOTS == 512u,
              "k_mark_walk: the hot rows fit under the entry list, 256 threads stage them");
static_assert(kMwOffE >= kMwStage, "staged text must fit under the entry cells");
static_assert(kTileBytes + kLABytes + 4u <= kMwStage - 16u && kTileBytes + kLABytes + 4u <= kTileBytes + 64u,
              "lookahead bytes are staged and have document bits");
static_assert(kMwLds + 16u <= 163840u / 8u, "k_mark_walk: 8 workgroups per CU");
// utf8.DecodeRune (Go rules, as jb_decode) at a lead byte (>= 0xC0), without
// branches: the phase-1 lead loop runs every lane's leads in step, so a
// branchy decode diverged on every byte class (k_mark_walk 0.601 -> 0.598 ms).
__device__ __forceinline__ uint32_t dec_lead(uint32_t x, uint32_t lim, uint32_t* rune) {
    const uint32_t b0 = x & 0xFFu, b1 = (x >> 8) & 0xFFu, b2 = (x >> 16) & 0xFFu, b3 = x >> 24;
    const uint32_t n = b0 >= 0xF0u ? 4u : (b0 >= 0xE0u ? 3u : 2u);
    uint32_t lo = b0 == 0xE0u ? 0xA0u : 0x80u;
    lo = b0 == 0xF0u ? 0x90u : lo;
    uint32_t hi = b0 == 0xEDu ? 0x9Fu : 0xBFu;
    hi = b0 == 0xF4u ? 0x8Fu : hi;
    const bool ok = (b0 - 0xC2u <= 0xF4u - 0xC2u) & (b1 >= lo) & (b1 <= hi) &
                    ((n < 3u) | ((b2 & 0xC0u) == 0x80u)) & ((n < 4u) | ((b3 & 0xC0u) == 0x80u)) & (n <= lim);
    const uint32_t m0 = n == 2u ? 0x1Fu : (n == 3u ? 0x0Fu : 0x07u);
    uint32_t cp = ((b0 & m0) << 6) | (b1 & 0x3Fu);
    cp = n >= 3u ? ((cp << 6) | (b2 & 0x3Fu)) : cp;
    cp = n == 4u ? ((cp << 6) | (b3 & 0x3Fu)) : cp;
    *rune = ok ? cp : 0xFFFDu;
    return ok ? n : 1u;
}

// entry: rune (bits 0-17; Han runes are < 0x40000) | tile offset (bits 18-29)
constexpr uint32_t kEntCont = 0x40000000u;  // the next entry continues the run
constexpr uint32_t kEntEdge = 0x80000000u;  // the run may continue past the tile
// entry: rune code [0,17) | 4-byte rune [17] | tile offset [18,30) | flags [30,32)
__device__ __forceinline__ uint32_t ent_code(uint32_t e) { return e & 0x1FFFFu; }
__device__ __forceinline__ uint32_t ent_pos(uint32_t e) { return (e >> 18) & 0xFFFu; }
__device__ __forceinline__ uint32_t ent_w(uint32_t e) { return 3u + ((e >> 17) & 1u); }

// The Han rune encoded by x (Go-valid, within `lim` bytes), or 0.  A 3-byte
// form with a Han value cannot be overlong (E0) or a surrogate (ED), and a
// 4-byte form with a Han value is >= U+16FF0, so the bit patterns suffice.
__device__ __forceinline__ uint32_t han_rune(uint32_t x, uint32_t lim, uint32_t* w) {
    const uint32_t b0 = x & 0xFFu;
    if ((x & 0x00C0C0F0u) == 0x008080E0u) {
        const uint32_t r = ((b0 & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu);
        if (lim < 3u || !han_cp(r)) return 0u;
        *w = 3u;
        return r;
    }
    if ((x & 0xC0C0C0F8u) == 0x808080F0u) {
        const uint32_t r =
            ((b0 & 0x07u) << 18) | (((x >> 8) & 0x3Fu) << 12) | (((x >> 16) & 0x3Fu) << 6) | ((x >> 24) & 0x3Fu);
        if (lim < 4u || !han_cp(r)) return 0u;
        *w = 4u;
        return r;
    }
    return 0u;
}

// One trie step in the double array: the cell that holds rune r (code k) under
// the node whose cell is c; a hit when its check names that node.
__device__ __forceinline__ uint32_t rune_code(const DevImage& im, uint32_t r) {
    return im.code[jb_row(im.pagemap, r)];
}
__device__ __forceinline__ uint32_t dat_slot_k(uint64_t c, uint32_t k) { return jb_cell_base(c) + k; }
__device__ __forceinline__ uint32_t dat_slot(const DevImage& im, uint64_t c, uint32_t r) {
    return dat_slot_k(c, rune_code(im, r));
}
__device__ __forceinline__ bool dat_hit(uint64_t child, uint32_t id) { return jb_cell_check(child) == id + 1u; }

// k_mark_walk: one workgroup per 4 KiB tile, staged in LDS, two phases.
//
// (1) Blocks (zh regex + splitText, tokenizer.go:21,154-155,165-210): 16
// bytes per lane; the lane's window is [p0-4, p0+20).  Only lead bytes
// (>= 0xC0) can start a multi-byte rune, so the lane decodes (Go
// utf8.DecodeRune, bounded by the document end) at its lead bytes only; a
// valid sequence covers its continuation bytes, every other byte is a rune of
// its own (Go's range loop takes an invalid byte as one U+FFFD).  A block
// starts at a rune start that is a document start or changes Han-ness.
// Output per lane: bits 0-15 block starts, bits 16-31 of those the Han ones,
// and the tile's (blocks, Han blocks) counts.
//
// (2) DAG edges of every Han rune of the tile (buildDag, tokenizer.go:462-497).
// The tile's Han runes go to an LDS entry list in text order: rune value,
// tile offset, and whether the next entry is the next rune of the same Han
// run (adjacent, same document).  Every lane runs one walk at a time as a
// small state machine — one trie probe per loop trip, the next rune read from
// the entry list — and takes the next walk start from the tile's queue as soon
// as its walk ends, so lanes stay busy however long the walks are.  The trie
// is a double array: a walk starts at its rune's level-1 cell (loaded for
// every entry while the list is built) and each further rune is one 8-byte
// load, cell base + row(rune), a hit when that cell's check names the current
// node.  It stops at the first string that is not a key (:475-478), at a node
// without children, or at the end of the Han run.  A run that goes past the
// tile is walked again at the end, from global memory.
//
// Output per rune, slot = byte offset / 3 (Han runes are >= 3 bytes, so slots
// never collide), one u64 record erec[slot]:
//   bits 0-7    bit L-1 set for an edge of L runes (:479-481)
//   bits 8-63   four 14-bit fields, field k at bit 8 + 14k: weight index + 1.
//               The n edges fill the LAST n fields in ascending L; the first
//               4 - n fields are 0, a "phantom" edge whose weight is -Inf
//               (DevImage::wtab1[0]), which k_zh's fold passes over (rec_fold_a3).
// A rune with more than 4 edges, an edge longer than 8 runes or a weight index
// past kRecIdxMax gets the record 0 (a Han rune always has at least one edge);
// k_zh then walks that rune itself.  A rune that is absent or has count 0 gets
// the single edge L = 1 (:468-471) with weight index 0 (Log(1) - Log(size)) or
// that of Log(0) - Log(size) = -Inf.
// At most 80 SGPRs (the rest spill to VGPR lanes) and 20.2 KB of LDS: 8
// workgroups per CU instead of 6 (k_mark_walk is latency-bound: 0.695 -> 0.618 ms).
#ifndef JB_MW_SGPR
#define JB_MW_SGPR 80
#endif
#ifndef JB_MW_WALKS
#define JB_MW_WALKS 1  // trie walks per lane at once (2 measured slower)
#endif
#define JB_MW_ATTR __attribute__((amdgpu_num_sgpr(JB_MW_SGPR), amdgpu_waves_per_eu(8, 8)))
__global__ __launch_bounds__(256) JB_MW_ATTR void k_mark_walk(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                   const uint32_t* __restrict__ docbits, DevImage im,
                                                   uint32_t* __restrict__ lanemask, uint2* __restrict__ tile_cnt,
                                                   uint64_t* __restrict__ erec, uint32_t* __restrict__ tile4,
                                                   uint64_t* __restrict__ alnum16, uint32_t* __restrict__ sbits,
                                                   uint32_t* __restrict__ ebits, uint32_t diag,
                                                   uint64_t* __restrict__ dbg, uint32_t split) {
    // LDS: 20.2 KB, so that 8 workgroups fit a CU (160 KB).  The staged text is
    // dead once the entries are decoded; the entry cells/records reuse its bytes.
    __shared__ __attribute__((aligned(16))) uint8_t s_raw[kMwLds];
    uint64_t* const s_c = reinterpret_cast<uint64_t*>(s_raw);  // level-1 cell of each entry's rune, then its record
    uint8_t* const s_t = s_raw;                                 // bytes [t0-16, t0+4096+48) (phase 1 and decode)
    uint32_t* const s_e = reinterpret_cast<uint32_t*>(s_raw + kMwOffE);
    uint32_t* const s_db = reinterpret_cast<uint32_t*>(s_raw + kMwOffDb);  // document starts of the tile
    uint16_t* const s_wl = reinterpret_cast<uint16_t*>(s_raw + kMwOffWl);  // walk list
    uint32_t* const lds = reinterpret_cast<uint32_t*>(s_raw + kMwOffScan);
    __shared__ uint32_t s_nla, s_nwl;
#if JB_STAMPS
    const bool stamps = (diag & 0x100u) != 0;  // diagnostic per-wave phase clocks (make STAMPS=1)
#else
    const bool stamps = false;
#endif
    uint64_t c0 = stamps ? __builtin_amdgcn_s_memtime() : 0, c1 = 0, c2 = 0, c3 = 0, c0b = 0, c1b = 0;
    uint32_t trips = 0;
    // split s > 0 (small batches, fewer tiles than CUs): 2^s workgroups per tile; all run the
    // tile's phases 1 and 2 (their stores are the same values), and each walks and writes the
    // records of its 2^-s of the tile's entries, by entry index (the walk list's order comes
    // from LDS atomics, so it differs between them and cannot be what splits the work)
    const uint32_t tile = blockIdx.x >> split, part = blockIdx.x & ((1u << split) - 1u);
    const uint64_t t0 = (uint64_t)tile * kTileBytes;
    // The prologue's global loads (the staged text, the tile's document words and the
    // lane's window words for M below) are all issued before any is waited on: as a
    // staging loop and separate stores they were four round trips in a row.
    static_assert(kMwStage / 16 > 256u && kMwStage / 16 <= 512u, "the staged text is two loads per thread at most");
    uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
    {
        const int64_t g = (int64_t)t0 - 16 + 16 * (int64_t)threadIdx.x, g2 = g + 16 * 256;
        if (g >= 0 && (uint64_t)g + 16 <= nbytes + 64) va = *reinterpret_cast<const uint4*>(text + g);
        if (threadIdx.x < kMwStage / 16 - 256u && (uint64_t)g2 + 16 <= nbytes + 64)
            vb = *reinterpret_cast<const uint4*>(text + g2);
    }
    // the hot level-1 rows (512 values and tags), staged into the entry list's space (free
    // until the entries are written, after the level-1 lookups that read them)
    const uint4 hv4 = reinterpret_cast<const uint4*>(im.hot)[threadIdx.x];
    const uint32_t ht2 = reinterpret_cast<const uint32_t*>(im.hot + JB_HOT_SLOTS)[threadIdx.x];
    const uint64_t lastw = (nbytes + 31) >> 5;
    uint32_t dbw = 0;
    if (threadIdx.x < kTileBytes / 32 + 3) {
        const uint64_t wi = (t0 >> 5) + threadIdx.x;
        dbw = wi < lastw ? docbits[wi] : 0u;
    }
    if (threadIdx.x == 0) {
        s_nla = 0;
        s_nwl = 0;
    }
#if JB_MW_SORT
    uint32_t* const s_hist = reinterpret_cast<uint32_t*>(s_raw + kMwOffHist);
    if (threadIdx.x < kMwSortB) s_hist[threadIdx.x] = 0u;
#endif
    const uint64_t p0 = t0 + threadIdx.x * 16u;
    // doc-start / past-the-end mask, bit k <-> byte p0 - 4 + k (k < 24)
    uint64_t M;
    {
        const int64_t base = (int64_t)p0 - 4;
        if (base >= 0) {
            const uint64_t wi = (uint64_t)base >> 5;
            const uint32_t off = (uint32_t)base & 31u;
            const uint64_t lo = wi < lastw ? docbits[wi] : 0u;
            const uint64_t hi = wi + 1 < lastw ? docbits[wi + 1] : 0u;
            M = ((hi << 32) | lo) >> off;
        } else {
            M = (uint64_t)docbits[0] << 4;  // p0 == 0: window bytes -4..-1 do not exist (zeros)
        }
        if (nbytes < p0 + 20) {  // bytes at or past the end stop every decode
            const int64_t endk = (int64_t)nbytes - base;
            if (endk <= 0) M = ~0ull;
            else M |= ~0ull << endk;
        }
    }
    reinterpret_cast<uint4*>(s_t)[threadIdx.x] = va;
    if (threadIdx.x < kMwStage / 16 - 256u) reinterpret_cast<uint4*>(s_t)[threadIdx.x + 256u] = vb;
    if (threadIdx.x < kTileBytes / 32 + 3) s_db[threadIdx.x] = dbw;
    reinterpret_cast<uint4*>(s_raw + kMwOffHot)[threadIdx.x] = hv4;
    reinterpret_cast<uint32_t*>(s_raw + kMwOffHot + 8u * JB_HOT_SLOTS)[threadIdx.x] = ht2;
    {  // clear the tile's words of the token bitmaps (k_zh and k_nonzh OR into them): no memset pass
        const uint64_t wz = (t0 >> 5) + (threadIdx.x & 127u);
        if (wz < lastw + 2u) __builtin_nontemporal_store(0u, (threadIdx.x < 128u ? sbits : ebits) + wz);
    }
    __syncthreads();
    if (stamps) c0b = __builtin_amdgcn_s_memtime();  // (text staged)
    const uint8_t* win = s_t + 12 + threadIdx.x * 16u;  // window index 0
    // The window's words, read once (one LDS round trip): as separate reads behind the
    // alnum test's short-circuit || and then again for the leads, they were six round
    // trips in a row (ISA audit).
    // Words 1-4 are the lane's own 16 bytes, one 16-byte read (16-byte aligned, so without
    // the 4-way bank conflicts of 4-byte reads at a 16-byte lane stride); word 0 is the
    // previous lane's word 4, by a DPP wave shift (lane 0 of the wave reads it).
    uint32_t xw[5];
    {
        const uint4 v4 = *reinterpret_cast<const uint4*>(win + 4);
        xw[1] = v4.x;
        xw[2] = v4.y;
        xw[3] = v4.z;
        xw[4] = v4.w;
        uint32_t w0 = 0;
        if ((threadIdx.x & 63u) == 0u) w0 = reinterpret_cast<const uint32_t*>(win)[0];
        xw[0] = (uint32_t)__builtin_amdgcn_update_dpp((int)w0, (int)xw[4], 0x138, 0xF, 0xF, false);  // wave_shr:1
    }
    {  // some [0-9A-Za-z] byte in the lane's 16 bytes (k_nonzh skips blocks without one; padding
       // bytes past the batch can only add false positives)
        const bool al = ((uint32_t)jb_any_alnum4(xw[1]) | (uint32_t)jb_any_alnum4(xw[2]) |
                         (uint32_t)jb_any_alnum4(xw[3]) | (uint32_t)jb_any_alnum4(xw[4])) != 0u;
        const uint64_t am = __ballot(al);
        if ((threadIdx.x & 63u) == 0) alnum16[(t0 >> 10) + (threadIdx.x >> 6)] = am;
    }
    // lead bytes (>= 0xC0) at window indices 0..19
    uint32_t lead = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t x = xw[j];
        const uint32_t f = (x & (x << 1) & 0x80808080u) >> 7;  // bit 0/8/16/24
        lead |= ((f * 0x204081u) >> 21 & 0xFu) << (4 * j);
    }
    uint32_t covered = 0, hanb = 0;
    uint64_t cl[7];        // level-1 rows of the lane's Han starts, by slot (see below)
    uint32_t hsm = 0, kp = 0;  // slots holding one; their byte offsets in the lane, 4 bits per slot
    uint32_t rowp[4] = {0u, 0u, 0u, 0u};  // their level-1 rows, 16 bits per slot
    {  // Plain 3-byte leads (E1..EC, EE, EF: no overlong or surrogate bound on the
       // second byte) with a common Han value or none, the leads of nearly all
       // Chinese text, in a short loop; every other lead (2- and 4-byte forms, E0,
       // ED, the rare Han ranges) goes to the general decode below.
        constexpr uint64_t k3000 = (1ull << 5) | (1ull << 7) | (0x1FFull << 0x21) | (0xFull << 0x38);
        // Unrolled over the first 7 leads (a 20-byte window of 3-byte runes has at most
        // 7), so that each lead has fixed registers: a Han rune of the common ranges
        // starting in the lane's own bytes issues its level-1 load here (slot i),
        // in flight during the block scan.  Leads past the 7th go to the general decode.
        // The seven leads' positions first, then their 4-byte reads all at once (one LDS
        // round trip; read inside the per-lead branch they were seven in a row), then the
        // branch-free classification.  A missing lead (fewer than 7) reads position 0 and is
        // masked out.
        uint32_t l = lead, slow = 0, xs[7], vm = 0;
        uint64_t kq = 0;  // the leads' positions, 5 bits each (registers: 63 VGPRs, 8 waves per SIMD)
#pragma unroll
        for (int i = 0; i < 7; i++) {
            vm |= (l != 0u ? 1u : 0u) << i;
            const uint32_t k = l ? (uint32_t)__builtin_ctz(l) : 0u;
            kq |= (uint64_t)k << (5 * i);
            xs[i] = lds4(win, k);
            l &= l - 1u;
        }
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const bool v = (vm >> i) & 1u;
            const uint32_t k = (uint32_t)(kq >> (5 * i)) & 31u, x = xs[i];
            const uint32_t b0 = x & 0xFFu;
            const uint32_t r = ((b0 & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu);
            const bool plain = (b0 - 0xE1u < 12u) | (b0 - 0xEEu < 2u);
            const bool rare = (r - 0x2E80u < 0x180u) | (r - 0xF900u < 0x200u);
            const bool ok = ((x & 0x00C0C000u) == 0x00808000u) & (((uint32_t)(M >> (k + 1u)) & 3u) == 0u);
            const uint32_t o = r - 0x3000u;
            const bool h = (r - 0x4E00u <= 0x9FFCu - 0x4E00u) | (r - 0x3400u <= 0x4DBFu - 0x3400u) |
                           ((o < 64u) & (((k3000 >> (o & 63u)) & 1ull) != 0ull));
            const bool fast = plain & !(ok & rare);
            slow |= ((v & !fast) ? 1u : 0u) << k;
            covered |= ((v & fast & ok) ? 3u : 0u) << (k + 1u);
            hanb |= ((v & fast & ok & h) ? 7u : 0u) << k;
            const bool dr = v & fast & ok & h & (k >= 4u) & (r >= JB_DIRECT_LO);  // (rows of U+3400..U+9FFF are direct)
            rowp[i >> 1] |= (dr ? r - 0x3300u : 0u) << (16 * (i & 1));
            hsm |= (dr ? 1u : 0u) << i;
            kp |= (dr ? k - 4u : 0u) << (4 * i);
        }
        slow |= l;
        lead = slow;
    }
    while (lead) {
        const uint32_t k = __builtin_ctz(lead);
        lead &= lead - 1u;
        const uint32_t lim = 1u + (uint32_t)__builtin_ctzll(((M >> (k + 1)) & 7ull) | 8ull);
        uint32_t r;
        const uint32_t w = dec_lead(lds4(win, k), lim, &r);
        covered |= ((1u << (w - 1u)) - 1u) << (k + 1u);  // (nothing for w == 1)
        if (w >= 3u && han_cp(r)) hanb |= ((1u << w) - 1u) << k;
    }
    if (p0 == 0) hanb &= ~0xFu;
    uint32_t valid = 0xFFFF0u;  // window indices 4..19 that are inside the batch
    if (nbytes < p0 + 16) valid = nbytes > p0 ? ((1u << (uint32_t)(nbytes - p0)) - 1u) << 4 : 0u;
    const uint32_t bs = ~covered & valid & ((uint32_t)M | (hanb ^ (hanb << 1)));
    const uint32_t bmask = (bs >> 4) & 0xFFFFu, zmask = ((bs & hanb) >> 4) & 0xFFFFu;
    __builtin_nontemporal_store(bmask | (zmask << 16), lanemask + tile * 256u + threadIdx.x);  // (read on other XCDs)
    uint32_t tot;
    block_scan_u32(__popc(bmask) | (__popc(zmask) << 16), lds, &tot);
    if (threadIdx.x == 0) tile_cnt[tile] = make_uint2(tot & 0xFFFFu, tot >> 16);
    if (stamps) c1 = __builtin_amdgcn_s_memtime();

    // ---- (2) Han rune entries of the tile, in text order ---------------------------
    uint32_t hs = ((hanb & ~covered & valid) >> 4) & 0xFFFFu;  // Han rune starts of the lane's bytes
    {  // the level-1 rows, in flight during the entry scan: a hot rune's from LDS, the rest
       // gathered (a gather costs the L1 one cycle per active lane, so the hot runes' are
       // taken out of it, not just served faster)
        const uint64_t* s_hv = reinterpret_cast<const uint64_t*>(s_raw + kMwOffHot);
        const uint16_t* s_ht = reinterpret_cast<const uint16_t*>(s_raw + kMwOffHot + 8u * JB_HOT_SLOTS);
        // every slot's tag and value read at once (14 LDS reads, one round trip; behind the
        // tag test's && and the hit branch they were fourteen in a row), then the misses gathered
        uint32_t hit = 0, tg[7];
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const uint32_t r = ((rowp[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) + 0x3300u;
            tg[i] = s_ht[jb_hot_slot(r)];
            cl[i] = s_hv[jb_hot_slot(r)];
        }
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const uint32_t r = ((rowp[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) + 0x3300u;
            hit |= (((hsm >> i) & 1u) & (tg[i] == r ? 1u : 0u)) << i;
        }
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const uint32_t row = (rowp[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
            if (!((hit >> i) & 1u)) cl[i] = 0ull;
            if ((~hit & hsm) >> i & 1u) cl[i] = im.l1row[row];
        }
    }
    uint32_t nent;
    uint32_t o = block_scan_u32(__popc(hs), lds, &nent);
    bool has4 = false;  // a 4-byte Han rune starts in the lane's bytes
    {
        // Slot i of the lane holds its Han rune number popc(hsm & ((1 << i) - 1)).
        // A lane with a Han start the fast loop did not take (a 4-byte rune, the
        // U+3000 page, past 7 leads) decodes all of its starts again here, slots =
        // rune numbers (at most 6 Han runes start in 16 bytes).
        uint32_t w4m = 0;
        if (__popc(hs) != __popc(hsm)) {
            const uint32_t ne = __popc(hs);
            uint32_t h2 = hs;
            hsm = 0;
            kp = 0;
#pragma unroll
            for (int i = 0; i < 6; i++) {
                cl[i] = 0ull;
                if ((uint32_t)i < ne) {
                    const uint32_t k = (uint32_t)__builtin_ctz(h2);
                    h2 &= h2 - 1u;
                    const uint32_t x = lds4(win, k + 4u);
                    const uint32_t r = (x & 0xF0u) == 0xE0u
                                           ? ((x & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu)
                                           : ((x & 0x07u) << 18) | (((x >> 8) & 0x3Fu) << 12) |
                                                 (((x >> 16) & 0x3Fu) << 6) | ((x >> 24) & 0x3Fu);
                    cl[i] = im.l1row[jb_row(im.pagemap, r)];  // code and level-1 cell: one load per rune
                    hsm |= 1u << i;
                    kp |= k << (4 * i);
                    w4m |= (r >= 0x10000u ? 1u : 0u) << i;
                }
            }
            cl[6] = 0ull;
        }
        has4 = w4m != 0u;
        const uint32_t top = hsm ? 31u - (uint32_t)__builtin_clz(hsm) : 0u;
        const uint32_t lastend =  // window index past the lane's last Han rune
            hsm ? ((kp >> (4u * top)) & 15u) + 4u + 3u + ((w4m >> top) & 1u) : 0u;
        // (the lookahead's decode and code loads, issued before the level-1 loads are
        // waited on, so that the last wave does not add a round trip before the barrier)
        const uint32_t le255 = __builtin_amdgcn_readlane(lastend, 63);  // (meaningful in the last wave)
        const bool la = threadIdx.x >= 192u && le255 >= 20u;
        uint32_t law = 0, lar = 0, lacd = 0;
        if (la) {
            const uint32_t j = threadIdx.x & 63u, q = kTileBytes + j;
            if (j < kLABytes) {
                const uint64_t db = ((((uint64_t)s_db[(q >> 5) + 1u]) << 32) | s_db[q >> 5]) >> (q & 31u);
                uint32_t lim = 1u + (uint32_t)__builtin_ctzll(((db >> 1) & 7ull) | 8ull);
                const uint64_t gq = t0 + q;
                if (gq + lim > nbytes) lim = gq < nbytes ? (uint32_t)(nbytes - gq) : 0u;
                lar = (db & 1ull) ? 0u : han_rune(lds4(s_t, q + 16u), lim, &law);
            }
            lacd = lar ? rune_code(im, lar) : 0u;
        }
#pragma unroll
        for (int i = 0; i < 7; i++) {  // (s_e is not under the staged text)
            if ((hsm >> i) & 1u)
                s_e[o + __popc(hsm & ((1u << i) - 1u))] = jb_l1row_code(cl[i]) | (((w4m >> i) & 1u) << 17) |
                                                          ((threadIdx.x * 16u + ((kp >> (4 * i)) & 15u)) << 18);
            cl[i] = ((hsm >> i) & 1u) ? jb_l1row_cell(cl[i]) : 0ull;
        }
        // Lookahead (the last lane, while the cell loads fly): when the tile's last
        // Han rune ends at or past the tile end, the runes that continue its run
        // (same document, Go-valid, Han) in the next kLABytes bytes become entries
        // nent.. so that walks go on through them like any other (their records
        // belong to the next tile and are not written here).  A walk that reaches
        // past the last of them gets record 0: k_zh walks that rune itself.
        // The last wave does it, one candidate position per lane: lane j decodes at
        // tile offset kTileBytes + j (j < kLABytes) and loads that rune's code;
        // the chain from the rune after lane 255's last one is then walked on the
        // ballot masks (scalar), and each lane on it writes its entry.  (One lane
        // stepping rune by rune took a long serial chain and a large code body.)
        if (la) {
            const uint32_t j = threadIdx.x & 63u;
            const uint32_t w = law, r = lar, cdj = lacd;
            const uint64_t hm = __ballot(r != 0u), w4b = __ballot(w == 4u);
            // the chain (wave-uniform): runes at jj, jj + w, ... while Han, at most kLA
            uint64_t chain = 0;
            uint32_t jj = le255 - 20u, n = 0;
            bool go = true;
#pragma unroll
            for (int i = 0; i < (int)kLA; i++) {
                if (go && jj < kLABytes && ((hm >> jj) & 1ull)) {
                    chain |= 1ull << jj;
                    n++;
                    jj += ((w4b >> jj) & 1ull) ? 4u : 3u;
                } else {
                    go = false;
                }
            }
            if ((chain >> j) & 1ull) {  // the last one: the run may go on (all kLA decoded) or ends
                const uint32_t ix = (uint32_t)__popcll(chain & ((1ull << j) - 1ull));
                s_e[nent + ix] = cdj | ((w == 4u ? 1u : 0u) << 17) | (ix + 1u < n ? kEntCont : (go ? kEntEdge : 0u));
            }
            if (j == 0u) s_nla = n;
        }
        __syncthreads();  // every lane has decoded from s_t: its bytes now take the cells
        if (stamps) c1b = __builtin_amdgcn_s_memtime();  // (codes, cells and lookahead in)
#pragma unroll
        for (int i = 0; i < 7; i++)
            if ((hsm >> i) & 1u) s_c[o + __popc(hsm & ((1u << i) - 1u))] = cl[i];
    }
    __syncthreads();
    // Run links, then level 1 of every entry: a rune that is absent, has count 0,
    // has no children or ends its Han run gets its record now (in its LDS cell,
    // which only its own walk would read); the others go on the walk list.
    const uint32_t nla = s_nla;
    [[maybe_unused]] uint32_t wm = 0;  // (JB_MW_SORT) which of the thread's entries went on the walk list
    for (uint32_t i = threadIdx.x, k = 0; i < nent; i += 256u, k++) {
        const uint32_t e = s_e[i];
        const uint32_t nxt = ent_pos(e) + ent_w(e);
        uint32_t f = 0;
        if (nxt >= kTileBytes) f = nla ? kEntCont : 0u;  // (the tile's last rune: the lookahead goes on)
        else if (i + 1u < nent && ent_pos(s_e[i + 1u]) == nxt && !((s_db[nxt >> 5] >> (nxt & 31u)) & 1u)) f = kEntCont;
        s_e[i] = e | f;
        const uint64_t c1 = s_c[i];
        const uint32_t fc = jb_cell_fc(c1), wi = jb_cell_widx(c1);
        uint64_t r1 = 0;
        bool go = false;
        if (jb_cell_check(c1) != JB_CHECK_ROOT) {
            r1 = 1ull | ((uint64_t)(JB_WIDX_ABSENT + 1u) << kRecTop);  // absent: the single edge only, Log(1) (:468-471)
        } else if (wi > kRecIdxMax && fc != JB_FC_NEG) {
            r1 = 0ull;  // the weight index does not fit a record: k_zh walks this rune
        } else if (fc == JB_FC_ZERO) {
            r1 = 1ull | ((uint64_t)(wi + 1u) << kRecTop);  // count 0: the single edge only, Log(0) = -Inf
        } else {
            if (fc == JB_FC_POS) r1 = 1ull | ((uint64_t)(wi + 1u) << kRecTop);  // (a negative count has no edge)
            go = jb_cell_hc(c1) != 0u && f != 0u;
        }
        if (!im.plainw) {  // weights that are +Inf or NaN: k_zh folds every rune literally
            r1 = 0ull;
            go = false;
        }
        if (!go) {
            s_c[i] = r1;
        } else if (i < ((nent * part) >> split) || i >= ((nent * (part + 1u)) >> split)) {
            // (another workgroup of the tile walks it)
        } else {
#if JB_MW_SORT
            // Walks whose first probes fall in one 128-byte line of cells go next to each
            // other on the list, so that a wave's gather asks L2 for fewer lines: a
            // counting sort by a hash of that line (the order within a bucket does not
            // matter).  The bucket and the rank in it wait in the entry cell's check
            // field, which a walk never reads (its check is the root).
            const uint32_t ln = (jb_cell_base(c1) + ent_code(s_e[i + 1u])) >> 4;
            const uint32_t b = (ln * 0x9E3779B1u) >> 26;
            static_assert(kMwSortB == 64u && kTileEX <= 2048u, "bucket (6 bits) and rank (11 bits) in the check field");
            const uint32_t rk = atomicAdd(&s_hist[b], 1u);
            s_c[i] = (c1 & ~0x3FFFFFull) | (b << 11) | rk;
            wm |= 1u << k;
#else
            s_wl[atomicAdd(&s_nwl, 1u)] = (uint16_t)i;
#endif
        }
    }
    const int any4 = __syncthreads_or(has4);  // (also the barrier after the run links)
    if (threadIdx.x == 0) tile4[tile] = any4 ? 1u : 0u;  // k_zh: general rune stepping near this tile
#if JB_MW_SORT
    if (threadIdx.x < 64u) {  // bucket offsets: wave 0, a bucket per lane
        const uint32_t h = s_hist[threadIdx.x];
        const uint32_t x = wave_incl_scan(h);
        s_hist[threadIdx.x] = x - h;
        if (threadIdx.x == 63u) s_nwl = x;
    }
    __syncthreads();
    for (uint32_t k = 0; wm >> k; k++) {
        if ((wm >> k) & 1u) {
            const uint32_t i = threadIdx.x + 256u * k;
            const uint32_t ck = (uint32_t)s_c[i] & 0x3FFFFFu;
            s_wl[s_hist[ck >> 11] + (ck & 2047u)] = (uint16_t)i;
        }
    }
    __syncthreads();
#endif
    if (stamps) c2 = __builtin_amdgcn_s_memtime();
    // ---- walks: wave w takes a quarter of the walk list ------------------------------
    const uint32_t* ent = s_e;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t nwl = s_nwl;
    uint32_t head = (nwl * wv) >> 2;
    const uint32_t hi = (nwl * (wv + 1u)) >> 2;
    // Walk state per lane: entry j of the current node's rune, start entry js,
    // the current node's cell index id and base.  The record builds as an edge
    // mask m and a shift register rw of weight indices + 1 (each new one enters
    // at the last field, kRecTop, pushing the earlier ones a field down: after n
    // edges they fill the last n fields, the record's layout, and the first
    // 4 - n fields are still 0).  One trip = one probe per walk, with selects
    // instead of branches.  Each lane runs JB_MW_WALKS walks side by side (two:
    // two probes in flight per lane and trip, so the wave pays the probe round
    // trip half as often; the walk phase is latency-bound).
    struct Walk {
        bool act, ovf;
        uint32_t j, js, id, base, len, nedge, m, en;
        uint64_t rw;
    };
    Walk wk[JB_MW_WALKS];
#pragma unroll
    for (int q = 0; q < JB_MW_WALKS; q++) {
        wk[q].act = wk[q].ovf = false;
        wk[q].j = wk[q].js = wk[q].id = wk[q].base = wk[q].len = wk[q].nedge = wk[q].m = wk[q].en = 0u;
        wk[q].rw = 0ull;
    }
    for (;;) {
#pragma unroll
        for (int q = 0; q < JB_MW_WALKS; q++) {  // idle walks take the next starts of the wave's list
            Walk& w = wk[q];
            const uint64_t need = __ballot(!w.act);
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            const uint32_t j0 = head + rank;
            const bool fresh = !w.act && j0 < hi;
            head = min(hi, head + (uint32_t)__popcll(need));
            if (fresh) {  // a walk from the list: its rune has children and the run goes on in the tile
                w.js = s_wl[j0];
                w.j = w.js;
                const uint64_t c = s_c[w.j];
                w.id = ent_code(ent[w.j]);  // its level-1 cell
                w.base = jb_cell_base(c);
                const bool pos = jb_cell_fc(c) == JB_FC_POS;  // (weight index < 2^14: checked by the run links)
                w.m = pos ? 1u : 0u;
                w.nedge = w.m;
                w.rw = pos ? (uint64_t)(jb_cell_widx(c) + 1u) << kRecTop : 0ull;
                w.len = 1u;
                w.ovf = false;
                w.act = true;
                w.en = ent[w.j + 1u];
            }
        }
        uint64_t child[JB_MW_WALKS];
        uint32_t tt[JB_MW_WALKS], en2[JB_MW_WALKS];
#pragma unroll
        for (int q = 0; q < JB_MW_WALKS; q++) {  // every walk's probe issued before any is used
            tt[q] = wk[q].base + ent_code(wk[q].en);
            child[q] = wk[q].act ? im.cells[tt[q]] : 0ull;
            en2[q] = ent[wk[q].j + 2u];  // (used only when the walk goes on: then entry j + 2 exists)
        }
#pragma unroll
        for (int q = 0; q < JB_MW_WALKS; q++) {
            Walk& w = wk[q];
            if (w.act) {
                const uint64_t ch = child[q];
                const bool hit = dat_hit(ch, w.id);
                ++w.len;
                const uint32_t wi = jb_cell_widx(ch);
                const bool pos = hit && jb_cell_fc(ch) == JB_FC_POS;
                const bool bad = pos && (w.len > kEdgeMaxL || w.nedge >= 4u || wi > kRecIdxMax);
                const bool add = pos && !bad;
                w.ovf |= bad;
                w.m |= add ? 1u << ((w.len - 1u) & 7u) : 0u;
                w.rw = add ? (w.rw >> kEdgeIdxBits) | ((uint64_t)(wi + 1u) << kRecTop) : w.rw;
                w.nedge += add ? 1u : 0u;
                const bool more = hit && jb_cell_hc(ch) && !w.ovf;
                const bool go = more && (w.en & kEntCont);
                const bool dfr = more && !(w.en & kEntCont) && (w.en & kEntEdge);  // past the lookahead: k_zh walks it
                ++w.j;
                w.en = en2[q];
                w.id = tt[q];
                w.base = jb_cell_base(ch);
                if (!go) {  // the record goes to the start entry's LDS cell (read when the walk began)
                    s_c[w.js] = (w.ovf || dfr) ? 0ull : ((uint64_t)w.m | w.rw);
                    w.act = false;
                }
            }
        }
        trips++;
        bool any = false;
#pragma unroll
        for (int q = 0; q < JB_MW_WALKS; q++) any |= wk[q].act;
        if (!__any(any) && head >= hi) break;
    }
    if (stamps) c3 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    // records out in entry (= text) order: consecutive lanes, mostly consecutive slots
    // (non-temporal: k_zh reads them on another XCD; kept out of this L2, where the trie's hot lines live)
    {
        const uint32_t e0 = (nent * part) >> split, e1 = (nent * (part + 1u)) >> split;
        for (uint32_t i = e0 + threadIdx.x; i < e1; i += 256u)
            __builtin_nontemporal_store(s_c[i], erec + (t0 + ent_pos(s_e[i])) / 3u);
    }
    if (stamps && part == 0u && (threadIdx.x & 63u) == 0) {  // per-wave phase clocks, summed on the host
        uint64_t* o = dbg + ((uint64_t)tile * 4u + (threadIdx.x >> 6)) * 8u;
        o[0] = c1 - c0;
        o[1] = c2 - c1;
        o[2] = c3 - c2;
        o[3] = __builtin_amdgcn_s_memtime() - c3;
        o[4] = trips;
        o[5] = 1;
        o[6] = c0b - c0;
        o[7] = c1b - c1;
    }
}

// The first block start after chunk c (16 bytes each), or nbytes: the rest of c's
// tile chunk by chunk, then whole tiles by their block counts (tile_cnt.x).
__device__ uint32_t nz_block_end(const uint32_t* __restrict__ lanemask, const uint2* __restrict__ tile_cnt,
                                 uint32_t ntiles, uint32_t nbytes, uint32_t c) {
    const uint32_t nch = ntiles * 256u;
    uint32_t k = c + 1u;
    while (k < nch) {
        if ((k & 255u) == 0u) {
            uint32_t t = k >> 8;
            while (t < ntiles && tile_cnt[t].x == 0u) t++;
            if (t >= ntiles) break;
            k = t * 256u;
        }
        const uint32_t m = lanemask[k] & 0xFFFFu;
        if (m) return min(nbytes, k * 16u + (uint32_t)__builtin_ctz(m));
        k++;
    }
    return nbytes;
}

// The end of the block that starts at byte bs: the next block start of any kind
// (k_mark_walk's lane masks), or nbytes.
__device__ uint32_t block_end_at(const uint32_t* __restrict__ lanemask, const uint2* __restrict__ tile_cnt,
                                 uint32_t ntiles, uint32_t nbytes, uint32_t bs) {
    const uint32_t c = bs >> 4;
    const uint32_t above = lanemask[c] & 0xFFFFu & ~((2u << (bs & 15u)) - 1u);
    if (above) return c * 16u + (uint32_t)__builtin_ctz(above);
    return nz_block_end(lanemask, tile_cnt, ntiles, nbytes, c);
}

// ---------------------------------------------------------------------------
// k_zh: Han blocks (cutZh, tokenizer.go:221-255), balanced over a wave's lanes.
//
// Work unit: a group = the zh blocks that start in one kZhGroupBytes span of
// text (read from k_mark_walk's block-start masks), taken by whole waves.  The group's
// blocks (in chunks of at most kZhChunk) are ranked by length and dealt to
// the 64 lanes in a snake (lane i gets ranks i, 127-i, 128+i, ...), so every
// lane carries about the same number of runes.  Per lane, one flattened
// backward loop runs the DP over all of its blocks (calcDagProba, :502-548):
// a rune's edges (i, i+L) from k_mark_walk, ascending in L as the DAG lists
// them, fold into maxIndexProba's running state (:565-578) with
// pieceProba = w + best(i+L) (:519-529); best(n) is the {n, 0.0} sentinel
// (:522-525).  best(i+L) for L <= 8 comes from an 8-entry LDS ring; a block
// with a longer edge (rare) is redone with every best value also stored in
// gbest (index be/3 - c, inside the block's slot range).  The chosen piece
// length goes to the rune's slot in LDS; the forward walk (findDagPath,
// :552-562) then emits pieces or, with HMM, gathers runs of single-rune pieces
// for the Viterbi (:228-253).  Token bits collect in LDS (over the ring, which
// is dead by then) and leave with one atomicOr per word.  A block that ends
// past the group window (kZhWin bytes) runs the same code on global memory.
// ---------------------------------------------------------------------------
constexpr uint32_t kZhRing = 8;                            // LDS best ring per lane (runes)
#ifndef JB_ZH_SLACK
#define JB_ZH_SLACK 1024
#endif
#ifndef JB_ZH_CHUNK
#define JB_ZH_CHUNK 192
#endif
constexpr uint32_t kZhWin = kZhGroupBytes + JB_ZH_SLACK;  // window: group span + slack for the last blocks
constexpr uint32_t kZhChunk = JB_ZH_CHUNK;                // blocks ranked together (kZhPer per lane)
constexpr uint32_t kZhPer = kZhChunk / 64u;
static_assert(kZhChunk % 64u == 0u && kZhPer >= 1u && kZhPer <= 4u, "k_zh: 1-4 blocks per lane and chunk");
// (a block whose end lm_collect did not find spans its round and the lookahead round
// after it, so it is over 1 KiB long: a group has at most one per KiB, plus one)
static_assert(kZhGroupBytes / 1024u + 1u <= 64u, "k_zh: a chunk's unresolved blocks fit the wave's 64 hist words");
constexpr uint32_t kZhWinWords = kZhWin / 32u + 1u;        // token bitmap words of a window
static_assert(kZhGroupBytes % 32u == 0u && kZhGroupSmall % 32u == 0u && kZhGroupSmall <= kZhGroupBytes,
              "k_zh groups are whole token-bitmap words");
static_assert(2u * kZhWinWords <= 2u * kZhRing * 64u, "token bitmaps fit over the ring");
// the wave's run list (zh_fwd_a3 -> viterbi_fwd_runs) sits in the ring area too, past the bitmaps
constexpr uint32_t kZhPool = 512u;  // (u32 word offset in the wave's ring)
constexpr uint32_t kZhBlBytes = kZhWin / 3u + 4u;
// LDS of the wide form: per wave the slots, ring, block table and histogram, plus the
// length table and the weight table; all of it within one CU's 160 KiB
static_assert(kZhWgWide * (((kZhBlBytes + 15u) & ~15u) + 8u * kZhRing * 64u + 4u * kZhChunk + 256u + 4u) + 2048u +
                      8u * kZhWtabWide <= 163840u,
              "k_zh wide form: LDS");
static_assert(kZhWin < 65536u, "window offsets are packed in 16 bits");
// k_zh stages a group's lane-mask words plus two 64-word rounds after them (lm_collect reads
// round rw and its lookahead rw + 64, with rw < the group's words) into the wave's ring area.
// (A 12 KiB group once read 64 unstaged ring words here, built garbage block bounds from
// them and faulted on global memory: the staged count now follows the group size.)
constexpr uint32_t kZhStageWords = kZhGroupBytes / 16u + 128u;
constexpr uint32_t kZhStagePer = (kZhStageWords + 63u) / 64u;  // words per lane
static_assert(kZhStagePer * 64u <= 2u * kZhRing * 64u,
              "k_zh: a group's lane-mask words and their lookahead must fit the wave's ring (JB_ZH_GROUP <= 14336)");

// A3: every rune of the block is 3 bytes (no 4-byte Han), so rune steps are
// plain arithmetic instead of dependent byte reads.
template <bool A3>
struct GrpZvT {  // text from HBM, slots of the group window in LDS
    static constexpr bool all3 = A3;
    const uint8_t* text;
    uint8_t* bls;
    uint32_t wb;
    __device__ __forceinline__ uint32_t b(uint32_t q) const { return text[q]; }
    __device__ __forceinline__ uint32_t x4(uint32_t q) const { return ld4(text, q); }
    __device__ __forceinline__ uint8_t& bl(uint32_t q) const { return bls[(q - wb) / 3u]; }
};
struct GlbZv {  // the same, slots in HBM (blocks past the window)
    static constexpr bool all3 = false;
    const uint8_t* text;
    uint8_t* gbl;
    __device__ __forceinline__ uint32_t b(uint32_t q) const { return text[q]; }
    __device__ __forceinline__ uint32_t x4(uint32_t q) const { return ld4(text, q); }
    __device__ __forceinline__ uint8_t& bl(uint32_t q) const { return gbl[q / 3u]; }
};

template <class V>
__device__ __forceinline__ uint32_t z_dec(const V& v, uint32_t q, uint32_t* w) {  // Han rune at q
    const uint32_t x = v.x4(q);
    const uint32_t b0 = x & 0xFFu;
    if (V::all3 || b0 < 0xF0u) {
        *w = 3;
        return ((b0 & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu);
    }
    *w = 4;
    return ((b0 & 0x07u) << 18) | (((x >> 8) & 0x3Fu) << 12) | (((x >> 16) & 0x3Fu) << 6) | ((x >> 24) & 0x3Fu);
}
template <class V>
__device__ __forceinline__ uint32_t z_w(const V& v, uint32_t q) {
    if (V::all3) return 3u;
    return v.b(q) < 0xF0u ? 3u : 4u;
}
template <class V>
__device__ __forceinline__ uint32_t z_prev(const V& v, uint32_t q, uint32_t lo) {  // rune that ends at q
    if (V::all3) return q - 3u;  // (q > lo: a whole rune lies before q)
    if (q - lo < 4u) return lo;
    return (v.b(q - 3u) & 0xF0u) == 0xE0u ? q - 3u : q - 4u;
}

__device__ __forceinline__ void load_emit(const DevImage& im, uint32_t r, double e[4]) {
    const double2* p = reinterpret_cast<const double2*>(im.emit) + (size_t)jb_row(im.pagemap, r) * 2u;
    const double2 a = p[0], b = p[1];
    e[0] = a.x; e[1] = a.y; e[2] = b.x; e[3] = b.y;
}

// stateTransitionRoute (tokenizer.go:736-756): candidates in stateChange
// order, strict '>' against minFloat; code 0/1 = candidate, 2 = no route ("").
// An exact tie a == b > minFloat is counted in nt: the reference picks either
// one, in Go's randomized map order (:748-753, Q12); here the first wins.
__device__ __forceinline__ void route2(double a, double b, uint32_t* code, double* p, uint32_t& nt) {
    uint32_t c = 2u;
    double best = JB_MIN_FLOAT;
    if (a > best) { c = 0u; best = a; }
    if (b > best) { c = 1u; best = b; }
    nt += (a == b && a > JB_MIN_FLOAT) ? 1u : 0u;
    *code = c;
    *p = best;
}

// viterbi (tokenizer.go:668-730) over the m runes [rs, re) + cutHMM (:273-285).
// Back-pointers (2 bits per state) go to each rune's slot; the traceback
// stops at the first "" route: the reference's path then restarts at that
// step (fullPath[""] is nil, :715) and cutHMM labels runes from the run start.
// The traceback + cutHMM half of viterbi (tokenizer.go:715-729, 273-285):
// back-pointers are in the runes' slots, st is the final state.
template <class V, class E>
__device__ void viterbi_back(const V& v, uint32_t rs, uint32_t re, uint32_t m, uint32_t st, E& em) {
    uint32_t t = m - 1, reset = 0;
    uint32_t qt = z_prev(v, re, rs);
    for (;;) {
        if (t == 0) {
            v.bl(qt) = (uint8_t)st;
            break;
        }
        const uint32_t code = (v.bl(qt) >> (2u * st)) & 3u;
        v.bl(qt) = (uint8_t)st;
        if (code == 2u) {
            reset = t;
            break;
        }
        st = (st == JB_B || st == JB_S) ? 2u + code : code;  // B,S <- {E,S}; M,E <- {B,M}
        --t;
        qt = z_prev(v, qt, rs);
    }
    uint32_t qa = rs, qb = qt, ts = rs;
    for (uint32_t k = 0; k < m - reset; k++) {
        const uint32_t lab = v.bl(qb);
        qa += z_w(v, qa);
        qb += z_w(v, qb);
        if (lab >= (uint32_t)JB_E) {
            em.token(ts, qa);
            ts = qa;
        }
    }
}

// viterbi (tokenizer.go:668-730) over the m runes [rs, re) + cutHMM (:273-285).
// Back-pointers (2 bits per state) go to each rune's slot; the traceback
// stops at the first "" route: the reference's path then restarts at that
// step (fullPath[""] is nil, :715) and cutHMM labels runes from the run start.
template <class V, class E>
__device__ void viterbi_run(const V& v, const DevImage& im, uint32_t rs, uint32_t re, uint32_t m, E& em) {
    if (m == 1) {  // always "S" for a single rune (:672-674)
        em.token(rs, re);
        return;
    }
    uint32_t w;
    double e[4], en[4];
    uint32_t r = z_dec(v, rs, &w);
    load_emit(im, r, e);
    double vB = START_B + e[0], vM = JB_MIN_FLOAT + e[1], vE = JB_MIN_FLOAT + e[2], vS = START_S + e[3];
    uint32_t q = rs + w;
    if (q < re) load_emit(im, z_dec(v, q, &w), e);
    while (q < re) {
        const uint32_t qn = q + w;
        uint32_t wn = 0;
        if (qn < re) load_emit(im, z_dec(v, qn, &wn), en);  // next rune's emissions, in flight
        uint32_t cB, cM, cE, cS;
        double pB, pM, pE, pS;
        route2(vE + T_EB, vS + T_SB, &cB, &pB, em.ties);  // B <- E, S
        route2(vB + T_BM, vM + T_MM, &cM, &pM, em.ties);  // M <- B, M
        route2(vB + T_BE, vM + T_ME, &cE, &pE, em.ties);  // E <- B, M
        route2(vE + T_ES, vS + T_SS, &cS, &pS, em.ties);  // S <- E, S
        vB = pB + e[0];
        vM = pM + e[1];
        vE = pE + e[2];
        vS = pS + e[3];
        v.bl(q) = (uint8_t)(cB | (cM << 2) | (cE << 4) | (cS << 6));
        q = qn;
        w = wn;
        e[0] = en[0]; e[1] = en[1]; e[2] = en[2]; e[3] = en[3];
    }
    viterbi_back(v, rs, re, m, vE > vS ? (uint32_t)JB_E : (uint32_t)JB_S, em);  // (:723-729)
}

// A lane's blocks of the current chunk: LDS table entries t[j * 64] for
// j < nseg, (bs - wb) | (be - wb) << 16, ~0u = none.
struct TblSrc {
    const uint32_t* t;
    uint32_t nseg, wb;
    __device__ __forceinline__ bool next(uint32_t& j, uint32_t& bs, uint32_t& be) const {
        while (j < nseg) {
            const uint32_t x = t[j * 64u];
            j++;
            if (x != ~0u) {
                bs = wb + (x & 0xFFFFu);
                be = wb + (x >> 16);
                return true;
            }
        }
        return false;
    }
};
struct TblPeek {  // (the lane's block after the current one, TblSrc::peek)
    uint32_t bs, be;
    bool ok;
};
__device__ __forceinline__ TblPeek tbl_peek(const TblSrc& src, uint32_t j) {
    TblPeek p{0u, 0u, false};
    while (j < src.nseg) {
        const uint32_t x = src.t[j * 64u];
        j++;
        if (x != ~0u) {
            p.bs = src.wb + (x & 0xFFFFu);
            p.be = src.wb + (x >> 16);
            p.ok = true;
            break;
        }
    }
    return p;
}
// The same blocks read into registers once (a lane holds at most kZhChunk / 64 = 3, and
// only the last can be ~0u): a block change in the DP then takes its next block and the
// one after it from registers, not from LDS.  A lane's blocks end at different steps, so
// nearly every DP step has some lane changing block, and as TblSrc loops those were two
// LDS round trips (next, then the peek for the prefetch) on the wave's path.
struct RegSrc {
    uint32_t x[kZhPer];  // the lane's next entries, ~0u past its last
    uint32_t wb;
    __device__ __forceinline__ explicit RegSrc(const TblSrc& s) : wb(s.wb) {
#pragma unroll
        for (uint32_t i = 0; i < kZhPer; i++) x[i] = s.nseg > i ? s.t[64u * i] : ~0u;
    }
    __device__ __forceinline__ bool next(uint32_t& j, uint32_t& bs, uint32_t& be) {  // j: the block's ordinal + 1
        if (x[0] == ~0u) return false;
        j++;
        bs = wb + (x[0] & 0xFFFFu);
        be = wb + (x[0] >> 16);
#pragma unroll
        for (uint32_t i = 0; i + 1u < kZhPer; i++) x[i] = x[i + 1u];
        x[kZhPer - 1u] = ~0u;
        return true;
    }
};
__device__ __forceinline__ TblPeek tbl_peek(const RegSrc& src, uint32_t) {
    return TblPeek{src.wb + (src.x[0] & 0xFFFFu), src.wb + (src.x[0] >> 16), src.x[0] != ~0u};
}
struct OneSrc {  // a single block
    uint32_t bs0, be0;
    __device__ __forceinline__ bool next(uint32_t& j, uint32_t& bs, uint32_t& be) const {
        if (j) return false;
        j = 1;
        bs = bs0;
        be = be0;
        return true;
    }
};

// DP over all of a lane's blocks in one backward loop: when a block's first
// rune is done the loop moves on to the lane's next block, so a lane's trip
// count is its total rune count, not the per-block maximum over the wave.
// Returns the number of DP steps (diagnostics).
struct DpFold {  // maxIndexProba's running state over one rune's DAG items (:565-578)
    double prevP = JB_MIN_FLOAT, bestP = JB_MIN_FLOAT;
    uint32_t bestL = 0, lastL = 0;
    bool redo = false;
    __device__ __forceinline__ void item(uint32_t L, double wt, uint32_t c, const double* ring, bool longm,
                                         const double* __restrict__ gbest, uint32_t key0) {
        double nb;
        if (L == c) nb = 0.0;  // the {n, 0.0} sentinel
        else if (L <= kZhRing) nb = ring[((c - L) & (kZhRing - 1u)) * 64u];
        else if (longm) nb = gbest[key0 - (c - L)];
        else {
            redo = true;
            nb = 0.0;
        }
        const double pp = wt + nb;
        if (pp >= prevP) {
            bestL = L;
            bestP = pp;
        }
        prevP = pp;
        lastL = L;
    }
    __device__ __forceinline__ void finish() {
        if (bestL == 0) {  // no item qualified: the last item (or {-1, minFloat})
            bestL = lastL;
            bestP = prevP;
        }
    }
};

// A rune whose record overflowed (more than 4 edges, or an edge past 8 runes,
// or a weight index past 14 bits): walk it here by the rules of k_mark_walk.
template <class V>
__device__ __forceinline__ void dp_walk_rune(const V& v, const DevImage& im, uint32_t q, uint32_t be, DpFold& f,
                                             uint32_t c, const double* ring, bool longm,
                                             const double* __restrict__ gbest, uint32_t key0) {
    uint32_t w0;
    const uint32_t r0 = z_dec(v, q, &w0);
    uint32_t id = rune_code(im, r0);
    uint64_t cc = im.cells[id];
    if (jb_cell_check(cc) != JB_CHECK_ROOT) {
        f.item(1u, im.wtab[JB_WIDX_ABSENT], c, ring, longm, gbest, key0);
    } else if (jb_cell_fc(cc) == JB_FC_ZERO) {
        f.item(1u, im.wtab[jb_cell_widx(cc)], c, ring, longm, gbest, key0);
    } else {
        if (jb_cell_fc(cc) == JB_FC_POS) f.item(1u, im.wtab[jb_cell_widx(cc)], c, ring, longm, gbest, key0);
        uint32_t qq = q + w0, len = 1;
        bool go = jb_cell_hc(cc) != 0u;
        while (go && qq < be) {
            uint32_t wr;
            const uint32_t r = z_dec(v, qq, &wr);
            const uint32_t tt = dat_slot(im, cc, r);
            const uint64_t ch = im.cells[tt];
            if (!dat_hit(ch, id)) break;
            ++len;
            qq += wr;
            if (jb_cell_fc(ch) == JB_FC_POS) f.item(len, im.wtab[jb_cell_widx(ch)], c, ring, longm, gbest, key0);
            go = jb_cell_hc(ch) != 0u;
            id = tt;
            cc = ch;
        }
    }
}

// The weights of a record's four fields: four loads issued now, with no branch
// (a phantom field, index + 1 = 0, loads wtab1[0] = -Inf), so the compiler's
// vmcnt bookkeeping stays exact and later waits do not drain other loads.  Each
// address is the image's wtab1 plus a 32-bit byte offset (the saddr form of the
// load: no 64-bit address arithmetic).
//
// WL: the whole table sits in LDS (s_wt, k_zh's wide workgroups), so the four
// reads are ds_read_b64 instead of global gathers.  A global gather whose 64
// lanes hit different cache lines costs the CU's vector L1 one cycle per lane
// (64 cycles per wave instruction; tools/diag/gather.hip), and the DP's four per
// step kept that unit saturated; LDS reads take the LDS pipe instead.
typedef const __attribute__((address_space(1))) char gchar;  // global memory, whatever inference concludes
typedef const __attribute__((address_space(3))) char lchar;  // LDS
__shared__ __attribute__((aligned(32))) double s_wt[kZhWtabWide];  // wtab1 in LDS (k_zh<.., kZhWgWide>: one copy per CU)
template <bool WL = false>
__device__ __forceinline__ void rec_weights(const DevImage& im, uint64_t rc, double w[4]) {
    gchar* const wb = (gchar*)im.wtab1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t off = (uint32_t)(rc >> (8 + kEdgeIdxBits * k - 3)) & (((1u << kEdgeIdxBits) - 1u) << 3);
        if constexpr (WL) w[k] = *(const __attribute__((address_space(3))) double*)((lchar*)s_wt + off);
        else w[k] = *(const __attribute__((address_space(1))) double*)(wb + off);
    }
}

// A record's edge lengths by its 8-bit mask, a 16-bit field per record field k
// holding L << 9 (the byte stride of a ring slot): the mask's n set bits + 1 in
// the last n fields, ascending, and L = 1 in the phantom fields before them.
// A 256-entry LDS table that k_zh (and k_long_dp) fill at their start.
__shared__ uint64_t s_ltab[256];
__device__ __forceinline__ uint64_t ltab_entry(uint32_t m) {
    uint32_t L[4] = {1u, 1u, 1u, 1u}, n = 0;
    for (uint32_t b = 0; b < 8u; b++)
        if ((m >> b) & 1u) {
            L[0] = L[1];
            L[1] = L[2];
            L[2] = L[3];
            L[3] = b + 1u;
            n++;
        }
    (void)n;
    uint64_t v = 0;
    for (int k = 0; k < 4; k++) v |= (uint64_t)(L[k] << 9) << (16 * k);
    return m ? v : (v | 0x8000u);  // record 0 (mask 0): overflowed (zh_dp_a3's kLtabOvf)
}

// maxIndexProba (:565-578) over a record's four fields, phantoms first.
//
// The reference keeps the last item whose proba is >= its predecessor's, with
// {-1, minFloat} before the first, and falls back to the last item when none
// qualified.  Every proba here is finite (> minFloat) or -Inf (count 0 gives
// Log(0); plainw excludes +Inf and NaN weights), and that rule gives the same
// item when the first item is compared with -Inf instead of minFloat: the
// first item then always qualifies, and when it is -Inf (where the reference
// skips it) with a second item behind it, the second qualifies in both forms;
// with none behind it, the fallback returns it anyway.  A phantom field's
// proba is -Inf + best(i + 1) = -Inf, so it qualifies against -Inf and leaves
// the state as it was before any item: the phantoms pass over, the real items
// fold as the reference folds them, and the last field is always real, so the
// chosen length is never a phantom's.  No per-field presence test, no
// fallback step: the first field is taken outright, each later one by one
// compare and three selects.
//
// Ring addresses: best(i + L) of this lane is in ring slot (c - L) & 7 at byte
// ((c - L) << 9 & 0xE00) | lb, where lb = wave ring offset + lane * 8 (bits 3-8
// and 12-13: disjoint from 0xE00, so the OR is an add) and rb0 is the ring
// array's LDS base (folded into the instruction offset).  cs = c << 9, lp the
// record's s_ltab entry.  Returns the chosen L << 9 and its proba.
__device__ __forceinline__ uint32_t ring_off(uint32_t x, uint32_t lb) {  // (x & 0xE00) | lb in one VALU
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(0xE00u), "v"(lb));
    return r;
}
__device__ __forceinline__ double rec_fold_a3(uint64_t lp, const double w[4], uint32_t cs, const char* rb0, uint32_t lb,
                                              uint32_t& bls) {
    double pp[4], rv[4];
    uint32_t Ls[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        Ls[k] = (uint32_t)(lp >> (16 * k));  // (bits past the field: no effect on & 0xE00, nor on (uint8_t)(Ls >> 9))
        rv[k] = *reinterpret_cast<const double*>(rb0 + ring_off(cs - Ls[k], lb));
    }
    __builtin_amdgcn_sched_barrier(0);  // the four ring reads issue back to back
#pragma unroll
    for (int k = 0; k < 4; k++) pp[k] = w[k] + rv[k];
    uint32_t bL = Ls[0];
    double bP = pp[0];
#pragma unroll
    for (int k = 1; k < 4; k++) {
        const bool take = pp[k] >= pp[k - 1];
        bL = take ? Ls[k] : bL;
        bP = take ? pp[k] : bP;
    }
    bls = bL;
    return bP;
}

// The same fold on a per-lane ring pointer (slot stride 64 doubles).  Returns L.
__device__ __forceinline__ double rec_fold_g(uint64_t lp, const double w[4], uint32_t c, const double* ring,
                                             uint32_t& bl) {
    double pp[4];
    uint32_t L[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        L[k] = (uint32_t)(lp >> (16 * k + 9)) & 0x7Fu;
        pp[k] = w[k] + ring[((c - L[k]) & (kZhRing - 1u)) * 64u];
    }
    uint32_t bL = L[0];
    double bP = pp[0];
#pragma unroll
    for (int k = 1; k < 4; k++) {
        const bool take = pp[k] >= pp[k - 1];
        bL = take ? L[k] : bL;
        bP = take ? pp[k] : bP;
    }
    bl = bL;
    return bP;
}

// General form (any rune widths): the next rune's record is loaded one step ahead.
// best(n) = 0.0 (the {n, 0.0} sentinel) sits in ring slot 0 from each (re)start:
// the edge with L == c reads slot (c - L) & 7 = 0, which step 8 is the first to
// overwrite (after its reads).
template <class V, class Src>
__device__ __forceinline__ uint32_t zh_dp(const V& v, const DevImage& im, const uint64_t* __restrict__ erec,
                          double* __restrict__ gbest, double* ring, const Src& src) {
    uint32_t j = 0, bs = 0, be = 0;
    if (!src.next(j, bs, be)) return 0;
    uint32_t key0 = be / 3u, steps = 0;
    bool longm = false;
    uint32_t q = z_prev(v, be, bs), c = 1;
    uint64_t rc = erec[q / 3u];
    ring[0] = 0.0;
    for (;;) {
        const bool more = q > bs;
        uint32_t qn = 0, bL = 0;
        uint64_t rn = 0;
        double bP;
        bool redo = false;
        if (rc) {
            double w4[4];
            rec_weights(im, rc, w4);
            if (more) {  // next rune's record, in flight while this rune folds
                qn = z_prev(v, q, bs);
                rn = erec[qn / 3u];
            }
            bP = rec_fold_g(s_ltab[(uint32_t)rc & 0xFFu], w4, c, ring, bL);
        } else {
            if (more) {
                qn = z_prev(v, q, bs);
                rn = erec[qn / 3u];
            }
            DpFold f;
            dp_walk_rune(v, im, q, be, f, c, ring, longm, gbest, key0);
            f.finish();
            bL = f.bestL;
            bP = f.bestP;
            redo = f.redo;
        }
        ring[(c & (kZhRing - 1u)) * 64u] = bP;
        if (longm) gbest[key0 - c] = bP;
        v.bl(q) = (uint8_t)bL;
        steps++;
        if (redo) {  // an edge past the ring: this block again, every best value kept in gbest
            longm = true;
            q = z_prev(v, be, bs);
            c = 1;
            rc = erec[q / 3u];
            ring[0] = 0.0;
            continue;
        }
        if (more) {
            q = qn;
            rc = rn;
            ++c;
            continue;
        }
        if (!src.next(j, bs, be)) break;
        key0 = be / 3u;
        longm = false;
        q = z_prev(v, be, bs);
        c = 1;
        rc = erec[q / 3u];
        ring[0] = 0.0;
    }
    return steps;
}

// All-3-byte form, software-pipelined.  Rune k steps back has slot s - k.  Per
// step, in this issue order: the weights of the NEXT rune (its record landed
// long ago), then, every other step, the record pair of the runes four and five
// back, then the fold of this rune with the weights loaded one step ago.
// Records come two per 16-byte load into two register pairs X and Y that
// alternate, so a pair is loaded three steps before its first use; vmcnt
// retires loads in issue order and the pair is issued after the weights, so
// the next step's wait for those weights does not wait for it, and it has two
// whole steps to land (with one pair register set a record had one step: the
// DP waited for an HBM round trip every other step).  Four step kinds cycle:
//   0: A_X  uses X.lo = E(s-1), reloads X = (E(s-5), E(s-4))
//   1: B_Y  uses Y.hi = E(s-1)
//   2: A_Y  uses Y.lo = E(s-1), reloads Y = (E(s-5), E(s-4))
//   3: B_X  uses X.hi = E(s-1)
// The ring is addressed as rec_fold_a3 describes (rb0 + lb: this lane's slot 0),
// the chosen length goes to the window slot bi = (q - wb) / 3, counted down
// with q.  Length-table entries carry kLtabOvf for record 0 (an overflowed
// record: dp_walk_rune folds that rune).
constexpr uint64_t kLtabOvf = 0x8000u;  // (bit 15 of field 0: no effect on a ring offset)
// A block with an edge past the ring (an overflowed record's walk found L > kZhRing) is
// left at once, its ordinal set in redom, and the caller redoes it with zh_dp, which keeps
// every best value in gbest.  So the loop has no global store: stores and loads pending
// together on vmcnt made the compiler wait for vmcnt(0) at every wait in it (gfx9 counts
// both on one counter, and their order is not known), which drained the record pairs
// loaded steps ahead once per four steps.
template <bool WL, class Src>
__device__ uint32_t zh_dp_a3(const GrpZvT<true>& v, const DevImage& im, const uint64_t* __restrict__ erec,
                             double* __restrict__ gbest, double* ring, const char* rb0, uint32_t lb, Src src,
                             uint32_t& redom) {
    uint32_t j = 0, bs = 0, be = 0;
    if (!src.next(j, bs, be)) return 0;
    uint32_t steps = 0, q = 0, c = 1, s = 0, bi = 0;
    uint64_t lc = 0;
    // Slots before a block (or before the text: erec has kErecPad slots of padding in
    // front) are garbage that `more` masks at the use.
    uint64_t xl = 0, xh = 0, yl = 0, yh = 0;
    auto ld_pair = [&](uint32_t k, uint64_t& lo, uint64_t& hi) __attribute__((always_inline)) {  // slots k, k+1
        typedef uint64_t u64x2 __attribute__((ext_vector_type(2), aligned(8)));
        const u64x2 x = *reinterpret_cast<const u64x2*>(erec + (int32_t)k);
        lo = x.x;
        hi = x.y;
    };
    auto ring_at = [&](uint32_t cs) -> double& {
        return *reinterpret_cast<double*>(const_cast<char*>(rb0) + ring_off(cs, lb));
    };
    auto setup = [&]() __attribute__((always_inline)) {  // (re)start at the last rune of [bs, be)
        q = be - 3u;
        c = 1;
        s = q / 3u;
        bi = (q - v.wb) / 3u;
        ring_at(0u) = 0.0;  // best(n), the {n, 0.0} sentinel
    };
    // The records of the lane's NEXT block's last two runes, E(s'-1) and E(s'), in one
    // 16-byte load issued when this block starts (after everything else of its prime),
    // so a block change finds them landed instead of waiting for HBM twice (its last
    // rune's record, then the record the first step reads).
    typedef uint64_t u64x2v __attribute__((ext_vector_type(2), aligned(8)));
    u64x2v pre = {0ull, 0ull}, pre0 = {0ull, 0ull};  // E(s'-1), E(s') and E(s'-3), E(s'-2)
    auto load_pre = [&]() __attribute__((always_inline)) {
        const TblPeek nb = tbl_peek(src, j);
        if (nb.ok) {
            const u64x2v* p = reinterpret_cast<const u64x2v*>(erec + (int32_t)((nb.be - 3u) / 3u - 3u));
            pre0 = p[0];
            pre = p[1];
        }
    };
    // The pairs a step of kind P at slot s (the block's last rune) and the steps after it
    // read.  e1: (E(s-1), E(s)), e0: (E(s-3), E(s-2)), from pre or (a redo) loaded here.
    auto prime = [&](const int P, double (&wn)[4], const u64x2v e1, const u64x2v e0) __attribute__((always_inline)) {
        const uint64_t rc = e1.y;
        if (P == 0) {
            xl = e1.x;
            xh = e1.y;
            yl = e0.x;
            yh = e0.y;
        } else if (P == 1) {
            yl = e0.y;
            yh = e1.x;
            ld_pair(s - 4u, xl, xh);
        } else if (P == 2) {
            yl = e1.x;
            yh = e1.y;
            xl = e0.x;
            xh = e0.y;
        } else {
            xl = e0.y;
            xh = e1.x;
            ld_pair(s - 4u, yl, yh);
        }
        lc = s_ltab[(uint32_t)rc & 0xFFu];
        rec_weights<WL>(im, rc, wn);
        load_pre();
    };
    auto ld_e = [&](int d) -> u64x2v { return *reinterpret_cast<const u64x2v*>(erec + (int32_t)(s - 1u - d)); };
    // One rune.  wc: this rune's weights (loaded a step ago); wn: gets the next rune's.
    // Weight registers alternate between steps, so nothing is copied out of a
    // load's destination (a copy would wait for the load).
    auto step = [&](const int P, double (&wc)[4], double (&wn)[4]) __attribute__((always_inline)) -> bool {
        const bool more = q > bs;
        const uint64_t nx = P == 0 ? xl : (P == 1 ? yh : (P == 2 ? yl : xh));
        // the next rune's record when it exists; past the block's first rune it is whatever
        // precedes, and what it loads is replaced at the restart (prime) unused: with the
        // weights in LDS a garbage index only reads other LDS words, from memory it could
        // fault, so only that form masks it
        const uint64_t r1v = (WL || more) ? nx : 0ull;
        const uint64_t ln = s_ltab[(uint32_t)r1v & 0xFFu];
        rec_weights<WL>(im, r1v, wn);
        if (P == 0) ld_pair(s - 5u, xl, xh);
        if (P == 2) ld_pair(s - 5u, yl, yh);
        const uint32_t cs = c << 9;
        uint32_t bLs;
        double bP = rec_fold_a3(lc, wc, cs, rb0, lb, bLs);
        bool redo = false;
        if (lc & kLtabOvf) {  // overflowed record (rare)
            DpFold f;
            dp_walk_rune(v, im, q, be, f, c, ring, false, gbest, 0u);
            f.finish();
            bLs = f.bestL << 9;
            bP = f.bestP;
            redo = f.redo;
        }
        ring_at(cs) = bP;
        v.bls[bi] = (uint8_t)(bLs >> 9);
        steps++;
        const bool restart = redo || !more;
        if (!restart) {
            q -= 3u;
            s -= 1u;
            bi -= 1u;
            lc = ln;
            ++c;
            return false;
        }
        if (redo) redom |= 1u << (j - 1u);  // an edge past the ring: the caller redoes this block
        if (!src.next(j, bs, be)) return true;
        setup();
        prime((P + 1) & 3, wn, pre, pre0);  // the next step is the next kind
        return false;
    };
    double wa[4], wb[4];
    setup();
    prime(0, wa, ld_e(0), ld_e(2));
    for (;;) {
        if (step(0, wa, wb)) break;
        if (step(1, wb, wa)) break;
        if (step(2, wa, wb)) break;
        if (step(3, wb, wa)) break;
    }
    return steps;
}

// A lane's deferred Viterbi runs (all-3-byte chunks): LDS words t[r * 64],
// (rs - wb) | (re - wb) << 16.  The forward walk only lists the runs; the
// Viterbis then run with every lane on its r-th run at once, instead of one
// divergent Viterbi whenever some lane's walk reaches the end of a run.
#ifndef JB_ZH_RUNS
#define JB_ZH_RUNS 4
#endif
constexpr uint32_t kZhRuns = JB_ZH_RUNS;
static_assert(2u * kZhWinWords <= kZhPool && kZhPool + kZhRuns * 64u <= 2u * kZhRing * 64u,
              "k_zh: token bitmaps, then the run list, within the wave's ring");
struct RunList {
    uint32_t* t;
    uint32_t wb;
    uint32_t n;
    uint32_t* pool = nullptr;  // zh_fwd_a3: the wave's run list (kZhRuns * 64 entries) and its count
    uint32_t* cnt = nullptr;
};

// The forward half of viterbi for all of a lane's deferred runs (all-3-byte
// chunk) in one loop: one rune per step, runs back to back, so a lane's trip
// count is its total run length.  The text of the rune two steps ahead and
// the emissions of the next rune are in flight during each step, in two
// register sets that alternate between steps (nothing copied out of a load's
// destination).  Returns the final states, bit r set for E (:723-729).
template <class E>
__device__ uint32_t viterbi_fwd_runs(const GrpZvT<true>& v, const DevImage& im, const uint32_t* runs, uint32_t n,
                                     uint32_t& nt) {
    // rune cursor: position q and run r of the current, next and next-but-one rune
    uint32_t q0 = 0, r0 = 0, q1 = 0, r1 = 0, q2 = 0, r2 = 0, t = 0;
    auto rs_of = [&](uint32_t r) { return v.wb + (runs[r * 64u] & 0xFFFFu); };
    auto re_of = [&](uint32_t r) { return v.wb + (runs[r * 64u] >> 16); };
    auto adv = [&](uint32_t& q, uint32_t& r) {  // the rune after (q, r); r == n past the last
        if (r >= n) return;
        if (q + 3u < re_of(r)) {
            q += 3u;
        } else {
            ++r;
            if (r < n) q = rs_of(r);
        }
    };
    uint32_t stbits = 0;
    if (n == 0) return 0;
    q0 = rs_of(0);
    q1 = q0;
    r1 = 0;
    adv(q1, r1);
    q2 = q1;
    r2 = r1;
    adv(q2, r2);
    double vB = 0, vM = 0, vE = 0, vS = 0;
    uint32_t xa = 0, xb = 0;  // text dwords (rune two ahead), alternating
    double ea[4], eb[4];      // emissions (rune one ahead), alternating
    uint32_t w0;
    load_emit(im, z_dec(v, q0, &w0), ea);
    xa = v.x4(q1);
    bool act = true;
    auto step = [&](uint32_t& xn, uint32_t& xnn, double (&ec)[4], double (&en)[4]) {
        // xn: text of rune 1 ahead (landed); xnn: gets rune 2 ahead; ec: this rune's emissions
        if (r2 < n) xnn = v.x4(q2);
        if (r1 < n) {
            const uint32_t x = xn;
            const uint32_t rn = ((x & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu);
            load_emit(im, rn, en);
        }
        uint32_t cB, cM, cE, cS;
        double pB, pM, pE, pS;
        uint32_t tt = 0;  // (a run's first rune takes no route: its values are the previous run's)
        route2(vE + T_EB, vS + T_SB, &cB, &pB, tt);  // B <- E, S
        route2(vB + T_BM, vM + T_MM, &cM, &pM, tt);  // M <- B, M
        route2(vB + T_BE, vM + T_ME, &cE, &pE, tt);  // E <- B, M
        route2(vE + T_ES, vS + T_SS, &cS, &pS, tt);  // S <- E, S
        const bool first = t == 0;
        nt += first ? 0u : tt;
        vB = (first ? START_B : pB) + ec[0];
        vM = (first ? JB_MIN_FLOAT : pM) + ec[1];
        vE = (first ? JB_MIN_FLOAT : pE) + ec[2];
        vS = (first ? START_S : pS) + ec[3];
        v.bl(q0) = (uint8_t)(cB | (cM << 2) | (cE << 4) | (cS << 6));  // (unread for the first rune)
        const bool last = r1 != r0;
        if (last) stbits |= (vE > vS ? 1u : 0u) << r0;
        t = last ? 0u : t + 1u;
        q0 = q1;
        r0 = r1;
        q1 = q2;
        r1 = r2;
        adv(q2, r2);
        act = r0 < n;
    };
    while (act) {
        step(xa, xb, ea, eb);
        if (!act) break;
        step(xb, xa, eb, ea);
    }
    return stbits;
}

// Forward walk of one block (findDagPath) + HMM runs.  Returns false where the
// reference panics (a rune on the chosen path with no DAG edge: cutDAG slices
// with tail index -1).
template <bool HMM, class V, class E>
__device__ __forceinline__ bool zh_fwd(const V& v, const DevImage& im, uint32_t bs, uint32_t be, E& em, RunList* rl) {
    auto run_end = [&](uint32_t rs, uint32_t re, uint32_t m) {
        if (m == 1u) em.token(rs, re);  // a single rune is always "S" (:672-674)
        else if (rl && rl->n < kZhRuns) {
            rl->t[rl->n * 64u] = (rs - rl->wb) | ((re - rl->wb) << 16);
            rl->n++;
        } else viterbi_run(v, im, rs, re, m, em);
    };
    uint32_t p = bs, run_s = 0, run_n = 0;
    while (p < be) {
        const uint32_t L = v.bl(p);
        if (L == 0) return false;  // tail index -1: cutDAG's slice panics in the reference
        uint32_t pe = p;
        if (V::all3) pe += 3u * L;
        else
            for (uint32_t k = 0; k < L; k++) pe += z_w(v, pe);
        if (!HMM) {
            em.token(p, pe);
        } else if (L == 1) {
            if (run_n == 0) run_s = p;
            run_n++;
        } else {
            if (run_n) {
                run_end(run_s, p, run_n);
                run_n = 0;
            }
            em.token(p, pe);
        }
        p = pe;
    }
    if (HMM && run_n) run_end(run_s, be, run_n);
    return true;
}

// The forward walk over all of a lane's blocks in one loop (a lane's trip
// count is its total piece count, not the per-block maximum over the wave).
template <bool HMM, class V, class E, class Src>
__device__ bool zh_fwd_lane(const V& v, const DevImage& im, const Src& src, E& em, RunList* rl) {
    auto run_end = [&](uint32_t rs, uint32_t re, uint32_t m) {
        if (m == 1u) em.token(rs, re);  // a single rune is always "S" (:672-674)
        else if (rl && rl->n < kZhRuns) {
            rl->t[rl->n * 64u] = (rs - rl->wb) | ((re - rl->wb) << 16);
            rl->n++;
        } else viterbi_run(v, im, rs, re, m, em);
    };
    uint32_t j = 0, bs = 0, be = 0;
    bool ok = true;
    if (!src.next(j, bs, be)) return ok;
    uint32_t p = bs, run_s = 0, run_n = 0;
    for (;;) {
        if (p >= be) {  // the block is done: its last run, then the lane's next block
            if (HMM && run_n) run_end(run_s, be, run_n);
            run_n = 0;
            if (!src.next(j, bs, be)) break;
            p = bs;
            continue;
        }
        const uint32_t L = v.bl(p);
        if (L == 0) {  // tail index -1: cutDAG's slice panics in the reference
            ok = false;
            p = be;
            run_n = 0;
            continue;
        }
        uint32_t pe = p;
        if (V::all3) pe += 3u * L;
        else
            for (uint32_t k = 0; k < L; k++) pe += z_w(v, pe);
        if (!HMM) {
            em.token(p, pe);
        } else if (L == 1) {
            if (run_n == 0) run_s = p;
            run_n++;
        } else {
            if (run_n) {
                run_end(run_s, p, run_n);
                run_n = 0;
            }
            em.token(p, pe);
        }
        p = pe;
    }
    return ok;
}

// The same for an all-3-byte window (the common case), leaner: a piece's length is
// read by slot ((q - wb) / 3 kept beside q, no division), the lane's blocks come from
// registers (RegSrc: a block change is no LDS loop), and each token ORs its two bits
// straight into the wave's LDS bitmaps (two LDS atomics, no register state to flush
// when the word changes).  Runs of single-rune pieces go to the run list as before
// (a run of one rune is "S", its own token).
template <bool HMM, class Src>
__device__ __forceinline__ bool zh_fwd_a3(const GrpZvT<true>& v, const DevImage& im, Src src,
                                          uint32_t* sb, uint32_t* eb, LdsEmitter& le, RunList* rl) {
    const uint32_t w0 = v.wb >> 5;
    auto token = [&](uint32_t a, uint32_t b) __attribute__((always_inline)) {
        atomicOr(sb + ((a >> 5) - w0), 1u << (a & 31u));
        atomicOr(eb + (((b - 1u) >> 5) - w0), 1u << ((b - 1u) & 31u));
    };
    // A run of more than one rune goes to the wave's run list (one LDS atomic), whose
    // entries are then dealt to the lanes round-robin: runs are short (2-4 runes,
    // about one per two blocks), and a lane's own runs would leave most lanes idle
    // while a few work through several.  A full list (rare) cuts the run here.
    auto run_end = [&](uint32_t rs, uint32_t re, uint32_t m) __attribute__((always_inline)) {
        if (m == 1u) token(rs, re);  // a single rune is always "S" (:672-674)
        else {
            const uint32_t k = atomicAdd(rl->cnt, 1u);
            if (k < kZhRuns * 64u) rl->pool[k] = (rs - rl->wb) | ((re - rl->wb) << 16);
            else viterbi_run(v, im, rs, re, m, le);
        }
    };
    uint32_t j = 0, bs = 0, be = 0;
    bool ok = true;
    if (!src.next(j, bs, be)) return ok;
    uint32_t p = bs, sp = (bs - v.wb) / 3u, run_s = 0, run_n = 0;  // sp: GrpZvT::bl's slot of p
    for (;;) {
        if (p >= be) {  // the block is done: its last run, then the lane's next block
            if (HMM && run_n) run_end(run_s, be, run_n);
            run_n = 0;
            if (!src.next(j, bs, be)) break;
            p = bs;
            sp = (bs - v.wb) / 3u;
            continue;
        }
        const uint32_t L = v.bls[sp];
        if (L == 0) {  // tail index -1: cutDAG's slice panics in the reference
            ok = false;
            p = be;
            run_n = 0;
            continue;
        }
        const uint32_t pe = p + 3u * L;
        if (HMM && L == 1u) {
            run_s = run_n ? run_s : p;
            run_n++;
        } else {
            if (HMM && run_n) {
                run_end(run_s, p, run_n);
                run_n = 0;
            }
            token(p, pe);
        }
        p = pe;
        sp += L;
    }
    return ok;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// any 4-byte UTF-8 lead byte (>= 0xF0) in the 16-byte words covering [bs, be)
// (bytes of neighbours in the same words may give a false positive: that only
// selects the general rune stepping)
__device__ __forceinline__ bool text_has4(const uint8_t* __restrict__ text, uint32_t bs, uint32_t be) {
    uint32_t acc = 0;
    for (uint32_t a = bs & ~15u; a < be; a += 16u) {
        const uint4 x = *reinterpret_cast<const uint4*>(text + a);
        acc |= (x.x & (x.x << 1) & (x.x << 2) & (x.x << 3)) | (x.y & (x.y << 1) & (x.y << 2) & (x.y << 3)) |
               (x.z & (x.z << 1) & (x.z << 2) & (x.z << 3)) | (x.w & (x.w << 1) & (x.w << 2) & (x.w << 3));
    }
    return (acc & 0x80808080u) != 0u;
}

template <bool HMM, bool A3, bool WL>
__device__ __forceinline__ void zh_chunk_main(const uint8_t* __restrict__ text, const DevImage& im,
                              const uint64_t* __restrict__ erec, double* __restrict__ gbest, uint8_t* bls,
                              double* ring, const char* rb0, uint32_t lb, uint32_t* rb32, uint32_t* runs,
                              uint32_t* nrun,
                              const TblSrc& src, uint32_t wb, uint32_t lane,
                              uint32_t* __restrict__ counters, uint32_t winw, uint32_t& nties, uint64_t* st) {
    const GrpZvT<A3> v{text, bls, wb};
    uint32_t steps;
#ifndef JB_ZH_REGSRC
#define JB_ZH_REGSRC 1
#endif
    if constexpr (A3) {
        uint32_t redom = 0;
#if JB_ZH_REGSRC
        steps = zh_dp_a3<WL>(v, im, erec, gbest, ring, rb0, lb, RegSrc(src), redom);
#else
        steps = zh_dp_a3<WL>(v, im, erec, gbest, ring, rb0, lb, src, redom);
#endif
        while (redom) {  // (rare) blocks with an edge past the ring, best values in gbest
            const uint32_t k = (uint32_t)__builtin_ctz(redom);
            redom &= redom - 1u;
            const uint32_t x = src.t[k * 64u];
            steps += zh_dp(v, im, erec, gbest, ring, OneSrc{wb + (x & 0xFFFFu), wb + (x >> 16)});
        }
    } else {
        steps = zh_dp(v, im, erec, gbest, ring, src);
    }
    wave_sync();  // ring dead: its space takes the window's token bitmaps
    if (st) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        st[1] += t - st[7];
        st[7] = t;
        st[4] += steps;
        uint32_t mx = steps;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
        st[5] += mx;
    }
    uint32_t* sb = rb32;
    uint32_t* eb = rb32 + kZhWinWords;
    for (uint32_t k = lane; k < winw; k += 64u) {
        sb[k] = 0u;
        eb[k] = 0u;
    }
    wave_sync();
    {
        LdsEmitter le(sb, eb, wb >> 5);
        bool ok;
        RunList rl{runs, wb, 0u, runs - lane, nrun};
        RunList* const rlp = (HMM && A3) ? &rl : nullptr;
        if constexpr (A3) {
            if (lane == 0u) *nrun = 0u;
            wave_sync();
#if JB_ZH_REGSRC
            ok = zh_fwd_a3<HMM>(v, im, RegSrc(src), sb, eb, le, &rl);
#else
            ok = zh_fwd_a3<HMM>(v, im, src, sb, eb, le, &rl);
#endif
            wave_sync();
            const uint32_t nr = min(*nrun, kZhRuns * 64u);  // the pool's entries k = lane + 64 r are this lane's
            rl.n = nr > lane ? (nr - lane + 63u) / 64u : 0u;
            if (st) {  // Viterbi lane use: the lanes' summed run lengths against 64 x their maximum
                uint32_t s = 0, l1 = 0;
                for (uint32_t r = 0; r < rl.n; r++) {
                    const uint32_t y = runs[r * 64u];
                    const uint32_t len = ((y >> 16) - (y & 0xFFFFu)) / 3u;
                    s += len;
                    l1 = max(l1, len);
                }
                uint32_t mx = s, sm = s;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) {
                    mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
                    sm += (uint32_t)__shfl_xor((int)sm, d, 64);
                    l1 = max(l1, (uint32_t)__shfl_xor((int)l1, d, 64));
                }
                st[10] += sm;
                st[11] += mx;
                st[12] += l1;              // the longest single run: no dealing goes below it
                st[13] += (sm + 63u) / 64u;  // the wave's runes split evenly over its lanes
            }
        } else {
            ok = zh_fwd_lane<HMM>(v, im, src, le, rlp);
        }
        if (st) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            st[8] += t - st[7];
            st[7] = t;
        }
        if constexpr (HMM && A3) {
            const uint32_t stb = viterbi_fwd_runs<LdsEmitter>(v, im, runs, rl.n, le.ties);
            if (st) {
                const uint64_t t = __builtin_amdgcn_s_memtime();
                st[9] += t - st[7];
                st[7] = t;
            }
            for (uint32_t r = 0; r < kZhRuns; r++)
                if (r < rl.n) {
                    const uint32_t x = runs[r * 64u];
                    const uint32_t rs = wb + (x & 0xFFFFu), re = wb + (x >> 16);
                    viterbi_back(v, rs, re, (re - rs) / 3u, ((stb >> r) & 1u) ? (uint32_t)JB_E : (uint32_t)JB_S,
                                 le);
                }
        }
        le.flush();
        nties += le.ties;
        if (!ok) atomicOr(counters + CNT_ERR, 1u);
    }
    wave_sync();
}

// The next m zh blocks of a k_zh group, in text order, from its lane-mask words
// staged in LDS (lmv: group word i at lmv[i]; gnw words hold the group's starts,
// the rest are lookahead for block ends).  Rounds of 64 words, one per lane; rw is
// the current round, used how many of its zh starts earlier chunks took.  Entries
// tbl[0..m): in-window blocks as (bs - wb) | (be - wb) << 16, the others as
// 0x80000000 | (bs - wb).  Returns the new (rw, used).  Not inlined: its registers
// would otherwise stay allocated across k_zh's DP (3 waves per SIMD instead of 4).
__device__ __noinline__ uint2 lm_collect(const uint32_t* lmv, uint32_t* tbl, uint32_t lane, uint32_t gw0, uint32_t gnw,
                                         uint32_t nlw, uint32_t nbytes, uint32_t wb, uint32_t wend, uint32_t m,
                                         uint32_t rw, uint32_t used) {
    for (uint32_t have = 0; have < m;) {
        const uint32_t xa = lmv[rw + lane], xb = lmv[rw + 64u + lane];  // this round and its lookahead
        const uint32_t bm = xa & 0xFFFFu;
        const uint32_t zm = (rw + lane < gnw) ? (xa >> 16) : 0u;
        const uint32_t cz = (uint32_t)__popc(zm);
        const uint32_t incl = wave_incl_scan(cz);  // inclusive prefix over the lanes
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        // the first block start after this lane's word: in a later lane of this round, else
        // in the lookahead round, else past it (0xFFFFFFFF: found later) or the batch end
        const uint64_t la = __ballot(bm != 0u), lb = __ballot((xb & 0xFFFFu) != 0u);
        const uint64_t later = la & ~((2ull << lane) - 1ull);
        const uint32_t j = later ? (uint32_t)__builtin_ctzll(later) : (lb ? (uint32_t)__builtin_ctzll(lb) : 0u);
        const uint32_t lo_a = bm ? (uint32_t)__builtin_ctz(bm) : 0u;
        const uint32_t lo_b = (xb & 0xFFFFu) ? (uint32_t)__builtin_ctz(xb & 0xFFFFu) : 0u;
        const uint32_t sa = (uint32_t)__shfl((int)lo_a, (int)j, 64), sb = (uint32_t)__shfl((int)lo_b, (int)j, 64);
        const uint32_t wr = gw0 + rw;
        uint32_t nxt = 0xFFFFFFFFu;
        if (later) nxt = (wr + j) * 16u + sa;
        else if (lb) nxt = (wr + 64u + j) * 16u + sb;
        else if (wr + 128u >= nlw) nxt = (uint32_t)nbytes;  // no block starts after this one
        const uint32_t take = min(total - used, m - have);
        uint32_t z = zm, r = incl - cz;
        while (z) {
            const uint32_t k = (uint32_t)__builtin_ctz(z);
            z &= z - 1u;
            if (r >= used && r < used + take) {
                const uint32_t bs = (wr + lane) * 16u + k;
                const uint32_t above = bm & ~((2u << k) - 1u);
                const uint32_t be = above ? (wr + lane) * 16u + (uint32_t)__builtin_ctz(above) : nxt;
                tbl[have + r - used] = (be <= wend) ? (bs - wb) | ((be - wb) << 16) : (0x80000000u | (bs - wb));
            }
            r++;
        }
        have += take;
        used += take;
        if (used == total) {  // next round
            rw += 64u;
            used = 0;
        }
    }
    return make_uint2(rw, used);
}

// ---------------------------------------------------------------------------
// k_nonzh: one lane per non-Han block (cutNonZh, tokenizer.go:289-310)
// ---------------------------------------------------------------------------
// cutNonZh for one block [bs, be) (tokenizer.go:289-310).  The block's bytes
// come in 16-byte loads issued together (a byte-by-byte walk over global
// memory made every byte a dependent round trip); the tokenizing pass reads
// them from the lane's 80-byte LDS window.
__device__ __forceinline__ uint32_t nz_keep(uint32_t base, uint32_t bs, uint32_t be) {  // bytes in [bs, be)
    const uint32_t lo = bs > base ? min(bs - base, 4u) : 0u, hi = be > base ? min(be - base, 4u) : 0u;
    if (hi <= lo) return 0u;
    return (uint32_t)(((1ull << (8u * hi)) - 1ull) & ~((1ull << (8u * lo)) - 1ull));
}
// W: the bytes tokenized per round of loads (64 with the lane's 80-byte window; 48 with a
// 64-byte one)
__device__ __forceinline__ uint32_t alnum_mask16(uint4 x);
// Bit k for each byte k of the 16 bytes x: >= 0x80 (hi), an ASCII space (sp: 0x09-0x0D, 0x20)
__device__ __forceinline__ void hi_space_mask16(uint4 x, uint32_t& hi, uint32_t& sp) {
    const uint32_t v[4] = {x.x, x.y, x.z, x.w};
    hi = sp = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t h = (v[j] & 0x80808080u) >> 7;
        const uint32_t s = (jb_bytes_between(v[j], 0x08u, 0x0Eu) | jb_bytes_between(v[j], 0x1Fu, 0x21u)) >> 7;
        hi |= ((h * 0x204081u) >> 21 & 0xFu) << (4 * j);
        sp |= ((s * 0x204081u) >> 21 & 0xFu) << (4 * j);
    }
}
template <uint32_t W>
__device__ void nonzh_block(const uint8_t* __restrict__ text, uint32_t bs, uint32_t be, Emitter& em, uint8_t* buf) {
    static_assert(W == 64u, "the 80-byte window");
    const uint32_t a0 = bs & ~15u;
    if (be <= a0 + 64u) {
        // The block lies in one round of four loads: its tokens come from bit masks over
        // those 64 bytes (the byte-at-a-time walk below: k_nonzh 0.165 -> 0.139 ms at 1 GiB).
        // alnum runs -> one token each; other ASCII bytes -> one token each unless a space;
        // runes from bytes >= 0x80 (never alnum, never ASCII) are decoded one by one.
        uint4 c[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            c[k] = (a0 + 16u * k < be) ? *reinterpret_cast<const uint4*>(text + a0 + 16u * k) : make_uint4(0, 0, 0, 0);
        const uint32_t lo = bs - a0, hb = be - a0;  // the block's bytes: [lo, hb) of the 64, hb in 1..64
        const uint64_t inb = (hb == 64u ? ~0ull : (1ull << hb) - 1ull) & ~((1ull << lo) - 1ull);
        uint64_t A = 0, H = 0, S = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t h, s;
            hi_space_mask16(c[k], h, s);
            A |= (uint64_t)alnum_mask16(c[k]) << (16 * k);
            H |= (uint64_t)h << (16 * k);
            S |= (uint64_t)s << (16 * k);
        }
        A &= inb;
        if (!A) return;  // alnum.FindAllIndex found nothing -> no tokens (:290-293)
        H &= inb;
        const uint64_t O = inb & ~(A | H | S);  // one-byte tokens
        uint64_t st = (A & ~(A << 1)) | O, en = (A & ~(A >> 1)) | O;
        if (H) {
#pragma unroll
            for (int k = 0; k < 4; k++) reinterpret_cast<uint4*>(buf)[k] = c[k];
            do {
                const uint32_t p = (uint32_t)__builtin_ctzll(H);
                uint32_t r;
                const uint32_t w = jb_decode(lds4(buf, p), min(4u, hb - p), &r);  // (lds4 reads up to byte 66)
                if (!jb_is_space(r)) {
                    st |= 1ull << p;
                    en |= 1ull << (p + w - 1u);
                }
                H &= p + w >= 64u ? 0ull : ~((1ull << (p + w)) - 1ull);
            } while (H);
        }
        // 64 bits from a0 (a0 % 32 is 0 or 16) -> bitmap words a0 / 32 .. + 2
        const uint32_t sh = a0 & 31u, w0 = a0 >> 5;
        em.bits(w0, (uint32_t)st << sh, (uint32_t)en << sh);
        em.bits(w0 + 1u, (uint32_t)((st << sh) >> 32), (uint32_t)((en << sh) >> 32));
        if (sh) em.bits(w0 + 2u, (uint32_t)(st >> 48), (uint32_t)(en >> 48));
        return;
    }
    bool has = false;  // alnum.FindAllIndex found nothing -> no tokens (:290-293)
    for (uint32_t a = bs & ~15u; a < be && !has; a += 64u) {
        uint4 c[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            c[k] = (a + 16u * k < be) ? *reinterpret_cast<const uint4*>(text + a + 16u * k) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t b = a + 16u * k;
            has |= jb_any_alnum4(c[k].x & nz_keep(b, bs, be)) || jb_any_alnum4(c[k].y & nz_keep(b + 4u, bs, be)) ||
                   jb_any_alnum4(c[k].z & nz_keep(b + 8u, bs, be)) || jb_any_alnum4(c[k].w & nz_keep(b + 12u, bs, be));
        }
    }
    if (!has) return;
    uint32_t p = bs, run = 0;
    bool in_run = false;
    while (p < be) {
        const uint32_t a = p & ~15u;
#pragma unroll
        for (int k = 0; k < (int)(W / 16u) + 1; k++)  // bytes up to be + 3 (decode reads 4; padding follows the text)
            if (a + 16u * k < be + 4u)
                reinterpret_cast<uint4*>(buf)[k] = *reinterpret_cast<const uint4*>(text + a + 16u * k);
        const uint32_t pe = min(be, a + W);
        while (p < pe) {
            const uint32_t x = lds4(buf, p - a);
            if (jb_is_alnum(x & 0xFFu)) {  // alnum runs are kept whole
                if (!in_run) {
                    in_run = true;
                    run = p;
                }
                p++;
                continue;
            }
            if (in_run) {
                em.token(run, p);
                in_run = false;
            }
            uint32_t r;
            const uint32_t w = jb_decode(x, min(4u, be - p), &r);
            if (!jb_is_space(r)) em.token(p, p + w);  // one token per rune; spaces dropped
            p += w;
        }
    }
    if (in_run) em.token(run, be);
}

// Bit k set for each byte k of the 16 bytes x that is [0-9A-Za-z] (jb_is_alnum).
__device__ __forceinline__ uint32_t alnum_mask16(uint4 x) {
    const uint32_t v[4] = {x.x, x.y, x.z, x.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t f = (jb_bytes_between(v[j], 0x2Fu, 0x3Au) | jb_bytes_between(v[j] | 0x20202020u, 0x60u, 0x7Bu)) >> 7;
        m |= ((f * 0x204081u) >> 21 & 0xFu) << (4 * j);  // bits 0/8/16/24 -> 0..3
    }
    return m;
}

// The non-Han blocks whose first alnum byte lies in chunk c (text tx, lane mask lm).
template <uint32_t W>
__device__ __forceinline__ void nonzh_chunk(const uint8_t* __restrict__ text, uint32_t nbytes,
                                            const uint32_t* __restrict__ lanemask, const uint2* __restrict__ tile_cnt,
                                            uint32_t ntiles, const uint64_t* __restrict__ alnum16, uint32_t c, uint4 tx,
                                            uint32_t lm, Emitter& em, uint8_t* buf) {
    {
        const uint32_t c0 = c * 16u;
        uint32_t A = alnum_mask16(tx);
        if (c0 + 16u > nbytes) A &= (1u << (nbytes - c0)) - 1u;
        const uint32_t bm = lm & 0xFFFFu;
        while (A) {  // a block with an alnum byte in this chunk
            const uint32_t i = (uint32_t)__builtin_ctz(A);
            const uint32_t le = bm & ((2u << i) - 1u), after = bm & ~((2u << i) - 1u);
            A &= after ? ~((1u << __builtin_ctz(after)) - 1u) : 0u;  // the block's bytes of this chunk
            uint32_t bs;
            bool own = true;
            if (le) {
                bs = c0 + 31u - (uint32_t)__builtin_clz(le);
            } else {  // the block began before this chunk: walk back to its start
                uint32_t k = c;
                bs = 0;
                while (k > 0u) {  // (byte 0 starts a block, so the walk ends there at the latest)
                    --k;
                    const uint32_t m = lanemask[k] & 0xFFFFu;
                    const bool al = (alnum16[k >> 6] >> (k & 63u)) & 1ull;
                    if (m) {
                        const uint32_t o = 31u - (uint32_t)__builtin_clz(m);
                        bs = k * 16u + o;
                        if (al) own = (alnum_mask16(*reinterpret_cast<const uint4*>(text + k * 16u)) >> o) == 0u;
                        break;
                    }
                    if (al) {
                        own = false;
                        break;
                    }
                }
            }
            if (!own) continue;
            const uint32_t be = after ? c0 + (uint32_t)__builtin_ctz(after)
                                      : nz_block_end(lanemask, tile_cnt, ntiles, nbytes, c);
            nonzh_block<W>(text, bs, be, em, buf);
        }
    }
}

// k_nonzh's unit is a wave's 64 alnum16 words (64 KiB of text).  Their chunks with an
// alnum byte (about 0.8 per KiB on C_syn, up to 8 in one word) are dealt to the
// wave's lanes in order through an LDS list, kNzCap per round (two per lane, their
// loads issued together): a lane per word instead made every wave as slow as its
// busiest word's serial chain of dependent loads.
#ifndef JB_NZ_CAP
#define JB_NZ_CAP 128
#endif
constexpr uint32_t kNzCap = JB_NZ_CAP;
static_assert(kNzCap % 64u == 0u && kNzCap >= 64u && kNzCap <= 256u, "whole rounds of the wave's lanes");
struct NzLds {
    uint8_t win[256][80];          // the lanes' nonzh_block windows
    uint32_t list[4][kNzCap];      // each wave's chunks of the round
};
template <uint32_t W>
__device__ __forceinline__ void nonzh_waves(const uint8_t* __restrict__ text, uint32_t nbytes, uint32_t nch,
                                            const uint32_t* __restrict__ lanemask, const uint2* __restrict__ tile_cnt,
                                            uint32_t ntiles, const uint64_t* __restrict__ alnum16, uint32_t wave,
                                            uint32_t nwaves, Emitter& em, NzLds& L) {
    const uint32_t lane = threadIdx.x & 63u, nw = (nch + 63u) >> 6;
    uint32_t* const list = L.list[threadIdx.x >> 6];
    uint8_t* const buf = L.win[threadIdx.x];
    for (uint32_t w0 = wave * 64u; w0 < nw; w0 += nwaves * 64u) {  // (uniform in the wave)
        const uint32_t wi = w0 + lane;
        uint64_t a = wi < nw ? alnum16[wi] : 0ull;
        const uint32_t cnt = (uint32_t)__builtin_popcountll(a);
        const uint32_t inc = wave_incl_scan(cnt);
        const uint32_t total = (uint32_t)__shfl((int)inc, 63, 64);
        uint32_t pos = inc - cnt;  // this lane's next chunk's place in the wave's order
        for (uint32_t r0 = 0; r0 < total; r0 += kNzCap) {
            for (; a && pos < r0 + kNzCap; pos++, a &= a - 1ull) list[pos - r0] = wi * 64u + (uint32_t)__builtin_ctzll(a);
            wave_sync();
            const uint32_t m = min(kNzCap, total - r0);
            uint32_t c[kNzCap / 64u], lm[kNzCap / 64u];
            uint4 tx[kNzCap / 64u];
#pragma unroll
            for (uint32_t j = 0; j < kNzCap / 64u; j++) {
                c[j] = lane + 64u * j < m ? list[lane + 64u * j] : ~0u;
                tx[j] = make_uint4(0, 0, 0, 0);
                lm[j] = 0;
                if (c[j] < nch) {  // (chunks past the batch: padding)
                    tx[j] = *reinterpret_cast<const uint4*>(text + c[j] * 16u);
                    lm[j] = lanemask[c[j]];
                }
            }
            wave_sync();  // the list is read before the next round writes it
#pragma unroll
            for (uint32_t j = 0; j < kNzCap / 64u; j++)
                if (c[j] < nch) nonzh_chunk<W>(text, nbytes, lanemask, tile_cnt, ntiles, alnum16, c[j], tx[j], lm[j], em, buf);
        }
    }
}

// k_nonzh's arguments, for its work inside k_long<.., true>
struct NzArgs {
    uint32_t nbytes, ntiles, ndocs;
    const uint32_t* lanemask;
    const uint2* tile_cnt;
    const uint64_t* alnum16;
    uint32_t* docbits;
    const uint64_t* doc_off;
};

// At least 4 waves per SIMD (at most 128 VGPRs): the DP is latency-bound and
// needs them; left alone the allocator lands just above 128 (3 waves, k_zh +17 %).
#ifndef JB_ZH_WAVES
#define JB_ZH_WAVES 4
#endif
#define JB_ZH_ATTR __attribute__((amdgpu_waves_per_eu(JB_ZH_WAVES)))
// NW waves per workgroup: 4, or kZhWgWide = 16 (one workgroup per CU) with the
// weight table in LDS for the DP (rec_weights<true>), when it fits (kZhWtab).
template <bool HMM, uint32_t NW>
__global__ __launch_bounds__(NW * 64) JB_ZH_ATTR void k_zh(const uint8_t* __restrict__ text, uint64_t nbytes,
                                            const uint32_t* __restrict__ lanemask, const uint2* __restrict__ tile_cnt,
                                            const uint32_t* __restrict__ tile4,
                                            uint32_t* __restrict__ counters, DevImage im,
                                            const uint64_t* __restrict__ erec, uint8_t* __restrict__ gbl,
                                            double* __restrict__ gbest,
                                            uint32_t* __restrict__ sbits, uint32_t* __restrict__ ebits,
                                            uint2* __restrict__ longblk, uint32_t* __restrict__ lsegb, uint32_t grp,
                                            uint32_t g1, uint32_t sgrp, uint32_t diag, uint64_t* __restrict__ dbg) {
    constexpr bool WL = NW == kZhWgWide;
    __shared__ uint8_t s_bl[NW][kZhBlBytes];
    __shared__ double s_rb[NW][kZhRing * 64];  // DP ring, then the window's token bitmaps and run list
    __shared__ uint32_t s_tbl[NW][kZhChunk];   // the chunk's blocks as found, then as dealt to the lanes
    __shared__ uint32_t s_hist[NW][64];
    __shared__ uint32_t s_nrun[NW];  // entries in a wave's run list (zh_fwd_a3)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    double* ring = s_rb[wv] + lane;
    const char* const rb0 = reinterpret_cast<const char*>(&s_rb[0][0]);  // (rec_fold_a3's ring addressing)
    const uint32_t lb = wv * (uint32_t)sizeof(s_rb[0]) + lane * 8u;
    static_assert(sizeof(s_rb[0]) == 4096u, "a wave's ring is 8 slots x 64 lanes x 8 bytes (offsets 0xE00 | lb)");
    uint32_t* rb32 = reinterpret_cast<uint32_t*>(s_rb[wv]);
    uint32_t* tbl = s_tbl[wv];
    uint32_t* hist = s_hist[wv];
    // groups 0..g1-1 are grp bytes, the rest (the batch's tail) sgrp <= grp bytes: the
    // persistent grid's last claims are short, so its waves finish closer together
    const uint32_t tail0 = g1 * grp;
    const uint32_t ngroups = g1 + (tail0 < nbytes ? (uint32_t)((nbytes - tail0 + sgrp - 1u) / sgrp) : 0u);
    const uint32_t ntiles = (uint32_t)((nbytes + kTileBytes - 1u) / kTileBytes);
    const uint32_t nlw = ntiles * 256u;                                  // lane-mask words (16 bytes each)
    const uint32_t winw = (grp + (kZhWin - kZhGroupBytes)) / 32u + 1u;  // token words of a window (<= kZhWinWords)
    auto lmw = [&](uint32_t w) -> uint32_t { return w < nlw ? lanemask[w] : 0u; };
    if (threadIdx.x < 256u) s_ltab[threadIdx.x] = ltab_entry(threadIdx.x);
    if constexpr (WL)  // the weights, once per CU (the host launches this form only when they fit)
        for (uint32_t i = threadIdx.x; i < im.nw1; i += NW * 64u) s_wt[i] = im.wtab1[i];
    __syncthreads();
    // diagnostic per-wave clocks (JB_ABLATE bit 8): [0] setup [1] DP [2] forward+Viterbi+flush [3] chunks
    // [4] sum of lane DP steps [5] sum of per-chunk max lane DP steps [6] blocks past the window [7] scratch
    uint64_t stv[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // [8] forward walk [9] Viterbi forward half
    // [14] sum over chunks of the chunk's longest in-window block (runes): no dealing takes the DP below it
    // [10] lanes' summed Viterbi run runes [11] 64 x max ... (Viterbi lane use)
#if JB_STAMPS
    uint64_t* st = (diag & 0x100u) ? stv : nullptr;
#else
    uint64_t* const st = nullptr;  // built without the diagnostic clocks (make STAMPS=1)
#endif
    const uint64_t tk0 = st ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t nties = 0;  // Viterbi route ties
    // Wave w takes group w first, then the next unclaimed one from the counter: only
    // waves that finished a group touch the counter (4096 waves all claiming their
    // first group on one address cost ~80 us on a one-sentence batch).
    const uint32_t nwv = gridDim.x * (blockDim.x >> 6);
    uint32_t g = blockIdx.x * (blockDim.x >> 6) + wv;
    auto next_group = [&]() -> uint32_t {
        if (nwv >= ngroups) return ngroups;  // every group was some wave's first: no claim (a round trip) needed
        uint32_t x = 0;
        if (lane == 0) x = atomicAdd(counters + CNT_WORK, 1u);
        return nwv + __builtin_amdgcn_readfirstlane(x);
    };
    for (;; ) {
        if (g >= ngroups) break;
        const uint32_t gl = g < g1 ? grp : sgrp;
        const uint32_t wb = g < g1 ? g * grp : tail0 + (g - g1) * sgrp, wend = wb + gl + (kZhWin - kZhGroupBytes);
        // The group's zh blocks are the Han block starts (lane-mask bits 16-31) in its
        // words; a block ends at the next block start of any kind (bits 0-15).
        const uint32_t gw0 = wb >> 4;
        const uint32_t gnw = (uint32_t)((min((uint64_t)wb + gl, nbytes) - wb + 15u) >> 4);
        // The group's lane-mask words and the two rounds after them (block ends) are
        // staged in the wave's ring area, which is free until the DP.
        uint32_t* const lmv = rb32;
        // (returns the lane's count of Han block starts in the group's words, from the
        // registers: read back from LDS it was a round trip per word)
        auto stage = [&]() -> uint32_t {
            uint32_t v[kZhStagePer];
#pragma unroll
            for (uint32_t k = 0; k < kZhStagePer; k++) v[k] = lmw(gw0 + lane + 64u * k);
            uint32_t c = 0;
#pragma unroll
            for (uint32_t k = 0; k < kZhStagePer; k++) {
                lmv[lane + 64u * k] = v[k];
                c += lane + 64u * k < gnw ? (uint32_t)__popc(v[k] >> 16) : 0u;
            }
            wave_sync();
            return c;
        };
        uint32_t n = 0;
        {
            n = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(stage()), 63);
        }
        if (n == 0u) {  // no Han block starts here
            g = next_group();
            continue;
        }
        // all-3-byte window: no 4-byte Han rune starts in the tiles under it
        bool any4 = false;
        {
            const uint32_t t0 = wb / kTileBytes, t1 = (uint32_t)((min((uint64_t)wend, nbytes) - 1u) / kTileBytes);
            if (lane <= t1 - t0 && t0 + lane < ntiles) any4 = tile4[t0 + lane] != 0u;
        }
        const bool all3 = __ballot(any4) == 0ull;
        const uint32_t nch = (n + kZhChunk - 1u) / kZhChunk;
        const uint32_t cs = (n + nch - 1u) / nch;  // even chunks
        uint32_t rw = 0, used = 0;  // current round: group words [rw, rw + 64); zh starts of it already taken
        for (uint32_t c0 = 0; c0 < n; c0 += cs) {
            if (st) stv[7] = __builtin_amdgcn_s_memtime();
            const uint32_t m = min(cs, n - c0);
            if (c0) stage();  // (the previous chunk's DP and bitmaps used the ring)
            // the chunk's m zh blocks in text order: in-window ones as (bs - wb) | (be - wb) << 16,
            // the others as 0x80000000 | (bs - wb) (their end is found later)
            {
                const uint2 ru = lm_collect(lmv, tbl, lane, gw0, gnw, nlw, (uint32_t)nbytes, wb, wend, m, rw, used);
                rw = ru.x;
                used = ru.y;
            }
            wave_sync();
            // this lane's items k = lane + 64 i of the chunk.  Blocks whose end lm_collect did
            // not find in its two rounds (at least 1 KiB long; they may still end inside the
            // window) are cut one by one after the chunk: their starts wait in the wave's
            // hist words meanwhile, so nothing of them stays in registers across the DP.
            uint32_t bsi[kZhPer], bei[kZhPer];
            bool in[kZhPer], out[kZhPer];
#pragma unroll
            for (int i = 0; i < (int)kZhPer; i++) {
                const uint32_t k = lane + 64u * (uint32_t)i;
                const uint32_t x = k < m ? tbl[k] : 0x80000000u;
                in[i] = !(x & 0x80000000u);
                out[i] = k < m && !in[i];
                bsi[i] = wb + (x & 0xFFFFu);
                bei[i] = in[i] ? wb + (x >> 16) : bsi[i];
            }
            // rank in-window blocks by length (descending; counting sort on len/4)
            hist[lane] = 0u;
            wave_sync();
            for (uint32_t k = lane; k < kZhChunk; k += 64u) tbl[k] = ~0u;
            uint32_t bkt[kZhPer], idx[kZhPer];
#pragma unroll
            for (int i = 0; i < (int)kZhPer; i++) {
                bkt[i] = min(63u, (bei[i] - bsi[i]) >> 2);
                idx[i] = in[i] ? atomicAdd(hist + bkt[i], 1u) : 0u;
            }
            wave_sync();
            {  // start of each bucket in descending order: sum of the counts of longer buckets
                const uint32_t incl = wave_incl_scan(hist[lane]);  // (buckets 0..lane)
                const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                wave_sync();
                hist[lane] = total - incl;  // (buckets lane+1..63)
            }
            wave_sync();
            uint32_t nin = 0;
#pragma unroll
            for (int i = 0; i < (int)kZhPer; i++) {
                nin += (uint32_t)__popcll(__ballot(in[i]));
                if (in[i]) {
                    const uint32_t r = hist[bkt[i]] + idx[i];
                    const uint32_t sg = r >> 6, ps = r & 63u;
                    const uint32_t ln = (sg & 1u) ? 63u - ps : ps;
                    tbl[sg * 64u + ln] = (bsi[i] - wb) | ((bei[i] - wb) << 16);
                }
            }
            wave_sync();
            uint32_t nout = 0;  // (hist is free once the blocks are dealt)
#pragma unroll
            for (int i = 0; i < (int)kZhPer; i++) {
                const uint64_t ob = __ballot(out[i]);
                if (out[i]) hist[nout + __builtin_amdgcn_mbcnt_hi((uint32_t)(ob >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ob, 0u))] = bsi[i];
                nout += (uint32_t)__popcll(ob);
            }
            wave_sync();
            const TblSrc src{tbl + lane, (nin + 63u) >> 6, wb};
            if (st) {
                uint32_t lb3 = 0;
#pragma unroll
                for (int i = 0; i < (int)kZhPer; i++) lb3 = max(lb3, in[i] ? (bei[i] - bsi[i]) / 3u : 0u);
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) lb3 = max(lb3, (uint32_t)__shfl_xor((int)lb3, d, 64));
                stv[14] += lb3;
            }
            if (st) {
                const uint64_t t = __builtin_amdgcn_s_memtime();
                stv[0] += t - stv[7];
                stv[7] = t;
                stv[3]++;
            }
            if (all3)
                zh_chunk_main<HMM, true, WL>(text, im, erec, gbest, s_bl[wv], ring, rb0, lb, rb32, rb32 + kZhPool + lane,
                                             &s_nrun[wv], src, wb, lane, counters, winw, nties, st);
            else
                zh_chunk_main<HMM, false, WL>(text, im, erec, gbest, s_bl[wv], ring, rb0, lb, rb32, rb32 + kZhPool + lane,
                                              &s_nrun[wv], src, wb, lane, counters, winw, nties, st);
            // the window's token words: consecutive words per lane, one OR each (edge
            // words are shared with neighbouring groups and with k_nonzh)
            {
                const uint32_t w0 = wb >> 5;
                const uint32_t* sb = rb32;
                const uint32_t* eb = rb32 + kZhWinWords;
                for (uint32_t k = lane; k < winw; k += 64u) {
                    const uint32_t a = sb[k], b = eb[k];
                    if (a) atomicOr(sbits + w0 + k, a);
                    if (b) atomicOr(ebits + w0 + k, b);
                }
            }
            wave_sync();  // bitmaps read: the ring is free again
            // blocks whose end was not found in the staged rounds (rare): one per lane, each
            // on its own in HBM (or, from 8 KiB, by the k_long_* kernels)
            if (st) stv[6] += nout;
            if (lane < nout) {
                const uint32_t obs = hist[lane];
                const uint32_t obe = block_end_at(lanemask, tile_cnt, ntiles, (uint32_t)nbytes, obs);
                if (obe - obs >= kZhLongMin) {  // the k_long_* kernels cut it
                    // block index and first segment from one atomic, so lsegb ascends with the index
                    const uint32_t nsg = ((obe - obs) / 3u + kSeg - 1u) / kSeg;
                    const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long*>(counters + CNT_NLONG),
                                                             ((unsigned long long)nsg << 32) | 1ull);
                    longblk[(uint32_t)old] = make_uint2(obs, obe);
                    lsegb[(uint32_t)old] = (uint32_t)(old >> 32);
                } else {
                    Emitter em(sbits, ebits);
                    const GlbZv gv{text, gbl};
                    zh_dp(gv, im, erec, gbest, ring, OneSrc{obs, obe});
                    if (!zh_fwd<HMM>(gv, im, obs, obe, em, nullptr)) atomicOr(counters + CNT_ERR, 1u);
                    em.flush();
                    nties += em.ties;
                }
            }
            wave_sync();
            if (st) {
                const uint64_t t = __builtin_amdgcn_s_memtime();
                stv[2] += t - stv[7];
                stv[7] = t;
            }
        }
        g = next_group();
    }
    {
        uint32_t t = nties;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) t += (uint32_t)__shfl_xor((int)t, d, 64);
        if (lane == 0 && t) atomicAdd(counters + CNT_TIES, t);
    }
    if (st) {
        // lane DP steps summed over the wave
        uint64_t sum = stv[4];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)sum, d, 64);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(sum >> 32), d, 64);
            sum += ((uint64_t)hi << 32) | lo;
        }
        if (lane == 0) {
            uint64_t* o = dbg + (blockIdx.x * NW + wv) * 16u;
            o[8] = stv[8];
            o[9] = stv[9];
            o[10] = stv[10];
            o[11] = stv[11];
            o[12] = stv[12];
            o[13] = stv[13];
            o[14] = stv[14];
            o[0] = stv[0];
            o[1] = stv[1];
            o[2] = stv[2];
            o[3] = stv[3];
            o[4] = sum;
            o[5] = stv[5];
            o[6] = __builtin_amdgcn_s_memtime() - tk0;
            o[7] = stv[6];
        }
    }
}

// ---------------------------------------------------------------------------
// Long zh blocks (>= kZhLongMin bytes; e.g. an unpunctuated document, BASELINE
// config 5b), all 3-byte runes.  Their DP is one serial chain: best(i) is built
// from best(i+L) with float64 adds in the reference's order (:519-529), which
// must not be re-associated, so no two runes' values can be computed in
// parallel.  Everything around the chain is parallel:
//   k_long_dp    one workgroup per long block.  Waves 1-3 turn each rune's DAG
//                record into a descriptor in LDS (its item weights and the LDS
//                addresses of the best values they add to), two windows of 256
//                runes ahead of the chain, and copy finished best values to
//                HBM.  Wave 0 runs the chain on one lane, from LDS only, one
//                step software-pipelined and without a branch.
//   k_long_seg   one lane per 64-rune segment: the chosen lengths (maxIndexProba
//                over the same sums again, from the best values in HBM) and a
//                speculative path walked from the segment's first rune.
//   k_long_path  one wave per long block: findDagPath's true path through the
//                segments (:552-562).  Where it enters a segment off the
//                speculative path it walks until the two meet (within a few
//                pieces, in practice) and fixes the segment's path bits.
//   k_long_tail  one lane per segment: tokens of the marked pieces, and the
//                Viterbi (+ cutHMM) of every run of single-rune pieces that
//                starts there (the runs are independent, :229-253).
// A long block with a 4-byte Han rune takes k_zh's one-lane path in k_long_dp.
// ---------------------------------------------------------------------------
constexpr uint32_t kLongGrid = 64;    // k_long_dp workgroups (persistent over the long-block list)
#if JB_STAMPS
constexpr uint32_t kDbgLong = 65536u * 4u;  // k_long_dp's diagnostic clocks in the debug buffer (u64 index)
constexpr uint32_t kDbgLongWin = 65536u * 8u;  // per-window chain clocks and group counts of block 0
constexpr uint32_t kDbgLongWinMax = 65536u * 2u;
#endif
constexpr uint32_t kLdWin = 256;      // runes per descriptor window
constexpr uint32_t kLdDesc = 1024;    // descriptor ring: 4 windows
constexpr uint32_t kLdRing = 512;     // best-value ring (edges are at most 255 runes)
constexpr uint32_t kLdSide = 256;     // items of slow runes, per window
constexpr uint32_t kLdWalk = 0xFFFFFFFFu;  // descriptor flag: the chain walks the rune itself
static_assert(kSeg == 64u, "segments are one 64-bit mask");

// A rune's DP step in LDS.  Fast form (flag 0): items L = 1 < L2 < L3 < L4,
// absent ones with a NaN weight (their sums are NaN, every compare with them
// is false and fmax drops them).
struct LDesc {
    double w[4];    // item weights, ascending L
    uint32_t a[3];  // byte offsets in the best ring of best(i + L_k), k = 2..4
    uint32_t flag;  // 0: fast; 1 | off << 1 | m << 16: m items at side[off]; kLdWalk
};
struct LItem {
    double w;
    uint32_t L, pad;
};
// c ? a : b for a mask c of all ones or zero, as two v_bfi_b32 (a select the compiler
// keeps: it turns ternaries whose arms are loads into exec-mask branches)
__device__ __forceinline__ double bitsel64(uint32_t m, double a, double b) {
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    uint32_t lo, hi;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(lo) : "v"(m), "v"((uint32_t)ua), "v"((uint32_t)ub));
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(hi) : "v"(m), "v"((uint32_t)(ua >> 32)), "v"((uint32_t)(ub >> 32)));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

struct LSpec {  // a rune's speculative choice (k_long_spec) as the decided chain takes it
    double w;     // the chosen item's weight
    uint32_t ra;  // byte offset in dring of best(i + L)
    uint32_t m1;  // all ones if L is 1
};
struct LDecided {  // the decided chain's LDS (rune i at i & 1023)
    LSpec spec[16 + kLdDesc];  // (rune i at 16 + (i & 1023): the chain's prefetch past a window reads the 16 below)
    double dring[kLdDesc];  // best(i): the chain writes, the helpers verify and publish
    uint32_t m2[16 + kLdDesc];  // all ones if L is 2 (as spec)
    uint32_t L[kLdDesc];    // the chosen length (verification)
};
constexpr uint32_t kSpWin = 256;  // the decided chain's window (ring slots (j & 3) * 256 ..: no wrap inside): 16 loop trips of 4 groups
// Path states at segment boundaries (findDagPath, :552-562, over a long block cut
// in 64-rune segments).  Where the path goes on at the start of a segment is one
// byte x, the same code k_long_seg writes for each rune:
//   0..254  the next piece starts x runes past the segment's start (x >= 64: the
//           piece before spans the whole segment)
//   0xFF    it starts at offset 0, and the piece before is one rune (so a run of
//           single-rune pieces enters the segment)
// Crossing segment s maps x to the state at the next boundary: kLpNext.  The
// state at every boundary follows from composing these maps, which is integer
// work: exact in any association (unlike the f64 values).
__device__ __forceinline__ uint32_t lp_next(const uint8_t* codes, uint32_t x) {  // codes: the segment's 64 exit codes
    return x >= 64u && x != 0xFFu ? x - 64u : codes[x == 0xFFu ? 0u : x];
}
// the segment's entry as k_long_tail takes it: first piece start | a one-rune piece ends there << 8;
// 0xFFFFFFFF when no piece starts in it (or the path ended: runes past the block's n)
__device__ __forceinline__ uint32_t lp_entry(uint32_t x, uint32_t a, uint32_t n) {
    const uint32_t o = x == 0xFFu ? 0u : x;
    if (o >= 64u || a + o >= n) return 0xFFFFFFFFu;
    return o | (x == 0xFFu ? 256u : 0u);
}
constexpr uint32_t kLpMap = 256;    // a chunk map: next state for each of the 256 states
constexpr uint32_t kLpBatch = 128;  // chunk maps k_long_path stages in LDS at a time (32 KB)

// The 256-entry map of a chunk (64 consecutive segments of one block, each segment's
// 64 exit codes at sc[k]): the state at the chunk's end for each state at its start,
// four states per lane walked through the segments (a wave; k_long_spec, k_long_seg).
__device__ __forceinline__ void lp_compose(const uint8_t (*sc)[kSeg], uint8_t* __restrict__ m, uint32_t lane) {
    uint32_t x0 = lane, x1 = lane + 64u, x2 = lane + 128u, x3 = lane + 192u;
    for (uint32_t k = 0; k < kSeg; k++) {  // (four independent chains per lane)
        x0 = lp_next(sc[k], x0);
        x1 = lp_next(sc[k], x1);
        x2 = lp_next(sc[k], x2);
        x3 = lp_next(sc[k], x3);
    }
    m[lane] = (uint8_t)x0;
    m[lane + 64u] = (uint8_t)x1;
    m[lane + 128u] = (uint8_t)x2;
    m[lane + 192u] = (uint8_t)x3;
}

// The path chain's LDS (k_long_dp, round 5): window jw of kSpWin runes in buffer jw & 3,
// rune i at ring slot i & 1023.
struct LPath {
    double pw[4][kSpWin];     // the window's path runes right to left: w_D, then (fill) best
    double ck[4][kSpWin / 8u + 2u];  // the chain's sum before the window, then after every 8 path runes
    double dring[kLdDesc];    // best(i)
    double wd[kLdDesc];       // w_D(i): the decided item's weight (k_long_spec)
    uint8_t L[kLdDesc];       // D(i): the decided item's length
    uint64_t pbits[4][kSpWin / kSeg];  // the window's path runes, a bit each
    uint32_t pcnt[4];
};
struct LongLds {
    double ring[kLdRing];  // best(i) at i & 511
    union {
        LDesc desc[kLdDesc];   // rune i at i & 1023
        LDecided dc;           // (the decided chain)
        LPath lp;              // (the path chain)
    };
    uint8_t cls[kLdDesc];  // rune i's step form: 0 items L = 1..m (m <= 4), 1 other fast forms, 3 slow
    LItem side[4][kLdSide];
    uint32_t sidecnt[4], wslow[4], bad;
};

// DAG items (L, weight) of rune i of an all-3-byte block [bs, be), ascending L
// (buildDag's pieces and calcDagProba's pieceFreq, :462-497,511-519): from the
// rune's record, or by walking the trie when the record overflowed.
// (long_items_rc: the rune's record rc = erec[bs / 3 + i] already loaded)
template <class F>
__device__ __forceinline__ void long_items_rc(const uint8_t* __restrict__ text, const DevImage& im, uint64_t rc,
                                              uint32_t bs, uint32_t be, uint32_t i, F&& f) {
    const uint32_t q = bs + 3u * i;
    uint32_t mk = (uint32_t)rc & 0xFFu;
    if (mk) {  // the edges are in the last popc(mk) fields (the first ones are phantoms)
        for (int k = 4 - __popc(mk); k < 4; k++) {
            const uint32_t L = (uint32_t)__builtin_ctz(mk) + 1u;
            mk &= mk - 1u;
            f(L, im.wtab1[(uint32_t)(rc >> (8 + kEdgeIdxBits * k)) & ((1u << kEdgeIdxBits) - 1u)]);
        }
        return;
    }
    auto dec3 = [&](uint32_t p) {
        const uint32_t x = ld4(text, p);
        return ((x & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu);
    };
    uint32_t id = rune_code(im, dec3(q));
    uint64_t cc = im.cells[id];
    if (jb_cell_check(cc) != JB_CHECK_ROOT) {  // not a key: the rune alone, tf 1.0 (:468-471,515-518)
        f(1u, im.wtab[JB_WIDX_ABSENT]);
        return;
    }
    if (jb_cell_fc(cc) == JB_FC_ZERO) {  // count == 0: the rune alone, Log(0) (:468-471)
        f(1u, im.wtab[jb_cell_widx(cc)]);
        return;
    }
    if (jb_cell_fc(cc) == JB_FC_POS) f(1u, im.wtab[jb_cell_widx(cc)]);
    uint32_t qq = q + 3u, len = 1;
    bool go = jb_cell_hc(cc) != 0u;
    while (go && qq < be) {
        const uint32_t tt = dat_slot(im, cc, dec3(qq));
        const uint64_t ch = im.cells[tt];
        if (!dat_hit(ch, id)) break;  // (:475-478)
        ++len;
        qq += 3u;
        if (jb_cell_fc(ch) == JB_FC_POS) f(len, im.wtab[jb_cell_widx(ch)]);
        go = jb_cell_hc(ch) != 0u;
        id = tt;
        cc = ch;
    }
}

template <class F>
__device__ __forceinline__ void long_items(const uint8_t* __restrict__ text, const DevImage& im,
                                           const uint64_t* __restrict__ erec, uint32_t bs, uint32_t be, uint32_t i,
                                           F&& f) {
    long_items_rc(text, im, erec[bs / 3u + i], bs, be, i, f);
}

// max of two float64 sums that are never NaN: one v_max_f64 (fmax would add a
// canonicalizing v_max_f64 of an operand the compiler cannot prove canonical)
__device__ __forceinline__ double max_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// maxIndexProba's rule on one item (:565-578), for a DpFold
__device__ __forceinline__ void fold_item(DpFold& f, uint32_t L, double pp) {
    if (pp >= f.prevP) {
        f.bestL = L;
        f.bestP = pp;
    }
    f.prevP = pp;
    f.lastL = L;
}

// the long block that segment g belongs to (lsegb: first segment of each block, ascending)
__device__ __forceinline__ uint32_t long_block_of(const uint32_t* __restrict__ lsegb, uint32_t nlong, uint32_t g) {
    uint32_t lo = 0, hi = nlong;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (lsegb[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

// k_long_spec: the speculative choices of the long blocks' runes, in parallel.
// One lane per 64-rune segment (grid-stride; the lane's DP ring in LDS): the DP
// of calcDagProba + maxIndexProba (:502-578) from kSpecOver runes past the
// segment, where best is taken as 0.0 (a guess; at the block's end it is the
// true best(n) = 0.0), down to the segment's first rune.  Past a few hundred
// runes the choices no longer depend on the guess (config 5b: none differ at
// 1024, 1.1 % at 64: tools/spec_sim.cpp).  For each rune of the segment it
// writes the chosen length to gbl and the chosen item's weight to gbest, which
// k_long_dp's decided chain turns into the exact best values and verifies.
constexpr uint32_t kSpecOver = 1024;
constexpr uint32_t kSpecRing = 128;  // best values kept per lane (an item longer takes the guess)
constexpr uint32_t kSpecGrid = 256;  // 64-lane workgroups, one per CU (140 KB of LDS each)
// the weight table in LDS when it fits (kZhWtab entries, as k_zh's wide form: else nullptr,
// and k_long_spec gathers the weights), and the records' length table (one wave)
__device__ __forceinline__ double* long_spec_setup(const DevImage& im, double* s_wtl) {
    const uint32_t lane = threadIdx.x & 63u;
    double* const s_wt = im.nw1 <= kZhWtab ? s_wtl : nullptr;
    if (s_wt)
        for (uint32_t k = lane; k < im.nw1; k += 64u) s_wt[k] = im.wtab1[k];
    for (uint32_t k = lane; k < 256u; k += 64u) s_ltab[k] = ltab_entry(k);
    wave_sync();
    return s_wt;
}
__device__ __forceinline__ void long_spec_body(const uint8_t* __restrict__ text, DevImage im,
                                                  const uint64_t* __restrict__ erec, const uint2* __restrict__ longblk,
                                                  const uint32_t* __restrict__ lsegb, const uint32_t* __restrict__ counters,
                                                  const uint32_t* __restrict__ tile4, uint8_t* __restrict__ gbl,
                                                  double* __restrict__ gbest, uint8_t* __restrict__ lcode,
                                                  uint8_t* __restrict__ lmap, uint32_t* __restrict__ lflag, uint32_t mode,
        uint32_t wg, uint32_t ng, double (*s_ring)[64], uint8_t (*s_cd)[kSeg], double* s_wt, double (*s_bw)[kSeg]) {
    const uint32_t nlong = counters[CNT_NLONG], nseg = counters[CNT_NLSEG], lane = threadIdx.x & 63u;
    if (!im.plainw) return;  // (k_long_dp runs the exact chain)
    for (uint32_t g0 = wg * 64u; g0 < nseg; g0 += ng * 64u) {  // (wave-uniform)
        const uint32_t g = g0 + lane;
        const bool act = g < nseg;
        const uint32_t bi = act ? long_block_of(lsegb, nlong, g) : 0xFFFFFFFFu;
        // A block with a 4-byte Han rune takes k_long_dp's general path, which ignores these
        // choices; its runes are not all 3 bytes, so slots bs / 3 + i are not all rune starts
        // written in this batch (a record there may be stale), and it is skipped.  The
        // wave checks the tile4 flags of its segments' blocks, one block at a time.
        bool skip = !act;
        for (uint64_t pend = __ballot(act); pend;) {
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bi, (int)__builtin_ctzll(pend));
            const uint2 bb0 = longblk[b0];
            bool f = false;
            for (uint32_t t = bb0.x / kTileBytes + lane; t <= (bb0.y - 1u) / kTileBytes; t += 64u) f |= tile4[t] != 0u;
            const bool has4 = __ballot(f) != 0ull;
            if (bi == b0) skip = has4;
            pend &= ~__ballot(bi == b0);
        }
        // the block's flag: 3 for k_long_dp's path chain (k_long_path and k_long_pbits find
        // the path of these choices first); 0 for the others (k_long_dp writes every flag)
        if (act && g == lsegb[bi]) lflag[bi] = skip || mode == 3u ? 0u : 3u;
        uint32_t n = 0, a = 0;
        if (!skip) {
        const uint2 bb = longblk[bi];
        const uint32_t bs = bb.x, be = bb.y, s0 = bs / 3u;
        n = (be - bs) / 3u;
        a = (g - lsegb[bi]) * kSeg;
        const uint32_t lim = min(a + kSeg, n), top = min(lim + kSpecOver, n);
        // By groups of four runes g .. g + 3, from the top down.  The records are loaded
        // three groups ahead (the DP waits only on LDS).  With the weight table in LDS (WL:
        // at most kZhWtab weights) a group's 16 weights are LDS reads at its start; else
        // they are gathered a group ahead.  An item of kSpecRing runes or more takes the
        // guess 0.0 for best(i + L), as past the top (only the speculation's quality depends
        // on it: k_long_dp verifies every choice).
        // (unconditional loads, the index clamped into the block: a rune past the top or a
        // group below the segment is never used, and a conditional load made every later
        // write of its register wait for all loads in flight)
        auto ld_rc = [&](int32_t g, uint64_t (&rc)[4]) __attribute__((always_inline)) {
#pragma unroll
            for (int32_t r = 0; r < 4; r++) {
                const int32_t i = min(max(g + r, 0), (int32_t)n - 1);
                rc[r] = erec[s0 + (uint32_t)i];
            }
        };
        auto fidx = [](uint64_t rc, uint32_t k) {
            return (uint32_t)(rc >> (8 + kEdgeIdxBits * k)) & ((1u << kEdgeIdxBits) - 1u);
        };
        auto ld_w = [&](const uint64_t (&rc)[4], double (&w)[4][4], const double* __restrict__ wt)
                        __attribute__((always_inline)) {
#pragma unroll
            for (uint32_t r = 0; r < 4u; r++)
#pragma unroll
                for (uint32_t k = 0; k < 4u; k++) w[r][k] = wt[fidx(rc[r], k)];
        };
        const int32_t gtop = (int32_t)(a + ((top - a + 3u) & ~3u)) - 4;
        double bnx = 0.0;  // speculative best(i + 1)
        // the DP of group g's runes, right to left, its weights in wc
        auto group = [&](int32_t g, const uint64_t (&rcg)[4], const double (&wc)[4][4]) __attribute__((always_inline)) {
#pragma unroll
            for (int32_t r = 3; r >= 0; r--) {
                const uint32_t i = (uint32_t)(g + r);
                if (i >= top) continue;  // (the first group's runes past the top)
                double prevP = JB_MIN_FLOAT, bestP = JB_MIN_FLOAT, bestW = 0.0, lastW = 0.0;
                uint32_t bestL = 0, lastL = 0;
                const uint32_t mk = (uint32_t)rcg[r] & 0xFFu;
                if (mk) {
                    // the record's four fields, phantoms (weight -Inf, L = 1) first, by k_zh's
                    // fold (rec_fold_a3's reading of maxIndexProba: the first field taken
                    // outright, each later one if its proba is >= the one before; the same item
                    // under plainw).  best(i + L) for i + L >= top is 0.0 from the ring (set
                    // below the top before the loop), best(i + 1) from a register.
                    const uint64_t lt = s_ltab[mk];
                    double prv = 0.0;
#pragma unroll
                    for (uint32_t k = 0; k < 4u; k++) {
                        const uint32_t L = (uint32_t)(lt >> (16u * k + 9u)) & 0x7Fu;
                        const double rv = s_ring[(i + L) & (kSpecRing - 1u)][lane];
                        const double wt = wc[r][k];
                        const double pp = wt + (L == 1u ? bnx : rv);
                        const bool take = k == 0u || pp >= prv;
                        bestL = take ? L : bestL;
                        bestP = take ? pp : bestP;
                        bestW = take ? wt : bestW;
                        prv = pp;
                    }
                } else {  // an overflowed record: walk the trie
                    long_items_rc(text, im, 0ull, bs, be, i, [&](uint32_t L, double wt) {
                        const uint32_t j = i + L;
                        const double b = j >= top || L >= kSpecRing
                                             ? 0.0
                                             : (L == 1u ? bnx : s_ring[j & (kSpecRing - 1u)][lane]);
                        const double pp = wt + b;
                        if (pp >= prevP) {
                            bestL = L;
                            bestP = pp;
                            bestW = wt;
                        }
                        prevP = pp;
                        lastL = L;
                        lastW = wt;
                    });
                }
                if (bestL == 0) {  // (walk) no item qualified: the last item (or none)
                    bestL = lastL;
                    bestP = prevP;
                    bestW = lastW;
                }
                s_ring[i & (kSpecRing - 1u)][lane] = bestP;
                bnx = bestP;
                // the choice and its weight into the lane's 64 slots in LDS, unconditionally: a rune
                // past the segment is overwritten by the segment's own rune there later (no global
                // store in the loop: its wait counts made every trip wait for the record loads)
                // (mode 2, testing only: some choices made wrong on purpose, so that
                // k_long_dp's verification and exact chain run)
                s_cd[lane][(i - a) & (kSeg - 1u)] = (uint8_t)(mode == 2u && i % 97u == 0u && bestL > 1u ? 1u : bestL);
                s_bw[lane][(i - a) & (kSeg - 1u)] = bestW;
            }
        };
        // best = 0.0 (the guess) for the 8 runes from the top up (a record's items are at most
        // 8 runes long; the walk path tests i + L >= top itself)
#pragma unroll
        for (uint32_t t = 0; t < 8u; t++) s_ring[(top + t) & (kSpecRing - 1u)][lane] = 0.0;
        if (s_wt) {
            // four record sets in rotation, four groups per loop trip: a set is reloaded for
            // the group four ahead right after its own group (copying the sets instead made
            // every trip wait for the loads it had just issued)
            uint64_t r0[4], r1[4], r2[4], r3[4];
            ld_rc(gtop, r0);
            ld_rc(gtop - 4, r1);
            ld_rc(gtop - 8, r2);
            ld_rc(gtop - 12, r3);
            auto step = [&](int32_t g, uint64_t (&rc)[4]) __attribute__((always_inline)) {
                double wc[4][4];
                ld_w(rc, wc, s_wt);
                group(g, rc, wc);
                ld_rc(g - 16, rc);
            };
            for (int32_t g = gtop; g >= (int32_t)a; g -= 16) {
                step(g, r0);
                if (g - 4 < (int32_t)a) break;
                step(g - 4, r1);
                if (g - 8 < (int32_t)a) break;
                step(g - 8, r2);
                if (g - 12 < (int32_t)a) break;
                step(g - 12, r3);
            }
        } else {
            uint64_t rcc[4], rcn[4];
            double wc[4][4];
            ld_rc(gtop, rcc);
            ld_w(rcc, wc, im.wtab1);
            ld_rc(gtop - 4, rcn);
            for (int32_t g = gtop; g >= (int32_t)a; g -= 4) {
                uint64_t rcnn[4];
                ld_rc(g - 8, rcnn);
                double wn[4][4];
                ld_w(rcn, wn, im.wtab1);
                group(g, rcc, wc);
#pragma unroll
                for (uint32_t r = 0; r < 4u; r++) {
                    rcc[r] = rcn[r];
                    rcn[r] = rcnn[r];
#pragma unroll
                    for (uint32_t k = 0; k < 4u; k++) wc[r][k] = wn[r][k];
                }
            }
        }
        // the segment's exit codes under these choices (k_long_seg's rule; the path chain
        // finds the path of the decisions from them)
        for (uint32_t p = lim; p-- > a;) {
            const uint32_t d = s_cd[lane][p - a];
            gbl[s0 + p] = (uint8_t)d;
            gbest[s0 + p] = s_bw[lane][p - a];
            const uint32_t L = max(1u, d), q = p + L;
            const uint8_t c = q >= lim ? (L == 1u ? (uint8_t)0xFFu : (uint8_t)(q - lim)) : s_cd[lane][q - a];
            s_cd[lane][p - a] = c;
            lcode[s0 + p] = c;
        }
        }
        // the chunk map of the wave's 64 segments (one block's, with more of it after them)
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bi);
        if (__ballot(!skip && bi == b0 && a + kSeg < n) == ~0ull) {
            wave_sync();
            lp_compose(s_cd, lmap + (uint64_t)(g0 / kSeg) * kLpMap, lane);
        }
        wave_sync();  // (the next iteration overwrites s_cd)
    }
}

__global__ __launch_bounds__(64) void k_long_spec(const uint8_t* __restrict__ text, DevImage im,
                                                  const uint64_t* __restrict__ erec, const uint2* __restrict__ longblk,
                                                  const uint32_t* __restrict__ lsegb, const uint32_t* __restrict__ counters,
                                                  const uint32_t* __restrict__ tile4, uint8_t* __restrict__ gbl,
                                                  double* __restrict__ gbest, uint8_t* __restrict__ lcode,
                                                  uint8_t* __restrict__ lmap, uint32_t* __restrict__ lflag, uint32_t mode) {
    __shared__ double s_ring[kSpecRing][64];
    __shared__ uint8_t s_cd[64][kSeg];  // the lane's segment: its decisions, then its exit codes
    __shared__ double s_wt[kZhWtab];
    __shared__ double s_bw[64][kSeg];  // the lane's segment's chosen weights
    double* const wt = long_spec_setup(im, s_wt);
    long_spec_body(text, im, erec, longblk, lsegb, counters, tile4, gbl, gbest, lcode, lmap, lflag, mode, blockIdx.x,
                   gridDim.x, s_ring, s_cd, wt, s_bw);
}

template <bool HMM>
__device__ __forceinline__ void long_dp_body(const uint8_t* __restrict__ text, DevImage im,
                                                 const uint64_t* __restrict__ erec, uint8_t* __restrict__ gbl,
                                                 double* __restrict__ gbest, const uint2* __restrict__ longblk,
                                                 uint32_t* __restrict__ counters, uint32_t* __restrict__ sbits,
                                                 uint32_t* __restrict__ ebits, uint32_t* __restrict__ lflag,
                                                 const uint32_t* __restrict__ lsegb, const uint64_t* __restrict__ lpath,
                                                 uint64_t* __restrict__ dbg, uint32_t spec,
        uint32_t wg, uint32_t ng, LongLds& S) {
#if JB_STAMPS
    uint64_t st_run = 0, st_bar = 0, st_n = 0, st_slow = 0;  // diagnostic clocks (lane 0 of each wave)
    uint64_t st_p[4] = {0, 0, 0, 0};  // sub-phase clocks (the path chain's fill and verify)
#endif
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint32_t nlong = counters[CNT_NLONG];
    const char* const rb = reinterpret_cast<const char*>(S.ring);
    s_ltab[tid] = ltab_entry(tid);  // (zh_dp's record lengths; 256 threads, read after the barriers below)
    for (uint32_t bi = wg; bi < nlong; bi += ng) {
        const uint2 bb = longblk[bi];
        const uint32_t bs = bb.x, be = bb.y;
        bool any4 = false;  // a 4-byte Han rune (lead >= 0xF0) anywhere in the block
        for (uint32_t a = (bs & ~15u) + 16u * tid; a < be; a += 4096u) {
            const uint4 x = *reinterpret_cast<const uint4*>(text + a);
            any4 |= ((x.x & (x.x << 1) & (x.x << 2) & (x.x << 3)) | (x.y & (x.y << 1) & (x.y << 2) & (x.y << 3)) |
                     (x.z & (x.z << 1) & (x.z << 2) & (x.z << 3)) | (x.w & (x.w << 1) & (x.w << 2) & (x.w << 3))) &
                    0x80808080u;
        }
        if (__syncthreads_or(any4)) {  // the general one-lane path (k_zh's); the later kernels skip the block
            if (tid == 0) {
                lflag[bi] = 0u;
                Emitter em(sbits, ebits);
                const GlbZv gv{text, gbl};
                zh_dp(gv, im, erec, gbest, S.ring, OneSrc{bs, be});
                if (!zh_fwd<HMM>(gv, im, bs, be, em, nullptr)) atomicOr(counters + CNT_ERR, 1u);
                em.flush();
                if (em.ties) atomicAdd(counters + CNT_TIES, em.ties);
            }
            __syncthreads();
            continue;
        }
        const uint32_t n = (be - bs) / 3u, s0 = bs / 3u;  // rune i: bytes bs + 3i, slot s0 + i
        const int32_t J = (int32_t)((n + kLdWin - 1u) / kLdWin);  // windows; runes [n, 256 J) are dummies
        const uint32_t lf = lflag[bi];  // (k_long_spec's; every thread reads it before thread 0 rewrites it)
        if (lf == 3u) {
            // ---- the path chain (round 5): only the runes on findDagPath's path through
            // k_long_spec's choices (k_long_pbits' lpath bits) are a serial chain, best(p) =
            // w_D(p) + best(next path rune), one f64 add each on lane 0 (wave 0); from their
            // values every other rune's, best(i) = w_D(i) + best(i + L_D(i)), in parallel (wave
            // 2: the decided paths off the path soon join it); then every rune's choice is
            // verified by maxIndexProba over these values (wave 3), as for the decided chain:
            // the same adds of the same values, so if all choices pass, all values are exact.
            // Window jw of kSpWin runes: stage (wave 1) at step jw + 1, chain at jw, fill at
            // jw - 1, verify at jw - 2; buffers jw & 3 (4 windows in flight), a barrier per step. ----
            const int32_t Jd = (int32_t)((n + kSpWin - 1u) / kSpWin);
            const uint32_t sb = lsegb[bi];
            if (tid == 0u) {
                S.bad = 0u;
                S.lp.dring[n & (kLdDesc - 1u)] = 0.0;  // best(n), when rune n is past the last window
            }
            // window jw's choices (wave 1): w_D and L_D of every rune at its ring slot, and the
            // path runes' w_D right to left in pw.  Its loads
            // are issued a step before (stage_load; a barrier does not wait for them).
            struct StageIn {
                uint64_t pm[4];  // the four segments' path bits
                double w[4];     // w_D of rune base + 64 q + lane
                uint32_t L[4];   // L_D
            };
            auto stage_load = [&](int32_t jw, StageIn& X) {
                const uint32_t base = (uint32_t)jw * kSpWin;
#pragma unroll
                for (uint32_t q = 0; q < 4u; q++) {
                    const uint32_t i = base + kSeg * q + lane;
                    X.pm[q] = base + kSeg * q < n ? lpath[sb + (uint32_t)jw * 4u + q] : 0ull;
                    X.w[q] = i < n ? gbest[s0 + i] : 0.0;
                    X.L[q] = i < n ? (uint32_t)gbl[s0 + i] : 1u;
                }
            };
            auto stage = [&](int32_t jw, const StageIn& X) {
                const uint32_t b = (uint32_t)jw & 3u, kb = b * kSpWin;
                const uint32_t c3 = (uint32_t)__popcll(X.pm[3]), c2 = (uint32_t)__popcll(X.pm[2]);
                const uint32_t c1 = (uint32_t)__popcll(X.pm[1]), c0 = (uint32_t)__popcll(X.pm[0]);
                const uint32_t above[4] = {c3 + c2 + c1, c3 + c2, c3, 0u};  // path runes in the words above
                const uint32_t cnt = c3 + c2 + c1 + c0;
                bool none = false;
#pragma unroll
                for (uint32_t q = 0; q < 4u; q++) {
                    const uint32_t r = kSeg * q + lane;
                    none |= X.L[q] == 0u;  // no item (the reference panics later): the exact chain
                    S.lp.wd[kb + r] = X.w[q];
                    S.lp.L[kb + r] = (uint8_t)max(1u, X.L[q]);
                    const uint64_t hi = X.pm[q] >> lane;
                    if (hi & 1ull) S.lp.pw[b][above[q] + (uint32_t)__popcll(hi >> 1)] = X.w[q];
                }
                if (none) S.bad = 1u;
                // (the chain runs to a multiple of 16: x + -0.0 is x, bit for bit)
                if (cnt + lane < ((cnt + 15u) & ~15u)) S.lp.pw[b][cnt + lane] = -0.0;
                if (lane == 0u) {
                    S.lp.pcnt[b] = cnt;
#pragma unroll
                    for (uint32_t q = 0; q < 4u; q++) S.lp.pbits[b][q] = X.pm[q];
                }
            };
            // the chain over window j's path runes (wave 0, lane 0): 16 at a time from
            // registers, the next 16 loaded meanwhile.  It stores only its sum before the window
            // and after every 8 runes (ck): one wave's LDS stores cost it more than its adds
            // (a 16-byte store per two sums: 24 cycles per sum against 12.6 with these
            // checkpoints, tools/diag/pchain.hip); fill redoes the same adds from them.
            double acc = 0.0;  // best of the path rune after the window (best(n) = 0.0 first)
            auto chain = [&](int32_t j) {
                const uint32_t b = (uint32_t)j & 3u;
                const uint32_t c16 = (uint32_t)__builtin_amdgcn_readfirstlane((int)((S.lp.pcnt[b] + 15u) & ~15u));
                double* const pw = S.lp.pw[b];
                struct V16 {
                    double v[16];
                };
                V16 A, B;
                auto ld = [&](V16& X, uint32_t k) __attribute__((always_inline)) {
#pragma unroll
                    for (int t = 0; t < 8; t++) {
                        const double2 v = *reinterpret_cast<const double2*>(pw + k + 2u * t);
                        X.v[2 * t] = v.x;
                        X.v[2 * t + 1] = v.y;
                    }
                };
                double* const ck = S.lp.ck[b];
                auto run = [&](const V16& X, uint32_t k) __attribute__((always_inline)) {
#pragma unroll
                    for (int t = 0; t < 8; t++) acc = X.v[t] + acc;
                    const double a8 = acc;
#pragma unroll
                    for (int t = 8; t < 16; t++) acc = X.v[t] + acc;
                    __builtin_amdgcn_sched_barrier(0);
                    ck[k / 8u + 1u] = a8;
                    ck[k / 8u + 2u] = acc;
                };
#if JB_STAMPS
                st_slow += c16;
#endif
                ck[0] = acc;
                ld(A, 0u);  // (loads past c16 stay inside S and are not used)
                for (uint32_t k = 0; k < c16; k += 32u) {
                    ld(B, k + 16u);
                    __builtin_amdgcn_sched_barrier(0);
                    run(A, k);
                    // B used here, before the branch: otherwise the compiler sinks its loads past
                    // the branch to their use, and the half waits a whole LDS round trip (the
                    // loads are done by now: this costs nothing)
                    asm volatile("" ::"v"(B.v[0]), "v"(B.v[2]), "v"(B.v[4]), "v"(B.v[6]), "v"(B.v[8]), "v"(B.v[10]),
                                 "v"(B.v[12]), "v"(B.v[14]));
                    if (k + 16u >= c16) break;
                    ld(A, k + 32u);
                    run(B, k + 16u);
                }
            };
            // window jw's best values into the ring (wave 2): the path runes', then each other
            // rune's once its successor's is known, by rounds.  An unknown value is a NaN in the
            // ring (under plainw no best value is NaN: weights are finite or -Inf, and nothing
            // adds +Inf); a rune's w_D and successor slot stay in registers, and every round
            // reads all four successors' values at once.
            auto fill = [&](int32_t jw) {
                const uint32_t b = (uint32_t)jw & 3u, base = (uint32_t)jw * kSpWin, kb = b * kSpWin;
#if JB_STAMPS
                const uint64_t f0 = __builtin_amdgcn_s_memtime();
#endif
                // (the lane's inputs first: their reads do not wait for the stores below)
                const uint32_t r0 = 4u * lane;
                uint64_t pm[4];
#pragma unroll
                for (uint32_t q = 0; q < 4u; q++) pm[q] = S.lp.pbits[b][q];
                const uint32_t wsel = lane >> 4;  // the word of the lane's four bits
                const uint64_t pmw = wsel == 0u ? pm[0] : wsel == 1u ? pm[1] : wsel == 2u ? pm[2] : pm[3];
                const uint32_t c3 = (uint32_t)__popcll(pm[3]), c2 = (uint32_t)__popcll(pm[2]);
                const uint32_t c1 = (uint32_t)__popcll(pm[1]);
                const uint32_t abv = wsel == 0u ? c3 + c2 + c1 : wsel == 1u ? c3 + c2 : wsel == 2u ? c3 : 0u;
                const uint32_t L4 = *reinterpret_cast<const uint32_t*>(S.lp.L + kb + r0);
                const double2 w01 = *reinterpret_cast<const double2*>(S.lp.wd + kb + r0);
                const double2 w23 = *reinterpret_cast<const double2*>(S.lp.wd + kb + r0 + 2u);
                {  // the path runes' values: the chain's adds again, 8 per lane from its checkpoints
                    const uint32_t c16 = (S.lp.pcnt[b] + 15u) & ~15u;
                    if (lane < c16 / 8u) {
                        double a = S.lp.ck[b][lane];
                        double* const pw = S.lp.pw[b] + 8u * lane;
                        double x[8];
#pragma unroll
                        for (int t = 0; t < 4; t++) {
                            const double2 v = reinterpret_cast<const double2*>(pw)[t];
                            x[2 * t] = v.x;
                            x[2 * t + 1] = v.y;
                        }
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            a = x[t] + a;
                            x[t] = a;
                        }
#pragma unroll
                        for (int t = 0; t < 4; t++) reinterpret_cast<double2*>(pw)[t] = make_double2(x[2 * t], x[2 * t + 1]);
                    }
                }
#if JB_STAMPS
                const uint64_t f1 = __builtin_amdgcn_s_memtime();
#endif
                // each lane four consecutive runes r0 .. r0 + 3: a successor inside the lane is
                // taken from the register of its value in the same round (the four right to left),
                // so a run of off-path runes resolves a lane at a time
                const double wq[4] = {w01.x, w01.y, w23.x, w23.y};
                uint32_t tq[4];
                double vq[4];
                // a path rune's value from pw (its rank from the right), a rune past the block
                // 0.0 (so best(n) = 0.0), any other NaN
#pragma unroll
                for (uint32_t q = 0; q < 4u; q++) {
                    const uint64_t hi = (pmw >> ((r0 + q) & 63u));
                    const double pv = S.lp.pw[b][(abv + (uint32_t)__popcll(hi >> 1)) & (kSpWin - 1u)];
                    vq[q] = (hi & 1ull) ? pv : base + r0 + q >= n ? 0.0 : __builtin_nan("");
                    tq[q] = r0 + q + ((L4 >> (8u * q)) & 0xFFu);  // the successor's window offset
                }
                double2* const dw = reinterpret_cast<double2*>(S.lp.dring + kb + r0);
                dw[0] = make_double2(vq[0], vq[1]);
                dw[1] = make_double2(vq[2], vq[3]);
#if JB_STAMPS
                const uint64_t f2 = __builtin_amdgcn_s_memtime();
#endif
                // a round: every rune still NaN takes w_D + its successor's value (NaN while
                // that is unknown); the ring reads, the lane's runes right to left, two stores
                uint32_t rounds = 0;
                while (__ballot(vq[0] != vq[0] || vq[1] != vq[1] || vq[2] != vq[2] || vq[3] != vq[3]) != 0ull) {
                    double v[4];
#pragma unroll
                    for (uint32_t q = 0; q < 4u; q++) v[q] = S.lp.dring[(kb + tq[q]) & (kLdDesc - 1u)];
#pragma unroll
                    for (int q = 3; q >= 0; q--) {
                        double sv = v[q];
                        if (q <= 2) sv = tq[q] == r0 + 3u ? vq[3] : sv;
                        if (q <= 1) sv = tq[q] == r0 + 2u ? vq[2] : sv;
                        if (q == 0) sv = tq[q] == r0 + 1u ? vq[1] : sv;
                        vq[q] = vq[q] != vq[q] ? wq[q] + sv : vq[q];
                    }
                    dw[0] = make_double2(vq[0], vq[1]);
                    dw[1] = make_double2(vq[2], vq[3]);
                    rounds++;
                }
#if JB_STAMPS
                st_slow += rounds;
                const uint64_t f3 = __builtin_amdgcn_s_memtime();
                st_p[0] += f1 - f0;  // the path runes' values
                st_p[1] += f2 - f1;  // setup
                st_p[2] += f3 - f2;  // rounds
#else
                (void)rounds;
#endif
            };
            // every rune's choice by maxIndexProba over the values (wave 3).  A record's items
            // are the last popc(mk) of its four fields, lengths the bits of mk ascending; an
            // overflowed record (mk 0) walks the trie (long_items_rc).  The loads run two steps
            // ahead: at step j the records of window j, the weights of window j + 1 (all 16
            // fields of each lane's four runes at once), the fold of window j + 2.
            // Runes 64 q + lane for q in [Q0, Q1): wave 3 takes q = 0..2, wave 1 (after its
            // stage) q = 3, each with its own loads in flight (VState).
            struct VState {
                uint64_t vrc[4];    // records of window j + 1 (loaded the step before)
                double vwv[4][4];   // weights of window j + 2
                uint32_t vmk = 0;   // its item masks, a byte per rune
            };
            auto verify = [&](int32_t j, auto Q0c, auto Q1c, VState& vs) {
                constexpr uint32_t Q0 = decltype(Q0c)::value, Q1 = decltype(Q1c)::value;
                uint64_t(&vrc)[4] = vs.vrc;
                double(&vwv)[4][4] = vs.vwv;
                uint32_t& vmk = vs.vmk;
#if JB_STAMPS
                const uint64_t v0 = __builtin_amdgcn_s_memtime();
#endif
                uint64_t rn[4];
                if (j >= 0) {
#pragma unroll
                    for (uint32_t q = Q0; q < Q1; q++) {
                        const uint32_t i = (uint32_t)j * kSpWin + kSeg * q + lane;
                        rn[q] = i < n ? erec[s0 + i] : 0x1ull;  // (past the block: one phantom item)
                    }
                }
                double wn[4][4];
                uint32_t mkn = 0;
                if (j + 1 >= 0 && j + 1 < Jd) {
#pragma unroll
                    for (uint32_t q = Q0; q < Q1; q++) {
                        mkn |= ((uint32_t)vrc[q] & 0xFFu) << (8u * q);
#pragma unroll
                        for (uint32_t k = 0; k < 4u; k++)
                            wn[q][k] = im.wtab1[(uint32_t)(vrc[q] >> (8 + kEdgeIdxBits * k)) & ((1u << kEdgeIdxBits) - 1u)];
                    }
                }
#if JB_STAMPS
                const uint64_t v1 = __builtin_amdgcn_s_memtime();
                uint64_t v2 = v1, v3 = v1;
#endif
                if (j + 2 < Jd) {
                    // the items' sums: all 16 ring reads at once (an absent field reads best(i + 1),
                    // unused; the ring holds best(n) = 0.0, so no case for i + L = n), then
                    // maxIndexProba (:565-578) by selects over the present items, ascending L
                    const int32_t jv = j + 2;
                    const uint32_t kb = ((uint32_t)jv & 3u) * kSpWin, base = (uint32_t)jv * kSpWin;
                    uint32_t Lk[4][4];
                    double rv[4][4];
#pragma unroll
                    for (uint32_t q = Q0; q < Q1; q++) {
                        const uint32_t i = base + kSeg * q + lane;
                        uint32_t mk = (vmk >> (8u * q)) & 0xFFu;
                        const uint32_t k0 = 4u - (uint32_t)__popc(mk);
#pragma unroll
                        for (uint32_t k = 0; k < 4u; k++) {
                            const bool pres = k >= k0;
                            Lk[q][k] = pres ? (uint32_t)__builtin_ctz(mk) + 1u : 0u;
                            mk = pres ? mk & (mk - 1u) : mk;
                            rv[q][k] = S.lp.dring[(i + max(1u, Lk[q][k])) & (kLdDesc - 1u)];
                        }
                    }
#if JB_STAMPS
                    v2 = __builtin_amdgcn_s_memtime();
#endif
                    bool bad = false;
#pragma unroll
                    for (uint32_t q = Q0; q < Q1; q++) {
                        const uint32_t i = base + kSeg * q + lane;
                        double prevP = JB_MIN_FLOAT;
                        uint32_t bestL = 0, lastL = 0;
#pragma unroll
                        for (uint32_t k = 0; k < 4u; k++) {
                            const uint32_t L = Lk[q][k];
                            const double pp = vwv[q][k] + rv[q][k];
                            bestL = L != 0u && pp >= prevP ? L : bestL;
                            prevP = L != 0u ? pp : prevP;
                            lastL = L != 0u ? L : lastL;
                        }
                        bestL = bestL ? bestL : lastL;
#if JB_STAMPS
                        st_slow += (uint64_t)__popcll(__ballot(((vmk >> (8u * q)) & 0xFFu) == 0u && i < n));
#endif
                        if (((vmk >> (8u * q)) & 0xFFu) == 0u && i < n) {  // an overflowed record: walk
                            DpFold f;
                            long_items_rc(text, im, 0ull, bs, be, i, [&](uint32_t L, double wt) {
                                fold_item(f, L, wt + (i + L == n ? 0.0 : S.lp.dring[(i + L) & (kLdDesc - 1u)]));
                            });
                            f.finish();
                            bestL = f.bestL;
                        }
                        bad |= i < n && bestL != S.lp.L[kb + kSeg * q + lane];
                    }
                    if (bad) S.bad = 1u;
#if JB_STAMPS
                    v3 = __builtin_amdgcn_s_memtime();
#endif
                }
#if JB_STAMPS
                st_p[0] += v1 - v0;  // loads issued
                st_p[1] += v2 - v1;  // ring reads
                st_p[2] += v3 - v2;  // fold
#endif
#pragma unroll
                for (uint32_t q = Q0; q < Q1; q++) {
                    vrc[q] = rn[q];
#pragma unroll
                    for (uint32_t k = 0; k < 4u; k++) vwv[q][k] = wn[q][k];
                }
                vmk = mkn;
            };
            // steps j = Jd - 1 .. -2, a barrier each (verify's first fold, of window Jd - 1, at
            // step Jd - 3); each wave its own loop (one loop with a branch per wave merged the
            // waves' registers at its join, and waited there for verify's loads in flight)
#if JB_STAMPS
#define JB_LP_STEP(body)                                          \
    for (int32_t j = Jd - 1; j >= -2; --j) {                      \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();         \
        body;                                                     \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();         \
        __syncthreads();                                          \
        st_run += t1 - t0;                                        \
        st_bar += __builtin_amdgcn_s_memtime() - t1;              \
        st_n++;                                                   \
    }
#else
#define JB_LP_STEP(body)                     \
    for (int32_t j = Jd - 1; j >= -2; --j) { \
        body;                                \
        __syncthreads();                     \
    }
#endif
            if (wave == 0u) {
                __syncthreads();
                JB_LP_STEP(if (j >= 0 && lane == 0u) chain(j));
            } else if (wave == 1u) {
                StageIn sx;
                stage_load(Jd - 1, sx);
                stage(Jd - 1, sx);
                if (Jd >= 2) stage_load(Jd - 2, sx);
                __syncthreads();
                VState vs;
                JB_LP_STEP(if (j >= 1) {
                    stage(j - 1, sx);
                    if (j >= 2) stage_load(j - 2, sx);
                } verify(j, std::integral_constant<uint32_t, 3>{}, std::integral_constant<uint32_t, 4>{}, vs));
            } else if (wave == 2u) {
                __syncthreads();
                JB_LP_STEP(if (j >= -1 && j + 1 < Jd) fill(j + 1));
            } else {
                VState vs;
                __syncthreads();
                JB_LP_STEP(verify(j, std::integral_constant<uint32_t, 0>{}, std::integral_constant<uint32_t, 3>{}, vs));
            }
#undef JB_LP_STEP
            const bool bad = S.bad != 0u;
#if JB_STAMPS
            st_slow += bad ? 1000000u : 0u;  // (a block sent to the exact chain)
#endif
            if (!bad) {
                if (tid == 0u) lflag[bi] = 1u;  // the path is the decided one: k_long_seg, k_long_path skip it
                __syncthreads();
                continue;
            }
            __syncthreads();  // (every thread has read S.bad: the exact chain below reuses the LDS)
        } else if (spec == 3u && im.plainw) {
            // ---- the decided chain (round 4, JB_LONG_SPEC=3): best(s) = w_D(s) + best(s + L_D(s)) from k_long_spec's
            // choices (the reference's pieceProba add for the chosen item, :519-529), one add
            // per rune on lane 0; the helper waves stage the choices two windows ahead and
            // verify each finished window: every rune's choice by maxIndexProba over the
            // exact values.  The rightmost wrong choice would be the first one found, and
            // every value right of it is exact; any wrong choice sends the block to the exact
            // chain below, which recomputes all of it. ----
            const int32_t Jd = (int32_t)((n + kSpWin - 1u) / kSpWin);  // windows; runes [n, 192 Jd) are dummies
            if (tid == 0u) S.bad = 0u;
            __syncthreads();
            auto stage = [&](int32_t jw, uint32_t t, uint32_t nt) {
                for (uint32_t r = t; r < kSpWin; r += nt) {
                    const int32_t i = jw * (int32_t)kSpWin + (int32_t)r;
                    const uint32_t k = (uint32_t)i & (kLdDesc - 1u);
                    const bool real = i >= 0 && (uint32_t)i < n;  // (past the block: best = 0.0 + best(i + 1) = 0.0)
                    uint32_t L = real ? (uint32_t)gbl[s0 + (uint32_t)i] : 1u;
                    if (L == 0u) {  // no item (the reference panics later): the exact chain
                        S.bad = 1u;
                        L = 1u;
                    }
                    S.dc.spec[16u + k].w = real ? gbest[s0 + (uint32_t)i] : 0.0;
                    S.dc.spec[16u + k].ra = (((uint32_t)i + L) & (kLdDesc - 1u)) * 8u;
                    S.dc.spec[16u + k].m1 = L == 1u ? ~0u : 0u;
                    S.dc.m2[16u + k] = L == 2u ? ~0u : 0u;
                    S.dc.L[k] = L;
                }
            };
            // every rune's choice by maxIndexProba over the exact values; then the window's
            // values go to gbest (k_long_seg, k_long_path read them)
            auto verify = [&](int32_t jv, uint32_t t, uint32_t nt) {
                bool bad = false;
                for (uint32_t r = t; r < kSpWin; r += nt) {
                    const uint32_t i = (uint32_t)jv * kSpWin + r;
                    if (i >= n) continue;
                    DpFold f;
                    long_items(text, im, erec, bs, be, i, [&](uint32_t L, double wt) {
                        fold_item(f, L, wt + (i + L == n ? 0.0 : S.dc.dring[(i + L) & (kLdDesc - 1u)]));
                    });
                    f.finish();
                    bad |= f.bestL != S.dc.L[i & (kLdDesc - 1u)];
                    gbest[s0 + i] = S.dc.dring[i & (kLdDesc - 1u)];
                }
                if (bad) S.bad = 1u;
            };
            stage(Jd - 1, tid, 256u);
            stage(Jd - 2, tid, 256u);
            if (tid == 0u) S.dc.dring[n & (kLdDesc - 1u)] = 0.0;  // best(n), when rune n is no dummy
            __syncthreads();
            if (wave == 0u) {
                // best(s + 1), best(s + 2) in registers; best(s + L) for L >= 3 from dring, read
                // two to three runes ahead (right after rune s + 3 is written: LDS accesses of a wave
                // complete in order).  A group's choices are loaded three groups ahead into one of
                // four register sets (four groups per loop trip, so the sets rotate without
                // copies); a window's slots do not wrap, so a trip's loads and stores are one base
                // address and immediate offsets.  Values are taken by bit selects, which the
                // compiler cannot turn into branches.  Per rune: four v_bfi_b32, one v_add_f64,
                // one LDS write and one LDS read.
                double H0 = 0.0, H1 = 0.0;  // best(s + 1), best(s + 2)
                double inner = 0.0;  // the next rune's L = 2 / L >= 3 select, made one step ahead
                // a zero the compiler cannot see through: the choices stay in VGPRs (uniform,
                // the compiler moved them to SGPRs and branched on them: 288 cycles per rune)
                uint32_t dz;
                asm volatile("v_mov_b32 %0, 0" : "=v"(dz));
                const char* const ringb = reinterpret_cast<const char*>(S.dc.dring);
                for (int32_t j = Jd - 1; j >= 0; --j) {
#if JB_STAMPS
                    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
                    if (lane == 0u) {
                        struct Set {
                            double w[4];
                            uint32_t ra[4], m1[4], m2[4];
                        };
                        const uint32_t kwin = ((uint32_t)j & 3u) * kSpWin;  // the window's first slot
                        const LSpec* const sp = S.dc.spec + (16u + kwin + dz);
                        const uint32_t* const mp = S.dc.m2 + (16u + kwin + dz);
                        double* const rw = S.dc.dring + kwin;
                        // the group at window offset p (a multiple of 4, >= -16)
                        auto load = [&](Set& X, int32_t p) {
#pragma unroll
                            for (int r = 0; r < 4; r++) {
                                const LSpec d = sp[p + r];
                                X.w[r] = d.w;
                                X.ra[r] = d.ra;
                                X.m1[r] = d.m1;
                            }
                            const uint4 m2 = *reinterpret_cast<const uint4*>(mp + p);
                            X.m2[0] = m2.x;
                            X.m2[1] = m2.y;
                            X.m2[2] = m2.z;
                            X.m2[3] = m2.w;
                        };
                        double rv[4];  // best(s + L) of rune s at index s & 3
                        // group p from set X (the ring reads of the next group from set Y); set Z
                        // (the last group's) loaded for the group three ahead
                        auto group = [&](const Set& X, const Set& Y, Set& Z, int32_t p) {
                            load(Z, p - 12);
                            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                            for (int u = 0; u < 4; u++) {
                                const int r = 3 - u;
                                const double b = bitsel64(X.m1[r], H0, inner);
                                // the inner select of rune p + r - 1 (its best(s + 2) is H0 now)
                                // between this rune's select and add (after the add instead, a
                                // hazard s_nop per rune and 5.8 % slower: profiles/ab/r04z6_chain_order_ab.txt)
                                inner = r ? bitsel64(X.m2[r - 1], H0, rv[r - 1]) : bitsel64(Y.m2[3], H0, rv[3]);
                                __builtin_amdgcn_sched_barrier(0);
                                const double P = X.w[r] + b;
                                __builtin_amdgcn_sched_barrier(0);
                                rw[p + r] = P;
                                // rune p + r - 3: p from X, p - 1 .. p - 3 from Y
                                rv[(r + 1) & 3] = *reinterpret_cast<const double*>(ringb + (r == 3 ? X.ra[0] : Y.ra[r + 1]));
                                H1 = H0;
                                H0 = P;
                                __builtin_amdgcn_sched_barrier(0);
                            }
                        };
                        Set A, B, C, D;
                        const int32_t top = (int32_t)kSpWin;
                        load(A, top - 4);
                        load(B, top - 8);
                        load(C, top - 12);
#pragma unroll
                        for (int r = 1; r < 4; r++) rv[r] = *reinterpret_cast<const double*>(ringb + A.ra[r]);
                        // (the window's top rune: a dummy or rune n - 1, L = 1, in the top window)
                        inner = bitsel64(A.m2[3], H1, rv[3]);
                        for (int32_t p = top - 4; p > 0; p -= 16) {
                            group(A, B, D, p);
                            group(B, C, A, p - 4);
                            group(C, D, B, p - 8);
                            group(D, A, C, p - 12);
                        }
                    }
#if JB_STAMPS
                    const uint64_t t1 = __builtin_amdgcn_s_memtime();
#endif
                    __syncthreads();
#if JB_STAMPS
                    st_run += t1 - t0;
                    st_bar += __builtin_amdgcn_s_memtime() - t1;
                    st_n++;
#endif
                }
                __syncthreads();
            } else {
                const uint32_t ht = tid - 64u;
                for (int32_t j = Jd - 1; j >= 0; --j) {
#if JB_STAMPS
                    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
                    stage(j - 2, ht, 192u);
                    if (j + 1 < Jd) verify(j + 1, ht, 192u);
#if JB_STAMPS
                    const uint64_t t1 = __builtin_amdgcn_s_memtime();
#endif
                    __syncthreads();
#if JB_STAMPS
                    st_run += t1 - t0;
                    st_bar += __builtin_amdgcn_s_memtime() - t1;
                    st_n++;
#endif
                }
                verify(0, ht, 192u);
                __syncthreads();
            }
            const bool bad = S.bad != 0u;
#if JB_STAMPS
            st_slow += bad ? 1000000u : 0u;  // (a block sent to the exact chain)
#endif
            if (!bad) {
                if (tid == 0u) lflag[bi] = 2u;  // DP done here; k_long_path sets 1 (entries found)
                __syncthreads();
                continue;
            }
            __syncthreads();  // (every thread has read S.bad: the exact chain below reuses the LDS)
        }
        if (tid < 4u) {
            S.sidecnt[tid] = 0u;
            S.wslow[tid] = 0u;
        }
        if (tid == 0u) lflag[bi] = 2u;  // DP done here; k_long_path sets 1 (entries found)
        __syncthreads();
        // descriptors of window jw (buffer jw & 3) by threads t, t + nt, ...
        auto fill = [&](int32_t jw, uint32_t t, uint32_t nt) {
            const uint32_t b = (uint32_t)jw & 3u;
            for (uint32_t r = t; r < kLdWin; r += nt) {
                const int32_t i = jw * (int32_t)kLdWin + (int32_t)r;
                LDesc& d = S.desc[(uint32_t)i & (kLdDesc - 1u)];
                const double nan = __builtin_nan("");
                uint8_t& cl = S.cls[(uint32_t)i & (kLdDesc - 1u)];
                if (i < 0 || (uint32_t)i >= n) {  // past the block: best = 0.0 + 0.0 (so best(n) = 0.0, :522-525)
                    cl = 0u;
                    d.w[0] = 0.0;
                    d.w[1] = d.w[2] = d.w[3] = nan;
                    d.a[0] = d.a[1] = d.a[2] = 0u;
                    d.flag = 0u;
                    continue;
                }
                uint32_t m = 0, L[4] = {0, 0, 0, 0};
                double w[4] = {nan, nan, nan, nan};
                long_items(text, im, erec, bs, be, (uint32_t)i, [&](uint32_t Lk, double wk) {
#pragma unroll
                    for (uint32_t k = 0; k < 4u; k++) {  // (no dynamic register index: no scratch)
                        L[k] = m == k ? Lk : L[k];
                        w[k] = m == k ? wk : w[k];
                    }
                    m++;
                });
                if (im.plainw && m >= 1u && m <= 4u && L[0] == 1u) {  // (the classes assume no +Inf/NaN weight)
#pragma unroll
                    for (int k = 0; k < 4; k++) d.w[k] = w[k];
#pragma unroll
                    for (int k = 1; k < 4; k++) d.a[k - 1] = (uint32_t)k < m ? (((uint32_t)i + L[k]) & (kLdRing - 1u)) * 8u : 0u;
                    d.flag = 0u;
                    // 0: items exactly L = 1..m (the chain's register form), 1: other gaps
                    cl = (m < 2u || L[1] == 2u) && (m < 3u || L[2] == 3u) && (m < 4u || L[3] == 4u) ? 0u : 1u;
                } else {  // more than 4 items, or none, or no L = 1 item (a negative count)
                    cl = 3u;
                    const uint32_t off = atomicAdd(&S.sidecnt[b], m);
                    if (off + m <= kLdSide) {
                        uint32_t k = 0;
                        long_items(text, im, erec, bs, be, (uint32_t)i, [&](uint32_t Lk, double wk) {
                            S.side[b][off + k].w = wk;
                            S.side[b][off + k].L = Lk;
                            k++;
                        });
                        d.flag = 1u | (off << 1) | (m << 16);
                    } else {
                        d.flag = kLdWalk;
                    }
                    d.a[0] = d.a[1] = d.a[2] = 0u;
                    atomicOr(&S.wslow[b], 1u);
                }
            }
        };
        auto copy = [&](int32_t jw, uint32_t t, uint32_t nt) {  // finished best values of window jw -> gbest
            for (uint32_t r = t; r < kLdWin; r += nt) {
                const uint32_t i = (uint32_t)jw * kLdWin + r;
                if (i < n) gbest[s0 + i] = S.ring[i & (kLdRing - 1u)];
            }
        };
        fill(J - 1, tid, 256u);
        fill(J - 2, tid, 256u);
        if (tid == 0u) S.ring[n & (kLdRing - 1u)] = 0.0;
        __syncthreads();
        if (wave == 0u) {
            // ---- the chain (calcDagProba + maxIndexProba, :502-578), lane 0 ----
            // By groups of four runes g..g+3 (taken g+3 first): the group's descriptors
            // were loaded into registers during the group before (two register sets,
            // alternate groups, no copies), and best(s+1 .. s+4) are in registers (H).
            // A group whose runes all have items exactly L = 1..m (m <= 4; class word 0,
            // most groups) folds from registers only.  Another group reads best(s + L_k)
            // from the ring, one rune ahead, and its slow runes walk their item lists.
            // The reference's rule over items p1..p4 (:565-578) is "the last k with
            // p_k >= p_(k-1)" (p_0 = minFloat).  With L1 = 1 and NaN for absent items
            // that is: p4 if p4 >= p3, else p3 if p3 >= p2, else max(p1, p2) (p1 <
            // minFloat only when p1 = -Inf, and then p2 >= p1 whenever item 2 exists;
            // equal values are the same value; tests/test_long_fold.py checks this
            // form against the oracle's rule).
            struct DSet {
                double w[4][4];
                uint32_t a[4][3], f[4];
            };
            DSet D0, D1;
            double H[4] = {0.0, 0.0, 0.0, 0.0};  // best(s + 1 .. s + 4) before rune s
            // a zero the compiler cannot see through: the descriptor addresses are
            // uniform, and it would otherwise keep the loaded sets in SGPRs and wait
            // for each load at once to move it there (readfirstlane), not a group later
            uint32_t dz;
            asm volatile("v_mov_b32 %0, 0" : "=v"(dz));
            double RV[2][3];
            auto ld_grp = [&](DSet& D, int32_t g) __attribute__((always_inline)) {  // descriptors of runes g .. g+3 (index s & 3)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const char* p = reinterpret_cast<const char*>(S.desc) + (((uint32_t)(g + r) & (kLdDesc - 1u)) * 48u + dz);
                    const double2 x = *reinterpret_cast<const double2*>(p);
                    const double2 y = *reinterpret_cast<const double2*>(p + 16);
                    const uint4 z = *reinterpret_cast<const uint4*>(p + 32);
                    D.w[r][0] = x.x;
                    D.w[r][1] = x.y;
                    D.w[r][2] = y.x;
                    D.w[r][3] = y.y;
                    D.a[r][0] = z.x;
                    D.a[r][1] = z.y;
                    D.a[r][2] = z.z;
                    D.f[r] = z.w;
                }
            };
            auto ld_rv = [&](uint32_t k, const DSet& D, int r) __attribute__((always_inline)) {
#pragma unroll
                for (int q = 0; q < 3; q++) RV[k][q] = *reinterpret_cast<const double*>(rb + D.a[r][q]);
            };
            auto push = [&](double P) __attribute__((always_inline)) {
                H[3] = H[2];
                H[2] = H[1];
                H[1] = H[0];
                H[0] = P;
            };
            auto group = [&](auto chk, int32_t g, const DSet& C, DSet& N, uint32_t cw, uint32_t b) __attribute__((always_inline)) {
                constexpr bool CHK = decltype(chk)::value;
                ld_grp(N, g - 4);  // (the next group's, a whole group ahead)
                char* const rw = reinterpret_cast<char*>(S.ring) + ((uint32_t)g & (kLdRing - 1u)) * 8u;
                if (cw == 0u) {
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int r = 3 - u;
                        const double p1 = C.w[r][0] + H[0];
                        const double p2 = C.w[r][1] + H[1];
                        const double p3 = C.w[r][2] + H[2];
                        const double p4 = C.w[r][3] + H[3];
                        const double R = max_f64(p1, p2);
                        const bool k3 = p3 >= p2, k4 = p4 >= p3;
                        const double p34 = k4 ? p4 : p3;
                        const double P = (k3 || k4) ? p34 : R;
                        *reinterpret_cast<double*>(rw + (uint32_t)r * 8u) = P;
                        push(P);
                    }
                    return;
                }
                ld_rv(1u, C, 3);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int r = 3 - u;
                    const uint32_t rs = (uint32_t)(u + 1) & 1u;  // this rune's ring values (set 1 at u = 0)
                    if (u < 3) ld_rv(rs ^ 1u, C, r - 1);  // the next rune's, a step ahead
                    double P;
                    const uint32_t cl = (cw >> (8 * r)) & 3u;
                    if (CHK && cl == 3u) {
                        const uint32_t s = (uint32_t)(g + r), fl = C.f[r];
                        DpFold f;
                        if (fl == kLdWalk) {
                            long_items(text, im, erec, bs, be, s, [&](uint32_t L, double wt) {
                                fold_item(f, L, wt + S.ring[(s + L) & (kLdRing - 1u)]);
                            });
                        } else {
                            const uint32_t m = fl >> 16, off = (fl >> 1) & 0x7FFFu;
                            for (uint32_t k = 0; k < m; k++) {
                                const LItem it = S.side[b][off + k];
                                fold_item(f, it.L, it.w + S.ring[(s + it.L) & (kLdRing - 1u)]);
                            }
                        }
                        f.finish();
                        P = f.bestP;
                    } else {
                        const double p1 = C.w[r][0] + H[0];
                        const double p2 = C.w[r][1] + RV[rs][0];
                        const double p3 = C.w[r][2] + RV[rs][1];
                        const double p4 = C.w[r][3] + RV[rs][2];
                        const double R = max_f64(p1, p2);
                        const bool k3 = p3 >= p2, k4 = p4 >= p3;
                        const double p34 = k4 ? p4 : p3;
                        P = (k3 || k4) ? p34 : R;
                    }
                    *reinterpret_cast<double*>(rw + (uint32_t)r * 8u) = P;
                    push(P);
                    __builtin_amdgcn_sched_barrier(0);
                }
            };
            const int32_t top = (int32_t)kLdWin * J - 4;  // the first group
            uint32_t cwn = 0;
            if (lane == 0u) {
                ld_grp(D0, top);
                cwn = *reinterpret_cast<const uint32_t*>(S.cls + ((uint32_t)top & (kLdDesc - 1u)));
            }
#if JB_STAMPS
            uint32_t st_wf = 0, st_w1 = 0, st_w3 = 0;  // per window: register-form groups, class-1 and class-3 runes
            auto st_count = [&](uint32_t cw) {
                const uint32_t x = cw & 0x03030303u;
                st_wf += cw == 0u ? 1u : 0u;
                st_w1 += (uint32_t)__popc(x & ~(x >> 1) & 0x01010101u);
                st_w3 += (uint32_t)__popc(x & (x >> 1) & 0x01010101u);
            };
#else
            auto st_count = [](uint32_t) {};
#endif
            auto run = [&](auto chk, int32_t j) {
                const uint32_t b = (uint32_t)j & 3u;
                for (int32_t g = (int32_t)kLdWin * j + (int32_t)kLdWin - 4; g >= (int32_t)kLdWin * j; g -= 8) {
                    uint32_t cw = __builtin_amdgcn_readfirstlane(cwn);
                    cwn = *reinterpret_cast<const uint32_t*>(S.cls + ((uint32_t)(g - 4) & (kLdDesc - 1u)));
                    st_count(cw);
                    group(chk, g, D0, D1, cw, b);
                    cw = __builtin_amdgcn_readfirstlane(cwn);
                    cwn = *reinterpret_cast<const uint32_t*>(S.cls + ((uint32_t)(g - 8) & (kLdDesc - 1u)));
                    st_count(cw);
                    group(chk, g - 4, D1, D0, cw, b);
                }
            };
            static_assert(kLdWin % 8u == 0u, "two groups per loop trip");
            for (int32_t j = J - 1; j >= 0; --j) {
#if JB_STAMPS
                const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
                if (lane == 0u) {
                    if (S.wslow[j & 3]) run(std::true_type{}, j);
                    else run(std::false_type{}, j);
                }
#if JB_STAMPS
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
                st_slow += S.wslow[j & 3] ? 1u : 0u;
                if (wg == 0u && lane == 0u && (uint32_t)j < kDbgLongWinMax) {  // per window of block 0
                    uint64_t* o = dbg + kDbgLongWin + (uint64_t)j * 4u;
                    o[0] = t1 - t0;
                    o[1] = st_wf;
                    o[2] = st_w1;
                    o[3] = st_w3;
                }
                st_wf = st_w1 = st_w3 = 0u;
#endif
                __syncthreads();
#if JB_STAMPS
                st_run += t1 - t0;
                st_bar += __builtin_amdgcn_s_memtime() - t1;
                st_n++;
#endif
            }
        } else {
            const uint32_t ht = tid - 64u;  // helper thread 0..191
            for (int32_t j = J - 1; j >= 0; --j) {
                if (ht == 0u) {  // buffer of window j - 3 (last used by window j + 1, done): filled next trip
                    S.sidecnt[(uint32_t)(j - 3) & 3u] = 0u;
                    S.wslow[(uint32_t)(j - 3) & 3u] = 0u;
                }
#if JB_STAMPS
                const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
                fill(j - 2, ht, 192u);
                if (j + 1 < J) copy(j + 1, ht, 192u);
#if JB_STAMPS
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
#endif
                __syncthreads();
#if JB_STAMPS
                st_run += t1 - t0;
                st_bar += __builtin_amdgcn_s_memtime() - t1;
                st_n++;
#endif
            }
            copy(0, ht, 192u);
        }
        __syncthreads();
    }
#if JB_STAMPS
    if (lane == 0u) {  // per wave w, [4w .. 4w + 3]: run, barrier, windows, slow (wave 0: the chain)
        uint64_t* o = dbg + kDbgLong + wg * 16u + wave * 4u;
        o[0] = st_run;
        o[1] = st_bar;
        o[2] = st_n;
        o[3] = st_slow;
        uint64_t* p = dbg + kDbgLong + 64u * 16u + wg * 16u + wave * 4u;
        for (int k = 0; k < 4; k++) p[k] = st_p[k];
    }
#else
    (void)dbg;
#endif
}

template <bool HMM>
__global__ __launch_bounds__(256) void k_long_dp(const uint8_t* __restrict__ text, DevImage im,
                                                 const uint64_t* __restrict__ erec, uint8_t* __restrict__ gbl,
                                                 double* __restrict__ gbest, const uint2* __restrict__ longblk,
                                                 uint32_t* __restrict__ counters, uint32_t* __restrict__ sbits,
                                                 uint32_t* __restrict__ ebits, uint32_t* __restrict__ lflag,
                                                 const uint32_t* __restrict__ lsegb, const uint64_t* __restrict__ lpath,
                                                 uint64_t* __restrict__ dbg, uint32_t spec) {
    __shared__ LongLds S;
    long_dp_body<HMM>(text, im, erec, gbl, gbest, longblk, counters, sbits, ebits, lflag, lsegb, lpath, dbg, spec, blockIdx.x, gridDim.x, S);
}


// k_long_seg: one lane per 64-rune segment of a long block that k_long_dp ran
// the chain for.  The chosen lengths are maxIndexProba over the same sums
// w + best(i + L) the chain formed (the same float64 adds of the same values),
// so they are the chain's choices.  Then, backwards over the segment, each
// rune's exit code: where findDagPath, entering the segment at that rune, first
// lands at or past the segment's end (its offset past the end, 0..254), or
// 0xFF when that is the end itself and the last piece before it is one rune
// (so the next segment knows a run of single-rune pieces enters it).
// A wave holds 64 consecutive segments, chunk c = g / 64.  When they are all one
// block's and the block goes on past them, the wave composes their boundary maps
// into the chunk's map (lmap[c]: state at the chunk's start -> state at its end),
// four states per lane walked through the 64 segments' codes in LDS.
__device__ __forceinline__ void long_seg_body(const uint8_t* __restrict__ text, DevImage im,
                                                  const uint64_t* __restrict__ erec, const uint2* __restrict__ longblk,
                                                  const uint32_t* __restrict__ lsegb, const uint32_t* __restrict__ counters,
                                                  const uint32_t* __restrict__ lflag, const double* __restrict__ gbest,
                                                  uint8_t* __restrict__ gbl, uint8_t* __restrict__ lcode,
                                                  uint8_t* __restrict__ lmap,
        uint32_t wg, uint32_t ng, uint8_t (*s_bl)[kSeg]) {
    const uint32_t nlong = counters[CNT_NLONG], nseg = counters[CNT_NLSEG], lane = threadIdx.x & 63u;
    uint8_t* const my = s_bl[threadIdx.x];
    for (uint32_t gw = wg * blockDim.x + (threadIdx.x & ~63u); gw < nseg; gw += ng * blockDim.x) {
        const uint32_t g = gw + lane;  // (the loop is wave-uniform: the chunk map needs the whole wave)
        uint32_t bi = 0xFFFFFFFFu, n = 0, a = 0;
        bool act = g < nseg;
        if (act) {
            bi = long_block_of(lsegb, nlong, g);
            act = lflag[bi] == 2u;
        }
        if (act) {
            const uint2 bb = longblk[bi];
            const uint32_t bs = bb.x, be = bb.y, s0 = bs / 3u;
            n = (be - bs) / 3u;
            a = (g - lsegb[bi]) * kSeg;
            const uint32_t lim = min(a + kSeg, n);
            for (uint32_t i = a; i < lim; i++) {
                DpFold f;
                long_items(text, im, erec, bs, be, i, [&](uint32_t L, double wt) {
                    fold_item(f, L, wt + (i + L == n ? 0.0 : gbest[s0 + i + L]));
                });
                f.finish();
                my[i - a] = (uint8_t)f.bestL;
                gbl[s0 + i] = (uint8_t)f.bestL;
            }
            for (uint32_t p = lim; p-- > a;) {
                // (a rune with no piece walks on as if it had one: if the true path
                // comes to it, k_long_tail reports it)
                const uint32_t L = max(1u, (uint32_t)my[p - a]), q = p + L;
                const uint8_t c = q >= lim ? (L == 1u ? (uint8_t)0xFFu : (uint8_t)(q - lim)) : my[q - a];
                my[p - a] = c;
                lcode[s0 + p] = c;
            }
        }
        // the chunk map: 64 whole segments of one block, and more of the block after them
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bi);
        const bool inner = act && bi == b0 && a + kSeg < n;
        if (__ballot(inner) == ~0ull) {
            wave_sync();  // (every lane's codes are in LDS)
            lp_compose(s_bl + (threadIdx.x & ~63u), lmap + (uint64_t)(gw / kSeg) * kLpMap, lane);
        }
        wave_sync();  // (the next iteration's codes overwrite these)
    }
}

__global__ __launch_bounds__(256) void k_long_seg(const uint8_t* __restrict__ text, DevImage im,
                                                  const uint64_t* __restrict__ erec, const uint2* __restrict__ longblk,
                                                  const uint32_t* __restrict__ lsegb, const uint32_t* __restrict__ counters,
                                                  const uint32_t* __restrict__ lflag, const double* __restrict__ gbest,
                                                  uint8_t* __restrict__ gbl, uint8_t* __restrict__ lcode,
                                                  uint8_t* __restrict__ lmap) {
    __shared__ uint8_t s_bl[256][kSeg];
    long_seg_body(text, im, erec, longblk, lsegb, counters, lflag, gbest, gbl, lcode, lmap, blockIdx.x, gridDim.x, s_bl);
}

// k_long_path: one wave per long block: the path state (lp_next) at the start of
// every 64-segment chunk the block spans past its first (lcx[c]).  The segments
// before the first chunk boundary are crossed one by one (their codes staged in
// LDS), then each chunk by its map (k_long_seg), the maps staged kLpBatch at a
// time: one LDS lookup per chunk instead of one hop per segment (the serial walk
// over 15.6K segments of config 5b took 2.1 ms).  k_long_tail finds each
// segment's entry from these states.
__device__ __forceinline__ void long_path_body(const uint2* __restrict__ longblk, const uint32_t* __restrict__ lsegb,
                                                  const uint32_t* __restrict__ counters, uint32_t* __restrict__ lflag,
                                                  const uint8_t* __restrict__ lcode, const uint8_t* __restrict__ lmap,
                                                  uint8_t* __restrict__ lcx, uint32_t want, uint32_t set,
        uint32_t wg, uint32_t ng, uint32_t* s_m32) {
    const uint8_t* const s_m = reinterpret_cast<const uint8_t*>(s_m32);
    static_assert(kSeg * kSeg <= kLpBatch * kLpMap, "the first partial chunk's codes fit the map space");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nlong = counters[CNT_NLONG];
    for (uint32_t bi = wg; bi < nlong; bi += ng) {
        if (lflag[bi] != want) continue;
        const uint2 bb = longblk[bi];
        const uint32_t n = (bb.y - bb.x) / 3u, s0 = bb.x / 3u, sb = lsegb[bi];
        const uint32_t gend = sb + (n + kSeg - 1u) / kSeg;  // past the block's last segment
        const uint32_t g1 = min(gend, (sb + kSeg - 1u) & ~(kSeg - 1u));  // the first chunk boundary
        uint32_t x = 0;  // the state at the block's start: its first rune, no piece before
        if (g1 < gend) {
            if (g1 > sb) {  // the segments before it, one by one (lcode has 512 bytes of slack)
                const uint32_t nw = (g1 - sb) * (kSeg / 4u);
                for (uint32_t k = lane; k < nw; k += 64u) s_m32[k] = ld4(lcode, (uint64_t)s0 + 4u * k);
                wave_sync();
                for (uint32_t j = 0; j < g1 - sb; j++) x = lp_next(s_m + j * kSeg, x);
                wave_sync();
            }
            for (uint32_t c0 = g1 / kSeg; c0 * kSeg < gend; c0 += kLpBatch) {
                // chunks c0 .. (the maps of the ones wholly inside the block with more after them)
                const uint32_t cend = min(c0 + kLpBatch, (gend + kSeg - 1u) / kSeg);
                uint32_t cmap = cend;
                while (cmap > c0 && (cmap * kSeg >= gend)) --cmap;  // chunks c0..cmap-1 have a map
                const uint32_t nw = (cmap - c0) * (kLpMap / 4u);
                const uint32_t* gm = reinterpret_cast<const uint32_t*>(lmap + (uint64_t)c0 * kLpMap);
                for (uint32_t k = lane; k < nw; k += 64u) s_m32[k] = gm[k];
                wave_sync();
                for (uint32_t c = c0; c < cend; c++) {
                    if (lane == 0u) lcx[c] = (uint8_t)x;
                    if (c < cmap) x = s_m[(c - c0) * kLpMap + x];
                }
                wave_sync();
            }
        }
        if (lane == 0u) lflag[bi] = set;
    }
}

__global__ __launch_bounds__(64) void k_long_path(const uint2* __restrict__ longblk, const uint32_t* __restrict__ lsegb,
                                                  const uint32_t* __restrict__ counters, uint32_t* __restrict__ lflag,
                                                  const uint8_t* __restrict__ lcode, const uint8_t* __restrict__ lmap,
                                                  uint8_t* __restrict__ lcx, uint32_t want, uint32_t set) {
    __shared__ uint32_t s_m32[kLpBatch * kLpMap / 4u];
    long_path_body(longblk, lsegb, counters, lflag, lcode, lmap, lcx, want, set, blockIdx.x, gridDim.x, s_m32);
}

// k_long_pbits: for the blocks k_long_dp takes by the path chain (lflag 3), the path of
// findDagPath (:552-562) through k_long_spec's choices, one lane per segment: its entry
// as k_long_tail finds it (the wave's 64 segments' exit codes crossed in order from
// the chunk's state, k_long_path's lcx), then the pieces from there by the choices
// (in LDS); lpath[g] has a bit for each rune where a piece starts.
__device__ __forceinline__ void long_pbits_body(const uint2* __restrict__ longblk, const uint32_t* __restrict__ lsegb,
                                                    const uint32_t* __restrict__ counters,
                                                    const uint32_t* __restrict__ lflag, const uint8_t* __restrict__ gbl,
                                                    const uint8_t* __restrict__ lcode, const uint8_t* __restrict__ lcx,
                                                    uint64_t* __restrict__ lpath,
        uint32_t wg, uint32_t ng, uint4 (*s_cd)[kSeg / 16u]) {
    const uint32_t nlong = counters[CNT_NLONG], nseg = counters[CNT_NLSEG], lane = threadIdx.x & 63u;
    uint32_t* const d = reinterpret_cast<uint32_t*>(s_cd[threadIdx.x]);
    for (uint32_t gw = wg * blockDim.x + (threadIdx.x & ~63u); gw < nseg; gw += ng * blockDim.x) {
        const uint32_t g = gw + lane;  // (wave-uniform loop)
        uint32_t bi = 0, a = 0, n = 0, s0 = 0;
        bool act = g < nseg;
        if (act) {
            bi = long_block_of(lsegb, nlong, g);
            act = lflag[bi] == 3u;
        }
        bool first = false;  // the block's first segment
        if (act) {
            const uint2 bb = longblk[bi];
            const uint32_t sg = lsegb[bi];
            n = (bb.y - bb.x) / 3u;
            s0 = bb.x / 3u;
            a = (g - sg) * kSeg;
            first = g == sg;
#pragma unroll
            for (uint32_t k = 0; k < kSeg / 4u; k++) d[k] = ld4(lcode, (uint64_t)s0 + a + 4u * k);  // (256 bytes of slack)
        }
        const uint64_t am = __ballot(act), fm = __ballot(first);
        wave_sync();
        uint32_t x = lcx[gw / kSeg], ent = 0xFFFFFFFFu;
        for (uint32_t k = 0; k < 64u; k++) {
            if (!((am >> k) & 1ull)) continue;  // (uniform)
            if ((fm >> k) & 1ull) x = 0u;
            const uint32_t ak = (uint32_t)__builtin_amdgcn_readlane((int)a, (int)k);
            const uint32_t nk = (uint32_t)__builtin_amdgcn_readlane((int)n, (int)k);
            const uint32_t e = lp_entry(x, ak, nk);
            if (lane == k) ent = e;
            if (e != 0xFFFFFFFFu || (x != 0xFFu && x >= 64u))
                x = lp_next(reinterpret_cast<const uint8_t*>(s_cd[(threadIdx.x & ~63u) + k]), x);
        }
        wave_sync();  // (every lane is done with the codes)
        if (act) {
#pragma unroll
            for (uint32_t k = 0; k < kSeg / 4u; k++) d[k] = ld4(gbl, (uint64_t)s0 + a + 4u * k);  // (512 bytes of slack)
            const uint8_t* const dl = reinterpret_cast<const uint8_t*>(d);
            const uint32_t lim = min(kSeg, n - a);
            uint64_t bits = 0;
            if (ent != 0xFFFFFFFFu)
                for (uint32_t o = ent & 0xFFu; o < lim; o += max(1u, (uint32_t)dl[o])) bits |= 1ull << o;
            lpath[g] = bits;
        }
        wave_sync();  // (the next iteration overwrites the LDS rows)
    }
}

__global__ __launch_bounds__(256) void k_long_pbits(const uint2* __restrict__ longblk, const uint32_t* __restrict__ lsegb,
                                                    const uint32_t* __restrict__ counters,
                                                    const uint32_t* __restrict__ lflag, const uint8_t* __restrict__ gbl,
                                                    const uint8_t* __restrict__ lcode, const uint8_t* __restrict__ lcx,
                                                    uint64_t* __restrict__ lpath) {
    __shared__ uint4 s_cd[256][kSeg / 16u];  // each lane's segment's exit codes, then its choices
    long_pbits_body(longblk, lsegb, counters, lflag, gbl, lcode, lcx, lpath, blockIdx.x, gridDim.x, s_cd);
}

// Viterbi (tokenizer.go:668-730) + cutHMM (:273-285) of the run of single-rune
// pieces [q, r) (rune indices of a long block, all 3-byte): back-pointers in
// bp (slot bytes), the final state from v[E] > v[S] (:723-729).
template <class E>
__device__ void long_viterbi(const uint8_t* __restrict__ text, const DevImage& im, uint32_t bs, uint32_t s0,
                             uint32_t q, uint32_t r, uint8_t* __restrict__ bp, E& em) {
    auto rune_at = [&](uint32_t j) {
        const uint32_t x = ld4(text, bs + 3u * j);
        return ((x & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu);
    };
    double e[4], en[4];
    load_emit(im, rune_at(q), e);
    double vB = START_B + e[0], vM = JB_MIN_FLOAT + e[1], vE = JB_MIN_FLOAT + e[2], vS = START_S + e[3];
    if (q + 1u < r) load_emit(im, rune_at(q + 1u), e);
    for (uint32_t j = q + 1u; j < r; j++) {
        if (j + 1u < r) load_emit(im, rune_at(j + 1u), en);  // next rune's emissions, in flight
        uint32_t cB, cM, cE, cS;
        double pB, pM, pE, pS;
        route2(vE + T_EB, vS + T_SB, &cB, &pB, em.ties);  // B <- E, S
        route2(vB + T_BM, vM + T_MM, &cM, &pM, em.ties);  // M <- B, M
        route2(vB + T_BE, vM + T_ME, &cE, &pE, em.ties);  // E <- B, M
        route2(vE + T_ES, vS + T_SS, &cS, &pS, em.ties);  // S <- E, S
        vB = pB + e[0];
        vM = pM + e[1];
        vE = pE + e[2];
        vS = pS + e[3];
        bp[s0 + j] = (uint8_t)(cB | (cM << 2) | (cE << 4) | (cS << 6));
        e[0] = en[0]; e[1] = en[1]; e[2] = en[2]; e[3] = en[3];
    }
    // traceback from the final state; a "" route restarts the path there (:715),
    // and cutHMM labels runes from the run start (:273-285)
    const uint32_t m = r - q;
    uint32_t st = vE > vS ? (uint32_t)JB_E : (uint32_t)JB_S;
    uint32_t t = m - 1u, reset = 0, jt = r - 1u;
    for (;;) {
        if (t == 0u) {
            bp[s0 + jt] = (uint8_t)st;
            break;
        }
        const uint32_t code = (bp[s0 + jt] >> (2u * st)) & 3u;
        bp[s0 + jt] = (uint8_t)st;
        if (code == 2u) {
            reset = t;
            break;
        }
        st = (st == JB_B || st == JB_S) ? 2u + code : code;  // B,S <- {E,S}; M,E <- {B,M}
        --t;
        --jt;
    }
    uint32_t ja = q, jb = jt, ts = q;
    for (uint32_t k = 0; k < m - reset; k++) {
        const uint32_t lab = bp[s0 + jb];
        ++ja;
        ++jb;
        if (lab >= (uint32_t)JB_E) {
            em.token(bs + 3u * ts, bs + 3u * ja);
            ts = ja;
        }
    }
}

// k_long_tail: one lane per segment of a long block.  A wave holds the 64
// segments of chunk c = g / 64: it stages their exit codes in LDS and crosses
// them in order from the chunk's state (k_long_path's lcx[c], or the block's
// start state where a block begins), which gives each segment its entry (the
// hop-by-hop walk of findDagPath, :552-562, over 64 segments at a time).  From
// its entry each lane makes the pieces that start in its segment tokens, and
// runs every run of one-rune pieces that starts there through Viterbi (+ cutHMM);
// a run that entered from the previous segment belongs to that segment's lane.
// The Viterbi back-pointers go to bp (gbest's bytes, free by now), not over the
// exit codes other waves still read.
template <bool HMM>
__device__ __forceinline__ void long_tail_body(const uint8_t* __restrict__ text, DevImage im,
                                                   const uint8_t* __restrict__ gbl, const uint2* __restrict__ longblk,
                                                   const uint32_t* __restrict__ lsegb, const uint32_t* __restrict__ lflag,
                                                   uint32_t* __restrict__ counters, const uint8_t* __restrict__ lcode,
                                                   const uint8_t* __restrict__ lcx, uint8_t* __restrict__ bp,
                                                   uint32_t* __restrict__ sbits, uint32_t* __restrict__ ebits,
        uint32_t wg, uint32_t ng, uint4 (*s_cd)[kSeg / 16u]) {
    const uint32_t nlong = counters[CNT_NLONG], nseg = counters[CNT_NLSEG], lane = threadIdx.x & 63u;
    Emitter em(sbits, ebits);
    bool bad = false;
    for (uint32_t gw = wg * blockDim.x + (threadIdx.x & ~63u); gw < nseg; gw += ng * blockDim.x) {
        const uint32_t g = gw + lane;  // (wave-uniform loop)
        uint32_t bi = 0, a = 0, n = 0;
        bool act = g < nseg;
        if (act) {
            bi = long_block_of(lsegb, nlong, g);
            act = lflag[bi] == 1u;  // (else cut by the one-lane path)
        }
        bool first = false;  // the block's first segment
        if (act) {
            const uint2 bb = longblk[bi];
            const uint32_t sg = lsegb[bi];
            n = (bb.y - bb.x) / 3u;
            a = (g - sg) * kSeg;
            first = g == sg;
            uint32_t* d = reinterpret_cast<uint32_t*>(s_cd[threadIdx.x]);  // (lcode has 256 bytes of slack)
#pragma unroll
            for (uint32_t k = 0; k < kSeg / 4u; k++) d[k] = ld4(lcode, (uint64_t)bb.x / 3u + a + 4u * k);
        }
        const uint64_t am = __ballot(act), fm = __ballot(first);
        wave_sync();
        // the wave's segments in order: every lane runs the same walk (LDS reads of one
        // address: broadcast) and keeps its own segment's entry
        uint32_t x = lcx[gw / kSeg], ent = 0xFFFFFFFFu;
        for (uint32_t k = 0; k < 64u; k++) {
            if (!((am >> k) & 1ull)) continue;  // (uniform)
            if ((fm >> k) & 1ull) x = 0u;
            const uint32_t ak = (uint32_t)__builtin_amdgcn_readlane((int)a, (int)k);
            const uint32_t nk = (uint32_t)__builtin_amdgcn_readlane((int)n, (int)k);
            const uint32_t e = lp_entry(x, ak, nk);
            if (lane == k) ent = e;
            if (e != 0xFFFFFFFFu || (x != 0xFFu && x >= 64u))
                x = lp_next(reinterpret_cast<const uint8_t*>(s_cd[(threadIdx.x & ~63u) + k]), x);
        }
        wave_sync();  // (the next iteration overwrites the codes)
        if (!act || ent == 0xFFFFFFFFu) continue;  // no piece starts here
        const uint2 bb = longblk[bi];
        const uint32_t bs = bb.x, s0 = bs / 3u;
        auto len = [&](uint32_t j) { return (uint32_t)gbl[s0 + j]; };
        const uint32_t c0 = a, c1 = min(n, c0 + kSeg);
        uint32_t q = c0 + (ent & 0xFFu);
        if (HMM && (ent >> 8))  // a run of one-rune pieces enters: its owner cuts it
            while (q < n && len(q) == 1u) q++;
        while (q < c1) {
            const uint32_t Ln = len(q);
            if (Ln == 0u) {  // tail index -1: cutDAG's slice panics in the reference
                bad = true;
                break;
            }
            if (!HMM || Ln > 1u) {
                em.token(bs + 3u * q, bs + 3u * (q + Ln));
                q += Ln;
                continue;
            }
            uint32_t r = q + 1u;
            while (r < n && len(r) == 1u) r++;
            if (r - q == 1u) em.token(bs + 3u * q, bs + 3u * r);  // a single rune is always "S" (:672-674)
            else long_viterbi(text, im, bs, s0, q, r, bp, em);
            q = r;
        }
    }
    em.flush();
    if (bad) atomicOr(counters + CNT_ERR, 1u);
    uint32_t t = em.ties;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) t += (uint32_t)__shfl_xor((int)t, d, 64);
    if ((threadIdx.x & 63u) == 0u && t) atomicAdd(counters + CNT_TIES, t);
}

template <bool HMM>
__global__ __launch_bounds__(256) void k_long_tail(const uint8_t* __restrict__ text, DevImage im,
                                                   const uint8_t* __restrict__ gbl, const uint2* __restrict__ longblk,
                                                   const uint32_t* __restrict__ lsegb, const uint32_t* __restrict__ lflag,
                                                   uint32_t* __restrict__ counters, const uint8_t* __restrict__ lcode,
                                                   const uint8_t* __restrict__ lcx, uint8_t* __restrict__ bp,
                                                   uint32_t* __restrict__ sbits, uint32_t* __restrict__ ebits) {
    __shared__ uint4 s_cd[256][kSeg / 16u];  // each lane's segment's exit codes
    long_tail_body<HMM>(text, im, gbl, longblk, lsegb, lflag, counters, lcode, lcx, bp, sbits, ebits, blockIdx.x, gridDim.x, s_cd);
}


// k_nonzh: cutNonZh (tokenizer.go:289-310) for exactly the non-Han blocks that hold
// a [0-9A-Za-z] byte; every other non-Han block has no tokens (:290-293).  An alnum
// byte is never Han, so it always lies in a non-Han block.  One wave per 64 alnum16
// words (64 KiB of text), their alnum chunks dealt over its lanes (nonzh_waves); for
// each such chunk and each block with an alnum byte there, the lane cuts the block
// when this chunk holds the block's first alnum byte (the block starts in the chunk,
// or walking back from it to the block start meets no alnum byte).  Block bounds come
// from the lane masks of k_mark_walk, so the kernel touches neither the block list nor
// the Han blocks.
__device__ __forceinline__ void nonzh_body(const uint8_t* __restrict__ text, uint32_t nbytes,
                                           const uint32_t* __restrict__ lanemask, const uint2* __restrict__ tile_cnt,
                                           uint32_t ntiles, const uint64_t* __restrict__ alnum16,
                                           uint32_t* __restrict__ sbits, uint32_t* __restrict__ ebits,
                                           uint32_t* __restrict__ docbits, const uint64_t* __restrict__ doc_off,
                                           uint32_t ndocs, uint32_t wg, uint32_t ng, NzLds& L) {
    const uint32_t nch = (nbytes + 15u) >> 4;
    // the words k_docbits set back to zero for the next run (k_mark_walk, their only
    // reader, is done): one store per document
    for (uint32_t d = wg * 256u + threadIdx.x; d < ndocs; d += ng * 256u) {
        const uint64_t o = doc_off[d];
        if (o < nbytes) docbits[o >> 5] = 0u;
    }
    Emitter em(sbits, ebits);
    nonzh_waves<64>(text, nbytes, nch, lanemask, tile_cnt, ntiles, alnum16, wg * 4u + (threadIdx.x >> 6), ng * 4u, em, L);
    em.flush();
}
__global__ __launch_bounds__(256) void k_nonzh(const uint8_t* __restrict__ text, uint32_t nbytes,
                                               const uint32_t* __restrict__ lanemask,
                                               const uint2* __restrict__ tile_cnt, uint32_t ntiles,
                                               const uint64_t* __restrict__ alnum16, uint32_t* __restrict__ sbits,
                                               uint32_t* __restrict__ ebits, uint32_t* __restrict__ docbits,
                                               const uint64_t* __restrict__ doc_off, uint32_t ndocs) {
    __shared__ __attribute__((aligned(16))) NzLds s_nz;
    nonzh_body(text, nbytes, lanemask, tile_cnt, ntiles, alnum16, sbits, ebits, docbits, doc_off, ndocs, blockIdx.x,
               gridDim.x, s_nz);
}

// ---------------------------------------------------------------------------
// token bitmaps -> spans
// ---------------------------------------------------------------------------
#ifndef JB_TOK_CAP
#define JB_TOK_CAP 3072
#endif
constexpr uint32_t kTokCap = JB_TOK_CAP;  // tokens per tile staged in LDS (k_tok's write pass)
// block `blk` of `nblk` (the write pass: token tile blk; the count pass: tiles 2 blk, 2 blk + 1)
template <bool WRITE>
__device__ __forceinline__ void tok_body(const uint32_t* __restrict__ sbits, const uint32_t* __restrict__ ebits,
                                         uint64_t nwords, uint2* __restrict__ tile_cnt,
                                         const uint2* __restrict__ supt, uint32_t* __restrict__ counters,
                                         uint32_t* __restrict__ tok_start, uint32_t* __restrict__ tok_end,
                                         uint32_t blk, uint32_t nblk, uint32_t* lds, uint32_t* s_s, uint32_t* s_e) {
    // bitmap words per lane: the write pass takes a token tile per workgroup, the count
    // pass two (16-byte loads, half the workgroups; a tile's count is the half's sum)
    constexpr uint32_t W = (WRITE ? 1u : 2u) * (kTokTileWords / 256);
    constexpr uint32_t kCap = kTokCap;
    const uint64_t w0 = ((uint64_t)blk * 256u + threadIdx.x) * W;
    PrefixLoads pl{0u, 0u};
    if (WRITE) pl = pf_load(tile_cnt, supt, blk);
    uint32_t s[W], e[W];
    if (w0 + W <= nwords) {
        if constexpr (W == 4u) {
            const uint4 a = *reinterpret_cast<const uint4*>(sbits + w0);
            const uint4 b = *reinterpret_cast<const uint4*>(ebits + w0);
            s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
            e[0] = b.x; e[1] = b.y; e[2] = b.z; e[3] = b.w;
        } else {
            const uint2 a = *reinterpret_cast<const uint2*>(sbits + w0);
            const uint2 b = *reinterpret_cast<const uint2*>(ebits + w0);
            s[0] = a.x; s[1] = a.y;
            e[0] = b.x; e[1] = b.y;
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < W; k++) {
            s[k] = w0 + k < nwords ? sbits[w0 + k] : 0u;
            e[k] = w0 + k < nwords ? ebits[w0 + k] : 0u;
        }
    }
    uint32_t cs = 0, ce = 0;
#pragma unroll
    for (uint32_t k = 0; k < W; k++) {
        cs += __popc(s[k]);
        ce += __popc(e[k]);
    }
    uint32_t ts, te;
    const uint32_t xs = block_scan_u32(cs, lds, &ts);
    const uint32_t xe = block_scan_u32(ce, lds, &te);
    if (!WRITE) {  // lanes 0-127 hold the first tile: its count is lane 128's exclusive prefix
        if (threadIdx.x == 128u) {
            tile_cnt[2u * blk] = make_uint2(xs, xe);
            tile_cnt[2u * blk + 1u] = make_uint2(ts - xs, te - xe);
        }
        return;
    }
    const uint2 to = pf_sum(pl, lds);
    if (blk == nblk - 1u && threadIdx.x == 0) {  // token totals
        counters[CNT_NTOK] = to.x + ts;
        counters[CNT_NTOKE] = to.y + te;
        *reinterpret_cast<uint64_t*>(counters + CNT_NWORDS) = to.x + ts;
    }
    // spans go to LDS in tile order, then out in one coalesced pass (a lane's own
    // tokens are ~60 bytes apart in the output: direct stores touch a line each)
    const bool staged = ts <= kCap && te <= kCap;
    // staged at LDS index (output index mod 4) + k, so that LDS and output share their
    // 16-byte alignment and the copy-out moves four spans per lane and store
    // (k_tok_write 0.298 -> 0.288 ms at 1 GiB; caller arrays not 16-byte aligned: one each)
    const bool v4 = (((uintptr_t)tok_start | (uintptr_t)tok_end) & 15u) == 0u;
    const uint32_t shs = v4 ? (to.x & 3u) : 0u, she = v4 ? (to.y & 3u) : 0u;
    uint32_t* os = staged ? s_s + shs : tok_start + to.x;
    uint32_t* oe = staged ? s_e + she : tok_end + to.y;
    uint32_t gs = xs, ge = xe;
#pragma unroll
    for (uint32_t k = 0; k < W; k++) {
        const uint32_t base = (uint32_t)((w0 + k) << 5);
        uint32_t m = s[k];
        while (m) {
            os[gs++] = base + (uint32_t)__builtin_ctz(m);
            m &= m - 1;
        }
        m = e[k];
        while (m) {
            oe[ge++] = base + (uint32_t)__builtin_ctz(m) + 1u;
            m &= m - 1;
        }
    }
    if (staged) {
        __syncthreads();
        if (v4) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            auto out = [&](const uint32_t* a, uint32_t sh, uint32_t n, uint32_t* g) {  // g: output at LDS index 0
                const uint32_t lo = (sh + 3u) & ~3u, hi = (sh + n) & ~3u;  // whole vectors: [lo, hi)
                if (lo < hi) {
                    for (uint32_t p = lo + 4u * threadIdx.x; p < hi; p += 1024u)
                        __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(a + p), reinterpret_cast<u32x4*>(g + p));
                    if (threadIdx.x < lo - sh) __builtin_nontemporal_store(a[sh + threadIdx.x], g + sh + threadIdx.x);
                    if (threadIdx.x < sh + n - hi) __builtin_nontemporal_store(a[hi + threadIdx.x], g + hi + threadIdx.x);
                } else if (threadIdx.x < n) {
                    __builtin_nontemporal_store(a[sh + threadIdx.x], g + sh + threadIdx.x);
                }
            };
            out(s_s, shs, ts, tok_start + to.x - shs);
            out(s_e, she, te, tok_end + to.y - she);
            return;
        }
        for (uint32_t k = threadIdx.x; k < ts; k += 256u) __builtin_nontemporal_store(s_s[k], tok_start + to.x + k);
        for (uint32_t k = threadIdx.x; k < te; k += 256u) __builtin_nontemporal_store(s_e[k], tok_end + to.y + k);
    }
}
template <bool WRITE>
__global__ __launch_bounds__(256) void k_tok(const uint32_t* __restrict__ sbits, const uint32_t* __restrict__ ebits,
                                             uint64_t nwords, uint2* __restrict__ tile_cnt,
                                             const uint2* __restrict__ supt, uint32_t* __restrict__ counters,
                                             uint32_t* __restrict__ tok_start, uint32_t* __restrict__ tok_end) {
    __shared__ uint32_t lds[8];
    __shared__ __attribute__((aligned(16))) uint32_t s_s[WRITE ? kTokCap + 4 : 1], s_e[WRITE ? kTokCap + 4 : 1];
    tok_body<WRITE>(sbits, ebits, nwords, tile_cnt, supt, counters, tok_start, tok_end, blockIdx.x, gridDim.x, lds, s_s,
                    s_e);
}

// tokens of document d: [doc_tok[d], doc_tok[d+1]) = lower_bound over starts.
// G lanes per document.  G = 16 (a small batch: few documents, so the kernel's time
// is one search's dependent loads): each trip, lane k probes the last start of the
// k-th sixteenth of the range and a ballot counts the sixteenths wholly before the
// target, log16 loads instead of log2.  G = 1 (many documents: their searches hide
// each other's latency, and 16 lanes each would cost more loads in all): binary.
template <uint32_t G>
__device__ __forceinline__ void doc_tok_body(const uint64_t* __restrict__ doc_off, uint32_t ndocs,
                                             const uint32_t* __restrict__ tok_start,
                                             const uint32_t* __restrict__ counters, uint64_t* __restrict__ doc_tok,
                                             uint32_t g) {
    static_assert(G == 1u || G == 16u, "binary or 16-ary");
    const uint32_t d = g / G, k = threadIdx.x & (G - 1u), gsh = threadIdx.x & (63u & ~(G - 1u));
    if (d > ndocs) return;  // (whole groups: a group is one document)
    const uint32_t n = counters[CNT_NTOK];
    const uint64_t target = doc_off[d];
    uint32_t lo = 0, hi = n;  // the answer is in [lo, hi]
    if constexpr (G == 1u) {
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint64_t)tok_start[mid] < target) lo = mid + 1;
            else hi = mid;
        }
    } else {
        while (lo < hi) {
            const uint32_t s = (hi - lo + 15u) >> 4;  // a sixteenth, rounded up
            const uint32_t i = lo + (k + 1u) * s - 1u;
            const bool before = i < hi && (uint64_t)tok_start[i] < target;
            const uint32_t c = (uint32_t)__popcll((__ballot(before) >> gsh) & 0xFFFFull);
            const uint32_t nlo = lo + c * s;
            if (s == 1u || nlo >= hi) {
                lo = min(nlo, hi);
                break;
            }
            hi = min(hi, nlo + s - 1u);  // (the probe ending the c-th sixteenth is >= target)
            lo = nlo;
        }
    }
    if (k == 0u) doc_tok[d] = lo;
}
template <uint32_t G>
__global__ __launch_bounds__(256) void k_doc_tok(const uint64_t* __restrict__ doc_off, uint32_t ndocs,
                                                 const uint32_t* __restrict__ tok_start,
                                                 const uint32_t* __restrict__ counters, uint64_t* __restrict__ doc_tok) {
    doc_tok_body<G>(doc_off, ndocs, tok_start, counters, doc_tok, blockIdx.x * blockDim.x + threadIdx.x);
}
constexpr uint32_t kDocTokWide = 16384;  // documents from which k_doc_tok searches one lane each

// k_tok1: the span kernels in one pass (round 5): k_tok's count pass, k_sup, its write
// pass and k_doc_tok.  A workgroup takes the next token tile by a ticket (tiles in
// claim order), counts its tokens, publishes the count, and finds its exclusive prefix
// by looking back over the tiles before it (decoupled look-back: a tile's status word is
// its count, flag 1, or its inclusive prefix, flag 2; it waits only on tiles claimed
// before it, so by running workgroups).  Then it writes its spans as k_tok's write pass
// does, and the per-document first tokens of the documents that start in its bytes
// (k_doc_tok's lower bound, here over the tile's own starts in LDS).
// Status: flag << 62 | starts prefix (31 bits) << 31 | ends prefix (31 bits).
__device__ __forceinline__ uint64_t ts_pack(uint32_t f, uint32_t x, uint32_t y) {
    return ((uint64_t)f << 62) | ((uint64_t)x << 31) | (uint64_t)y;
}
__global__ __launch_bounds__(256) void k_tok1(const uint32_t* __restrict__ sbits, const uint32_t* __restrict__ ebits,
                                              uint64_t nwords, uint32_t ntt, uint64_t* __restrict__ tstat,
                                              uint32_t* __restrict__ counters, uint32_t* __restrict__ tok_start,
                                              uint32_t* __restrict__ tok_end, const uint64_t* __restrict__ doc_off,
                                              uint32_t ndocs, uint64_t* __restrict__ doc_tok) {
    constexpr uint32_t W = kTokTileWords / 256u;
    constexpr uint32_t kCap = kTokCap;
    constexpr uint64_t TB = (uint64_t)kTokTileWords * 32u;  // bytes per token tile
    __shared__ uint32_t lds[8];
    __shared__ uint32_t s_t, s_d0;
    __shared__ uint2 s_to;
    __shared__ __attribute__((aligned(16))) uint32_t s_s[kCap + 4], s_e[kCap + 4];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0u) s_t = __hip_atomic_fetch_add(counters + CNT_TOKT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t t = s_t;
    const uint64_t w0 = ((uint64_t)t * 256u + threadIdx.x) * W;
    uint32_t s[W], e[W];
    if (w0 + W <= nwords) {
        const uint2 a = *reinterpret_cast<const uint2*>(sbits + w0);
        const uint2 b = *reinterpret_cast<const uint2*>(ebits + w0);
        s[0] = a.x; s[1] = a.y;
        e[0] = b.x; e[1] = b.y;
    } else {
#pragma unroll
        for (uint32_t k = 0; k < W; k++) {
            s[k] = w0 + k < nwords ? sbits[w0 + k] : 0u;
            e[k] = w0 + k < nwords ? ebits[w0 + k] : 0u;
        }
    }
    // the first document that starts in the tile (or after it): a JB_TOK1_ARY-ary lower bound
    // over doc_off (wave 1, its loads beside the bitmap loads)
#ifndef JB_TOK1_ARY
#define JB_TOK1_ARY 64
#endif
    static_assert(JB_TOK1_ARY == 16 || JB_TOK1_ARY == 64, "k_tok1's search: 16 or 64 lanes");
    if (wave == 1u) {
        constexpr uint32_t AR = JB_TOK1_ARY, SH = AR == 64u ? 6u : 4u;
        const uint64_t target = (uint64_t)t * TB;
        const uint32_t k = lane & (AR - 1u);
        uint32_t lo = 0, hi = ndocs + 1u;  // the answer in [lo, hi]
        while (lo < hi) {
            const uint32_t sx = (hi - lo + AR - 1u) >> SH;
            const uint32_t i = lo + (k + 1u) * sx - 1u;
            const bool before = i < hi && doc_off[i] < target;
            const uint32_t c = (uint32_t)__popcll(__ballot(before) & (AR == 64u ? ~0ull : 0xFFFFull));
            const uint32_t nlo = lo + c * sx;
            if (sx == 1u || nlo >= hi) {
                lo = min(nlo, hi);
                break;
            }
            hi = min(hi, nlo + sx - 1u);
            lo = nlo;
        }
        if (lane == 0u) s_d0 = lo;
    }
    uint32_t cs = 0, ce = 0;
#pragma unroll
    for (uint32_t k = 0; k < W; k++) {
        cs += __popc(s[k]);
        ce += __popc(e[k]);
    }
    uint32_t ts, te;
    const uint32_t xs = block_scan_u32(cs, lds, &ts);
    const uint32_t xe = block_scan_u32(ce, lds, &te);
    // publish the count, then look back (wave 0)
    if (threadIdx.x == 0u)
        __hip_atomic_store(tstat + t, ts_pack(t == 0u ? 2u : 1u, ts, te), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave == 0u) {
        uint32_t px = 0, py = 0;
        for (int64_t base = (int64_t)t - 1; base >= 0;) {
            const int64_t j = base - (int64_t)lane;
            uint64_t v = j >= 0 ? __hip_atomic_load(tstat + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ts_pack(2u, 0u, 0u);
            const uint64_t incl = __ballot((v >> 62) == 2u), ready = __ballot((v >> 62) != 0u);
            // the nearest inclusive prefix, and every tile between ready
            const uint32_t k2 = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
            const uint64_t need = k2 == 64u ? ~0ull : ((2ull << k2) - 1ull);
            if ((ready & need) != need) {
                __builtin_amdgcn_s_sleep(1);
                continue;  // (a tile before is still counting: read again)
            }
            uint32_t x = lane <= k2 ? (uint32_t)(v >> 31) & 0x7FFFFFFFu : 0u;
            uint32_t y = lane <= k2 ? (uint32_t)v & 0x7FFFFFFFu : 0u;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                x += (uint32_t)__shfl_xor((int)x, d, 64);
                y += (uint32_t)__shfl_xor((int)y, d, 64);
            }
            px += x;
            py += y;
            if (k2 < 64u) break;
            base -= 64;
        }
        if (lane == 0u) {
            s_to = make_uint2(px, py);
            if (t > 0u)
                __hip_atomic_store(tstat + t, ts_pack(2u, px + ts, py + te), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    const uint2 to = s_to;
    if (t == ntt - 1u && threadIdx.x == 0) {  // token totals
        counters[CNT_NTOK] = to.x + ts;
        counters[CNT_NTOKE] = to.y + te;
        *reinterpret_cast<uint64_t*>(counters + CNT_NWORDS) = to.x + ts;
    }
    // the spans (k_tok's write pass)
    const bool staged = ts <= kCap && te <= kCap;
    const bool v4 = (((uintptr_t)tok_start | (uintptr_t)tok_end) & 15u) == 0u;
    const uint32_t shs = v4 ? (to.x & 3u) : 0u, she = v4 ? (to.y & 3u) : 0u;
    uint32_t* os = staged ? s_s + shs : tok_start + to.x;
    uint32_t* oe = staged ? s_e + she : tok_end + to.y;
    uint32_t gs = xs, ge = xe;
#pragma unroll
    for (uint32_t k = 0; k < W; k++) {
        const uint32_t base = (uint32_t)((w0 + k) << 5);
        uint32_t m = s[k];
        while (m) {
            os[gs++] = base + (uint32_t)__builtin_ctz(m);
            m &= m - 1;
        }
        m = e[k];
        while (m) {
            oe[ge++] = base + (uint32_t)__builtin_ctz(m) + 1u;
            m &= m - 1;
        }
    }
    __syncthreads();  // (the staged starts, or this workgroup's global ones, for the documents below)
    // the documents that start in the tile (the last tile: all that are left, with the end
    // sentinel d = ndocs): their first token is the first start >= their offset
    {
        const uint32_t d0 = s_d0;
        const uint64_t hiB = t == ntt - 1u ? ~0ull : ((uint64_t)t + 1u) * TB;
        for (uint32_t d = d0 + threadIdx.x; d <= ndocs; d += 256u) {
            const uint64_t o = doc_off[d];
            if (o >= hiB) break;
            const uint32_t* st = staged ? s_s + shs : tok_start + to.x;
            uint32_t lo = 0, hi = ts;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if ((uint64_t)st[mid] < o) lo = mid + 1;
                else hi = mid;
            }
            doc_tok[d] = to.x + lo;
        }
    }
    if (!staged) return;
    if (v4) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        auto out = [&](const uint32_t* a, uint32_t sh, uint32_t n, uint32_t* g) {  // g: output at LDS index 0
            const uint32_t lo = (sh + 3u) & ~3u, hi = (sh + n) & ~3u;  // whole vectors: [lo, hi)
            if (lo < hi) {
                for (uint32_t p = lo + 4u * threadIdx.x; p < hi; p += 1024u)
                    __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(a + p), reinterpret_cast<u32x4*>(g + p));
                if (threadIdx.x < lo - sh) __builtin_nontemporal_store(a[sh + threadIdx.x], g + sh + threadIdx.x);
                if (threadIdx.x < sh + n - hi) __builtin_nontemporal_store(a[hi + threadIdx.x], g + hi + threadIdx.x);
            } else if (threadIdx.x < n) {
                __builtin_nontemporal_store(a[sh + threadIdx.x], g + sh + threadIdx.x);
            }
        };
        out(s_s, shs, ts, tok_start + to.x - shs);
        out(s_e, she, te, tok_end + to.y - she);
        return;
    }
    for (uint32_t k = threadIdx.x; k < ts; k += 256u) __builtin_nontemporal_store(s_s[k], tok_start + to.x + k);
    for (uint32_t k = threadIdx.x; k < te; k += 256u) __builtin_nontemporal_store(s_e[k], tok_end + to.y + k);
}

// ---------------------------------------------------------------------------
// k_long: the long-block kernels above as the phases of one launch (VERDICT r04
// item 5), so that a batch without a long block (CNT_NLONG 0: every batch of
// short documents) pays one launch instead of seven.
// A phase's work items (the separate kernel's workgroups) are claimed from a counter
// (CNT_PHASE + 2 p) by running workgroups, in phase order, and a workgroup adds its
// finished items to CNT_PHASE + 2 p + 1 (after an agent-scope release by every thread)
// and waits until the phase's count is complete (agent-scope atomic loads, then an
// agent-scope acquire: DESIGN §6's rule for inter-workgroup waits).  Since items are
// claimed in phase order, a workgroup only ever waits for items that running
// workgroups hold: the grid need not be resident all at once (another kernel, e.g. a
// second pipeline on the same GPU, may hold CUs), and no grid barrier is used.
// The wait is bounded in time, not in polls: it gives up only when the phase's done
// count has not moved for wait_ticks ticks of the 100 MHz real-time counter
// (JB_LONG_WAIT_US, default 20 s), so one legitimately long item (k_long_dp's chain
// over a very long block) is waited for as long as other items keep finishing.
// A workgroup whose wait gives up sets CNT_ERR bit 1 and leaves the kernel, as does
// every workgroup that then finds the bit set: nothing reads a phase's outputs
// before the phase is complete, and the host reports JB_EDEVICE.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wg_claim(uint32_t* ctr, uint32_t* s_x) {  // (the whole workgroup)
    if (threadIdx.x == 0u) *s_x = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t it = *s_x;
    __syncthreads();
    return it;
}
__device__ __forceinline__ uint32_t wave_claim(uint32_t* ctr) {  // (one wave)
    uint32_t it = 0;
    if ((threadIdx.x & 63u) == 0u) it = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)it);
}
// the end of a phase: every thread's stores released at agent scope, the workgroup's
// finished items (thread 0's count) added, then a wait until all nitems are done and an
// acquire.  Returns false (the workgroup must leave the kernel) when the wait gave up
// (no progress for wait_ticks) or another workgroup's did (CNT_ERR bit 1).
__device__ __forceinline__ bool phase_end(uint32_t* done, uint32_t mine, uint32_t nitems, uint32_t* err,
                                          uint32_t wait_ticks, uint32_t* s_x) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (threadIdx.x == 0u) {
        if (mine) __hip_atomic_fetch_add(done, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t ok = 1u, seen = 0xFFFFFFFFu;
        uint64_t since = 0;
        for (;;) {
            if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2u) {
                ok = 0u;  // a workgroup gave up: leave too (the kernel drains at once)
                break;
            }
            const uint32_t d = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d >= nitems) break;
            const uint64_t now = __builtin_amdgcn_s_memrealtime();  // (100 MHz)
            if (d != seen) {  // progress: the bound starts again
                seen = d;
                since = now;
            } else if (now - since > wait_ticks) {
                __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0u;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        *s_x = ok;
    }
    __syncthreads();
    const bool ok = *s_x != 0u;
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return ok;
}

union LongAll {  // the phases' LDS
    struct {
        double ring[kSpecRing][64];
        uint8_t cd[64][kSeg];
        double wt[kZhWtab];
        double bw[64][kSeg];
    } sp;                             // k_long_spec (wave 0)
    LongLds dp;                       // k_long_dp
    uint32_t m32[kLpBatch * kLpMap / 4u];  // k_long_path (wave 0)
    uint4 cd4[256][kSeg / 16u];       // k_long_pbits, k_long_tail
    uint8_t bl[256][kSeg];            // k_long_seg
    NzLds nz;                         // k_nonzh's windows and chunk lists (k_long<.., true>, before the long phases)
};

template <bool HMM, bool NZ>
__global__ __launch_bounds__(256) void k_long(const uint8_t* __restrict__ text, DevImage im,
                                              const uint64_t* __restrict__ erec, const uint2* __restrict__ longblk,
                                              const uint32_t* __restrict__ lsegb, uint32_t* __restrict__ counters,
                                              const uint32_t* __restrict__ tile4, uint8_t* __restrict__ gbl,
                                              double* __restrict__ gbest, uint8_t* __restrict__ lcode,
                                              uint8_t* __restrict__ lmap, uint8_t* __restrict__ lcx,
                                              uint64_t* __restrict__ lpath, uint32_t* __restrict__ lflag,
                                              uint32_t* __restrict__ sbits, uint32_t* __restrict__ ebits,
                                              uint64_t* __restrict__ dbg, uint32_t spec, NzArgs nz,
                                              uint32_t wait_ticks) {
    __shared__ __attribute__((aligned(16))) LongAll U;
    __shared__ uint32_t s_claim;
    if (NZ) {  // k_nonzh's work first (it needs only k_mark_walk's outputs): one launch less for small batches
        nonzh_body(text, nz.nbytes, nz.lanemask, nz.tile_cnt, nz.ntiles, nz.alnum16, sbits, ebits, nz.docbits,
                   nz.doc_off, nz.ndocs, blockIdx.x, gridDim.x, U.nz);
        __syncthreads();  // (U.nz is the long phases' LDS too)
    }
    const uint32_t nlong = counters[CNT_NLONG], nseg = counters[CNT_NLSEG];  // (k_zh wrote them before this launch)
    if (nlong == 0u) return;
    const bool w0 = threadIdx.x < 64u;  // (the one-wave phases)
    uint32_t* const ph = counters + CNT_PHASE;
    uint32_t* const err = counters + CNT_ERR;
    uint32_t p = 0;  // the phase
    // a phase of nitems items, f(item) on the whole workgroup / on wave 0 only; false:
    // the wait gave up, the workgroup leaves the kernel
    auto wg_phase = [&](uint32_t nitems, auto&& f) {
        uint32_t mine = 0;
        for (uint32_t it; (it = wg_claim(ph + 2u * p, &s_claim)) < nitems; mine++) f(it);
        return phase_end(ph + 2u * p + 1u, mine, nitems, err, wait_ticks, &s_claim) && (++p, true);
    };
    auto wave_phase = [&](uint32_t nitems, auto&& f) {
        uint32_t mine = 0;
        if (w0)
            for (uint32_t it; (it = wave_claim(ph + 2u * p)) < nitems; mine++) f(it);
        return phase_end(ph + 2u * p + 1u, mine, nitems, err, wait_ticks, &s_claim) && (++p, true);
    };
    const uint32_t nsg64 = (nseg + 63u) / 64u, nsg256 = (nseg + 255u) / 256u;
    {
        if (spec) {
            double* const wt = w0 ? long_spec_setup(im, U.sp.wt) : nullptr;
            if (!wave_phase(nsg64, [&](uint32_t it) {
                    long_spec_body(text, im, erec, longblk, lsegb, counters, tile4, gbl, gbest, lcode, lmap, lflag,
                                   spec, it, nsg64, U.sp.ring, U.sp.cd, wt, U.sp.bw);
                }))
                return;
            if (spec != 3u) {
                if (!wave_phase(nlong, [&](uint32_t it) {
                        long_path_body(longblk, lsegb, counters, lflag, lcode, lmap, lcx, 3u, 3u, it, nlong, U.m32);
                    }))
                    return;
                if (!wg_phase(nsg256, [&](uint32_t it) {
                        long_pbits_body(longblk, lsegb, counters, lflag, gbl, lcode, lcx, lpath, it, nsg256, U.cd4);
                    }))
                    return;
            } else {
                p += 2u;
            }
        } else {
            p += 3u;
        }
        if (!wg_phase(nlong, [&](uint32_t it) {
                long_dp_body<HMM>(text, im, erec, gbl, gbest, longblk, counters, sbits, ebits, lflag, lsegb, lpath,
                                  dbg, spec, it, nlong, U.dp);
            }))
            return;
        if (!wg_phase(nsg256, [&](uint32_t it) {
                long_seg_body(text, im, erec, longblk, lsegb, counters, lflag, gbest, gbl, lcode, lmap, it, nsg256,
                              U.bl);
            }))
            return;
        if (!wave_phase(nlong, [&](uint32_t it) {
                long_path_body(longblk, lsegb, counters, lflag, lcode, lmap, lcx, 2u, 1u, it, nlong, U.m32);
            }))
            return;
        // (the Viterbi back-pointers go to gbest's bytes: the exit codes in lcode are read to the end;
        // the last phase: nothing waits for it inside the kernel)
        for (uint32_t it; (it = wg_claim(ph + 2u * p, &s_claim)) < nsg256;)
            long_tail_body<HMM>(text, im, gbl, longblk, lsegb, lflag, counters, lcode, lcx,
                                reinterpret_cast<uint8_t*>(gbest), sbits, ebits, it, nsg256, U.cd4);
    }
}

// Boundary-mask output (jb_cut_batch_mask): a piece's token bitmaps (bit j = byte j
// of the piece, u32 words) into the range's u64 bitmaps at bit offset `rel`, bits
// of other pieces untouched: a word the piece shares with its neighbours (its first
// and last) is ORed in, the others stored.  Pieces of one range run in order on one
// stream over bitmaps cleared at the start.  Counts the piece's token starts and
// ends into the counters (the spans kernels do not run in this mode).
// A pipeline run's counters and summed tile block counts, written straight into
// mapped pinned host memory (cut_range: no copy-engine transfer on the kernels'
// stream, where it would queue behind the bulk copies of later pieces).
// out: u32[kSnapWords]: counters[0..CNT_CLEAR), then u64 blocks, u64 zh blocks.
__global__ __launch_bounds__(256) void k_snap(const uint32_t* __restrict__ counters, const uint2* __restrict__ tile_cnt,
                                              uint32_t ntiles, uint32_t* __restrict__ out) {
    __shared__ unsigned long long red[8];
    unsigned long long b = 0, z = 0;
    for (uint32_t t = threadIdx.x; t < ntiles; t += 256u) {
        const uint2 c = tile_cnt[t];
        b += c.x;
        z += c.y;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        b += (unsigned long long)__shfl_xor((long long)b, d, 64);
        z += (unsigned long long)__shfl_xor((long long)z, d, 64);
    }
    if ((threadIdx.x & 63u) == 0) {
        red[threadIdx.x >> 6] = b;
        red[4 + (threadIdx.x >> 6)] = z;
    }
    __syncthreads();
    if (threadIdx.x < CNT_CLEAR) out[threadIdx.x] = counters[threadIdx.x];
    if (threadIdx.x == 0) {
        const unsigned long long bs = red[0] + red[1] + red[2] + red[3], zs = red[4] + red[5] + red[6] + red[7];
        out[CNT_CLEAR] = (uint32_t)bs;
        out[CNT_CLEAR + 1] = (uint32_t)(bs >> 32);
        out[CNT_CLEAR + 2] = (uint32_t)zs;
        out[CNT_CLEAR + 3] = (uint32_t)(zs >> 32);
    }
    __threadfence_system();
}

// Zero n u32 words (instead of hipMemsetAsync, which may go to the copy engine and
// queue there behind the host pipeline's bulk transfers).
__global__ __launch_bounds__(256) void k_zero(uint32_t* __restrict__ p, uint64_t n, bool v4,
                                             uint32_t* __restrict__ p2, uint32_t n2) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u, t0 = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t0 < n2) p2[t0] = 0u;  // a second, small range (n2 <= 256) in the same launch
    const uint64_t n4 = v4 ? n / 4u : 0u;
    uint4* p4 = reinterpret_cast<uint4*>(p);
    for (uint64_t i = t0; i < n4; i += stride) p4[i] = make_uint4(0u, 0u, 0u, 0u);
    for (uint64_t i = 4u * n4 + t0; i < n; i += stride) p[i] = 0u;
}

hipError_t run_zero(void* p, uint64_t bytes, hipStream_t stream, void* p2, uint32_t bytes2) {
    const uint64_t n = bytes / 4u;  // (callers pass whole words)
    if (!n && !bytes2) return hipSuccess;
    const bool v4 = ((uintptr_t)p & 15u) == 0;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(2048u, (n / 4u + 255u) / 256u + 1u);
    hipLaunchKernelGGL(k_zero, dim3(grid), dim3(256), 0, stream, reinterpret_cast<uint32_t*>(p), n, v4,
                       reinterpret_cast<uint32_t*>(p2), bytes2 / 4u);
    return hipGetLastError();
}

hipError_t run_snap(const Work& w, uint64_t nbytes, uint32_t* out, hipStream_t stream) {
    const uint32_t ntiles = (uint32_t)((nbytes + kTileBytes - 1) / kTileBytes);
    hipLaunchKernelGGL(k_snap, dim3(1), dim3(256), 0, stream, w.counters, w.tile_cnt, ntiles, out);
    return hipGetLastError();
}

// Spans packed for the trip back to the host (jb_cut_batch's spans mode): token i as
// one u16, the gap from the previous token's end (0 for the first) in the low 6 bits and
// its length in the high 10, so the host link carries 2 bytes per token instead of 8 (on
// the C_syn corpus gaps stay under 63 bytes and tokens under 1,023: 0 escapes in 4.36M
// tokens).  A gap of 63 or more or a length of 1,023 or more is written as 0xFFFF, with
// the token's (index, start, end) appended to a side list.  hdr[b] is the end of the token
// before token b x kPackBlock (0 for b = 0), so the host decodes blocks of kPackBlock
// tokens independently.
__global__ __launch_bounds__(256) void k_span_pack(const uint32_t* __restrict__ ts, const uint32_t* __restrict__ te,
                                                   uint32_t* __restrict__ counters, uint16_t* __restrict__ pk,
                                                   uint32_t* __restrict__ hdr, uint4* __restrict__ side,
                                                   uint32_t side_cap) {
    const uint32_t nt = counters[CNT_NWORDS];  // (the u64 token count's low word: a piece has < 2^31 tokens)
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nt; i += gridDim.x * 256u) {
        const uint32_t a = ts[i], b = te[i], p = i ? te[i - 1u] : 0u;
        const uint32_t g = a - p, l = b - a;
        uint32_t x = g | (l << kPackGapBits);
        if (g >= kPackGapEsc || l >= kPackLenEsc) {
            x = 0xFFFFu;
            const uint32_t k = atomicAdd(counters + CNT_SIDE, 1u);
            if (k < side_cap) side[k] = make_uint4(i, a, b, 0u);
            else atomicOr(counters + CNT_ERR, 4u);  // (cannot happen: side_cap bounds the escapes)
        }
        pk[i] = (uint16_t)x;
        if ((i & (kPackBlock - 1u)) == 0u) hdr[i / kPackBlock] = p;
    }
}

hipError_t run_span_pack(const uint32_t* ts, const uint32_t* te, uint32_t* counters, uint16_t* pk, uint32_t* hdr,
                         uint4* side, uint32_t side_cap, uint64_t max_tokens, hipStream_t stream) {
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>(4096u, (max_tokens + 255u) / 256u));
    hipLaunchKernelGGL(k_span_pack, dim3(grid), dim3(256), 0, stream, ts, te, counters, pk, hdr, side, side_cap);
    return hipGetLastError();
}

constexpr uint32_t kMergeWords = 16;  // k_mask_merge: output words per thread
__global__ __launch_bounds__(256) void k_mask_merge(const uint32_t* __restrict__ sbits,
                                                    const uint32_t* __restrict__ ebits, uint64_t n, uint64_t rel,
                                                    uint64_t* __restrict__ ms, uint64_t* __restrict__ me,
                                                    uint32_t* __restrict__ counters) {
    __shared__ uint32_t red[8];
    const uint32_t sh = (uint32_t)(rel & 63u);
    const uint64_t nout = (sh + n + 63u) >> 6, nw32 = (n + 31u) >> 5;
    auto piece64 = [&](const uint32_t* b, int64_t i) -> uint64_t {  // piece bits [64i, 64i + 64)
        if (i < 0) return 0ull;
        const uint64_t lo = 2u * (uint64_t)i, hi = lo + 1u;
        return (lo < nw32 ? (uint64_t)b[lo] : 0ull) | ((hi < nw32 ? (uint64_t)b[hi] : 0ull) << 32);
    };
    uint32_t cs = 0, ce = 0;
    const uint64_t t0 = (uint64_t)blockIdx.x * (256u * kMergeWords) + threadIdx.x;
#pragma unroll 4
    for (uint32_t j = 0; j < kMergeWords; j++) {
        const uint64_t t = t0 + 256u * j;  // (consecutive threads: consecutive words)
        if (t >= nout) break;
        uint64_t os = piece64(sbits, (int64_t)t), oe = piece64(ebits, (int64_t)t);
        if (sh) {
            os = (os << sh) | (piece64(sbits, (int64_t)t - 1) >> (64u - sh));
            oe = (oe << sh) | (piece64(ebits, (int64_t)t - 1) >> (64u - sh));
        }
        const uint64_t w = (rel >> 6) + t;
        if (t == 0 || t == nout - 1u) {
            if (os) atomicOr(reinterpret_cast<unsigned long long*>(ms + w), (unsigned long long)os);
            if (oe) atomicOr(reinterpret_cast<unsigned long long*>(me + w), (unsigned long long)oe);
        } else {
            ms[w] = os;
            me[w] = oe;
        }
        cs += (uint32_t)__popcll(os);
        ce += (uint32_t)__popcll(oe);
    }
    // one set of counter atomics per workgroup (one per wave serialised on three addresses)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        cs += (uint32_t)__shfl_xor((int)cs, d, 64);
        ce += (uint32_t)__shfl_xor((int)ce, d, 64);
    }
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) {
        red[wv] = cs;
        red[4 + wv] = ce;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        cs = red[0] + red[1] + red[2] + red[3];
        ce = red[4] + red[5] + red[6] + red[7];
        if (cs | ce) {
            atomicAdd(counters + CNT_NTOK, cs);
            atomicAdd(counters + CNT_NTOKE, ce);
            atomicAdd(reinterpret_cast<unsigned long long*>(counters + CNT_NWORDS), (unsigned long long)cs);
        }
    }
}

// ---------------------------------------------------------------------------
// k_small: a whole small batch (<= kSmallBytes of text) in one workgroup, for
// single Cut calls (tokenizer.go:151-162; BASELINE config 1).  The eleven-kernel
// pipeline costs a dozen launches for a sentence; here one launch reads the
// text and document offsets straight from the caller's pinned host buffer,
// keeps everything in LDS and writes the spans back into pinned host memory.
// Same rules as the pipeline, in phases separated by barriers:
//   1  text -> LDS; document starts; per lead byte the Go utf8.DecodeRune width
//      (bounded by the document end) and Han-ness (zh regex, :21)
//   2  rune starts (bytes no valid sequence covers), block starts (document
//      starts and changes of Han-ness: splitText, :154-155,165-210)
//   3  the Han runes and the blocks in text order (workgroup scans)
//   4  per Han rune (one thread each): dense code and emissions -> LDS
//   5  per Han rune: its trie walk (buildDag, :462-497) -> up to 4 edges
//      (length, end byte, weight) in LDS; more edges: the DP walks it again
//   6  per block (one thread each): Han blocks get the backward DP
//      (calcDagProba + maxIndexProba, :502-578), the forward path (findDagPath,
//      :552-562) and the Viterbi of single-rune runs (:228-253,668-756), all
//      from LDS; other blocks get cutNonZh (:289-310)
//   7  token bitmaps -> spans, per-document first tokens, counters
// ---------------------------------------------------------------------------
constexpr uint32_t kSmallSlots = kSmallBytes / 3u + 2u;
constexpr uint32_t kSmZero = kSmallSlots - 1u;  // (Han ordinals are < kSmallBytes / 3 + 1)
constexpr uint32_t kSmM1 = 0x8000u;
constexpr uint32_t kSmallWords = kSmallBytes / 32u + 2u;

struct SmallLds {
    alignas(16) uint8_t txt[kSmallBytes + 128];
    uint8_t wd[kSmallBytes + 16];  // per byte: DecodeRune width at a lead byte (1 otherwise)
    uint32_t docb[kSmallWords];    // document starts
    uint32_t rsb[kSmallWords];     // rune starts
    uint32_t hsb[kSmallWords];     // Han rune starts
    uint32_t bsb[kSmallWords];     // block starts
    uint32_t sb[kSmallWords];      // token first bytes
    uint32_t eb[kSmallWords];      // token last bytes
    uint32_t swp[kSmallWords];     // token starts before each word
    uint32_t scan[16];
    uint64_t clk[22];  // phase clocks of thread 0 (JB_DEBUG): 0..15 realtime, 16..18 shader cycles of the last run,
                       // 19..21 shader cycles of the last DP (descriptors read, loop entered, done)
    uint32_t nh, nblk, nzh, err, ties;
    uint16_t doff[kSmallDocs + 1];  // document offsets
    uint16_t hpos[kSmallSlots];     // Han rune starts, text order
    uint16_t blist[kSmallBytes + 2];  // block starts, text order
    // per Han rune, at slot = byte / 3 (Han runes are >= 3 bytes)
    uint32_t scode[kSmallSlots];  // dense rune code, at slot = byte / 3 (Han runes are >= 3 bytes)
    uint16_t hord[kSmallSlots];   // Han ordinal, at the slot
    // per Han rune, by ordinal h (the runes of a block have consecutive ordinals)
    uint32_t rlw[kSmallSlots];       // DAG edge lengths, a byte each, ascending (0: none); 0xFF: more than 4
    alignas(16) double rw[kSmallSlots][4];  // their weights (pieceFreq, :511-519); NaN past the last
    alignas(8) uint16_t ra[kSmallSlots][4];  // byte offset in sbest of best(h + L) per item (kSmZero's at the block's end);
                                             // item 0's bit 15 (kSmM1): L = 1 inside the block (the chain's register)
    uint32_t slowb[kSmallSlots / 32u + 1u];  // by the ordinal of a block's first Han rune: the block needs the literal fold
    double sbest[kSmallSlots];       // (index kSmZero holds 0.0: best(n), :522-525)
    uint8_t sL[kSmallSlots];         // chosen piece length (0: none, the reference panics)
    uint8_t sbl[kSmallSlots];        // Viterbi labels (traceback)
    uint8_t bp4[kSmallSlots][4];     // Viterbi back-pointer of each state (quad lane = state)
    alignas(16) double sem[kSmallSlots][4];  // emissions B, M, E, S
};
static_assert(sizeof(SmallLds) <= 163840u, "k_small: one workgroup's LDS");

struct SmlZv {  // text and slots in LDS (viterbi_back, z_prev)
    static constexpr bool all3 = false;
    const uint8_t* tx;
    uint8_t* bls;
    __device__ __forceinline__ uint32_t b(uint32_t q) const { return tx[q]; }
    __device__ __forceinline__ uint32_t x4(uint32_t q) const { return lds4(tx, q); }
    __device__ __forceinline__ uint8_t& bl(uint32_t q) const { return bls[q / 3u]; }
};

__device__ __forceinline__ bool sm_bit(const uint32_t* b, uint32_t p) { return (b[p >> 5] >> (p & 31u)) & 1u; }

// The trie walk from the Han rune at p (dp_walk_rune's rules, :462-497): f(L, end
// byte, weight) for each DAG edge in ascending L.  The walk goes on while the
// next rune is a Han rune of the same block.
template <class F>
__device__ __forceinline__ void sm_walk(const SmallLds& s, const DevImage& im, uint32_t p, F&& f) {
    uint32_t id = s.scode[p / 3u];
    uint64_t cc = im.cells[id];
    const uint32_t w0 = s.wd[p];
    if (jb_cell_check(cc) != JB_CHECK_ROOT) {  // not a key: the rune alone, tf 1.0 (:468-471,515-518)
        f(1u, p + w0, im.wtab[JB_WIDX_ABSENT]);
        return;
    }
    if (jb_cell_fc(cc) == JB_FC_ZERO) {  // count == 0: the rune alone, Log(0) (:468-471)
        f(1u, p + w0, im.wtab[jb_cell_widx(cc)]);
        return;
    }
    if (jb_cell_fc(cc) == JB_FC_POS) f(1u, p + w0, im.wtab[jb_cell_widx(cc)]);
    uint32_t qq = p + w0, len = 1;
    bool go = jb_cell_hc(cc) != 0u;
    while (go && sm_bit(s.hsb, qq) && !sm_bit(s.bsb, qq)) {
        const uint32_t tt = dat_slot_k(cc, s.scode[qq / 3u]);
        const uint64_t ch = im.cells[tt];
        if (!dat_hit(ch, id)) break;  // (:475-478)
        ++len;
        qq += s.wd[qq];
        if (jb_cell_fc(ch) == JB_FC_POS) f(len, qq, im.wtab[jb_cell_widx(ch)]);
        go = jb_cell_hc(ch) != 0u;
        id = tt;
        cc = ch;
    }
}

// A float64 from another lane of the quad (DPP quad_perm; ctrl = src lane of lanes 0..3, 2 bits each)
template <int CTRL>
__device__ __forceinline__ double quad_perm_f64(double x) {
    const long long i = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)i, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(i >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// viterbi_run (:668-756) + viterbi_back + cutHMM (:273-285) for the m runes with
// ordinals [ha, ha + m) ending at byte re, by the four lanes of a quad: lane s holds
// state s (B, M, E, S: HMMstates order, :685) and takes its two candidates
// (stateChange, :24-29) from the other lanes with DPP, so a rune is one short
// chain instead of four serial routes.  Lane 0 then runs the traceback and emits.
template <class E>
__device__ void sm_viterbi(SmallLds& s, uint32_t ha, uint32_t re, uint32_t m, E& em, uint32_t ql,
                           uint64_t* xc = nullptr) {
    const uint32_t rs = s.hpos[ha];
    if (m == 1) {  // always "S" for a single rune (:672-674)
        if (ql == 0) em.token(rs, re);
        return;
    }
    // B <- (E, S), M <- (B, M), E <- (B, M), S <- (E, S)
    const double ta = ql == 0 ? T_EB : (ql == 1 ? T_BM : (ql == 2 ? T_BE : T_ES));
    const double tb = ql == 0 ? T_SB : (ql == 1 ? T_MM : (ql == 2 ? T_ME : T_SS));
    double vv = (ql == 0 ? START_B : (ql == 3 ? START_S : JB_MIN_FLOAT)) + s.sem[ha][ql];
    double en = s.sem[ha + 1u][ql];
    uint32_t nt = 0;
    for (uint32_t h = ha + 1u; h < ha + m; h++) {
        const double enn = s.sem[h + 1u][ql];  // (past the run: a harmless read)
        const double a = quad_perm_f64<2 | (0 << 2) | (0 << 4) | (2 << 6)>(vv) + ta;
        const double b = quad_perm_f64<3 | (1 << 2) | (1 << 4) | (3 << 6)>(vv) + tb;
        // stateTransitionRoute (:736-756): strict '>' against minFloat, code 2 = no route
        uint32_t c = 2u;
        double best = JB_MIN_FLOAT;
        if (a > best) { c = 0u; best = a; }
        if (b > best) { c = 1u; best = b; }
        nt += (a == b && a > JB_MIN_FLOAT) ? 1u : 0u;
        vv = best + en;
        s.bp4[h][ql] = (uint8_t)c;
        en = enn;
    }
    em.ties += nt;
    const double vE = quad_perm_f64<0xAA>(vv), vS = quad_perm_f64<0xFF>(vv);
    if (xc) xc[1] = __builtin_amdgcn_s_memtime();  // (JB_DEBUG sub-phase clocks: forward half done)
    if (ql != 0) return;
    // traceback (:715-729): stops at the first "" route, and cutHMM then labels the
    // runes from the run start (viterbi_back)
    uint32_t st = vE > vS ? (uint32_t)JB_E : (uint32_t)JB_S, t = m - 1u, reset = 0, h = ha + m - 1u;
    for (;;) {
        if (t == 0) {
            s.sbl[h] = (uint8_t)st;
            break;
        }
        const uint32_t code = s.bp4[h][st];
        s.sbl[h] = (uint8_t)st;
        if (code == 2u) {
            reset = t;
            break;
        }
        st = (st == JB_B || st == JB_S) ? 2u + code : code;  // B,S <- {E,S}; M,E <- {B,M}
        --t;
        --h;
    }
    if (xc) xc[2] = __builtin_amdgcn_s_memtime();  // (traceback done)
    uint32_t ts = rs;
    for (uint32_t k = 0; k < m - reset; k++) {
        const uint32_t lab = s.sbl[h + k];
        const uint32_t qa = ha + k + 1u < ha + m ? s.hpos[ha + k + 1u] : re;  // end of rune k
        if (lab >= (uint32_t)JB_E) {
            em.token(ts, qa);
            ts = qa;
        }
    }
}

// The end of a run's viterbi (:723-729) + traceback + cutHMM, after its forward half
// ran inside the fused forward walk (k_small): vv is lane ql's value of state ql at the
// run's last rune; the run is ordinals [ha, ha + m), ending at byte re.
template <class E>
__device__ void sm_vit_finish(SmallLds& s, uint32_t ha, uint32_t re, uint32_t m, double vv, E& em, uint32_t ql,
                              uint64_t* xc) {
    const uint32_t rs = s.hpos[ha];
    if (m == 1) {  // always "S" for a single rune (:672-674)
        if (ql == 0) em.token(rs, re);
        return;
    }
    const double vE = quad_perm_f64<0xAA>(vv), vS = quad_perm_f64<0xFF>(vv);
    if (xc) xc[1] = __builtin_amdgcn_s_memtime();
    if (ql != 0) return;
    // traceback (:715-729): stops at the first "" route, and cutHMM then labels the
    // runes from the run start (viterbi_back)
    uint32_t st = vE > vS ? (uint32_t)JB_E : (uint32_t)JB_S, t = m - 1u, reset = 0, h = ha + m - 1u;
    for (;;) {
        if (t == 0) {
            s.sbl[h] = (uint8_t)st;
            break;
        }
        const uint32_t code = s.bp4[h][st];
        s.sbl[h] = (uint8_t)st;
        if (code == 2u) {
            reset = t;
            break;
        }
        st = (st == JB_B || st == JB_S) ? 2u + code : code;  // B,S <- {E,S}; M,E <- {B,M}
        --t;
        --h;
    }
    if (xc) xc[2] = __builtin_amdgcn_s_memtime();
    uint32_t ts = rs;
    for (uint32_t k = 0; k < m - reset; k++) {
        const uint32_t lab = s.sbl[h + k];
        const uint32_t qa = ha + k + 1u < ha + m ? s.hpos[ha + k + 1u] : re;  // end of rune k
        if (lab >= (uint32_t)JB_E) {
            em.token(ts, qa);
            ts = qa;
        }
    }
}

// cutNonZh for the block [bs, be) from LDS (nonzh_block's rules, :289-310), four
// bytes per LDS read
template <class E>
__device__ void sm_nonzh(const uint8_t* tx, uint32_t bs, uint32_t be, E& em) {
    bool has = false;  // alnum.FindAllIndex found nothing -> no tokens (:290-293)
    for (uint32_t a = bs & ~3u; a < be && !has; a += 16u) {
#pragma unroll
        for (uint32_t k = 0; k < 4u; k++) {
            const uint32_t b = a + 4u * k;
            has |= jb_any_alnum4(*reinterpret_cast<const uint32_t*>(tx + b) & nz_keep(b, bs, be));
        }
    }
    if (!has) return;
    uint32_t p = bs, run = 0;
    bool in_run = false;
    while (p < be) {
        const uint32_t x = lds4(tx, p);
        if (jb_is_alnum(x & 0xFFu)) {  // alnum runs are kept whole
            if (!in_run) {
                in_run = true;
                run = p;
            }
            // the run's bytes of this word: the leading alnum bytes of x
            uint32_t k = 1;
            while (k < 4u && p + k < be && jb_is_alnum((x >> (8u * k)) & 0xFFu)) k++;
            p += k;
            continue;
        }
        if (in_run) {
            em.token(run, p);
            in_run = false;
        }
        uint32_t r;
        const uint32_t w = jb_decode(x, min(4u, be - p), &r);
        if (!jb_is_space(r)) em.token(p, p + w);  // one token per rune; spaces dropped
        p += w;
    }
    if (in_run) em.token(run, be);
}

// out: u32 header[kSmallHdr] (SM_*), then tok_start[kSmallBytes], tok_end[kSmallBytes],
// then doc_tok u64[ndocs + 1].  text is readable 16 bytes past nbytes.  Up to 1024
// threads, 4 bytes each in the byte phases (16 bytes each ran every phase as one long
// dependent instruction chain per wave); a batch gets as many waves as its bytes need.
constexpr uint32_t kSmallThreads = 1024;
static_assert(kSmallBytes / kSmallThreads == 4u, "4 bytes per thread at most in the byte phases");
constexpr uint32_t kSmallOneByte = 64;  // a batch up to this many bytes: one wave, one byte per lane

// PER: bytes per thread in the byte phases (a thread's bytes are one PER-bit field of a
// 32-bit bitmap word): 4, or 1 for a batch of at most kSmallOneByte bytes, whose one
// wave then runs every byte phase as one step instead of a loop of four (a sentence's
// widths phase took 1.6 us as four dependent rounds of LDS reads)
template <bool HMM, uint32_t PER>
__global__ __launch_bounds__(kSmallThreads) void k_small(const uint8_t* __restrict__ text, uint32_t nbytes,
                                                         const uint64_t* __restrict__ doc_off, uint32_t ndocs,
                                                         DevImage im, uint32_t* __restrict__ out, uint32_t seq,
                                                         SmallInline in) {
    __shared__ SmallLds s;
    const uint32_t t = threadIdx.x;
    const uint32_t nw = (nbytes + 31u) / 32u;
    uint64_t* const clk = s.clk;  // phase clocks (100 MHz), thread 0: header words SM_CLK.. (in LDS: no registers)
    uint64_t* const xc = s.clk + 16;  // sub-phase shader clocks of the last run (thread 0): header words 24..26
    uint64_t cyc0 = 0;
    if (t == 0) {
        clk[0] = __builtin_amdgcn_s_memrealtime();
        cyc0 = __builtin_amdgcn_s_memtime();
        xc[0] = xc[1] = xc[2] = xc[3] = xc[4] = xc[5] = 0;
    }
    const uint32_t nt = blockDim.x;  // a multiple of 64 with 4 * nt >= nbytes (run_small)
    // 1. text (zero past nbytes, up to 64 bytes on) and document offsets -> LDS (one
    // round trip), bitmaps cleared
    const uint8_t* const src = text ? text : in.txt;  // (inline: zero-padded by the host)
    for (uint32_t i = t; i < min((kSmallBytes + 128u) / 16u, (nbytes + 79u) / 16u); i += nt) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (16u * i < nbytes) {
            v = *reinterpret_cast<const uint4*>(src + 16u * i);
            uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t b = 16u * i + 4u * (uint32_t)k;
                if (b + 4u > nbytes) w[k] = b >= nbytes ? 0u : w[k] & ((1u << (8u * (nbytes - b))) - 1u);
            }
        }
        *reinterpret_cast<uint4*>(s.txt + 16u * i) = v;
    }
    for (uint32_t d = t; d <= ndocs; d += nt)
        s.doff[d] = doc_off ? (uint16_t)min(doc_off[d], (uint64_t)nbytes) : in.doff[d];
    for (uint32_t i = t; i < kSmallWords; i += nt) s.docb[i] = s.rsb[i] = s.hsb[i] = s.bsb[i] = s.sb[i] = s.eb[i] = 0u;
    for (uint32_t i = t; i < kSmallSlots / 32u + 1u; i += nt) s.slowb[i] = 0u;
    if (t == 0) s.err = s.ties = s.nzh = 0u;
    __syncthreads();
    if (t == 0) clk[1] = __builtin_amdgcn_s_memrealtime();
    for (uint32_t d = t; d < ndocs; d += nt) {
        const uint32_t o = s.doff[d];
        if (o < nbytes) atomicOr(&s.docb[o >> 5], 1u << (o & 31u));
    }
    __syncthreads();
    if (t == 0) clk[2] = __builtin_amdgcn_s_memrealtime();
    // widths at lead bytes: thread t owns bytes [4t, 4t + 4)
    static_assert(PER == 1u || PER == 4u, "PER bytes per thread");
    const uint32_t p0 = PER * t, sh = p0 & 31u;
    uint32_t hanm = 0;  // Han lead bytes of the thread's 4
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint32_t p = p0 + k;
        uint32_t w = 1;
        if (p < nbytes && s.txt[p] >= 0xC0u) {
            // bounded by the document end: the first document start in p+1 .. p+3
            const uint32_t nx = (uint32_t)(((((uint64_t)s.docb[(p >> 5) + 1u] << 32) | s.docb[p >> 5]) >> (p & 31u)) >> 1);
            const uint32_t lim = min(min(4u, nbytes - p), nx ? (uint32_t)__builtin_ctz(nx) + 1u : 4u);
            uint32_t r;
            w = dec_lead(lds4(s.txt, p), lim, &r);
            if (w >= 3u && han_cp(r)) hanm |= 1u << k;
        }
        s.wd[p] = (uint8_t)w;
    }
    __syncthreads();
    if (t == 0) clk[3] = __builtin_amdgcn_s_memrealtime();
    // 2. rune starts: bytes that no valid sequence of the 3 bytes before covers
    uint32_t rs4 = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint32_t p = p0 + k;
        const bool cov = (p >= 1u && s.wd[p - 1u] >= 2u) || (p >= 2u && s.wd[p - 2u] >= 3u) ||
                         (p >= 3u && s.wd[p - 3u] >= 4u);
        if (p < nbytes && !cov) rs4 |= 1u << k;
    }
    if (rs4) atomicOr(&s.rsb[p0 >> 5], rs4 << sh);
    if (hanm) atomicOr(&s.hsb[p0 >> 5], hanm << sh);
    __syncthreads();
    if (t == 0) clk[4] = __builtin_amdgcn_s_memrealtime();
    uint32_t bs4 = 0;
    for (uint32_t m = rs4; m; m &= m - 1u) {
        const uint32_t k = (uint32_t)__builtin_ctz(m), p = p0 + k;
        bool st = p == 0u || sm_bit(s.docb, p);
        if (!st) {  // Han-ness of the previous rune (it starts at most 4 bytes back)
            uint32_t q = p - 1u;
            while (!sm_bit(s.rsb, q)) q--;
            st = sm_bit(s.hsb, q) != ((hanm >> k) & 1u);
        }
        if (st) bs4 |= 1u << k;
    }
    if (bs4) atomicOr(&s.bsb[p0 >> 5], bs4 << sh);
    // 3. Han runes and blocks in text order: one scan of both counts (Han runes in
    // the low half: at most kSmallSlots; blocks in the high half: at most kSmallBytes)
    {
        uint32_t tot;
        const uint32_t x = block_scan_u32((uint32_t)__popc(hanm) | ((uint32_t)__popc(bs4) << 16), s.scan, &tot);
        uint32_t i = x & 0xFFFFu;
        for (uint32_t m = hanm; m; m &= m - 1u) {
            const uint32_t p = p0 + (uint32_t)__builtin_ctz(m);
            s.hord[p / 3u] = (uint16_t)i;
            s.hpos[i++] = (uint16_t)p;
        }
        i = x >> 16;
        uint32_t nz = 0;
        for (uint32_t m = bs4; m; m &= m - 1u) {
            const uint32_t k = (uint32_t)__builtin_ctz(m);
            s.blist[i++] = (uint16_t)(p0 + k);
            nz += (hanm >> k) & 1u;
        }
        if (nz) atomicAdd(&s.nzh, nz);
        if (t == 0) {
            s.nh = tot & 0xFFFFu;
            s.nblk = tot >> 16;
        }
    }
    __syncthreads();
    if (t == 0) clk[5] = __builtin_amdgcn_s_memrealtime();
    const uint32_t nh = s.nh, nblk = s.nblk;
    // 4. codes (and emissions) of the Han runes
    for (uint32_t h = t; h < nh; h += nt) {
        const uint32_t p = s.hpos[h];
        uint32_t r;
        (void)dec_lead(lds4(s.txt, p), 4u, &r);
        const uint32_t row = jb_row(im.pagemap, r);
        s.scode[p / 3u] = im.code[row];
        if (HMM) {
            const double2* ep = reinterpret_cast<const double2*>(im.emit) + (size_t)row * 2u;
            const double2 a = ep[0], b = ep[1];
            double* e = s.sem[h];
            e[0] = a.x; e[1] = a.y; e[2] = b.x; e[3] = b.y;
        }
    }
    __syncthreads();
    if (t == 0) clk[6] = __builtin_amdgcn_s_memrealtime();
    // 5. DAG edges of every Han rune, and the DP step's descriptor: weights (NaN for
    // absent items), where each item's best(h + L) is, and whether item 0 takes
    // best(h + 1) from the chain's register
    if (t == 0) s.sbest[kSmZero] = 0.0;
    for (uint32_t h = t; h < nh; h += nt) {
        const uint32_t p = s.hpos[h];
        uint32_t n = 0, lw = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            s.rw[h][k] = __builtin_nan("");
            s.ra[h][k] = (uint16_t)(kSmZero * 8u);
        }
        sm_walk(s, im, p, [&](uint32_t L, uint32_t qe, double w) {
            if (n < 4u) {
                lw |= L << (8u * n);
                s.rw[h][n] = w;
                // the piece ends at the block's end unless a Han rune of the same block starts at qe
                const bool inside = sm_bit(s.hsb, qe) && !sm_bit(s.bsb, qe);
                s.ra[h][n] = (uint16_t)((inside ? h + L : kSmZero) * 8u | (n == 0u && L == 1u && inside ? kSmM1 : 0u));
            }
            n++;
        });
        s.rlw[h] = n <= 4u ? lw : 0xFFu;
        if (n > 4u || n == 0u || !im.plainw) {  // (no item: the reference panics later)
            // the literal fold for this rune's block: its bit at the block's first Han rune
            uint32_t w = p >> 5, m = s.bsb[w] & (0xFFFFFFFFu >> (31u - (p & 31u)));
            while (!m) m = s.bsb[--w];
            const uint32_t h0 = s.hord[(32u * w + 31u - (uint32_t)__builtin_clz(m)) / 3u];
            atomicOr(&s.slowb[h0 >> 5], 1u << (h0 & 31u));
        }
    }
    __syncthreads();
    if (t == 0) clk[7] = __builtin_amdgcn_s_memrealtime();
    // 6. blocks, one quad of lanes each (the Viterbi takes all four; the rest is
    // run alike by the four lanes and written by lane 0)
    LdsEmitter em(s.sb, s.eb, 0u);
    const uint32_t ql = t & 3u;
    const SmlZv v{s.txt, s.sbl};  // (z_prev only)
    if (t == 0) clk[12] = clk[13] = clk[14] = 0;
    if (t == 0) clk[15] = __builtin_amdgcn_s_memrealtime();
    for (uint32_t k = t >> 2; k < nblk; k += nt / 4u) {
        const uint32_t bs = s.blist[k], be = k + 1u < nblk ? s.blist[k + 1u] : nbytes;
        if (!sm_bit(s.hsb, bs)) {
            if (ql == 0) sm_nonzh(s.txt, bs, be, em);
            continue;
        }
        // backward DP (calcDagProba, :502-548) over the block's runes, ordinals [h0, h1):
        // best(h) from best(h + L), best(h1) = 0.0.  A step is the chain of item 0's sum
        // (best(h + 1) from a register, or its LDS value) into the closed fold below; the
        // next rune's descriptor was read a step earlier and its best(h + L >= 2) values
        // are read at the start of this step (they were written by the steps before:
        // a wave's LDS accesses complete in order), so no LDS round trip is on the chain.
        const uint32_t h0 = s.hord[bs / 3u], h1 = s.hord[z_prev(v, be, bs) / 3u] + 1u;
        uint32_t h = h1 - 1u;
        if (t == 0) xc[3] = __builtin_amdgcn_s_memtime();
        if (!((s.slowb[h0 >> 5] >> (h0 & 31u)) & 1u)) {
            // Up to 4 items per rune without a branch: an absent item has a NaN weight, so
            // its sum is NaN and no compare takes it.  With finite or -Inf weights (plainw)
            // the reference's "last item k with p_k >= p_(k-1)" (p_0 = minFloat; none: the
            // last item) is then p3 if p3 >= p2, else p2 if p2 >= p1, else p1 if p1 >= p0,
            // else p0 (the first item alone, or -Inf).  The selects are v_bfi_b32 on masks
            // (bitsel64: as ternaries the compiler made branches of them), and the register
            // sets of three consecutive runes rotate by unrolling, not by copies.
            struct Rn {
                double w0, w1, w2, w3, b0, b1, b2, b3;
                uint32_t ra0, ra1, lw;
            };
            auto load_desc = [&](Rn& r, uint32_t i) {
                const double4 w = *reinterpret_cast<const double4*>(s.rw[i]);
                r.w0 = w.x; r.w1 = w.y; r.w2 = w.z; r.w3 = w.w;
                const uint2 a = *reinterpret_cast<const uint2*>(s.ra[i]);
                r.ra0 = a.x;
                r.ra1 = a.y;
                r.lw = s.rlw[i];
            };
            auto load_b = [&](Rn& r) {  // (item 0's L = 1 value is the chain's register)
                const char* const sb = reinterpret_cast<const char*>(s.sbest);
                r.b0 = *reinterpret_cast<const double*>(sb + (r.ra0 & 0x7FFFu));
                r.b1 = *reinterpret_cast<const double*>(sb + (r.ra0 >> 16));
                r.b2 = *reinterpret_cast<const double*>(sb + (r.ra1 & 0xFFFFu));
                r.b3 = *reinterpret_cast<const double*>(sb + (r.ra1 >> 16));
            };
            auto fold = [&](const Rn& r, uint32_t hh, double bnx) {
                const uint32_t m1 = (r.ra0 & kSmM1) ? ~0u : 0u;
                const double p0 = r.w0 + bitsel64(m1, bnx, r.b0);  // pieceProba (:519-529)
                const double p1 = r.w1 + r.b1, p2 = r.w2 + r.b2, p3 = r.w3 + r.b3;
                const uint32_t k3 = p3 >= p2 ? ~0u : 0u, k2 = p2 >= p1 ? ~0u : 0u, k1 = p1 >= p0 ? ~0u : 0u;
                const uint32_t kh = k3 | k2;
                const double best = bitsel64(kh, bitsel64(k3, p3, p2), bitsel64(k1, p1, p0));
                const uint32_t sh = (kh & k3 & 24u) | (kh & ~k3 & 16u) | (~kh & k1 & 8u);  // 8 x the item's index
                s.sbest[hh] = best;
                s.sL[hh] = (uint8_t)(r.lw >> sh);
                return best;
            };
            auto clampd = [&](uint32_t i, uint32_t d) { return i >= h0 + d ? i - d : h0; };
            Rn A, B, C;
            load_desc(A, h);
            load_b(A);
            load_desc(B, clampd(h, 1u));
            double bnx = 0.0;
            if (t == 0) xc[4] = __builtin_amdgcn_s_memtime();
            for (;;) {
                load_b(B);  // rune h - 1's best(h - 1 + L >= 2): written by the steps before
                load_desc(C, clampd(h, 2u));
                bnx = fold(A, h, bnx);
                if (h == h0) break;
                --h;
                load_b(C);
                load_desc(A, clampd(h, 2u));
                bnx = fold(B, h, bnx);
                if (h == h0) break;
                --h;
                load_b(A);
                load_desc(B, clampd(h, 2u));
                bnx = fold(C, h, bnx);
                if (h == h0) break;
                --h;
            }
        } else {
            // a rune with more than 4 edges (walked again), none, or +Inf/NaN weights: the
            // literal rule of maxIndexProba (:565-578) over the block, from LDS
            for (double bnx = 0.0;; --h) {
                double prevP = JB_MIN_FLOAT, bestP = JB_MIN_FLOAT;
                uint32_t bestL = 0, lastL = 0;
                auto item = [&](uint32_t L, double w) {
                    const double pp = w + (h + L == h1 ? 0.0 : (L == 1u ? bnx : s.sbest[h + L]));  // (:519-529)
                    const bool take = pp >= prevP;
                    bestL = take ? L : bestL;
                    bestP = take ? pp : bestP;
                    prevP = pp;
                    lastL = L;
                };
                const uint32_t lw = s.rlw[h];
                if (lw == 0xFFu) {
                    sm_walk(s, im, s.hpos[h], [&](uint32_t L, uint32_t, double w) { item(L, w); });
                } else {
                    const uint32_t L0 = lw & 0xFFu, L1 = (lw >> 8) & 0xFFu, L2 = (lw >> 16) & 0xFFu, L3 = lw >> 24;
                    if (L0) item(L0, s.rw[h][0]);
                    if (L1) item(L1, s.rw[h][1]);
                    if (L2) item(L2, s.rw[h][2]);
                    if (L3) item(L3, s.rw[h][3]);
                }
                if (bestL == 0) {  // no item qualified: the last item (or none: tail -1)
                    bestL = lastL;
                    bestP = prevP;
                }
                s.sbest[h] = bestP;
                s.sL[h] = (uint8_t)bestL;
                bnx = bestP;
                if (h == h0) break;
            }
        }
        if (t == 0) {
            xc[5] = __builtin_amdgcn_s_memtime();
            clk[12] = __builtin_amdgcn_s_memrealtime();
        }
#ifndef JB_SM_FUSED
#define JB_SM_FUSED 1
#endif
#if JB_SM_FUSED
        // forward path (findDagPath, :552-562) fused with the forward half of each HMM
        // run's viterbi (cutZh, :221-255; viterbi, :668-730): a single-rune piece is one
        // Viterbi step of the run it extends (lane ql of the quad holds state ql and takes
        // its two candidates from the other lanes by DPP).  The next piece's length, start
        // and emission are read a piece ahead, during this piece's step.
        bool ok = true;
        {
            // B <- (E, S), M <- (B, M), E <- (B, M), S <- (E, S)
            const double ta = ql == 0 ? T_EB : (ql == 1 ? T_BM : (ql == 2 ? T_BE : T_ES));
            const double tb = ql == 0 ? T_SB : (ql == 1 ? T_MM : (ql == 2 ? T_ME : T_SS));
            const double st0 = ql == 0 ? START_B : (ql == 3 ? START_S : JB_MIN_FLOAT);
            auto rd = [&](uint32_t i) { return min(i, kSmallSlots - 1u); };  // (reads past the block: unused)
            uint32_t nt = 0;
            h = h0;
            uint32_t L = s.sL[h];
            while (h < h1) {
                if (L == 0) {  // tail index -1: cutDAG's slice panics in the reference
                    ok = false;
                    break;
                }
                if (HMM && L == 1u) {
                    // a run of single-rune pieces from h: its viterbi's forward half rune by rune,
                    // the next rune's emission and piece length read a step ahead into register
                    // sets that alternate (nothing copied out of a load's destination)
                    const uint32_t ha = h;
                    double vv = st0 + s.sem[h][ql];
                    double ea = s.sem[rd(h + 1u)][ql], eb = 0.0;
                    uint32_t La = s.sL[rd(h + 1u)], Lb = 0, Lx;
                    auto vstep = [&](double e) {  // rune h + 1
                        const double a = quad_perm_f64<2 | (0 << 2) | (0 << 4) | (2 << 6)>(vv) + ta;
                        const double b = quad_perm_f64<3 | (1 << 2) | (1 << 4) | (3 << 6)>(vv) + tb;
                        // stateTransitionRoute (:736-756): strict '>' against minFloat, code 2 = no route
                        uint32_t c = 2u;
                        double best = JB_MIN_FLOAT;
                        if (a > best) { c = 0u; best = a; }
                        if (b > best) { c = 1u; best = b; }
                        nt += (a == b && a > JB_MIN_FLOAT) ? 1u : 0u;
                        vv = best + e;
                        s.bp4[h + 1u][ql] = (uint8_t)c;
                    };
                    for (;;) {
                        if (h + 1u >= h1 || La != 1u) {
                            Lx = La;
                            break;
                        }
                        eb = s.sem[rd(h + 2u)][ql];
                        Lb = s.sL[rd(h + 2u)];
                        vstep(ea);
                        ++h;
                        if (h + 1u >= h1 || Lb != 1u) {
                            Lx = Lb;
                            break;
                        }
                        ea = s.sem[rd(h + 2u)][ql];
                        La = s.sL[rd(h + 2u)];
                        vstep(eb);
                        ++h;
                    }
                    ++h;  // the run is [ha, h)
                    const uint32_t re = h < h1 ? s.hpos[h] : be;
                    if (t == 0) xc[0] = __builtin_amdgcn_s_memtime();  // (JB_DEBUG: the last run's forward half done)
                    sm_vit_finish(s, ha, re, h - ha, vv, em, ql, t == 0 ? xc : nullptr);
                    L = Lx;
                    continue;
                }
                const uint32_t hn = h + L, p = s.hpos[h];
                const uint32_t pn = hn < h1 ? s.hpos[hn] : be;
                const uint32_t Ln = s.sL[rd(hn)];
                if (ql == 0) em.token(p, pn);
                h = hn;
                L = Ln;
            }
            em.ties += nt;
        }
        if (!ok) {
            if (ql == 0) s.err = 1u;
            continue;
        }
#else
        // forward path (findDagPath, :552-562) + HMM runs (cutZh, :221-255)
        uint32_t run_h = 0, run_n = 0;
        bool ok = true;
        for (h = h0; h < h1;) {
            const uint32_t L = s.sL[h], p = s.hpos[h];
            if (L == 0) {  // tail index -1: cutDAG's slice panics in the reference
                ok = false;
                break;
            }
            const uint32_t pe = h + L < h1 ? s.hpos[h + L] : be;
            if (!HMM) {
                if (ql == 0) em.token(p, pe);
            } else if (L == 1) {
                if (run_n == 0) run_h = h;
                run_n++;
            } else {
                if (run_n) {
                    sm_viterbi(s, run_h, p, run_n, em, ql);
                    run_n = 0;
                }
                if (ql == 0) em.token(p, pe);
            }
            h += L;
        }
        if (!ok) {
            if (ql == 0) s.err = 1u;
            continue;
        }
        if (t == 0) xc[0] = __builtin_amdgcn_s_memtime();  // (forward walk done)
        if (HMM && run_n) sm_viterbi(s, run_h, be, run_n, em, ql, t == 0 ? xc : nullptr);
#endif
        if (t == 0) clk[13] = __builtin_amdgcn_s_memrealtime();
    }
    em.flush();
    if (t == 0) clk[14] = __builtin_amdgcn_s_memrealtime();
    if (em.ties) atomicAdd(&s.ties, em.ties);
    __syncthreads();
    if (t == 0) clk[8] = __builtin_amdgcn_s_memrealtime();
    // 7. spans, per-document first tokens, counters (starts in the low half of one
    // scan, ends in the high half: at most kSmallBytes each)
    const uint32_t sw_ = t < nw ? s.sb[t] : 0u, ew = t < nw ? s.eb[t] : 0u;
    uint32_t tot;
    const uint32_t x = block_scan_u32((uint32_t)__popc(sw_) | ((uint32_t)__popc(ew) << 16), s.scan, &tot);
    const uint32_t ts = tot & 0xFFFFu, te = tot >> 16;
    if (t == 0) clk[9] = __builtin_amdgcn_s_memrealtime();
    uint32_t* const os = out + kSmallHdr;
    uint32_t* const oe = os + kSmallBytes;
    if (t < nw) {
        s.swp[t] = x & 0xFFFFu;
        uint32_t g = x & 0xFFFFu;
        for (uint32_t m = sw_; m; m &= m - 1u) os[g++] = 32u * t + (uint32_t)__builtin_ctz(m);
        g = x >> 16;
        for (uint32_t m = ew; m; m &= m - 1u) oe[g++] = 32u * t + (uint32_t)__builtin_ctz(m) + 1u;
    }
    __syncthreads();
    if (t == 0) clk[10] = __builtin_amdgcn_s_memrealtime();
    uint64_t* const dt = reinterpret_cast<uint64_t*>(oe + kSmallBytes);
    for (uint32_t d = t; d <= ndocs; d += nt) {
        const uint32_t o = s.doff[d];
        uint32_t c = ts;
        if (o < nbytes) c = s.swp[o >> 5] + (uint32_t)__popc(s.sb[o >> 5] & ((1u << (o & 31u)) - 1u));
        dt[d] = c;
    }
    if (t == 0) {
        clk[11] = __builtin_amdgcn_s_memrealtime();
        out[SM_NTOK] = ts;
        out[SM_NTOKE] = te;
        out[SM_ERR] = s.err;
        out[SM_TIES] = s.ties;
        out[SM_BLOCKS] = nblk;
        out[SM_ZHBLOCKS] = s.nzh;
        for (int k = 1; k < 16; k++) out[SM_CLK + k - 1] = (uint32_t)(clk[k] - clk[0]);
        out[SM_CLK + 15] = (uint32_t)(__builtin_amdgcn_s_memtime() - cyc0);  // shader clock cycles
        for (int k = 0; k < 6; k++) out[SM_CLK + 16 + k] = xc[k] ? (uint32_t)(xc[k] - cyc0) : 0u;
    }
    // every thread's writes reach host memory before the completion word
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(out + SM_DONE, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
hipError_t run_small(const DevImage& im, const uint8_t* text, uint32_t nbytes, const uint64_t* doc_off,
                     uint32_t ndocs, bool hmm, uint32_t* out, uint32_t seq, const SmallInline& in,
                     hipStream_t stream) {
    if (nbytes > kSmallBytes || ndocs > kSmallDocs) return hipErrorInvalidValue;
    if ((!text || !doc_off) && (text || doc_off || nbytes > kSmallInline || ndocs > kSmallInlineDocs))
        return hipErrorInvalidValue;
    // as many waves as the byte phases need (4 bytes per thread): a sentence is one
    // wave, whose barriers and scans cost next to nothing (and up to 64 bytes, one byte per lane)
    const uint32_t nt = std::max(64u, (nbytes + 4u * 64u - 1u) / (4u * 64u) * 64u);
#define JB_SMALL_LAUNCH(H, P)                                                                                    \
    hipLaunchKernelGGL((k_small<H, P>), dim3(1), dim3(nt), 0, stream, text, nbytes, doc_off, ndocs, im, out, seq, in)
    if (nbytes <= kSmallOneByte) {
        if (hmm) JB_SMALL_LAUNCH(true, 1u);
        else JB_SMALL_LAUNCH(false, 1u);
    } else {
        if (hmm) JB_SMALL_LAUNCH(true, 4u);
        else JB_SMALL_LAUNCH(false, 4u);
    }
#undef JB_SMALL_LAUNCH
    return hipGetLastError();
}

template <bool HMM, uint32_t NW>
static uint32_t occ_zh() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_zh<HMM, NW>, NW * 64, 0) != hipSuccess || n <= 0) return 1;
    return (uint32_t)n;
}

uint32_t zh_waves_per_cu(bool hmm, bool wide) {
    if (wide) return kZhWgWide * (hmm ? occ_zh<true, kZhWgWide>() : occ_zh<false, kZhWgWide>());
    return 4u * (hmm ? occ_zh<true, 4>() : occ_zh<false, 4>());
}


#define JB_TIMED_ON(id, st, ...)                  \
    do {                                          \
        if (timer) timer->begin((id), (st));      \
        __VA_ARGS__;                              \
        if (timer) timer->end((id), (st));        \
    } while (0)
#define JB_TIMED(id, ...) JB_TIMED_ON(id, stream, __VA_ARGS__)

hipError_t run_pipeline(const DevImage& im, const Work& w, const uint8_t* d_text, uint64_t nbytes,
                        const uint64_t* d_doc_off, uint32_t ndocs, bool hmm, const LaunchCfg& lc,
                        hipStream_t stream, KernelTimer* timer, const MaskOut* mask) {
    const uint32_t diag = lc.diag;
    const uint64_t nwords = (nbytes + 31) / 32;
    const uint32_t ntiles = (uint32_t)((nbytes + kTileBytes - 1) / kTileBytes);
    // k_zh work unit: a small batch gets small groups, so that enough waves share it
    const uint32_t grp = lc.zh_group ? lc.zh_group : zh_group_for(nbytes);
    const uint32_t nttiles = (uint32_t)((nwords + kTokTileWords - 1) / kTokTileWords);
    // k_zh: a persistent grid, but no more 4-wave workgroups than the batch has groups
    // the last zh_tail bytes (at most) in groups of zh_tail_group (tail_groups)
    uint32_t g1, sgrp;
    const uint64_t ngroups = zh_tail_groups(nbytes, grp, lc, &g1, &sgrp);
    // the wide form (16 waves per workgroup, weights in LDS) for batches in 6 KiB groups whose
    // weight table fits; JB_ZH_WIDE (lc.zh_wide) forces either form
    const bool wide = im.nw1 <= kZhWtabWide && (lc.zh_wide > 0 || (lc.zh_wide < 0 && grp == kZhGroupBytes));
    const uint32_t nw = wide ? kZhWgWide : 4u;
    const uint32_t grid_zh = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>((wide ? lc.zh_waves_wide : lc.zh_waves) / nw, (ngroups + nw - 1) / nw));
    // No clearing pass: the document bitmap is all zeros between runs (k_nonzh clears
    // what k_docbits set; a fresh or dirty workspace is cleared by the caller), k_docbits
    // clears the counters and k_mark_walk the token bitmaps, tile by tile.
    if (nbytes == 0)  // (kernels, not hipMemsetAsync: see k_zero)
        return run_zero(w.doc_tok, (ndocs + 1) * sizeof(uint64_t), stream, w.counters, CNT_CLEAR * sizeof(uint32_t));
    JB_TIMED(K_DOCBITS, hipLaunchKernelGGL(k_docbits, dim3(std::max(1u, (std::max(ndocs, nttiles) + 255) / 256)),
                                           dim3(256), 0, stream, d_doc_off, ndocs, nbytes, w.docbits, w.counters,
                                           reinterpret_cast<uint64_t*>(w.ttile_cnt), nttiles));
    // a batch with fewer tiles than CUs: two workgroups per tile (k_mark_walk's split)
    const uint32_t mws = lc.mw_split >= 0 ? (uint32_t)lc.mw_split : (ntiles <= lc.ncu ? 1u : 0u);
    JB_TIMED(K_MARK_WALK, hipLaunchKernelGGL(k_mark_walk, dim3(ntiles << mws), dim3(256), 0, stream, d_text, nbytes,
                                             w.docbits, im, w.lanemask, w.tile_cnt, w.erec + kErecPad,
                                             w.tile4, w.alnum16, w.sbits, w.ebits, diag, w.dbg_walk, mws));
#define JB_ZH_LAUNCH(H, N)                                                                                      \
    JB_TIMED(K_ZH, hipLaunchKernelGGL((k_zh<H, N>), dim3(grid_zh), dim3((N) * 64), 0, stream, d_text, nbytes,       \
                                      w.lanemask, w.tile_cnt, w.tile4, w.counters, im, w.erec + kErecPad, w.gbl,     \
                                      w.gbest, w.sbits, w.ebits, w.longblk, w.lsegb, grp, g1, sgrp, diag, w.dbg))
    if (hmm) {
        if (wide) JB_ZH_LAUNCH(true, kZhWgWide);
        else JB_ZH_LAUNCH(true, 4u);
    } else {
        if (wide) JB_ZH_LAUNCH(false, kZhWgWide);
        else JB_ZH_LAUNCH(false, 4u);
    }
#undef JB_ZH_LAUNCH
    bool nz_done = false;  // (k_nonzh's work ran inside k_long)
    {
        // long blocks: the chain, then one lane per 64-rune segment (at most
        // nbytes / 192 + nbytes / kZhLongMin segments), one wave per block
        const uint64_t segs = nbytes / (3u * kSeg) + nbytes / kZhLongMin + 2u;
        const uint32_t gseg = (uint32_t)std::min<uint64_t>(1024u, (segs + 255u) / 256u);
        const uint32_t spec = lc.long_spec;
        if (lc.long_fused) {
            // one workgroup per 64 segments (k_long_spec's lanes), at most one per CU; a batch of at most
            // JB_NZ_FUSE_MIB MiB (default 4) runs k_nonzh's work in it too (one launch less)
            uint32_t gl = (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>(lc.ncu, (segs + 63u) / 64u));
            const bool nzf = nbytes <= ((uint64_t)lc.nz_fuse_mib << 20);
            const NzArgs nz{(uint32_t)nbytes, ntiles, ndocs, w.lanemask, w.tile_cnt, w.alnum16, w.docbits, d_doc_off};
            if (nzf) gl = std::max(gl, (uint32_t)((nbytes + 1023u) / 1024u + 255u) / 256u);
#define JB_LONG_LAUNCH(H, N)                                                                                           \
    JB_TIMED(K_LONG, hipLaunchKernelGGL((k_long<H, N>), dim3(gl), dim3(256), 0, stream, d_text, im, w.erec + kErecPad, \
                                        w.longblk, w.lsegb, w.counters, w.tile4, w.gbl, w.gbest, w.lbp, w.lmap, w.lcx, \
                                        w.lpath, w.lflag, w.sbits, w.ebits, w.dbg, spec, nz, lc.long_wait_ticks))
            if (hmm && nzf) JB_LONG_LAUNCH(true, true);
            else if (hmm) JB_LONG_LAUNCH(true, false);
            else if (nzf) JB_LONG_LAUNCH(false, true);
            else JB_LONG_LAUNCH(false, false);
#undef JB_LONG_LAUNCH
            nz_done = nzf;
        } else {
        if (spec)
            JB_TIMED(K_LONG_SPEC, hipLaunchKernelGGL(k_long_spec, dim3(kSpecGrid), dim3(64), 0, stream, d_text, im,
                                                     w.erec + kErecPad, w.longblk, w.lsegb, w.counters, w.tile4, w.gbl,
                                                     w.gbest, w.lbp, w.lmap, w.lflag, lc.long_spec));
        if (spec && lc.long_spec != 3u) {  // the path of the decided choices (the path chain's blocks, lflag 3)
            JB_TIMED(K_LONG_PATH, hipLaunchKernelGGL(k_long_path, dim3(kLongGrid), dim3(64), 0, stream, w.longblk,
                                                     w.lsegb, w.counters, w.lflag, w.lbp, w.lmap, w.lcx, 3u, 3u));
            JB_TIMED(K_LONG_PBITS, hipLaunchKernelGGL(k_long_pbits, dim3(gseg), dim3(256), 0, stream, w.longblk, w.lsegb,
                                                      w.counters, w.lflag, w.gbl, w.lbp, w.lcx, w.lpath));
        }
        if (hmm)
            JB_TIMED(K_LONG_DP, hipLaunchKernelGGL((k_long_dp<true>), dim3(kLongGrid), dim3(256), 0, stream, d_text, im,
                                                   w.erec + kErecPad, w.gbl, w.gbest, w.longblk, w.counters, w.sbits,
                                                   w.ebits, w.lflag, w.lsegb, w.lpath, w.dbg, spec));
        else
            JB_TIMED(K_LONG_DP, hipLaunchKernelGGL((k_long_dp<false>), dim3(kLongGrid), dim3(256), 0, stream, d_text, im,
                                                   w.erec + kErecPad, w.gbl, w.gbest, w.longblk, w.counters, w.sbits,
                                                   w.ebits, w.lflag, w.lsegb, w.lpath, w.dbg, spec));
        JB_TIMED(K_LONG_SEG, hipLaunchKernelGGL(k_long_seg, dim3(gseg), dim3(256), 0, stream, d_text, im,
                                                w.erec + kErecPad, w.longblk, w.lsegb, w.counters, w.lflag, w.gbest,
                                                w.gbl, w.lbp, w.lmap));
        JB_TIMED(K_LONG_PATH, hipLaunchKernelGGL(k_long_path, dim3(kLongGrid), dim3(64), 0, stream, w.longblk, w.lsegb,
                                                 w.counters, w.lflag, w.lbp, w.lmap, w.lcx, 2u, 1u));
        // (the Viterbi back-pointers go to gbest's bytes: the exit codes in lbp are read to the end)
        uint8_t* const bp = reinterpret_cast<uint8_t*>(w.gbest);
        if (hmm)
            JB_TIMED(K_LONG_TAIL, hipLaunchKernelGGL((k_long_tail<true>), dim3(gseg), dim3(256), 0, stream, d_text, im,
                                                     w.gbl, w.longblk, w.lsegb, w.lflag, w.counters, w.lbp, w.lcx, bp,
                                                     w.sbits, w.ebits));
        else
            JB_TIMED(K_LONG_TAIL, hipLaunchKernelGGL((k_long_tail<false>), dim3(gseg), dim3(256), 0, stream, d_text, im,
                                                     w.gbl, w.longblk, w.lsegb, w.lflag, w.counters, w.lbp, w.lcx, bp,
                                                     w.sbits, w.ebits));
        }
    }
    if (!nz_done) {
        const uint32_t nw = (uint32_t)((nbytes + 1023u) / 1024u);  // alnum16 words
        JB_TIMED(K_NONZH, hipLaunchKernelGGL(k_nonzh, dim3((nw + 255u) / 256u), dim3(256), 0, stream, d_text,
                                             (uint32_t)nbytes, w.lanemask, w.tile_cnt, ntiles, w.alnum16, w.sbits,
                                             w.ebits, w.docbits, d_doc_off, ndocs));
    }
    if (mask) {  // boundary masks instead of spans
        const uint64_t nout = ((mask->rel & 63u) + nbytes + 63u) >> 6;
        JB_TIMED(K_MASK_MERGE, hipLaunchKernelGGL(k_mask_merge,
                                                  dim3((uint32_t)((nout + 256u * kMergeWords - 1u) / (256u * kMergeWords))),
                                                  dim3(256), 0,
                                                  stream, w.sbits, w.ebits, nbytes, mask->rel, mask->s, mask->e,
                                                  w.counters));
        return hipGetLastError();
    }
    // the span kernels in one pass for batches of at most 256 token tiles (4 MiB): at 1 GiB
    // (65K tiles) the look-back chains cost more than the passes it saves (0.33 -> 0.84 ms)
    if (lc.tok1 && nttiles <= 256u) {
        JB_TIMED(K_TOK1, hipLaunchKernelGGL(k_tok1, dim3(nttiles), dim3(256), 0, stream, w.sbits, w.ebits, nwords,
                                            nttiles, reinterpret_cast<uint64_t*>(w.ttile_cnt), w.counters, w.tok_start,
                                            w.tok_end, d_doc_off, ndocs, w.doc_tok));
        return hipGetLastError();
    }
    JB_TIMED(K_TOK_COUNT, hipLaunchKernelGGL((k_tok<false>), dim3((nttiles + 1u) / 2u), dim3(256), 0, stream, w.sbits, w.ebits,
                                             nwords, w.ttile_cnt, w.supt, w.counters, nullptr, nullptr));
    if (nttiles > 256u)  // (k_tok's write pass reads the sums of whole groups of 256 tiles only)
        JB_TIMED(K_SCAN_TOK, hipLaunchKernelGGL(k_sup, dim3((nttiles + 255) / 256), dim3(256), 0, stream,
                                                w.ttile_cnt, nttiles, w.supt));
    JB_TIMED(K_TOK_WRITE, hipLaunchKernelGGL((k_tok<true>), dim3(nttiles), dim3(256), 0, stream, w.sbits, w.ebits,
                                             nwords, w.ttile_cnt, w.supt, w.counters, w.tok_start, w.tok_end));
    if (ndocs >= kDocTokWide)
        JB_TIMED(K_DOC_TOK, hipLaunchKernelGGL(k_doc_tok<1>, dim3((ndocs + 1 + 255) / 256), dim3(256), 0, stream,
                                               d_doc_off, ndocs, w.tok_start, w.counters, w.doc_tok));
    else
        JB_TIMED(K_DOC_TOK, hipLaunchKernelGGL(k_doc_tok<16>, dim3((16u * (ndocs + 1) + 255) / 256), dim3(256), 0,
                                               stream, d_doc_off, ndocs, w.tok_start, w.counters, w.doc_tok));
    return hipGetLastError();
}

}  // namespace jb
