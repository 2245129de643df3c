// jb_kernels.hip — gfx950 kernels of the jieba-go Cut path.
//
// Pipeline for one batch of documents (all in HBM, one stream):
//   k_docbits     document starts -> 1 bit per byte
//   k_blocks<0>   per 4 KiB tile: UTF-8 decode (Go rules), \p{Han} runs, count
//                 block starts                  (zh regex + splitText, tokenizer.go:21,154-155,165-210)
//   k_scan2       tile counts -> offsets
//   k_blocks<1>   write block list (start | zh<<31), zh ids, non-zh ids
//   k_zh          one lane per Han block, text staged per workgroup in LDS: trie
//                 walk + backward max-prob DP + forward path + BMES Viterbi on
//                 singleton runs (k_zh_long: blocks longer than an LDS window)
//                                               (cutZh/cutDAG/buildDag/calcDagProba/
//                                                findDagPath/maxIndexProba/viterbi/cutHMM,
//                                                tokenizer.go:221-285,462-578,668-756)
//   k_nonzh       one lane per non-Han block: alnum runs, single runes, spaces
//                 dropped, no-alnum blocks dropped (cutNonZh, tokenizer.go:289-310)
//   k_tok<0>/scan/k_tok<1>  token start/end bitmaps -> (start, end) spans
//   k_doc_tok     per document first token (Cut per document)
//
// Output format on the device: two bitmaps, 1 bit per input byte each (token
// first byte, token last byte), compacted to u32 spans.  All float64
// arithmetic is IEEE add/compare in the reference's order; the library is
// built with -ffp-contract=off and without fast-math (±Inf must propagate).
#include <hip/hip_runtime.h>

#include "jb_kernels.h"

namespace jb {

const char* const kKernelNames[K_NUM] = {"k_docbits", "k_blocks_count", "k_scan_blocks", "k_blocks_write",
                                         "k_zh", "k_zh_long", "k_nonzh", "k_tok_count", "k_scan_tok",
                                         "k_tok_write", "k_doc_tok"};

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
// 4 bytes at any offset: two aligned dword loads + v_alignbyte.  The text
// buffer is 4-byte aligned and readable 8 bytes past every offset used.
__device__ __forceinline__ uint32_t ld4(const uint8_t* __restrict__ t, uint64_t q) {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(t + (q & ~3ull));
    return __builtin_amdgcn_alignbyte(a[1], a[0], (uint32_t)(q & 3));
}

// Child of `parent` labelled r in the open-addressing edge hash.
__device__ __forceinline__ uint32_t child(const jb_node* __restrict__ nodes, uint32_t mask, uint32_t parent,
                                          uint32_t r, jb_node* out) {
    uint32_t h = jb_hash(parent, r) & mask;
    for (;;) {
        const jb_node n = nodes[h];
        if (n.parent == JB_EMPTY) return JB_EMPTY;
        if (n.parent == parent && (n.rune_fc & JB_RUNE_MASK) == r) {
            *out = n;
            return h;
        }
        h = (h + 1) & mask;
    }
}

// Token bitmaps: bits are accumulated per 32-byte word in registers and
// flushed with one atomicOr per word (neighbouring blocks may share a word).
struct Emitter {
    uint32_t* sb;
    uint32_t* eb;
    uint32_t word, s, e;
    __device__ Emitter(uint32_t* s_, uint32_t* e_) : sb(s_), eb(e_), word(0xFFFFFFFFu), s(0), e(0) {}
    __device__ __forceinline__ void flush() {
        if (s) atomicOr(sb + word, s);
        if (e) atomicOr(eb + word, e);
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
};

// ---------------------------------------------------------------------------
// k_docbits
// ---------------------------------------------------------------------------
__global__ void k_docbits(const uint64_t* __restrict__ doc_off, uint32_t ndocs, uint64_t nbytes,
                          uint32_t* __restrict__ bits) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
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
__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t* lds, uint32_t* total) {
    // exclusive scan over a 256-thread workgroup
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
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

template <bool WRITE>
__global__ __launch_bounds__(256) void k_blocks(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                const uint32_t* __restrict__ docbits, uint2* __restrict__ tile_cnt,
                                                const uint2* __restrict__ tile_off, uint32_t* __restrict__ blk,
                                                uint32_t* __restrict__ lists, uint32_t list_cap) {
    __shared__ uint32_t lds[8];
    const uint64_t p0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 16u;
    uint32_t wv[6];
    wv[0] = p0 >= 4 ? *reinterpret_cast<const uint32_t*>(text + p0 - 4) : 0u;
    if (p0 < nbytes) {
        const uint4 m = *reinterpret_cast<const uint4*>(text + p0);
        wv[1] = m.x; wv[2] = m.y; wv[3] = m.z; wv[4] = m.w;
    } else {
        wv[1] = wv[2] = wv[3] = wv[4] = 0u;
    }
    wv[5] = p0 + 16 < nbytes ? *reinterpret_cast<const uint32_t*>(text + p0 + 16) : 0u;
    // doc-start / past-the-end mask, bit k <-> byte p0 - 4 + k (k < 24)
    uint64_t M;
    {
        const int64_t base = (int64_t)p0 - 4;
        if (base >= 0) {
            const uint64_t wi = (uint64_t)base >> 5;
            const uint32_t off = (uint32_t)base & 31u;
            const uint64_t lastw = (nbytes + 31) >> 5;
            const uint64_t lo = wi < lastw ? docbits[wi] : 0u;
            const uint64_t hi = wi + 1 < lastw ? docbits[wi + 1] : 0u;
            M = ((hi << 32) | lo) >> off;
        } else {
            M = (uint64_t)docbits[0] << 4;  // p0 == 0: window bytes -4..-1 do not exist
        }
        // bytes at or past the end stop every decode
        if (nbytes < p0 + 20) {
            const int64_t endk = (int64_t)nbytes - base;  // first window index past the end
            if (endk <= 0) M = ~0ull;
            else M |= ~0ull << endk;
        }
    }
    // decode at window indices 0..19
    uint32_t dw[20];
    bool dv[20], dh[20], cont[20];
#pragma unroll
    for (int k = 0; k < 20; k++) {
        const int wi = k >> 2, sh = (k & 3) * 8;
        const uint32_t x = sh ? (wv[wi] >> sh) | (wv[wi + 1] << (32 - sh)) : wv[wi];
        const uint32_t lim = 1u + (uint32_t)__builtin_ctzll(((M >> (k + 1)) & 7ull) | 8ull);
        uint32_t r;
        const uint32_t w = jb_decode(x, lim, &r);
        dw[k] = w;
        dv[k] = !(w == 1 && r == 0xFFFDu);
        dh[k] = dv[k] && jb_is_han(r);
        cont[k] = (x & 0xC0u) == 0x80u;
    }
    // covering rune for window indices 3..19 (byte p0-1 .. p0+15)
    bool han[20], start[20];
#pragma unroll
    for (int k = 3; k < 20; k++) {
        int c = k;
#pragma unroll
        for (int d = 1; d <= 3; d++) {
            const int q = k - d;
            if (dv[q]) {
                if ((int)dw[q] > d) c = q;
                break;
            }
            if (!cont[q]) break;
        }
        // (c is a compile-time-unknown index; select through a small unrolled mux)
        bool h = dh[k];
#pragma unroll
        for (int d = 1; d <= 3; d++)
            if (c == k - d) h = dh[k - d];
        han[k] = h;
        start[k] = c == k;
    }
    if (p0 == 0) han[3] = false;
    uint32_t na = 0, nz = 0, bmask = 0;
#pragma unroll
    for (int k = 4; k < 20; k++) {
        const uint64_t p = p0 + (uint64_t)(k - 4);
        const bool bs = p < nbytes && start[k] && ((((M >> k) & 1ull) != 0) || han[k] != han[k - 1]);
        if (bs) {
            bmask |= 1u << (k - 4);
            na++;
            nz += han[k] ? 1u : 0u;
        }
    }
    uint32_t tot;
    const uint32_t ex = block_scan_u32(na | (nz << 16), lds, &tot);
    if (!WRITE) {
        if (threadIdx.x == 0) tile_cnt[blockIdx.x] = make_uint2(tot & 0xFFFFu, tot >> 16);
        return;
    }
    if (!bmask) return;
    const uint2 to = tile_off[blockIdx.x];
    uint32_t ga = to.x + (ex & 0xFFFFu);  // global block rank
    uint32_t gz = to.y + (ex >> 16);      // global zh rank
#pragma unroll
    for (int k = 4; k < 20; k++) {
        if (bmask & (1u << (k - 4))) {
            const uint32_t p = (uint32_t)(p0 + (uint64_t)(k - 4));
            blk[ga] = p | (han[k] ? 0x80000000u : 0u);
            if (han[k]) lists[gz++] = ga;
            else lists[list_cap - 1u - (ga - gz)] = ga;
            ga++;
        }
    }
}

// ---------------------------------------------------------------------------
// k_scan2: exclusive scan of n uint2 counts by one 1024-thread workgroup.
// Writes totals to tot[0], tot[1]; optional u64 copy of tot.x; optional sentinel.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan2(const uint2* __restrict__ cnt, uint32_t n, uint2* __restrict__ off,
                                                uint32_t* __restrict__ tot, uint64_t* __restrict__ tot64,
                                                uint32_t* __restrict__ sentinel_base, uint32_t sentinel_val) {
    __shared__ uint32_t la[16], lz[16];
    const uint32_t t = threadIdx.x, T = blockDim.x;
    const uint32_t chunk = (n + T - 1) / T;
    const uint32_t b = t * chunk, e = min(n, b + chunk);
    uint32_t sa = 0, sz = 0;
    for (uint32_t i = b; i < e; i++) {
        const uint2 c = cnt[i];
        sa += c.x;
        sz += c.y;
    }
    // workgroup exclusive scan of (sa, sz)
    const uint32_t lane = t & 63u, wid = t >> 6;
    uint32_t xa = sa, xz = sz;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t ya = __shfl_up(xa, d, 64), yz = __shfl_up(xz, d, 64);
        if (lane >= (uint32_t)d) { xa += ya; xz += yz; }
    }
    if (lane == 63) { la[wid] = xa; lz[wid] = xz; }
    __syncthreads();
    uint32_t ba = 0, bz = 0, ta = 0, tz = 0;
    for (uint32_t k = 0; k < (T >> 6); k++) {
        if (k < wid) { ba += la[k]; bz += lz[k]; }
        ta += la[k];
        tz += lz[k];
    }
    ba += xa - sa;
    bz += xz - sz;
    for (uint32_t i = b; i < e; i++) {
        const uint2 c = cnt[i];
        off[i] = make_uint2(ba, bz);
        ba += c.x;
        bz += c.y;
    }
    if (t == 0) {
        tot[0] = ta;
        tot[1] = tz;
        if (tot64) *tot64 = ta;
        if (sentinel_base) sentinel_base[ta] = sentinel_val;
    }
}

// ---------------------------------------------------------------------------
// Han blocks (cutZh, tokenizer.go:221-255).
//
// process_block() runs one block in one lane.  Backward over the block's runes
// (calcDagProba, :502-548): for rune i the lane walks the trie forward from i
// (buildDag, :462-497) and folds each edge (i, i+len) — in ascending len, as
// the DAG lists them — into maxIndexProba's running state (:565-578) with
// pieceProba = w + best(i+len) (:519-529); best(n) is the {n, 0.0} sentinel
// (:522-525).  best / the chosen length live per rune at index (byte offset)/3
// (Han runes are >= 3 bytes, so distinct runes never share an index).  The
// forward walk (findDagPath, :552-562) then emits pieces or, with HMM,
// gathers runs of single-rune pieces for the Viterbi (:228-253).
//
// A View supplies the text bytes, the per-rune slots and the token sink:
//   LdsView    — k_zh: the workgroup's window of text staged in LDS
//   GlobalView — k_zh_long: blocks longer than a window, straight from HBM
// ---------------------------------------------------------------------------
constexpr uint32_t kWin = 8192;  // k_zh window bytes (LDS)

__device__ __forceinline__ void load_emit(const DevImage& im, uint32_t r, double e[4]) {
    const double2* p = reinterpret_cast<const double2*>(im.emit) + (size_t)jb_row(im.pagemap, r) * 2u;
    const double2 a = p[0], b = p[1];
    e[0] = a.x; e[1] = a.y; e[2] = b.x; e[3] = b.y;
}

// stateTransitionRoute (tokenizer.go:736-756): candidates in stateChange
// order, strict '>' against minFloat; code 0/1 = candidate, 2 = no route ("").
__device__ __forceinline__ void route2(double a, double b, uint32_t* code, double* p) {
    uint32_t c = 2u;
    double best = JB_MIN_FLOAT;
    if (a > best) { c = 0u; best = a; }
    if (b > best) { c = 1u; best = b; }
    *code = c;
    *p = best;
}

struct LdsEmitter {  // token bits accumulated per word, OR-ed into the LDS bitmap
    uint32_t* ls;
    uint32_t* le;
    uint32_t w0, word, s, e;
    __device__ __forceinline__ void flush() {
        if (s) atomicOr(ls + (word - w0), s);
        if (e) atomicOr(le + (word - w0), e);
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

struct LdsView {
    const uint8_t* tx;  // tx[k] = text[wb + k]
    double* best;
    uint8_t* bl;
    uint32_t wb;
    LdsEmitter em;
    __device__ __forceinline__ uint32_t byte(uint32_t q) const { return tx[q - wb]; }
    __device__ __forceinline__ uint32_t load4(uint32_t q) const {
        const uint32_t k = q - wb;
        const uint32_t* a = reinterpret_cast<const uint32_t*>(tx + (k & ~3u));
        return __builtin_amdgcn_alignbyte(a[1], a[0], k & 3u);
    }
    __device__ __forceinline__ uint32_t slot(uint32_t q) const { return (q - wb) / 3u; }
    __device__ __forceinline__ void token(uint32_t a, uint32_t b) { em.token(a, b); }
};

struct GlobalView {
    const uint8_t* text;
    double* best;  // index q / 3
    uint8_t* bl;
    Emitter em;
    __device__ __forceinline__ uint32_t byte(uint32_t q) const { return text[q]; }
    __device__ __forceinline__ uint32_t load4(uint32_t q) const { return ld4(text, q); }
    __device__ __forceinline__ uint32_t slot(uint32_t q) const { return q / 3u; }
    __device__ __forceinline__ void token(uint32_t a, uint32_t b) { em.token(a, b); }
};

template <class V>
__device__ __forceinline__ uint32_t v_han(const V& v, uint32_t q, uint32_t* w) {
    const uint32_t x = v.load4(q);
    const uint32_t b0 = x & 0xFFu;
    if (b0 < 0xF0u) {
        *w = 3;
        return ((b0 & 0x0Fu) << 12) | (((x >> 8) & 0x3Fu) << 6) | ((x >> 16) & 0x3Fu);
    }
    *w = 4;
    return ((b0 & 0x07u) << 18) | (((x >> 8) & 0x3Fu) << 12) | (((x >> 16) & 0x3Fu) << 6) | ((x >> 24) & 0x3Fu);
}
template <class V>
__device__ __forceinline__ uint32_t v_width(const V& v, uint32_t q) { return v.byte(q) < 0xF0u ? 3u : 4u; }
template <class V>
__device__ __forceinline__ uint32_t v_prev(const V& v, uint32_t q, uint32_t lo) {  // rune ending at q
    if (q - lo < 4u) return lo;
    return (v.byte(q - 3u) & 0xF0u) == 0xE0u ? q - 3u : q - 4u;
}

// viterbi (tokenizer.go:668-730) over the m runes [rs, re) + cutHMM (:273-285).
// Back-pointers (2 bits per state) go to each rune's slot; the traceback stops
// at the first "" route: the reference's path then restarts at that step
// (fullPath[""] is nil, :715) and cutHMM labels runes from the run's start.
template <class V>
__device__ void viterbi_run(V& v, const DevImage& im, uint32_t rs, uint32_t re, uint32_t m) {
    if (m == 1) {  // always "S" for a single rune (:672-674)
        v.token(rs, re);
        return;
    }
    uint32_t w;
    double e[4];
    uint32_t r = v_han(v, rs, &w);
    load_emit(im, r, e);
    double vB = START_B + e[0], vM = JB_MIN_FLOAT + e[1], vE = JB_MIN_FLOAT + e[2], vS = START_S + e[3];
    uint32_t q = rs + w;
    while (q < re) {
        r = v_han(v, q, &w);
        load_emit(im, r, e);
        uint32_t cB, cM, cE, cS;
        double pB, pM, pE, pS;
        route2(vE + T_EB, vS + T_SB, &cB, &pB);  // B <- E, S
        route2(vB + T_BM, vM + T_MM, &cM, &pM);  // M <- B, M
        route2(vB + T_BE, vM + T_ME, &cE, &pE);  // E <- B, M
        route2(vE + T_ES, vS + T_SS, &cS, &pS);  // S <- E, S
        vB = pB + e[0];
        vM = pM + e[1];
        vE = pE + e[2];
        vS = pS + e[3];
        v.bl[v.slot(q)] = (uint8_t)(cB | (cM << 2) | (cE << 4) | (cS << 6));
        q += w;
    }
    uint32_t st = vE > vS ? (uint32_t)JB_E : (uint32_t)JB_S;  // (:723-729)
    uint32_t t = m - 1, reset = 0;
    uint32_t qt = v_prev(v, re, rs);
    for (;;) {
        const uint32_t sl = v.slot(qt);
        if (t == 0) {
            v.bl[sl] = (uint8_t)st;
            break;
        }
        const uint32_t code = (v.bl[sl] >> (2u * st)) & 3u;
        v.bl[sl] = (uint8_t)st;
        if (code == 2u) {
            reset = t;
            break;
        }
        st = (st == JB_B || st == JB_S) ? 2u + code : code;  // B,S <- {E,S}; M,E <- {B,M}
        --t;
        qt = v_prev(v, qt, rs);
    }
    uint32_t qa = rs, qb = qt, ts = rs;
    for (uint32_t k = 0; k < m - reset; k++) {
        const uint32_t lab = v.bl[v.slot(qb)];
        qa += v_width(v, qa);
        qb += v_width(v, qb);
        if (lab >= (uint32_t)JB_E) {
            v.token(ts, qa);
            ts = qa;
        }
    }
}

// One Han block [bs, be). Returns false when the reference would panic
// (a position with no DAG edge on the chosen path: cutDAG slices with -1).
template <bool HMM, class V>
__device__ bool process_block(V& v, const DevImage& im, uint32_t bs, uint32_t be) {
    // ---- backward DP ----------------------------------------------------------
    uint32_t q = be;
    while (q > bs) {
        q = v_prev(v, q, bs);
        uint32_t w0;
        const uint32_t r0 = v_han(v, q, &w0);
        double prevP = JB_MIN_FLOAT, bestP = JB_MIN_FLOAT;
        uint32_t bestL = 0, lastL = 0;
        auto edge = [&](uint32_t len, uint32_t end, double wt) {
            const double nb = end == be ? 0.0 : v.best[v.slot(end)];
            const double pp = wt + nb;
            if (pp >= prevP) {
                bestL = len;
                bestP = pp;
            }
            prevP = pp;
            lastL = len;
        };
        const jb_l1 l1 = im.l1[jb_row(im.pagemap, r0)];
        if (l1.fc == JB_FC_ABSENT || l1.fc == JB_FC_ZERO) {
            // absent or count 0: the single edge only (:468-471); w is -Log(size) or -Inf (:515-519)
            edge(1, q + w0, l1.w);
        } else {
            if (l1.fc == JB_FC_POS) edge(1, q + w0, l1.w);
            uint32_t id = l1.id, qq = q + w0, len = 1;
            while (qq < be) {
                uint32_t wr;
                const uint32_t r = v_han(v, qq, &wr);
                jb_node m;
                const uint32_t id2 = child(im.nodes, im.mask, id, r, &m);
                if (id2 == JB_EMPTY) break;  // (:475-478)
                ++len;
                qq += wr;
                if ((m.rune_fc >> JB_FC_SHIFT) == JB_FC_POS) edge(len, qq, m.w);  // (:479-481)
                id = id2;
            }
        }
        if (bestL == 0) {  // no item qualified: the last item (or {-1, minFloat})
            bestL = lastL;
            bestP = prevP;
        }
        const uint32_t sl = v.slot(q);
        v.best[sl] = bestP;
        v.bl[sl] = (uint8_t)bestL;
    }
    // ---- forward walk (findDagPath) + HMM runs ------------------------------------
    uint32_t p = bs, run_s = 0, run_n = 0;
    while (p < be) {
        const uint32_t L = v.bl[v.slot(p)];
        if (L == 0) return false;
        uint32_t pe = p;
        for (uint32_t k = 0; k < L; k++) pe += v_width(v, pe);
        if (!HMM) {
            v.token(p, pe);
        } else if (L == 1) {
            if (run_n == 0) run_s = p;
            run_n++;
        } else {
            if (run_n) {
                viterbi_run(v, im, run_s, p, run_n);
                run_n = 0;
            }
            v.token(p, pe);
        }
        p = pe;
    }
    if (HMM && run_n) viterbi_run(v, im, run_s, be, run_n);
    return true;
}

// k_zh: workgroups pull 256 consecutive Han blocks at a time from a global
// counter, stage the text window that holds them in LDS (coalesced 16-byte
// loads), run one block per lane out of LDS, and OR the window's token bits
// into the global bitmaps.  Blocks too long for a window go to k_zh_long.
template <bool HMM>
__global__ __launch_bounds__(256) void k_zh(const uint8_t* __restrict__ text, const uint32_t* __restrict__ blk,
                                            const uint32_t* __restrict__ lists, uint32_t* __restrict__ counters,
                                            DevImage im, uint32_t* __restrict__ sbits, uint32_t* __restrict__ ebits,
                                            uint32_t* __restrict__ longq) {
    __shared__ __attribute__((aligned(16))) uint8_t tx[kWin + 16];
    __shared__ double best[kWin / 3 + 2];
    __shared__ uint8_t bl[kWin / 3 + 2];
    __shared__ uint32_t ls[kWin / 32 + 2], le[kWin / 32 + 2];
    __shared__ uint32_t sh[4];
    const uint32_t tid = threadIdx.x;
    const uint32_t nzh = counters[CNT_NZH];
    for (;;) {
        if (tid == 0) sh[0] = atomicAdd(counters + CNT_WORK, 256u);
        __syncthreads();
        const uint32_t z0 = sh[0];
        if (z0 >= nzh) break;
        const uint32_t z = z0 + tid;
        bool todo = z < nzh;
        uint32_t bs = 0, be = 0;
        if (todo) {
            const uint32_t g = lists[z];
            bs = blk[g] & 0x7FFFFFFFu;
            be = blk[g + 1] & 0x7FFFFFFFu;
            if (be - bs > kWin - 32u) {
                longq[atomicAdd(counters + CNT_NLONG, 1u)] = z;
                todo = false;
            }
        }
        for (;;) {  // sub-rounds: the blocks whose bytes fit one window
            if (tid == 0) {
                sh[1] = 0xFFFFFFFFu;
                sh[2] = 0u;
            }
            __syncthreads();
            if (todo) atomicMin(&sh[1], bs);
            __syncthreads();
            const uint32_t first = sh[1];
            if (first == 0xFFFFFFFFu) break;
            const uint32_t wb = first & ~15u;
            const bool mine = todo && be - wb <= kWin;
            if (mine) atomicMax(&sh[2], be);
            __syncthreads();
            const uint32_t wend = sh[2];
            const uint32_t nld = (wend - wb + 8u + 15u) >> 4;
            for (uint32_t k = tid; k < nld; k += 256u)
                reinterpret_cast<uint4*>(tx)[k] = reinterpret_cast<const uint4*>(text + wb)[k];
            const uint32_t w0 = wb >> 5, nw = ((wend - 1u) >> 5) - w0 + 1u;
            for (uint32_t k = tid; k < nw; k += 256u) ls[k] = le[k] = 0u;
            __syncthreads();
            if (mine) {
                LdsView v{tx, best, bl, wb, LdsEmitter{ls, le, w0, 0xFFFFFFFFu, 0u, 0u}};
                if (!process_block<HMM>(v, im, bs, be)) atomicOr(counters + CNT_ERR, 1u);
                v.em.flush();
                todo = false;
            }
            __syncthreads();
            for (uint32_t k = tid; k < nw; k += 256u) {
                const uint32_t a = ls[k], b = le[k];
                if (a) atomicOr(sbits + w0 + k, a);
                if (b) atomicOr(ebits + w0 + k, b);
            }
            __syncthreads();
        }
    }
}

// k_zh_long: one lane per block longer than a window, text from HBM,
// per-rune slots in global scratch (index q / 3).
template <bool HMM>
__global__ __launch_bounds__(64) void k_zh_long(const uint8_t* __restrict__ text, const uint32_t* __restrict__ blk,
                                                const uint32_t* __restrict__ lists, uint32_t* __restrict__ counters,
                                                DevImage im, const uint32_t* __restrict__ longq, double* gbest,
                                                uint8_t* gbl, uint32_t* __restrict__ sbits,
                                                uint32_t* __restrict__ ebits) {
    const uint32_t n = counters[CNT_NLONG];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t g = lists[longq[i]];
        const uint32_t bs = blk[g] & 0x7FFFFFFFu, be = blk[g + 1] & 0x7FFFFFFFu;
        GlobalView v{text, gbest, gbl, Emitter(sbits, ebits)};
        if (!process_block<HMM>(v, im, bs, be)) atomicOr(counters + CNT_ERR, 1u);
        v.em.flush();
    }
}

// ---------------------------------------------------------------------------
// k_nonzh: one lane per non-Han block (cutNonZh, tokenizer.go:289-310)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_nonzh(const uint8_t* __restrict__ text, const uint32_t* __restrict__ blk,
                                               const uint32_t* __restrict__ lists, uint32_t list_cap,
                                               const uint32_t* __restrict__ counters, uint32_t* __restrict__ sbits,
                                               uint32_t* __restrict__ ebits) {
    const uint32_t nnz = counters[CNT_NBLK] - counters[CNT_NZH];
    Emitter em(sbits, ebits);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += gridDim.x * blockDim.x) {
        const uint32_t g = lists[list_cap - 1u - i];
        const uint32_t bs = blk[g] & 0x7FFFFFFFu, be = blk[g + 1] & 0x7FFFFFFFu;
        bool has = false;  // alnum.FindAllIndex found nothing -> no tokens (:290-293)
        for (uint32_t p = bs; p < be && !has; p += 4) {
            const uint32_t x = ld4(text, p);
            const uint32_t nb = min(4u, be - p);
            for (uint32_t k = 0; k < nb; k++) has |= jb_is_alnum((x >> (8 * k)) & 0xFFu);
        }
        if (!has) continue;
        uint32_t p = bs, run = 0;
        bool in_run = false;
        while (p < be) {
            const uint32_t x = ld4(text, p);
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
        if (in_run) em.token(run, be);
    }
    em.flush();
}

// ---------------------------------------------------------------------------
// token bitmaps -> spans
// ---------------------------------------------------------------------------
template <bool WRITE>
__global__ __launch_bounds__(256) void k_tok(const uint32_t* __restrict__ sbits, const uint32_t* __restrict__ ebits,
                                             uint64_t nwords, uint2* __restrict__ tile_cnt,
                                             const uint2* __restrict__ tile_off, uint32_t* __restrict__ tok_start,
                                             uint32_t* __restrict__ tok_end) {
    __shared__ uint32_t lds[8];
    const uint64_t w0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 4u;
    uint32_t s[4], e[4];
    if (w0 + 4 <= nwords) {
        const uint4 a = *reinterpret_cast<const uint4*>(sbits + w0);
        const uint4 b = *reinterpret_cast<const uint4*>(ebits + w0);
        s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
        e[0] = b.x; e[1] = b.y; e[2] = b.z; e[3] = b.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            s[k] = w0 + k < nwords ? sbits[w0 + k] : 0u;
            e[k] = w0 + k < nwords ? ebits[w0 + k] : 0u;
        }
    }
    uint32_t cs = 0, ce = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        cs += __popc(s[k]);
        ce += __popc(e[k]);
    }
    uint32_t ts, te;
    const uint32_t xs = block_scan_u32(cs, lds, &ts);
    const uint32_t xe = block_scan_u32(ce, lds, &te);
    if (!WRITE) {
        if (threadIdx.x == 0) tile_cnt[blockIdx.x] = make_uint2(ts, te);
        return;
    }
    const uint2 to = tile_off[blockIdx.x];
    uint32_t gs = to.x + xs, ge = to.y + xe;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t base = (uint32_t)((w0 + k) << 5);
        uint32_t m = s[k];
        while (m) {
            const uint32_t b = __builtin_ctz(m);
            tok_start[gs++] = base + b;
            m &= m - 1;
        }
        m = e[k];
        while (m) {
            const uint32_t b = __builtin_ctz(m);
            tok_end[ge++] = base + b + 1u;
            m &= m - 1;
        }
    }
}

// tokens of document d: [doc_tok[d], doc_tok[d+1]) = lower_bound over starts
__global__ void k_doc_tok(const uint64_t* __restrict__ doc_off, uint32_t ndocs, const uint32_t* __restrict__ tok_start,
                          const uint32_t* __restrict__ counters, uint64_t* __restrict__ doc_tok) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d > ndocs) return;
    const uint32_t n = counters[CNT_NTOK];
    const uint64_t target = doc_off[d];
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)tok_start[mid] < target) lo = mid + 1;
        else hi = mid;
    }
    doc_tok[d] = lo;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <bool HMM>
static uint32_t occ_zh() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_zh<HMM>, 256, 0) != hipSuccess || n <= 0) return 1;
    return (uint32_t)n;
}

uint32_t zh_blocks_per_cu(bool hmm) { return hmm ? occ_zh<true>() : occ_zh<false>(); }

uint32_t nonzh_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_nonzh, 256, 0) != hipSuccess || n <= 0) return 1;
    return (uint32_t)n;
}

#define JB_TIMED(id, stmt)                        \
    do {                                          \
        if (timer) timer->begin((id), stream);    \
        stmt;                                     \
        if (timer) timer->end((id), stream);      \
    } while (0)

hipError_t run_pipeline(const DevImage& im, const Work& w, const uint8_t* d_text, uint64_t nbytes,
                        const uint64_t* d_doc_off, uint32_t ndocs, bool hmm, uint32_t grid_zh, uint32_t grid_nz,
                        hipStream_t stream, KernelTimer* timer) {
    const uint64_t nwords = (nbytes + 31) / 32;
    const uint32_t ntiles = (uint32_t)((nbytes + kTileBytes - 1) / kTileBytes);
    const uint32_t nttiles = (uint32_t)((nwords + kTokTileWords - 1) / kTokTileWords);
    const uint32_t list_cap = (uint32_t)(nbytes + 2);
    hipError_t e;
    if ((e = hipMemsetAsync(w.counters, 0, CNT_NWORDS * sizeof(uint32_t) + sizeof(uint64_t), stream))) return e;
    if ((e = hipMemsetAsync(w.docbits, 0, (nwords + 2) * 4, stream))) return e;
    if ((e = hipMemsetAsync(w.sbits, 0, (nwords + 2) * 4, stream))) return e;
    if ((e = hipMemsetAsync(w.ebits, 0, (nwords + 2) * 4, stream))) return e;
    uint64_t* ntok64 = reinterpret_cast<uint64_t*>(w.counters + CNT_NWORDS);
    if (nbytes == 0) {
        if ((e = hipMemsetAsync(w.doc_tok, 0, (ndocs + 1) * sizeof(uint64_t), stream))) return e;
        return hipSuccess;
    }
    if (ndocs)
        JB_TIMED(K_DOCBITS, hipLaunchKernelGGL(k_docbits, dim3((ndocs + 255) / 256), dim3(256), 0, stream,
                                               d_doc_off, ndocs, nbytes, w.docbits));
    JB_TIMED(K_BLOCKS_COUNT, hipLaunchKernelGGL((k_blocks<false>), dim3(ntiles), dim3(256), 0, stream, d_text,
                                                nbytes, w.docbits, w.tile_cnt, nullptr, nullptr, nullptr, 0u));
    JB_TIMED(K_SCAN_BLOCKS, hipLaunchKernelGGL(k_scan2, dim3(1), dim3(1024), 0, stream, w.tile_cnt, ntiles,
                                               w.tile_off, w.counters + CNT_NBLK, nullptr, w.blk,
                                               (uint32_t)nbytes));
    JB_TIMED(K_BLOCKS_WRITE, hipLaunchKernelGGL((k_blocks<true>), dim3(ntiles), dim3(256), 0, stream, d_text,
                                                nbytes, w.docbits, nullptr, w.tile_off, w.blk, w.lists, list_cap));
    if (hmm)
        JB_TIMED(K_ZH, hipLaunchKernelGGL((k_zh<true>), dim3(grid_zh), dim3(256), 0, stream, d_text, w.blk, w.lists,
                                          w.counters, im, w.sbits, w.ebits, w.longq));
    else
        JB_TIMED(K_ZH, hipLaunchKernelGGL((k_zh<false>), dim3(grid_zh), dim3(256), 0, stream, d_text, w.blk, w.lists,
                                          w.counters, im, w.sbits, w.ebits, w.longq));
    if (hmm)
        JB_TIMED(K_ZH_LONG, hipLaunchKernelGGL((k_zh_long<true>), dim3(64), dim3(64), 0, stream, d_text, w.blk,
                                               w.lists, w.counters, im, w.longq, w.gbest, w.gbl, w.sbits, w.ebits));
    else
        JB_TIMED(K_ZH_LONG, hipLaunchKernelGGL((k_zh_long<false>), dim3(64), dim3(64), 0, stream, d_text, w.blk,
                                               w.lists, w.counters, im, w.longq, w.gbest, w.gbl, w.sbits, w.ebits));
    JB_TIMED(K_NONZH, hipLaunchKernelGGL(k_nonzh, dim3(grid_nz), dim3(256), 0, stream, d_text, w.blk, w.lists,
                                         list_cap, w.counters, w.sbits, w.ebits));
    JB_TIMED(K_TOK_COUNT, hipLaunchKernelGGL((k_tok<false>), dim3(nttiles), dim3(256), 0, stream, w.sbits, w.ebits,
                                             nwords, w.ttile_cnt, nullptr, nullptr, nullptr));
    JB_TIMED(K_SCAN_TOK, hipLaunchKernelGGL(k_scan2, dim3(1), dim3(1024), 0, stream, w.ttile_cnt, nttiles,
                                            w.ttile_off, w.counters + CNT_NTOK, ntok64, nullptr, 0u));
    JB_TIMED(K_TOK_WRITE, hipLaunchKernelGGL((k_tok<true>), dim3(nttiles), dim3(256), 0, stream, w.sbits, w.ebits,
                                             nwords, nullptr, w.ttile_off, w.tok_start, w.tok_end));
    JB_TIMED(K_DOC_TOK, hipLaunchKernelGGL(k_doc_tok, dim3((ndocs + 1 + 255) / 256), dim3(256), 0, stream,
                                           d_doc_off, ndocs, w.tok_start, w.counters, w.doc_tok));
    return hipGetLastError();
}

}  // namespace jb
