// jb_kernels.h — host-side launch interface of the gfx950 segmentation kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jb_common.h"

namespace jb {

// Device copy of the image (jb_common.h), passed by value to kernels.
struct DevImage {
    const uint16_t* pagemap;
    const double* emit;
    const uint32_t* code;   // dense rune code per row (0: in no key)
    const uint64_t* cells;  // double-array trie over codes; level-1 nodes at their codes
    const double* wtab;
    // wtab shifted by one: wtab1[0] = -Inf, wtab1[i + 1] = wtab[i].  DAG records hold
    // weight index + 1 per slot, so an unused slot gathers -Inf (k_mark_walk, k_zh)
    const double* wtab1;
    // per row: the rune's level-1 cell cells[code] with its check field
    // replaced by the code (bits 0-16) and bit 21 = "that check was the root",
    // so k_mark_walk gets code and level-1 cell in one load (jb_l1row_make)
    const uint64_t* l1row;
    // hot level-1 rows (jb_common.h JB_HOT_SLOTS): u64 l1row values, then u16 tags
    const uint64_t* hot;
    uint32_t nrows;
    uint32_t nw1;  // entries in wtab1 (distinct weights + 1)
    // 1: every weight is finite or -Inf (a dictionary whose size is > 0).  k_zh's
    // record fold relies on it; otherwise k_mark_walk writes only overflow records
    // and k_zh folds every rune with maxIndexProba's literal rule.
    uint32_t plainw;
};

// Device counters (u32 slots unless noted)
enum {
    CNT_NTOK = 2,   // token starts
    CNT_NTOKE = 3,  // token ends (== CNT_NTOK when consistent)
    CNT_ERR = 4,    // bit 0: a zh block reached a tail index -1 (the reference panics); bit 1: a k_long
                    // phase wait gave up (no progress for LaunchCfg::long_wait_ticks); bit 2: k_span_pack's
                    // side list overflowed (internal)
    CNT_WORK = 5,   // k_zh work counter: next group (kZhGroupBytes of text)
    CNT_SIDE = 6,   // k_span_pack: tokens in the side list
    CNT_TOKT = 30,  // k_tok1's tile tickets
    CNT_PHASE = 32, // k_long's phases: claimed items at 32 + 2 p, finished items at 33 + 2 p
    CNT_ALL = 64,   // (u32 slots of the counters buffer; k_docbits clears them all)
    CNT_TIES = 7,   // exact Viterbi route ties (Q12)
    CNT_NWORDS = 8, // u64 token count lives at u32 slots 8-9 (byte offset 32)
    CNT_NLONG = 10, // long zh blocks k_zh left to k_long_* (u64 with CNT_NLSEG: one atomic)
    CNT_NLSEG = 11, // their 64-rune segments
    CNT_CLEAR = 12  // u32 slots cleared per batch
};

constexpr int kTileBytes = 4096;       // k_blocks: 256 threads x 16 bytes
constexpr int kTokTileWords = 512;     // k_tok: 256 threads x 2 words (16 KiB of text)
#ifndef JB_ZH_GROUP
#define JB_ZH_GROUP 6144
#endif
constexpr uint32_t kErecPad = 8;  // erec slots before slot 0 (k_zh reads a few slots past a block's start)
// k_zh work unit: the zh blocks that start in one group of text bytes (a
// multiple of 32): kZhGroupBytes, or kZhGroupSmall for batches under
// kZhSmallBatch bytes so that a small batch still spreads over enough waves
constexpr uint32_t kZhGroupBytes = JB_ZH_GROUP;
constexpr uint32_t kZhGroupSmall = 1024;
constexpr uint64_t kZhSmallBatch = 16ull << 20;
constexpr uint32_t kZhLongMin = 8192;  // zh blocks of at least this many bytes go to k_long_*
constexpr uint32_t kSeg = 64;          // runes per segment of a long block (k_long_seg/path/tail)
inline uint32_t zh_group_for(uint64_t nbytes) { return nbytes < kZhSmallBatch ? kZhGroupSmall : kZhGroupBytes; }
// k_zh's wide form: 16-wave workgroups, one per CU, sharing one LDS copy of the weight
// table (up to kZhWtab entries of wtab1) for the DP's weight reads
constexpr uint32_t kZhWgWide = 16;
constexpr uint32_t kZhWtab = 5120;
// ... of which k_zh's wide form holds up to kZhWtabWide (its LDS also holds the per-wave slots
// and block tables, which larger groups make larger)
#ifndef JB_ZH_WTAB
#define JB_ZH_WTAB 5120
#endif
constexpr uint32_t kZhWtabWide = JB_ZH_WTAB;

// Per-call device workspace, sized for `nbytes` of text.
struct Work {
    uint32_t* docbits;     // 1 bit per byte: a document starts here
    uint32_t* sbits;       // 1 bit per byte: a token starts here
    uint32_t* ebits;       // 1 bit per byte: a token ends here (last byte)
    uint64_t bits_stride;  // words between docbits, sbits and ebits (one allocation)
    uint2* supt;           // per 256 token tiles: (starts, ends) (k_sup)
    uint2* tile_cnt;       // per k_mark_walk tile: (blocks, zh blocks) starting in it
    uint2* ttile_cnt;      // per token tile (starts, ends); k_tok1: its look-back status word
    uint64_t* alnum16;     // 1 bit per 16 bytes of text: some [0-9A-Za-z] byte there
    uint64_t* erec;        // per Han rune (slot = byte / 3): packed DAG edges (k_mark_walk -> k_zh)
    uint32_t* lanemask;    // per 16 bytes: block starts | Han block starts << 16 (k_zh and k_nonzh read
                           // their blocks from these bits: a block ends at the next start)
    uint2* longblk;        // (start, end) of each long zh block (k_zh -> k_long_*)
    uint32_t* lsegb;       // per long block: its first segment (ascending with the block index)
    uint8_t* lmap;         // per 64-segment chunk of a long block: its path-state map (k_long_seg -> k_long_path)
    uint8_t* lcx;          // per chunk: the path state at its start (k_long_path -> k_long_tail)
    uint64_t* lpath;       // per segment: the runes where a piece of the decided path starts (k_long_pbits -> k_long_dp)
    uint32_t* tile4;       // per tile: a 4-byte Han rune starts in it
    uint8_t* gbl;          // per Han rune: chosen piece length, then Viterbi back-pointers / labels
                           // (+512 bytes: k_zh_long reads 256-slot windows)
    uint32_t* lflag;       // per long block: 3 decided by k_long_spec (the path chain's), then k_long_dp's
                           // verdict: 0 cut by its one-lane path, 2 DP done, 1 entries found (or path verified)
    uint8_t* lbp;          // long blocks, per slot: path exit codes (k_long_seg -> k_long_path, k_long_tail)
    double* gbest;         // per Han rune: best proba, kept only for blocks with an edge > 8 runes
    uint32_t* tok_start;
    uint32_t* tok_end;
    uint64_t* doc_tok;
    uint32_t* counters;    // CNT_* (+ u64 ntok at counters + 8)
    uint64_t* dbg = nullptr;       // diagnostic per-wave clocks of k_zh (JB_ABLATE bit 8), 8 u64 per wave
    uint64_t* dbg_walk = nullptr;  // the same for k_mark_walk
    uint64_t cap_bytes = 0;
    uint32_t cap_docs = 0;
};

// Kernel ids for per-launch timing.
enum KernelId {
    K_DOCBITS = 0, K_MARK_WALK, K_ZH, K_NONZH,
    K_TOK_COUNT, K_SCAN_TOK, K_TOK_WRITE, K_DOC_TOK, K_LONG_SPEC, K_LONG_DP, K_LONG_SEG, K_LONG_PATH, K_LONG_TAIL, K_MASK_MERGE,
    K_LONG_PBITS, K_LONG, K_TOK1,
    K_NUM
};
extern const char* const kKernelNames[K_NUM];

// Optional per-launch timer (HIP events recorded on the launch stream).
struct KernelTimer {
    virtual void begin(int kernel_id, hipStream_t s) = 0;
    virtual void end(int kernel_id, hipStream_t s) = 0;
    virtual ~KernelTimer() {}
};

// Launch shape of one pipeline run (fixed per device at jb_open).
struct LaunchCfg {
    uint32_t zh_waves;       // persistent grid of k_zh, in waves (4-wave workgroups)
    uint32_t zh_waves_wide;  // ... of its wide form (kZhWgWide-wave workgroups)
    int32_t zh_wide;         // k_zh's wide form: -1 by batch size, 0 never, 1 whenever the weights fit
    uint32_t zh_group;  // k_zh group bytes (0: zh_group_for(nbytes))
    uint32_t diag;      // diagnostic clocks (STAMPS builds only; 0 otherwise)
    uint32_t small_max; // host batches up to this many bytes take k_small (0: never)
    uint32_t zh_tail;        // k_zh: about this many bytes at the batch end go in smaller groups (0: none)
    uint32_t zh_tail_group;  // ... of this many bytes (a multiple of 32, at most the group size)
    uint32_t long_spec;      // long blocks: speculative choices, then (JB_LONG_SPEC) 1 the path chain (default),
                             // 3 the decided chain (round 4), 0 neither (the exact chain); 2 testing: as 1 with
                             // some choices wrong on purpose, so that the exact chain redoes the block
    uint32_t long_fused;     // the long-block kernels as one launch, k_long (JB_LONG_FUSED: 1 default, 0 separate)
    uint32_t ncu;            // the device's CUs (k_long's grid: at most one workgroup per CU)
    uint32_t tok1;           // the span kernels as one pass, k_tok1, for batches of <= 256 token tiles
                             // (JB_TOK1: 1 default, 0 the count/write passes always)
    uint32_t nz_fuse_mib;    // k_nonzh's work inside k_long (fused) for batches of at most this many MiB
                             // (JB_NZ_FUSE_MIB: 4 default, 0 never)
    uint32_t long_wait_ticks;  // k_long: a phase wait gives up after this many 100 MHz ticks without progress
                               // (JB_LONG_WAIT_US x 100; default 20 s)
    int32_t mw_split;        // k_mark_walk: 2^s workgroups per tile, each walking its share of the entries
                             // (JB_MW_SPLIT: -1 = 1 when the batch has at most one tile per CU, else 0; 0-3 fixed)
};

// k_zh's group split: g1 groups of grp bytes, then groups of *sgrp bytes to the end.
// Returns the number of groups.
inline uint64_t zh_tail_groups(uint64_t nbytes, uint32_t grp, const LaunchCfg& lc, uint32_t* g1, uint32_t* sgrp) {
    *sgrp = grp;
    *g1 = (uint32_t)((nbytes + grp - 1) / grp);
    if (lc.zh_tail && lc.zh_tail_group && lc.zh_tail_group < grp && nbytes > lc.zh_tail) {
        *g1 = (uint32_t)((nbytes - lc.zh_tail) / grp);
        *sgrp = lc.zh_tail_group;
    }
    const uint64_t tail0 = (uint64_t)*g1 * grp;
    return *g1 + (tail0 < nbytes ? (nbytes - tail0 + *sgrp - 1) / *sgrp : 0);
}

// Boundary-mask output of one pipeline run (jb_cut_batch_mask): the batch's token
// start / end bits go into the u64 bitmaps s / e at bit offset rel (k_mask_merge)
// instead of becoming spans; the counters still receive the token count.
struct MaskOut {
    uint64_t* s;
    uint64_t* e;
    uint64_t rel;
};

// Enqueue the whole Cut pipeline on `stream`.  Returns hipSuccess or the first
// launch error.  d_text must be readable 64 bytes past nbytes.  mask != nullptr:
// boundary masks instead of spans (tok_start / tok_end / doc_tok are not written).
hipError_t run_pipeline(const DevImage& im, const Work& w, const uint8_t* d_text, uint64_t nbytes,
                        const uint64_t* d_doc_off, uint32_t ndocs, bool hmm, const LaunchCfg& lc,
                        hipStream_t stream, KernelTimer* timer, const MaskOut* mask = nullptr);

// One-workgroup path for small batches (k_small): the text and document offsets
// are read from `text`/`doc_off` (device or mapped pinned host memory; text
// readable 16 bytes past nbytes), the results written to `out`:
//   u32 header[kSmallHdr] (SM_*), u32 tok_start[kSmallBytes], u32 tok_end[kSmallBytes],
//   u64 doc_tok[ndocs + 1]
constexpr uint32_t kSmallBytes = 4096;  // 1024 threads x 4 bytes
constexpr uint32_t kSmallDocs = 4096;
constexpr uint32_t kSmallHdr = 32;
constexpr uint64_t kSmallOutBytes = 4ull * (kSmallHdr + 2ull * kSmallBytes) + 8ull * (kSmallDocs + 1ull);
enum { SM_NTOK = 0, SM_NTOKE, SM_ERR, SM_TIES, SM_BLOCKS, SM_ZHBLOCKS, SM_DONE, SM_CLK = 8 };  // SM_CLK..+10: phase clocks (10 ns ticks)
// A batch small enough to travel in the kernel arguments (text == nullptr): the
// kernel then reads it from the kernarg segment instead of host memory over PCIe.
constexpr uint32_t kSmallInline = 96;  // text bytes (zero-padded)
constexpr uint32_t kSmallInlineDocs = 7;
struct alignas(16) SmallInline {
    uint8_t txt[kSmallInline];
    uint16_t doff[kSmallInlineDocs + 1];  // document offsets, doff[ndocs] = nbytes
    uint32_t pad[4];
};
// out[SM_DONE] = seq is the kernel's last write (after a system-scope release).
hipError_t run_small(const DevImage& im, const uint8_t* text, uint32_t nbytes, const uint64_t* doc_off,
                     uint32_t ndocs, bool hmm, uint32_t* out, uint32_t seq, const SmallInline& in,
                     hipStream_t stream);

// After a pipeline run on `stream`: its counters (u32[CNT_CLEAR]) and the summed
// (blocks, zh blocks) of its tiles (two u64 after them) into `out`, mapped pinned
// host memory of kSnapWords u32, by a one-workgroup kernel.
constexpr uint32_t kSnapWords = CNT_CLEAR + 4;
// Zero `bytes` (a multiple of 4) at p with a kernel on `stream`.
// (and, in the same launch, bytes2 <= 1024 at p2)
hipError_t run_zero(void* p, uint64_t bytes, hipStream_t stream, void* p2 = nullptr, uint32_t bytes2 = 0);
hipError_t run_snap(const Work& w, uint64_t nbytes, uint32_t* out, hipStream_t stream);
// The spans of a pipeline run (ts/te, its counters' token count) packed for the host:
// pk[i] = gap from token i-1's end | length << kPackGapBits (u16), or 0xFFFF with
// (i, start, end) in the side list (counters[CNT_SIDE] entries, at most side_cap);
// hdr[b] = token b x kPackBlock - 1's end (0 for b = 0).  max_tokens bounds the count (the grid).
constexpr uint32_t kPackBlock = 4096;
constexpr uint32_t kPackGapBits = 6;
constexpr uint32_t kPackGapEsc = (1u << kPackGapBits) - 1u;         // gaps from here on are escaped
constexpr uint32_t kPackLenEsc = (1u << (16u - kPackGapBits)) - 1u;  // lengths from here on are escaped
// (an escaped gap covers >= 63 bytes, an escaped token >= 1,023: at most nbytes / 63 + nbytes / 1023 + 2)
inline uint32_t pack_side_cap(uint64_t nbytes) { return (uint32_t)(nbytes / kPackGapEsc + nbytes / kPackLenEsc + 4u); }
hipError_t run_span_pack(const uint32_t* ts, const uint32_t* te, uint32_t* counters, uint16_t* pk, uint32_t* hdr,
                         uint4* side, uint32_t side_cap, uint64_t max_tokens, hipStream_t stream);

// Resident k_zh waves per CU (occupancy API), 4-wave or wide workgroups.
uint32_t zh_waves_per_cu(bool hmm, bool wide);

}  // namespace jb
