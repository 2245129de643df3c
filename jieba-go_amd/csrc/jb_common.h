// jb_common.h — layout of the device-resident segmentation image, shared by the
// host builder (jb_image.cpp) and the gfx950 kernels (jb_kernels.hip).
//
// The image replaces the reference's two Go maps:
//   prefixDictionary.termFreq map[string]int  (tokenizer.go:381-387)
//   hiddenMarkovModel.emitP   map[string]map[string]float64 (tokenizer.go:616-621)
// with flat arrays that a wavefront can probe without strings:
//
//   pagemap[0x110000 >> 8]  u16   rune page -> dense page id (page 0 = empty page;
//                                 pages 0x34..0x9F, U+3400..U+9FFF, are always ids
//                                 1..108 so jb_row() skips the pagemap for them)
//   code[npages * 256]     u32   dense rune code, in order of occurrence in the
//                                 keys (0: the rune is in no key)
//   cells[ncells]           u64   the trie as a double array over rune codes: the
//                                 node of rune r under node s is cell base(s) +
//                                 code(r) when that cell's check is s; level-1
//                                 nodes (single-rune keys) are the cells at their
//                                 codes.
//                                 A cell holds {check, base, freq class,
//                                 has-children, weight index}; a node's id is its
//                                 cell index.
//   emit[npages * 256][4]   f64   emitP[B|M|E|S][string(rune)], minFloat if absent
//   wtab[nw]                f64   distinct weights w = math.Log(float64(freq)) -
//                                 math.Log(float64(size)) (Go's Log, on the host);
//                                 wtab[0] = Log(1.0) - Log(size) for absent runes
//
// Walking one more rune is one 8-byte load (none from a node without
// children).  Only keys that the reference's walk can reach are stored: keys
// made of valid Han runes whose every proper prefix is itself a key (buildDag
// breaks at the first absent string, tokenizer.go:475-478).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define JB_HD __host__ __device__ __forceinline__
#else
#define JB_HD static inline
#endif

#define JB_EMPTY 0xFFFFFFFFu
#define JB_ROOT 0xFFFFFFFEu
#define JB_NPAGES_MAX (0x110000u >> 8)

// freq class
#define JB_FC_ZERO 0u   // freq == 0: a prefix-only entry (e.g. "撙", tokenizer_test.go:126)
#define JB_FC_POS 1u    // freq > 0: a DAG edge (tokenizer.go:479)
#define JB_FC_NEG 2u    // freq < 0: present, no edge, walk continues
#define JB_FC_ABSENT 3u // (l1 only) the single rune is not a key
#define JB_WIDX_ABSENT 0u

// u64 cell: check[0,22) base[22,44) fc[44,46) has_child[46] widx[47,64).
// check = parent id + 1 (0: free cell), JB_CHECK_ROOT for level-1 nodes.
#define JB_CHECK_ROOT 0x3FFFFFu
#define JB_MAX_CELLS (JB_CHECK_ROOT - 2u)
#define JB_MAX_WIDX (1u << 17)
JB_HD uint64_t jb_cell_make(uint32_t check, uint32_t base, uint32_t fc, uint32_t hc, uint32_t widx) {
    return (uint64_t)check | ((uint64_t)base << 22) | ((uint64_t)fc << 44) | ((uint64_t)hc << 46) |
           ((uint64_t)widx << 47);
}
JB_HD uint32_t jb_cell_check(uint64_t c) { return (uint32_t)c & 0x3FFFFFu; }
JB_HD uint32_t jb_cell_base(uint64_t c) { return (uint32_t)(c >> 22) & 0x3FFFFFu; }
JB_HD uint32_t jb_cell_fc(uint64_t c) { return (uint32_t)(c >> 44) & 3u; }
JB_HD uint32_t jb_cell_hc(uint64_t c) { return (uint32_t)(c >> 46) & 1u; }
JB_HD uint32_t jb_cell_widx(uint64_t c) { return (uint32_t)(c >> 47); }

// Row-indexed level-1 table (device only, derived at upload): the cell
// cells[code] of a row with its check field holding the code instead (codes
// are < 2^17) and bit 21 set when that check was JB_CHECK_ROOT, i.e. when the
// single rune is a key.  jb_l1row_cell gives back a cell whose check is the
// root exactly when the original's was (0 otherwise: "absent").
#define JB_L1_ROOTBIT (1u << 21)
JB_HD uint64_t jb_l1row_make(uint32_t code, uint64_t cell) {
    return (cell & ~0x3FFFFFull) | code | (jb_cell_check(cell) == JB_CHECK_ROOT ? JB_L1_ROOTBIT : 0u);
}
JB_HD uint32_t jb_l1row_code(uint64_t v) { return (uint32_t)v & 0x1FFFFu; }
JB_HD uint64_t jb_l1row_cell(uint64_t v) {
    return (v & ~0x3FFFFFull) | (((uint32_t)v & JB_L1_ROOTBIT) ? (uint64_t)JB_CHECK_ROOT : 0ull);
}

// Hot level-1 rows (device only, derived at upload, jb_image.cpp build_hot_rows): the
// l1row values of the runes of U+3400..U+9FFF that text is likeliest to hold, in a
// direct-mapped table of JB_HOT_SLOTS slots (value u64, then tag u16 = the rune,
// 0 = empty).  k_mark_walk keeps it in LDS and gathers l1row only for the others.
#define JB_HOT_SLOTS 512u
JB_HD uint32_t jb_hot_slot(uint32_t r) { return (r * 0x9E3779B1u) >> 23; }

// Pages U+3400..U+9FFF (CJK Ext-A + URO) sit at fixed page ids 1..108.
#define JB_DIRECT_LO 0x3400u
#define JB_DIRECT_N 0x6C00u
#define JB_DIRECT_PAGES 108u

// Row of rune r in l1 / emit.
JB_HD uint32_t jb_row(const uint16_t* pagemap, uint32_t r) {
    if (r - JB_DIRECT_LO < JB_DIRECT_N) return r - 0x3300u;  // ((r>>8) - 0x33) * 256 + (r & 255)
    return (uint32_t)pagemap[r >> 8] * 256u + (r & 255u);
}


// tokenizer.go:19
#define JB_MIN_FLOAT (-3.14e100)

// HMM states in the reference's HMMstates order (tokenizer.go:685)
enum { JB_B = 0, JB_M = 1, JB_E = 2, JB_S = 3 };

// Unicode 13.0.0 Script=Han = Go 1.18 unicode.Han (the `zh` regex, tokenizer.go:21).
JB_HD bool jb_is_han(uint32_t r) {
    if (r >= 0x4E00u) {
        if (r <= 0x9FFCu) return true;
        if (r < 0xF900u) return false;
        if (r <= 0xFA6Du) return true;
        if (r < 0xFA70u) return false;
        if (r <= 0xFAD9u) return true;
        if (r < 0x16FF0u) return false;
        if (r <= 0x16FF1u) return true;
        if (r < 0x20000u) return false;
        if (r <= 0x2A6DDu) return true;
        if (r < 0x2A700u) return false;
        if (r <= 0x2B734u) return true;
        if (r < 0x2B740u) return false;
        if (r <= 0x2B81Du) return true;
        if (r < 0x2B820u) return false;
        if (r <= 0x2CEA1u) return true;
        if (r < 0x2CEB0u) return false;
        if (r <= 0x2EBE0u) return true;
        if (r < 0x2F800u) return false;
        if (r <= 0x2FA1Du) return true;
        if (r < 0x30000u) return false;
        return r <= 0x3134Au;
    }
    if (r >= 0x3400u) return r <= 0x4DBFu;
    if (r < 0x2E80u) return false;
    if (r <= 0x2E99u) return true;
    if (r < 0x2E9Bu) return false;
    if (r <= 0x2EF3u) return true;
    if (r < 0x2F00u) return false;
    if (r <= 0x2FD5u) return true;
    if (r == 0x3005u || r == 0x3007u) return true;
    if (r >= 0x3021u && r <= 0x3029u) return true;
    return r >= 0x3038u && r <= 0x303Bu;
}

// Go unicode.IsSpace (cutNonZh drops these runes, tokenizer.go:302-304).
JB_HD bool jb_is_space(uint32_t r) {
    if (r <= 0xFFu) return (r >= 0x09u && r <= 0x0Du) || r == 0x20u || r == 0x85u || r == 0xA0u;
    return r == 0x1680u || (r >= 0x2000u && r <= 0x200Au) || r == 0x2028u || r == 0x2029u ||
           r == 0x202Fu || r == 0x205Fu || r == 0x3000u;
}

// The `alnum` regex class [a-zA-Z0-9] (tokenizer.go:22).
JB_HD bool jb_is_alnum(uint32_t b) {
    return (b - 'a' < 26u) || (b - 'A' < 26u) || (b - '0' < 10u);
}

// Bytes of x with m < b < n (b < 0x80; m <= 127, n <= 128), bit 7 of each byte.
JB_HD uint32_t jb_bytes_between(uint32_t x, uint32_t m, uint32_t n) {
    const uint32_t t = x & 0x7F7F7F7Fu;
    return ((0x01010101u * (127u + n) - t) & ~x & (t + 0x01010101u * (127u - m))) & 0x80808080u;
}
// Some byte of x is [0-9A-Za-z] (jb_is_alnum), four at once.
JB_HD bool jb_any_alnum4(uint32_t x) {
    return (jb_bytes_between(x, 0x2Fu, 0x3Au) | jb_bytes_between(x | 0x20202020u, 0x60u, 0x7Bu)) != 0u;
}

// Go utf8.DecodeRune on the 4 bytes packed little-endian in x, with `lim`
// (1..4) bytes available. Invalid, truncated, surrogate and overlong sequences
// decode as U+FFFD with width 1. Returns width; writes the rune.
JB_HD uint32_t jb_decode(uint32_t x, uint32_t lim, uint32_t* rune) {
    const uint32_t b0 = x & 0xFFu, b1 = (x >> 8) & 0xFFu, b2 = (x >> 16) & 0xFFu, b3 = x >> 24;
    if (b0 < 0x80u) { *rune = b0; return 1; }
    uint32_t need, lo = 0x80u, hi = 0xBFu, cp;
    if (b0 >= 0xC2u && b0 <= 0xDFu) { need = 2; cp = b0 & 0x1Fu; }
    else if (b0 >= 0xE0u && b0 <= 0xEFu) {
        need = 3; cp = b0 & 0x0Fu;
        if (b0 == 0xE0u) lo = 0xA0u;
        if (b0 == 0xEDu) hi = 0x9Fu;
    } else if (b0 >= 0xF0u && b0 <= 0xF4u) {
        need = 4; cp = b0 & 0x07u;
        if (b0 == 0xF0u) lo = 0x90u;
        if (b0 == 0xF4u) hi = 0x8Fu;
    } else { *rune = 0xFFFDu; return 1; }
    if (need > lim || b1 < lo || b1 > hi) { *rune = 0xFFFDu; return 1; }
    cp = (cp << 6) | (b1 & 0x3Fu);
    if (need >= 3) {
        if ((b2 & 0xC0u) != 0x80u) { *rune = 0xFFFDu; return 1; }
        cp = (cp << 6) | (b2 & 0x3Fu);
    }
    if (need == 4) {
        if ((b3 & 0xC0u) != 0x80u) { *rune = 0xFFFDu; return 1; }
        cp = (cp << 6) | (b3 & 0x3Fu);
    }
    *rune = cp;
    return need;
}
