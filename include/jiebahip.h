/*
 * jiebahip.h — C ABI of libjiebahip.so, the MI355X (gfx950) segmentation path
 * behind jieba-go's Tokenizer API.
 *
 * The reference (ericlingit/jieba-go) is a pure-Go package with no FFI; its
 * boundary is its public Go API.  Each entry point below names
 * the reference interface it replaces.  A Go caller binds these through cgo
 * (INTEGRATION.md); the C++ mirror jieba-go_amd/host/tokenizer.hpp and the
 * Python ctypes binding jieba-go_amd/python/jiebahip.py sit on the same calls.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every function returns JB_OK (0) or a
 *    negative JB_E* code; the library never aborts the process (the reference
 *    calls log.Fatal / panic on load errors, tokenizer.go:397,405,416,443,452,656,660).
 *  - The caller owns every input buffer; nothing is retained past return.
 *  - Outputs returned in jb_spans are owned by the library until jb_spans_free.
 *  - A jb_ctx may be used by several threads at once for cutting (the reference
 *    takes pd.lock.RLock in Cut/CutParallel, tokenizer.go:82-83,152-153);
 *    jb_add_word takes the exclusive lock.
 *  - Token k of the output is the byte range [start[k], end[k]) of the input.
 *    A 1-byte token whose byte is >= 0x80 is an invalid UTF-8 byte, which the
 *    reference emits as "�" (range loop in cutNonZh, tokenizer.go:301-306).
 */
#ifndef JIEBAHIP_H
#define JIEBAHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JB_OK 0
#define JB_EINVAL (-1)  /* bad argument */
#define JB_EIO (-2)     /* file cannot be read (reference: log.Fatal, tokenizer.go:397,443) */
#define JB_EPARSE (-3)  /* dictionary / emission parse error (reference: log.Fatal / panic) */
#define JB_EDEVICE (-4) /* HIP runtime error (no device, launch failure, ...) */
#define JB_ENOMEM (-5)
#define JB_EPANIC (-6)  /* input on which the reference panics (cutDAG slice with tail -1) */
#define JB_ELIMIT (-7)  /* unsupported size (document >= 2 GiB, word > 255 runes) */

typedef struct jb_ctx jb_ctx;
typedef struct jb_image jb_image;

/* Dictionary semantics. */
#define JB_DICT_TXT 0    /* NewTokenizer(dictionaryFile): newPrefixDictionaryFromFile, tokenizer.go:61,389-437
                            (first occurrence wins, size = sum of first occurrences, no prefix entries) */
#define JB_DICT_PREFIX 1 /* dict.txt-format lines read as buildPrefixDictionary does, tokenizer.go:340-366
                            (last value wins, freq-0 prefix entries): the map prefix_dictionary.gob holds */
#define JB_DICT_GOB 2    /* NewJiebaTokenizer(): prefix_dictionary.gob itself, an encoding/gob map[string]int
                            (newJiebaPrefixDictionary, tokenizer.go:69,439-458); size = 60,101,967
                            (tokenizer.go:454) unless size_override > 0 */
#define JB_DICT_IMAGE 3  /* a serialized image written by jb_save / jb_image_save (dictionary, emission
                            table and device arrays; emit_path is ignored): skips parsing and the trie
                            build.  size_override > 0 and different from the saved size rebuilds the weights */
#define JB_JIEBA_SIZE 60101967 /* newJiebaPrefixDictionary's pd.size (tokenizer.go:454) */

typedef struct {
    const char *dict_path;   /* dictionary file in the dict_kind format; NULL: use dict_buf */
    const char *dict_buf;
    size_t dict_len;
    int dict_kind;           /* JB_DICT_TXT or JB_DICT_PREFIX */
    int64_t size_override;   /* > 0 replaces pd.size; NewJiebaTokenizer hard-codes 60_101_967 (tokenizer.go:454) */
    const char *emit_path;   /* prob_emit.json (tokenizer.go:654); NULL: use emit_buf */
    const char *emit_buf;
    size_t emit_len;
    int device;              /* first HIP device ordinal */
    int ndevices;            /* >= 1: documents are sharded over devices device..device+ndevices-1 */
    /* Optional caller-computed logarithms: log_vals[i] is the caller's
     * math.Log(float64(log_keys[i])).  calcDagProba's weights math.Log(tf) - math.Log(pd.size)
     * (tokenizer.go:503,515-519) use these values for the frequencies and the size they
     * cover, and the library's restatement of Go's math.Log (jb_go_log) for the rest, so a
     * Go caller that passes math.Log results gets the reference's weights by construction.
     * The keys a dictionary needs are listed by jb_image_log_keys.  nlog = 0: none. */
    const int64_t *log_keys;
    const double *log_vals;
    size_t nlog;
} jb_config;

typedef struct {
    uint64_t ntokens;
    uint64_t *start;   /* byte offset of each token in the batch */
    uint64_t *end;
    uint64_t *doc_tok; /* ndocs + 1 entries: tokens of document d are [doc_tok[d], doc_tok[d+1]) */
    uint32_t ndocs;
} jb_spans;

/* Replaces NewTokenizer (tokenizer.go:61) and NewJiebaTokenizer (tokenizer.go:69):
 * parse the dictionary and emission table, build the device image and upload it
 * to every configured device. */
int jb_open(const jb_config *cfg, jb_ctx **out);
/* jb_open from an image built by jb_image_build, so the trie is placed once: what the
 * Go binding calls after listing the image's log keys (jb_image_log_keys) and taking
 * math.Log of each (NewTokenizer / NewJiebaTokenizer, tokenizer.go:61-75).  Only
 * cfg->device, cfg->ndevices and the log table (log_keys, log_vals, nlog: the weights
 * are recomputed from them, tokenizer.go:503,515-519) are read.  `img` is consumed on
 * every path, success or not: do not jb_image_free it afterwards. */
int jb_open_image(jb_image *img, const jb_config *cfg, jb_ctx **out);
void jb_close(jb_ctx *ctx);
/* Last error message of the calling thread (never NULL). */
const char *jb_last_error(void);

/* Replaces Tokenizer.Cut (tokenizer.go:151) for one document. */
int jb_cut(jb_ctx *ctx, const uint8_t *text, size_t len, int hmm, jb_spans *out);

/* Replaces Tokenizer.CutParallel (tokenizer.go:81) and batches of Cut calls:
 * ndocs documents concatenated in `text`, document d = [doc_off[d], doc_off[d+1]).
 * Output tokens are in document order (CutParallel with ordered=true; the
 * reference's ordered=false is a block permutation of the same tokens). */
int jb_cut_batch(jb_ctx *ctx, const uint8_t *text, const uint64_t *doc_off, uint32_t ndocs, int hmm,
                 jb_spans *out);
void jb_spans_free(jb_spans *s);

/* jb_cut_batch into caller-owned arrays (no library allocation; what a Go
 * caller passes as slices): start/end hold up to `cap` tokens, doc_tok ndocs+1
 * entries.  *ntokens receives the token count; when it exceeds cap the call
 * returns JB_ELIMIT with *ntokens set and the caller retries with bigger arrays
 * (a batch of n bytes never has more than n tokens). */
int jb_cut_batch_into(jb_ctx *ctx, const uint8_t *text, const uint64_t *doc_off, uint32_t ndocs, int hmm,
                      uint64_t *start, uint64_t *end, uint64_t cap, uint64_t *doc_tok, uint64_t *ntokens);

/* jb_cut_batch_into with u32 outputs, offsets relative to the batch's first byte:
 * token k is the byte range [doc_off[0] + start[k], doc_off[0] + end[k]).  Half the
 * output of the u64 form (what a Go caller slices its strings with: the host side of
 * a host batch is bound by writing the spans, 16 bytes per token there, 8 here).  The
 * batch must be under 4 GiB (JB_ELIMIT otherwise; a caller cuts larger ones in parts);
 * JB_ELIMIT with *ntokens set when the arrays are too small, as jb_cut_batch_into. */
int jb_cut_batch_into32(jb_ctx *ctx, const uint8_t *text, const uint64_t *doc_off, uint32_t ndocs, int hmm,
                        uint32_t *start, uint32_t *end, uint64_t cap, uint64_t *doc_tok, uint64_t *ntokens);

/* Token boundaries as two bitmaps over the batch's bytes instead of spans (2 bits per
 * input byte; 268 MB per GiB instead of 8 bytes per token): bit i of `starts` (word
 * i / 64, bit i % 64) is set when a token begins at byte doc_off[0] + i, bit i of
 * `ends` when a token's last byte is doc_off[0] + i.  Each array holds nwords >=
 * (doc_off[ndocs] - doc_off[0] + 63) / 64 u64 words, and every one of them is written.
 * Tokens never cross a document boundary and never overlap, so start bit k pairs
 * with end bit k in order; a 1-byte token whose byte is >= 0x80 is "�" (as for spans).
 * *ntokens receives the token count.  The host text moves to the device in pieces
 * while earlier pieces are cut and their masks come back (three streams). */
int jb_cut_batch_mask(jb_ctx *ctx, const uint8_t *text, const uint64_t *doc_off, uint32_t ndocs, int hmm,
                      uint64_t *starts, uint64_t *ends, uint64_t nwords, uint64_t *ntokens);

/* Pinned (page-locked) host memory for batch text: a batch that lies in one such
 * allocation is copied to the device straight from it, without the staging copy
 * that pageable memory needs.  A Go caller builds its CutBatch buffer here (C
 * memory, so cgo's pointer rules allow it).  Free with jb_host_free. */
int jb_host_alloc(size_t n, void **p);
void jb_host_free(void *p);

/* Device-resident form for pipelines and benchmarks: d_text (nbytes, plus 64
 * readable padding bytes; 16-byte aligned) and d_doc_off (ndocs+1 offsets, d_doc_off[0] == 0,
 * d_doc_off[ndocs] == nbytes) are device pointers on ctx's first device; the
 * work is queued on `stream` (a hipStream_t; NULL = default stream) and the
 * call returns without synchronising.  Calls on one ctx may come from several
 * threads and streams: each pipeline waits on the device for the previous one
 * (the workspace is one per device).  Results stay in ctx-owned device memory
 * only until the next call on this ctx, from any thread: *d_start / *d_end (u32
 * token spans), *d_doc_tok (u64[ndocs+1]) and *d_ntok (u64 token count).
 * Concurrent callers use jb_cut_device_into. */
int jb_cut_device(jb_ctx *ctx, const uint8_t *d_text, uint64_t nbytes, const uint64_t *d_doc_off,
                  uint32_t ndocs, int hmm, void *stream, uint32_t **d_start, uint32_t **d_end,
                  uint64_t **d_doc_tok, uint64_t **d_ntok);
/* jb_cut_device into caller-owned device arrays, which nothing else writes: d_start /
 * d_end hold cap >= nbytes u32 entries (a batch of n bytes has at most n tokens),
 * d_doc_tok ndocs+1 u64 and *d_ntok the u64 token count, all valid once `stream`
 * reaches the end of this call's work.  Safe from several threads on one ctx. */
int jb_cut_device_into(jb_ctx *ctx, const uint8_t *d_text, uint64_t nbytes, const uint64_t *d_doc_off,
                       uint32_t ndocs, int hmm, void *stream, uint32_t *d_start, uint32_t *d_end, uint64_t cap,
                       uint64_t *d_doc_tok, uint64_t *d_ntok);

/* Error state of the last jb_cut_device / jb_cut_device_into pipeline on ctx's first
 * device (from any thread): synchronises `stream` (the one that call was queued on) and
 * the pipeline, then returns JB_OK, JB_EPANIC (input on which the reference panics:
 * the spans are not the reference's) or JB_EDEVICE (a long-block phase wait gave up,
 * JB_LONG_WAIT_US: the spans are incomplete).  The device calls themselves return
 * before their kernels run, so a caller that must know checks here (a host batch,
 * jb_cut_batch*, returns these codes itself). */
int jb_device_status(jb_ctx *ctx, void *stream);

/* Contiguous byte-balanced ranges of whole documents (the reference's
 * CutParallel deals blocks to goroutines instead, tokenizer.go:81-148), the partition
 * bench.py's one-process-per-GPU runs use (jb_cut_batch itself uses jb_split_points,
 * which may cut inside a document): part k owns documents
 * [cut[k], cut[k+1]), cut has nparts + 1 entries, cut[0] = 0 and
 * cut[nparts] = ndocs.  Host only. */
int jb_shard_bounds(const uint64_t *doc_off, uint32_t ndocs, uint32_t nparts, uint32_t *cut);

/* Byte-balanced split points that may fall inside a document (one
 * large document over several devices): cut has nparts + 1 entries, cut[0] =
 * doc_off[0], cut[nparts] = doc_off[ndocs], and cut[k] is the first document start
 * or Han-run start at or after doc_off[0] + total * k / nparts.  A Han-run start is
 * a byte where a Han rune begins (Go's DecodeRune over the document) and the rune
 * before it is not Han: cutting a document there leaves splitText's blocks
 * (tokenizer.go:165-210) unchanged, and blocks are cut independently
 * (tokenizer.go:158-160), so the parts' tokens are the whole's.  jb_cut_batch
 * shards over its devices with these points.  Host only. */
int jb_split_points(const uint8_t *text, const uint64_t *doc_off, uint32_t ndocs, uint32_t nparts, uint64_t *cut);

/* Replaces Tokenizer.AddWord (tokenizer.go:372; the reference deadlocks there,
 * :376 + :581).  freq < 1 takes suggestFreq's value (tokenizer.go:589-614).
 * Atomic: on any error (JB_ELIMIT for an all-Han word of more than 255 runes -- the
 * trie holds only all-Han keys, so a longer word with a non-Han rune is stored in
 * the dictionary and never walked; JB_EDEVICE, JB_ENOMEM) the dictionary, pd.size
 * and every device's image stay as they were. */
int jb_add_word(jb_ctx *ctx, const char *word, size_t len, int64_t freq);

/* suggestFreq (tokenizer.go:589-614): the frequency AddWord(word, freq < 1) would store. */
int jb_suggest_freq(jb_ctx *ctx, const char *word, size_t len, int64_t *freq);

/* Add caller-computed logarithms (as jb_config.log_keys/log_vals) to ctx's table: they
 * apply from the next image build, i.e. the next jb_add_word.  A Go AddWord passes
 * math.Log of the new frequency and of the new pd.size before calling jb_add_word. */
int jb_add_log(jb_ctx *ctx, const int64_t *keys, const double *vals, size_t n);

/* Dictionary introspection (prefixDictionary.termFreq / size, tokenizer.go:382-383). */
int jb_dict_get(jb_ctx *ctx, const char *word, size_t len, int64_t *freq); /* 1 found, 0 absent */
int64_t jb_dict_size(jb_ctx *ctx);

/* Counters of the last cut on each device of ctx, summed over the devices (a host
 * batch cut in pieces: summed over its pieces).  Synchronises the devices' streams.
 * After a device pipeline (jb_cut_device*) it fills *out and also returns that
 * pipeline's error state, as jb_device_status does.
 * Concurrent small calls (jb_cut of at most 4 KiB) are coalesced into shared k_small
 * batches: after one, the counters are those of the k_small batch that finished last
 * on the device, which may hold other callers' documents beside this caller's. */
typedef struct {
    uint64_t tokens;       /* tokens written */
    uint64_t blocks;       /* splitText blocks, zh and non-zh (tokenizer.go:165-210) */
    uint64_t zh_blocks;    /* of which Han runs (cutZh, tokenizer.go:221) */
    uint64_t long_blocks;  /* zh blocks of >= 8 KiB, cut by the long-block kernel */
    uint64_t viterbi_ties; /* exact stateTransitionRoute ties a == b > minFloat, which the reference
                              resolves in Go's random map order (tokenizer.go:748-753); here the first
                              candidate of stateChange wins */
} jb_stats;
int jb_last_stats(jb_ctx *ctx, jb_stats *out);

/* Per-kernel timing with HIP events on the launch stream (bench / profiling). */
int jb_profile_enable(jb_ctx *ctx, int on);
/* Fills up to cap entries: kernel name, total ms, launches. Synchronises. Returns #entries. */
int jb_profile_read(jb_ctx *ctx, const char **names, double *ms, uint64_t *launches, int cap);
int jb_profile_reset(jb_ctx *ctx);

/* Write ctx's current image (including words added by jb_add_word) to `path`,
 * to be opened later with dict_kind JB_DICT_IMAGE: the fast-start counterpart of
 * the reference shipping prefix_dictionary.gob instead of rebuilding the map
 * from dict.txt (tokenizer.go:439-458 vs :389-437). */
int jb_save(jb_ctx *ctx, const char *path);

/* ---- host-only image access (no GPU needed; used by CPU tests) ---------- */
int jb_image_build(const jb_config *cfg, jb_image **out);
void jb_image_free(jb_image *img);
int jb_image_save(const jb_image *img, const char *path);
/* prefixDictionary view of an image: number of termFreq entries and pd.size. */
int jb_image_dict_info(const jb_image *img, uint64_t *nentries, int64_t *size);
/* Look up a key as the device walk sees it: returns 1 if reachable, with freq and w. */
int jb_image_lookup(const jb_image *img, const char *word, size_t len, int64_t *freq, double *w);
/* nodes stored, hash capacity, pages, max key length in runes, size, -Log(size) */
int jb_image_stats(const jb_image *img, uint64_t *nodes, uint64_t *cap, uint32_t *npages, uint32_t *maxlen,
                   int64_t *size, double *w_absent);
/* emitP[state][string(rune)] as the device sees it (minFloat if absent). */
double jb_image_emit(const jb_image *img, int state, uint32_t rune);
/* The x whose math.Log(float64(x)) the image's weights use (every frequency of a key a
 * Han run can spell, 1 for absent pieces, and pd.size), ascending and distinct: what a
 * caller fills jb_config.log_keys with.  *n receives the count; returns JB_ELIMIT when
 * it exceeds cap (keys may be NULL with cap 0 to ask for the count). */
int jb_image_log_keys(const jb_image *img, int64_t *keys, size_t cap, size_t *n);
/* Go math.Log as used for the weights (src/math/log.go algorithm). */
double jb_go_log(double x);

#ifdef __cplusplus
}
#endif
#endif /* JIEBAHIP_H */
