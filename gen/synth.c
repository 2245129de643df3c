/*
 * gen/synth.c — seeded synthetic data for tests and bench.
 *
 * The real jieba data files are Git-LFS pointers in the reference, so every
 * measurement and parity test runs on synthetic data of the same shape:
 *   D_syn  dictionary (dict.txt format: "word freq tag" lines), seed 1
 *   E_syn  emission table (prob_emit.json format), seed 2
 *   C_syn  Zipf corpus documents, seed 3 + document index
 * Generation is deterministic in the seeds and independent of the caller's
 * sharding (document k always uses seed 3 + k), so ranks of a multi-GPU run
 * can each generate their own shard.
 *
 * This is test/bench infrastructure, not part of the shipped library.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define API __attribute__((visibility("default")))

typedef struct { uint64_t s; } rng_t;
static uint64_t rnext(rng_t *r) { /* splitmix64 */
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static double runif(rng_t *r) { return (double)(rnext(r) >> 11) * (1.0 / 9007199254740992.0); }
static uint32_t rint_(rng_t *r, uint32_t n) { return (uint32_t)(runif(r) * n); }

static int enc(uint32_t r, uint8_t *o) {
    if (r < 0x80) { o[0] = (uint8_t)r; return 1; }
    if (r < 0x800) { o[0] = 0xC0 | (r >> 6); o[1] = 0x80 | (r & 0x3F); return 2; }
    if (r < 0x10000) { o[0] = 0xE0 | (r >> 12); o[1] = 0x80 | ((r >> 6) & 0x3F); o[2] = 0x80 | (r & 0x3F); return 3; }
    o[0] = 0xF0 | (r >> 18); o[1] = 0x80 | ((r >> 12) & 0x3F); o[2] = 0x80 | ((r >> 6) & 0x3F); o[3] = 0x80 | (r & 0x3F);
    return 4;
}

#define HAN0 0x4E00u
#define NHAN (0x9FA5u - 0x4E00u + 1u) /* 20,902 chars */
#define MAXW 24

typedef struct {
    uint32_t nwords;
    uint32_t *wlen;   /* runes per word */
    uint32_t *wr;     /* runes, MAXW per word */
    int64_t *freq;
    double *wcdf;     /* Zipf(1.0) cumulative over word rank, for corpus sampling */
    uint32_t *chars;  /* chars by Zipf rank (permutation of the Han range) */
    double *ccdf;     /* Zipf(1.1) cumulative over char rank */
    uint32_t *zero1;  /* chars written as explicit "c 0" lines */
    uint32_t nzero1;
    uint32_t maxlen;
} syn_t;

static uint32_t sample_cdf(const double *cdf, uint32_t n, double u) {
    uint32_t lo = 0, hi = n - 1;
    double x = u * cdf[n - 1];
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* open-addressing set of words (hash of the rune sequence) */
typedef struct { uint64_t *h; uint32_t cap; } hset_t;
static uint64_t whash(const uint32_t *r, uint32_t n) {
    uint64_t h = 1469598103934665603ULL ^ n;
    for (uint32_t i = 0; i < n; i++) { h ^= r[i]; h *= 1099511628211ULL; h ^= h >> 29; }
    return h | 1;
}
static int hset_add(hset_t *s, uint64_t h) {
    uint32_t i = (uint32_t)h & (s->cap - 1);
    while (s->h[i]) { if (s->h[i] == h) return 0; i = (i + 1) & (s->cap - 1); }
    s->h[i] = h;
    return 1;
}

/* Build D_syn: nwords unique words, lengths 1:6% 2:55% 3:24% 4:12% 5-8:3%,
 * plus a few long words (9-16 runes) so walks and rings see longer entries. */
API void *syn_new(uint64_t seed, uint32_t nwords) {
    rng_t r = {seed};
    syn_t *s = calloc(1, sizeof(syn_t));
    s->chars = malloc(sizeof(uint32_t) * NHAN);
    for (uint32_t i = 0; i < NHAN; i++) s->chars[i] = HAN0 + i;
    for (uint32_t i = NHAN - 1; i > 0; i--) { uint32_t j = rint_(&r, i + 1); uint32_t t = s->chars[i]; s->chars[i] = s->chars[j]; s->chars[j] = t; }
    s->ccdf = malloc(sizeof(double) * NHAN);
    double acc = 0;
    for (uint32_t i = 0; i < NHAN; i++) { acc += 1.0 / pow((double)(i + 1), 1.1); s->ccdf[i] = acc; }
    /* 1% of chars (outside the top 2k) get an explicit freq-0 line; 2% more are
     * never single-char words, so the prefix semantics gives them freq 0. */
    uint8_t *nosingle = calloc(NHAN, 1);
    s->zero1 = malloc(sizeof(uint32_t) * NHAN);
    for (uint32_t i = 2000; i < NHAN; i++) {
        double u = runif(&r);
        if (u < 0.01) { s->zero1[s->nzero1++] = s->chars[i]; nosingle[i] = 1; }
        else if (u < 0.03) nosingle[i] = 1;
    }
    uint32_t nlong = nwords >= 10000 ? 40 : 0;
    s->nwords = nwords;
    s->wlen = malloc(sizeof(uint32_t) * nwords);
    s->wr = malloc(sizeof(uint32_t) * (size_t)nwords * MAXW);
    s->freq = malloc(sizeof(int64_t) * nwords);
    hset_t hs;
    hs.cap = 1;
    while (hs.cap < nwords * 4u) hs.cap <<= 1;
    hs.h = calloc(hs.cap, sizeof(uint64_t));
    uint32_t w = 0, guard = 0;
    while (w < nwords && guard < nwords * 50u) {
        guard++;
        uint32_t len;
        if (w >= nwords - nlong) len = 9 + rint_(&r, 8);
        else {
            double u = runif(&r);
            len = u < 0.06 ? 1 : u < 0.61 ? 2 : u < 0.85 ? 3 : u < 0.97 ? 4 : 5 + rint_(&r, 4);
        }
        uint32_t *rr = s->wr + (size_t)w * MAXW;
        for (uint32_t k = 0; k < len; k++) {
            uint32_t ci = sample_cdf(s->ccdf, NHAN, runif(&r));
            if (len == 1 && nosingle[ci]) { k--; continue; }
            rr[k] = s->chars[ci];
        }
        if (!hset_add(&hs, whash(rr, len))) continue;
        s->wlen[w] = len;
        if (len > s->maxlen) s->maxlen = len;
        w++;
    }
    s->nwords = w;
    /* Zipf(1.0) frequencies by rank (rank = generation order), total ~ 60,101,967 */
    double H = 0;
    for (uint32_t i = 0; i < w; i++) H += 1.0 / (i + 1);
    double C = 60101967.0 / H;
    s->wcdf = malloc(sizeof(double) * w);
    acc = 0;
    for (uint32_t i = 0; i < w; i++) {
        int64_t f = (int64_t)llround(C / (i + 1));
        s->freq[i] = f < 1 ? 1 : f;
        acc += 1.0 / (i + 1);
        s->wcdf[i] = acc;
    }
    free(hs.h);
    free(nosingle);
    return s;
}

API void syn_free(void *h) {
    syn_t *s = h;
    if (!s) return;
    free(s->wlen); free(s->wr); free(s->freq); free(s->wcdf); free(s->chars); free(s->ccdf); free(s->zero1);
    free(s);
}
API uint32_t syn_nwords(void *h) { return ((syn_t *)h)->nwords; }
API uint32_t syn_maxlen(void *h) { return ((syn_t *)h)->maxlen; }

/* dict.txt lines "word freq tag". Adds the explicit freq-0 single chars and
 * 0.1% duplicate lines with a different freq (first-wins vs last-wins). */
API long syn_write_dict(void *h, uint64_t seed, const char *path) {
    syn_t *s = h;
    rng_t r = {seed ^ 0xD1C7ULL};
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    static const char *tags[] = {"n", "v", "a", "d", "nr", "ns", "vn", "m"};
    uint8_t buf[MAXW * 4 + 8];
    long lines = 0;
    for (uint32_t i = 0; i < s->nwords; i++) {
        int l = 0;
        for (uint32_t k = 0; k < s->wlen[i]; k++) l += enc(s->wr[(size_t)i * MAXW + k], buf + l);
        fwrite(buf, 1, (size_t)l, f);
        fprintf(f, " %lld %s\n", (long long)s->freq[i], tags[rint_(&r, 8)]);
        lines++;
        if (runif(&r) < 0.001) {
            fwrite(buf, 1, (size_t)l, f);
            fprintf(f, " %lld %s\n", (long long)(1 + rint_(&r, 1000)), tags[rint_(&r, 8)]);
            lines++;
        }
    }
    for (uint32_t i = 0; i < s->nzero1; i++) {
        int l = enc(s->zero1[i], buf);
        fwrite(buf, 1, (size_t)l, f);
        fprintf(f, " 0\n");
        lines++;
    }
    fclose(f);
    return lines;
}

/* E_syn: S over the top 12k chars, B/E/M over 60%/60%/40% random subsets of
 * the top 7k; values uniform in [-16, -2], printed round-trip exact. */
API long syn_write_emit(void *h, uint64_t seed, const char *path) {
    syn_t *s = h;
    rng_t r = {seed};
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    const char *names[4] = {"B", "E", "M", "S"};
    const double frac[4] = {0.6, 0.6, 0.4, 1.0};
    const uint32_t top[4] = {7000, 7000, 7000, 12000};
    uint8_t buf[8];
    long n = 0;
    fprintf(f, "{");
    for (int st = 0; st < 4; st++) {
        fprintf(f, "%s\"%s\":{", st ? "," : "", names[st]);
        int first = 1;
        for (uint32_t i = 0; i < top[st] && i < NHAN; i++) {
            if (runif(&r) >= frac[st]) continue;
            double v = -2.0 - 14.0 * runif(&r);
            int l = enc(s->chars[i], buf);
            fprintf(f, "%s\"", first ? "" : ",");
            fwrite(buf, 1, (size_t)l, f);
            fprintf(f, "\":%.17g", v);
            first = 0;
            n++;
        }
        fprintf(f, "}");
    }
    fprintf(f, "}\n");
    fclose(f);
    return n;
}

/* ---- corpus ---------------------------------------------------------------- */
typedef struct {
    uint8_t *o;
    size_t n, cap;
    uint64_t runes;
    int overflow;
} out_t;

static void put(out_t *o, const uint8_t *b, size_t l, uint64_t runes) {
    if (o->n + l > o->cap) { o->overflow = 1; return; }
    memcpy(o->o + o->n, b, l);
    o->n += l;
    o->runes += runes;
}
static void put_rune(out_t *o, uint32_t r) { uint8_t b[4]; int l = enc(r, b); put(o, b, (size_t)l, 1); }

static void put_word(syn_t *s, rng_t *r, out_t *o) {
    uint32_t w = sample_cdf(s->wcdf, s->nwords, runif(r));
    for (uint32_t k = 0; k < s->wlen[w]; k++) put_rune(o, s->wr[(size_t)w * MAXW + k]);
}
static void put_oov(rng_t *r, out_t *o, uint32_t n) {
    for (uint32_t k = 0; k < n; k++) put_rune(o, 0x3400 + rint_(r, 0x4DBF - 0x3400 + 1)); /* CJK Ext-A */
}
static void put_ascii(rng_t *r, out_t *o) {
    uint8_t b[16];
    int l = 0;
    b[l++] = ' ';
    uint32_t nl = 2 + rint_(r, 7), nd = rint_(r, 4);
    for (uint32_t k = 0; k < nl; k++) b[l++] = (uint8_t)('a' + rint_(r, 26));
    for (uint32_t k = 0; k < nd; k++) b[l++] = (uint8_t)('0' + rint_(r, 10));
    b[l++] = ' ';
    put(o, b, (size_t)l, (uint64_t)l);
}

static const uint32_t JOIN[] = {0xFF0C, 0x3001, 0xFF1B, 0xFF1A};  /* ，、；： */
static const uint32_t END[] = {0x3002, 0xFF01, 0xFF1F};           /* 。！？ */
static const uint32_t ODD[] = {0x3000, 0xFF08, 0xFF09, 0x300C, 0x300D, 0xFF0E}; /* U+3000, （）「」．*/

static void put_clause(syn_t *s, rng_t *r, out_t *o) {
    uint32_t nw = 1 + rint_(r, 12);
    int ascii_at = runif(r) < 0.03 ? (int)rint_(r, nw) : -1;
    for (uint32_t k = 0; k < nw; k++) {
        if ((int)k == ascii_at) put_ascii(r, o);
        if (runif(r) < 0.05) put_oov(r, o, 1 + rint_(r, 3));
        else put_word(s, r, o);
    }
}
static void put_sentence(syn_t *s, rng_t *r, out_t *o) {
    uint32_t nc = 1 + rint_(r, 4);
    for (uint32_t c = 0; c < nc; c++) {
        put_clause(s, r, o);
        if (runif(r) < 0.01) put_rune(o, ODD[rint_(r, 6)]);
        if (c + 1 < nc) put_rune(o, JOIN[rint_(r, 4)]);
    }
    put_rune(o, END[rint_(r, 3)]);
}

/*
 * kind 0: C_syn documents (20-200 sentences each), document k seeded 3 + k,
 *         k = doc0, doc0+1, ... until target_bytes or max_docs is reached.
 * kind 1: S10k-style: each document one sentence of 10-40 runes.
 * kind 2: L1M punctuated: one document of target_runes runes.
 * kind 3: L1M unpunctuated, ~30% Ext-A OOV runes (long singleton runs).
 * Returns bytes written; doc_off gets ndocs+1 offsets.
 */
API long long syn_corpus(void *h, int kind, uint64_t doc0, uint64_t max_docs, uint64_t target_bytes,
                         uint64_t target_runes, uint8_t *out, uint64_t cap, uint64_t *doc_off,
                         uint64_t *ndocs_out, uint64_t *nrunes_out) {
    syn_t *s = h;
    out_t o = {out, 0, cap, 0, 0};
    uint64_t d = 0;
    doc_off[0] = 0;
    if (kind == 2 || kind == 3) {
        rng_t r = {3 + doc0};
        while (o.runes < target_runes && !o.overflow) {
            if (kind == 2) put_sentence(s, &r, &o);
            else if (runif(&r) < 0.33) put_oov(&r, &o, 1 + rint_(&r, 3));
            else put_word(s, &r, &o);
        }
        d = 1;
        doc_off[1] = o.n;
    } else {
        while (d < max_docs && o.n < target_bytes && !o.overflow) {
            rng_t r = {3 + doc0 + d};
            size_t before = o.n;
            uint64_t rb = o.runes;
            if (kind == 0) {
                uint32_t ns = 20 + rint_(&r, 181);
                for (uint32_t k = 0; k < ns; k++) put_sentence(s, &r, &o);
            } else {
                uint32_t want = 10 + rint_(&r, 31);
                while (o.runes - rb < want && !o.overflow) {
                    if (runif(&r) < 0.05) put_oov(&r, &o, 1 + rint_(&r, 3));
                    else put_word(s, &r, &o);
                    if (o.runes - rb + 2 < want && runif(&r) < 0.12) put_rune(&o, JOIN[rint_(&r, 4)]);
                }
                put_rune(&o, END[rint_(&r, 3)]);
            }
            if (o.overflow) { o.n = before; o.runes = rb; break; }
            d++;
            doc_off[d] = o.n;
        }
    }
    *ndocs_out = d;
    *nrunes_out = o.runes;
    return (long long)o.n;
}
