/*
 * oracle/jieba_oracle.c — TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * A plain-C, CPU-only restatement of ericlingit/jieba-go `tokenizer.go` (Go 1.18,
 * /root/reference/tokenizer.go).  It follows the reference's algorithm step by
 * step — string-keyed prefix map, DAG as per-position lists, backward
 * `calcDagProba`, `maxIndexProba`, forward `findDagPath`, Viterbi with literal
 * per-state path copying — so that its outputs can be compared with the
 * MI355X path.  Each function cites the reference file:line it restates.
 *
 * Who may use this file: only tests/, __graft_entry__.smoke() and bench.py's
 * `cpu_baseline` leg, and only as the checker / the timed CPU baseline.  The
 * product (libjiebahip.so) never links, loads or calls it.
 *
 * Pinning: the Go reference cannot be built or run in this image (no Go
 * toolchain; the jieba data files are Git-LFS pointers — SURVEY.md §8c).  This
 * restatement is pinned by the reference's own data-free known-answer tests
 * (tokenizer_test.go TestSplitText, TestMaxIndexProba, TestFindDagPath,
 * TestStateTransitionRoute, TestCutHMM, TestCutNonZh, TestBuildPrefixDict,
 * TestAddWord) restated as fixtures in tests/golden/, plus a mini dictionary
 * consistent with TestBuildDAG that reproduces TestCut "cut 8"/"cut 10".
 * Parity against real jieba data is unpinned (data absent).
 *
 * Deterministic choices where the reference is nondeterministic:
 *  - Viterbi exact route ties (tokenizer.go:748-753 iterate a Go map, random
 *    order): candidates are visited in `stateChange` order (:24-29) with the
 *    reference's strict `>`; every exact tie is counted in `ties` so tests can
 *    tell tie-ambiguous positions apart.
 *
 * Go semantics restated from the Go 1.18 standard library (no third-party
 * code in go.mod):
 *  - utf8.DecodeRune: invalid / truncated / surrogate / overlong sequences
 *    decode as U+FFFD with width 1.
 *  - unicode.Han (Unicode 13.0.0, 19 ranges) and unicode.IsSpace.
 *  - math.Log: the FreeBSD e_log.c algorithm of src/math/log.go (the amd64
 *    assembly computes the same operations in the same order).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define OR_API __attribute__((visibility("default")))

static const double minFloat = -3.14e100; /* tokenizer.go:19 */

/* ------------------------------------------------------------------------- */
/* Go math.Log (src/math/log.go, Go 1.18)                                      */
/* ------------------------------------------------------------------------- */
OR_API double or_go_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                 L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                 L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    if (isnan(x) || x == INFINITY) return x;
    if (x < 0) return NAN;
    if (x == 0) return -INFINITY;
    int ki;
    double f1 = frexp(x, &ki);
    if (f1 < 0.70710678118654752440 /* Sqrt2/2 */) {
        f1 *= 2;
        ki--;
    }
    double f = f1 - 1;
    double k = (double)ki;
    double s = f / (2 + f);
    double s2 = s * s;
    double s4 = s2 * s2;
    double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    double R = t1 + t2;
    double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

/* ------------------------------------------------------------------------- */
/* Go UTF-8 decoding + unicode tables                                          */
/* ------------------------------------------------------------------------- */
/* utf8.DecodeRune semantics; n = bytes available. */
static int go_decode(const uint8_t *s, size_t n, uint32_t *r) {
    if (n == 0) { *r = 0xFFFD; return 0; }
    uint8_t b0 = s[0];
    if (b0 < 0x80) { *r = b0; return 1; }
    int need; uint32_t lo = 0x80, hi = 0xBF, cp;
    if (b0 >= 0xC2 && b0 <= 0xDF) { need = 1; cp = b0 & 0x1F; }
    else if (b0 >= 0xE0 && b0 <= 0xEF) {
        need = 2; cp = b0 & 0x0F;
        if (b0 == 0xE0) lo = 0xA0;
        if (b0 == 0xED) hi = 0x9F;
    } else if (b0 >= 0xF0 && b0 <= 0xF4) {
        need = 3; cp = b0 & 0x07;
        if (b0 == 0xF0) lo = 0x90;
        if (b0 == 0xF4) hi = 0x8F;
    } else { *r = 0xFFFD; return 1; }
    if ((size_t)need + 1 > n) { *r = 0xFFFD; return 1; }
    uint8_t b1 = s[1];
    if (b1 < lo || b1 > hi) { *r = 0xFFFD; return 1; }
    cp = (cp << 6) | (b1 & 0x3F);
    for (int k = 2; k <= need; k++) {
        uint8_t b = s[k];
        if (b < 0x80 || b > 0xBF) { *r = 0xFFFD; return 1; }
        cp = (cp << 6) | (b & 0x3F);
    }
    *r = cp;
    return need + 1;
}

static int go_encode(uint32_t r, uint8_t *o) {
    if (r < 0x80) { o[0] = (uint8_t)r; return 1; }
    if (r < 0x800) { o[0] = 0xC0 | (r >> 6); o[1] = 0x80 | (r & 0x3F); return 2; }
    if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = 0xFFFD;
    if (r < 0x10000) {
        o[0] = 0xE0 | (r >> 12); o[1] = 0x80 | ((r >> 6) & 0x3F); o[2] = 0x80 | (r & 0x3F);
        return 3;
    }
    o[0] = 0xF0 | (r >> 18); o[1] = 0x80 | ((r >> 12) & 0x3F);
    o[2] = 0x80 | ((r >> 6) & 0x3F); o[3] = 0x80 | (r & 0x3F);
    return 4;
}

/* unicode.Han, Unicode 13.0.0 (Go 1.18 tables.go _Han) */
static const uint32_t han_ranges[][2] = {
    {0x2E80, 0x2E99}, {0x2E9B, 0x2EF3}, {0x2F00, 0x2FD5}, {0x3005, 0x3005}, {0x3007, 0x3007},
    {0x3021, 0x3029}, {0x3038, 0x303B}, {0x3400, 0x4DBF}, {0x4E00, 0x9FFC}, {0xF900, 0xFA6D},
    {0xFA70, 0xFAD9}, {0x16FF0, 0x16FF1}, {0x20000, 0x2A6DD}, {0x2A700, 0x2B734},
    {0x2B740, 0x2B81D}, {0x2B820, 0x2CEA1}, {0x2CEB0, 0x2EBE0}, {0x2F800, 0x2FA1D},
    {0x30000, 0x3134A}};

OR_API int or_is_han(uint32_t r) {
    for (size_t i = 0; i < sizeof(han_ranges) / sizeof(han_ranges[0]); i++)
        if (r >= han_ranges[i][0] && r <= han_ranges[i][1]) return 1;
    return 0;
}

/* unicode.IsSpace (Go 1.18 unicode/graphic.go + White_Space table) */
OR_API int or_is_space(uint32_t r) {
    if (r <= 0xFF) {
        switch (r) {
        case '\t': case '\n': case '\v': case '\f': case '\r': case ' ': case 0x85: case 0xA0:
            return 1;
        }
        return 0;
    }
    return r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 ||
           r == 0x202F || r == 0x205F || r == 0x3000;
}

static int is_alnum_byte(uint8_t b) {
    return (b >= 'a' && b <= 'z') || (b >= 'A' && b <= 'Z') || (b >= '0' && b <= '9');
}

/* ------------------------------------------------------------------------- */
/* string -> int map (Go map[string]int stand-in)                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    char *key;
    uint32_t klen;
    int64_t val;
    uint64_t hash;
} kv_t;

typedef struct {
    kv_t *slots;
    size_t cap, n;
} smap_t;

static uint64_t fnv1a(const void *p, size_t n) {
    const uint8_t *s = (const uint8_t *)p;
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; i++) { h ^= s[i]; h *= 1099511628211ULL; }
    return h ? h : 1;
}

static void smap_init(smap_t *m, size_t cap) {
    size_t c = 16;
    while (c < cap * 2) c <<= 1;
    m->slots = (kv_t *)calloc(c, sizeof(kv_t));
    m->cap = c;
    m->n = 0;
}

static void smap_free(smap_t *m) {
    for (size_t i = 0; i < m->cap; i++) free(m->slots[i].key);
    free(m->slots);
    m->slots = NULL;
}

static kv_t *smap_find_slot(const smap_t *m, const void *k, size_t kl, uint64_t h) {
    size_t mask = m->cap - 1, i = h & mask;
    for (;;) {
        kv_t *e = &m->slots[i];
        if (!e->hash) return e;
        if (e->hash == h && e->klen == kl && memcmp(e->key, k, kl) == 0) return e;
        i = (i + 1) & mask;
    }
}

static int smap_get(const smap_t *m, const void *k, size_t kl, int64_t *v) {
    kv_t *e = smap_find_slot(m, k, kl, fnv1a(k, kl));
    if (!e->hash) return 0;
    *v = e->val;
    return 1;
}

static void smap_grow(smap_t *m) {
    smap_t n2;
    n2.cap = m->cap * 2;
    n2.slots = (kv_t *)calloc(n2.cap, sizeof(kv_t));
    n2.n = m->n;
    for (size_t i = 0; i < m->cap; i++)
        if (m->slots[i].hash) *smap_find_slot(&n2, m->slots[i].key, m->slots[i].klen, m->slots[i].hash) = m->slots[i];
    free(m->slots);
    *m = n2;
}

static void smap_put(smap_t *m, const void *k, size_t kl, int64_t v) {
    if ((m->n + 1) * 2 > m->cap) smap_grow(m);
    uint64_t h = fnv1a(k, kl);
    kv_t *e = smap_find_slot(m, k, kl, h);
    if (!e->hash) {
        e->hash = h;
        e->key = (char *)malloc(kl ? kl : 1);
        memcpy(e->key, k, kl);
        e->klen = (uint32_t)kl;
        m->n++;
    }
    e->val = v;
}

/* ------------------------------------------------------------------------- */
/* strconv.Atoi (base 10, int64)                                              */
/* ------------------------------------------------------------------------- */
static int go_atoi(const char *s, size_t n, int64_t *out) {
    size_t i = 0;
    int neg = 0;
    if (n == 0) return -1;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i == n) return -1;
    uint64_t acc = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return -1;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (acc > (UINT64_MAX - d) / 10) return -1;
        acc = acc * 10 + d;
    }
    if (!neg && acc > (uint64_t)INT64_MAX) return -1;
    if (neg && acc > (uint64_t)INT64_MAX + 1) return -1;
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Tokenizer context                                                          */
/* ------------------------------------------------------------------------- */
typedef struct {
    smap_t tf;      /* prefixDictionary.termFreq (tokenizer.go:382) */
    int64_t size;   /* prefixDictionary.size (tokenizer.go:383) */
    smap_t emit[4]; /* hiddenMarkovModel.emitP, states B,M,E,S as double bits */
    int has_emit[4];
    long long ties; /* exact Viterbi route ties seen (Q12) */
    pthread_mutex_t mu;
} or_ctx;

enum { ST_B = 0, ST_M = 1, ST_E = 2, ST_S = 3, ST_NONE = -1 };
static const char ST_CH[4] = {'B', 'M', 'E', 'S'};

/* newJiebaHMM start/transition literals (tokenizer.go:629-652) */
static double startP(int s) {
    switch (s) {
    case ST_B: return -0.26268660809250016;
    case ST_E: return minFloat;
    case ST_M: return minFloat;
    default: return -1.4652633398537678;
    }
}
static double transP(int from, int to) {
    if (from == ST_B && to == ST_E) return -0.51082562376599;
    if (from == ST_B && to == ST_M) return -0.916290731874155;
    if (from == ST_E && to == ST_B) return -0.5897149736854513;
    if (from == ST_E && to == ST_S) return -0.8085250474669937;
    if (from == ST_M && to == ST_E) return -0.33344856811948514;
    if (from == ST_M && to == ST_M) return -1.2603623820268226;
    if (from == ST_S && to == ST_B) return -0.7211965654669841;
    if (from == ST_S && to == ST_S) return -0.6658631448798212;
    return NAN; /* never used: stateChange only names the pairs above */
}
/* stateChange (tokenizer.go:24-29) */
static const int stateChange[4][2] = {
    /* B */ {ST_E, ST_S}, /* M */ {ST_B, ST_M}, /* E */ {ST_B, ST_M}, /* S */ {ST_E, ST_S}};

/* ---- line splitting shared by both dictionary loaders -------------------- */
typedef struct {
    const char *p;
    size_t n;
} sv_t;

/* bufio.ScanLines: split at '\n', drop one trailing '\r'; the final
 * unterminated segment counts if non-empty. Returns 0 at end. */
static int next_line(const char *buf, size_t len, size_t *pos, sv_t *line) {
    if (*pos >= len) return 0;
    size_t s = *pos, e = s;
    while (e < len && buf[e] != '\n') e++;
    *pos = e < len ? e + 1 : e;
    size_t l = e - s;
    if (l > 0 && buf[s + l - 1] == '\r') l--;
    line->p = buf + s;
    line->n = l;
    return 1;
}

/* strings.SplitN(line, " ", 3): word = parts[0], parts[1] must exist. */
static int split_word_count(sv_t line, sv_t *word, int64_t *count) {
    const char *sp = memchr(line.p, ' ', line.n);
    if (!sp) return -2; /* parts[1] index out of range: the reference panics */
    word->p = line.p;
    word->n = (size_t)(sp - line.p);
    const char *c = sp + 1;
    size_t rest = line.n - word->n - 1;
    const char *sp2 = memchr(c, ' ', rest);
    size_t cl = sp2 ? (size_t)(sp2 - c) : rest;
    if (go_atoi(c, cl, count) != 0) return -3; /* log.Fatal(err) */
    return 0;
}

/* newPrefixDictionaryFromFile (tokenizer.go:389-437): first occurrence wins,
 * size sums first occurrences, no prefix entries. */
static int load_dict_txt(or_ctx *c, const char *buf, size_t len) {
    size_t pos = 0;
    sv_t line, word;
    int64_t cnt;
    smap_init(&c->tf, len / 14 + 16);
    c->size = 0;
    while (next_line(buf, len, &pos, &line)) {
        if (line.n > 65535) break; /* bufio.Scanner ErrTooLong ends the loop silently */
        int rc = split_word_count(line, &word, &cnt);
        if (rc) return rc;
        int64_t old;
        if (!smap_get(&c->tf, word.p, word.n, &old)) {
            smap_put(&c->tf, word.p, word.n, cnt);
            c->size += cnt;
        }
    }
    return 0;
}

/* buildPrefixDictionary (tokenizer.go:340-366): last value wins, total sums
 * every line, every proper rune-prefix inserted with 0 if absent. */
static int load_dict_prefix(or_ctx *c, const char *buf, size_t len) {
    size_t pos = 0;
    sv_t line, word;
    int64_t cnt, total = 0;
    smap_init(&c->tf, len / 7 + 16);
    uint8_t *piece = NULL;
    size_t piece_cap = 0;
    while (next_line(buf, len, &pos, &line)) {
        if (line.n > 65535) break;
        int rc = split_word_count(line, &word, &cnt);
        if (rc) { free(piece); return rc; }
        total += cnt;
        smap_put(&c->tf, word.p, word.n, cnt);
        /* wordR := []rune(word); for _, char := range wordR[:len(wordR)-1] */
        size_t nr = 0, q = 0;
        while (q < word.n) { uint32_t r; q += go_decode((const uint8_t *)word.p + q, word.n - q, &r); nr++; }
        if (nr == 0) { free(piece); return -2; } /* wordR[:-1] panics */
        if (piece_cap < word.n * 4 + 4) { piece_cap = word.n * 4 + 4; piece = realloc(piece, piece_cap); }
        size_t pl = 0;
        q = 0;
        for (size_t k = 0; k + 1 < nr; k++) {
            uint32_t r;
            q += go_decode((const uint8_t *)word.p + q, word.n - q, &r);
            pl += go_encode(r, piece + pl); /* piece += string(char) */
            int64_t old;
            if (!smap_get(&c->tf, piece, pl, &old)) smap_put(&c->tf, piece, pl, 0);
        }
    }
    free(piece);
    c->size = total;
    return 0;
}

/* ---- minimal JSON reader for prob_emit.json (encoding/json semantics) ---- */
typedef struct {
    const char *s;
    size_t n, i;
} js_t;

static void js_ws(js_t *j) {
    while (j->i < j->n && (j->s[j->i] == ' ' || j->s[j->i] == '\t' || j->s[j->i] == '\n' || j->s[j->i] == '\r')) j->i++;
}
static int js_hex4(js_t *j, uint32_t *v) {
    if (j->i + 4 > j->n) return -1;
    uint32_t x = 0;
    for (int k = 0; k < 4; k++) {
        char ch = j->s[j->i++];
        x <<= 4;
        if (ch >= '0' && ch <= '9') x |= ch - '0';
        else if (ch >= 'a' && ch <= 'f') x |= ch - 'a' + 10;
        else if (ch >= 'A' && ch <= 'F') x |= ch - 'A' + 10;
        else return -1;
    }
    *v = x;
    return 0;
}
/* Parse a JSON string into out (UTF-8). Returns length or -1. */
static long js_str(js_t *j, uint8_t *out, size_t cap) {
    js_ws(j);
    if (j->i >= j->n || j->s[j->i] != '"') return -1;
    j->i++;
    size_t o = 0;
    while (j->i < j->n) {
        uint8_t ch = (uint8_t)j->s[j->i];
        if (ch == '"') { j->i++; return (long)o; }
        if (o + 8 > cap) return -1;
        if (ch == '\\') {
            j->i++;
            if (j->i >= j->n) return -1;
            char e = j->s[j->i++];
            uint32_t r;
            switch (e) {
            case '"': out[o++] = '"'; break;
            case '\\': out[o++] = '\\'; break;
            case '/': out[o++] = '/'; break;
            case 'b': out[o++] = '\b'; break;
            case 'f': out[o++] = '\f'; break;
            case 'n': out[o++] = '\n'; break;
            case 'r': out[o++] = '\r'; break;
            case 't': out[o++] = '\t'; break;
            case 'u':
                if (js_hex4(j, &r)) return -1;
                if (r >= 0xD800 && r < 0xDC00) {
                    uint32_t r2;
                    size_t save = j->i;
                    if (j->i + 1 < j->n && j->s[j->i] == '\\' && j->s[j->i + 1] == 'u') {
                        j->i += 2;
                        if (js_hex4(j, &r2)) return -1;
                        if (r2 >= 0xDC00 && r2 < 0xE000) r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
                        else { r = 0xFFFD; j->i = save; }
                    } else r = 0xFFFD;
                } else if (r >= 0xDC00 && r < 0xE000) r = 0xFFFD;
                o += go_encode(r, out + o);
                break;
            default: return -1;
            }
        } else if (ch < 0x80) {
            out[o++] = ch;
            j->i++;
        } else {
            uint32_t r;
            int w = go_decode((const uint8_t *)j->s + j->i, j->n - j->i, &r);
            o += go_encode(r, out + o); /* invalid UTF-8 is replaced by U+FFFD */
            j->i += w;
        }
    }
    return -1;
}
static int js_num(js_t *j, double *v) {
    js_ws(j);
    size_t st = j->i;
    if (j->i < j->n && j->s[j->i] == '-') j->i++;
    while (j->i < j->n && ((j->s[j->i] >= '0' && j->s[j->i] <= '9') || j->s[j->i] == '.' ||
                           j->s[j->i] == 'e' || j->s[j->i] == 'E' || j->s[j->i] == '+' || j->s[j->i] == '-'))
        j->i++;
    if (j->i == st) return -1;
    char tmp[128];
    size_t l = j->i - st;
    if (l >= sizeof tmp) return -1;
    memcpy(tmp, j->s + st, l);
    tmp[l] = 0;
    char *end;
    *v = strtod(tmp, &end); /* correctly rounded, as strconv.ParseFloat */
    return *end ? -1 : 0;
}

/* newJiebaHMM emission part (tokenizer.go:653-661):
 * json.Unmarshal(data, &map[string]map[string]float64) */
static int load_emit(or_ctx *c, const char *buf, size_t len) {
    js_t j = {buf, len, 0};
    uint8_t key[4096], k2[4096];
    for (int s = 0; s < 4; s++) { smap_init(&c->emit[s], 8192); c->has_emit[s] = 0; }
    js_ws(&j);
    if (j.i >= j.n || buf[j.i] != '{') return -4;
    j.i++;
    js_ws(&j);
    if (j.i < j.n && buf[j.i] == '}') return 0;
    for (;;) {
        long kl = js_str(&j, key, sizeof key);
        if (kl < 0) return -4;
        js_ws(&j);
        if (j.i >= j.n || buf[j.i] != ':') return -4;
        j.i++;
        int st = -1;
        if (kl == 1) for (int s = 0; s < 4; s++) if (key[0] == (uint8_t)ST_CH[s]) st = s;
        if (st >= 0) { /* a repeated outer key decodes into a fresh inner map */
            smap_free(&c->emit[st]);
            smap_init(&c->emit[st], 8192);
            c->has_emit[st] = 0;
        }
        js_ws(&j);
        if (j.i < j.n && buf[j.i] == 'n' && j.i + 4 <= j.n && memcmp(buf + j.i, "null", 4) == 0) {
            j.i += 4; /* null leaves the inner map nil */
        } else {
            if (j.i >= j.n || buf[j.i] != '{') return -4;
            j.i++;
            if (st >= 0) c->has_emit[st] = 1;
            js_ws(&j);
            if (j.i < j.n && buf[j.i] == '}') j.i++;
            else for (;;) {
                long l2 = js_str(&j, k2, sizeof k2);
                if (l2 < 0) return -4;
                js_ws(&j);
                if (j.i >= j.n || buf[j.i] != ':') return -4;
                j.i++;
                double v;
                if (js_num(&j, &v)) return -4;
                if (st >= 0) {
                    int64_t bits;
                    memcpy(&bits, &v, 8);
                    smap_put(&c->emit[st], k2, (size_t)l2, bits);
                }
                js_ws(&j);
                if (j.i < j.n && buf[j.i] == ',') { j.i++; continue; }
                if (j.i < j.n && buf[j.i] == '}') { j.i++; break; }
                return -4;
            }
        }
        js_ws(&j);
        if (j.i < j.n && buf[j.i] == ',') { j.i++; continue; }
        if (j.i < j.n && buf[j.i] == '}') { j.i++; break; }
        return -4;
    }
    return 0;
}

/* kind: 0 = NewTokenizer(dict.txt) semantics, 1 = buildPrefixDictionary /
 * prefix_dictionary.gob semantics.  size_override > 0 replaces pd.size
 * (newJiebaPrefixDictionary hard-codes 60_101_967, tokenizer.go:454). */
OR_API void *or_open(const char *dict, size_t dict_len, int kind, long long size_override,
                     const char *emit, size_t emit_len, int *err) {
    or_ctx *c = (or_ctx *)calloc(1, sizeof(or_ctx));
    pthread_mutex_init(&c->mu, NULL);
    int rc = kind == 0 ? load_dict_txt(c, dict, dict_len) : load_dict_prefix(c, dict, dict_len);
    if (!rc && size_override > 0) c->size = size_override;
    if (!rc) rc = load_emit(c, emit, emit_len);
    if (err) *err = rc;
    if (rc) {
        smap_free(&c->tf);
        for (int s = 0; s < 4; s++) if (c->emit[s].slots) smap_free(&c->emit[s]);
        free(c);
        return NULL;
    }
    return c;
}

OR_API void or_close(void *h) {
    or_ctx *c = (or_ctx *)h;
    if (!c) return;
    smap_free(&c->tf);
    for (int s = 0; s < 4; s++) smap_free(&c->emit[s]);
    free(c);
}

OR_API long long or_dict_size(void *h) { return ((or_ctx *)h)->size; }
OR_API long long or_dict_count(void *h) { return (long long)((or_ctx *)h)->tf.n; }
OR_API int or_dict_get(void *h, const char *k, size_t kl, long long *v) {
    int64_t x;
    int f = smap_get(&((or_ctx *)h)->tf, k, kl, &x);
    if (f) *v = x;
    return f;
}
/* Iterate the map (for the TestBuildPrefixDict KAT): slot index -> key. */
OR_API long or_dict_iter(void *h, size_t slot, char *key, size_t cap, long long *v) {
    or_ctx *c = (or_ctx *)h;
    if (slot >= c->tf.cap) return -2;
    kv_t *e = &c->tf.slots[slot];
    if (!e->hash) return -1;
    if (e->klen > cap) return -3;
    memcpy(key, e->key, e->klen);
    *v = e->val;
    return (long)e->klen;
}
OR_API size_t or_dict_cap(void *h) { return ((or_ctx *)h)->tf.cap; }
/* addTerm (tokenizer.go:580-585) */
OR_API void or_add_term(void *h, const char *k, size_t kl, long long freq) {
    or_ctx *c = (or_ctx *)h;
    smap_put(&c->tf, k, kl, freq);
    c->size += freq;
}
OR_API long long or_ties(void *h) { return ((or_ctx *)h)->ties; }

/* emission lookup: hmm.emitP[s][string(r)] with "not found -> minFloat" */
static double emit_of(or_ctx *c, int s, uint32_t r) {
    uint8_t b[4];
    int l = go_encode(r, b);
    int64_t bits;
    if (!smap_get(&c->emit[s], b, l, &bits)) return minFloat;
    double v;
    memcpy(&v, &bits, 8);
    return v;
}
OR_API double or_emit(void *h, int s, uint32_t r, int *found) {
    or_ctx *c = (or_ctx *)h;
    uint8_t b[4];
    int l = go_encode(r, b);
    int64_t bits;
    *found = smap_get(&c->emit[s], b, l, &bits);
    if (!*found) return minFloat;
    double v;
    memcpy(&v, &bits, 8);
    return v;
}

/* ------------------------------------------------------------------------- */
/* Output buffer of token spans                                              */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint32_t *s, *e;
    size_t n, cap;
} spans_t;

static void sp_push(spans_t *o, size_t s, size_t e) {
    if (o->n == o->cap) {
        o->cap = o->cap ? o->cap * 2 : 256;
        o->s = realloc(o->s, o->cap * 4);
        o->e = realloc(o->e, o->cap * 4);
    }
    o->s[o->n] = (uint32_t)s;
    o->e[o->n] = (uint32_t)e;
    o->n++;
}

/* ------------------------------------------------------------------------- */
/* splitText (tokenizer.go:165-210) and the two regexes (:21-22)              */
/* ------------------------------------------------------------------------- */
typedef struct {
    size_t s, e;
    int doProcess;
} block_t;

/* zh.FindAllIndex: maximal runs of \p{Han} runes; alnum.FindAllIndex: maximal
 * runs of [a-zA-Z0-9]. Returns count, writes pairs. */
static size_t find_all(const uint8_t *t, size_t n, int want_han, size_t *pairs) {
    size_t cnt = 0, i = 0;
    int in = 0;
    size_t st = 0;
    while (i < n) {
        uint32_t r;
        int w = go_decode(t + i, n - i, &r);
        int m = want_han ? or_is_han(r) : (r < 0x80 && is_alnum_byte((uint8_t)r));
        if (m && !in) { in = 1; st = i; }
        if (!m && in) { in = 0; pairs[2 * cnt] = st; pairs[2 * cnt + 1] = i; cnt++; }
        i += w;
    }
    if (in) { pairs[2 * cnt] = st; pairs[2 * cnt + 1] = n; cnt++; }
    return cnt;
}

static size_t split_text(size_t n, const size_t *pairs, size_t np, block_t *out) {
    if (np == 0) { out[0].s = 0; out[0].e = n; out[0].doProcess = 0; return 1; }
    size_t nb = 0, prevTail = 0;
    for (size_t i = 0; i < np; i++) {
        if (pairs[2 * i] != prevTail) { out[nb].s = prevTail; out[nb].e = pairs[2 * i]; out[nb].doProcess = 0; nb++; }
        out[nb].s = pairs[2 * i]; out[nb].e = pairs[2 * i + 1]; out[nb].doProcess = 1; nb++;
        prevTail = pairs[2 * i + 1];
        if (i == np - 1 && pairs[2 * i + 1] != n) { out[nb].s = pairs[2 * i + 1]; out[nb].e = n; out[nb].doProcess = 0; nb++; }
    }
    return nb;
}

/* KAT entry: kind 0 = zh regex, 1 = alnum regex. out: 3 size_t per block. */
OR_API size_t or_split_text(const uint8_t *t, size_t n, int kind, size_t *out) {
    size_t *pairs = malloc(sizeof(size_t) * (2 * n + 2));
    block_t *b = malloc(sizeof(block_t) * (2 * n + 2));
    size_t np = find_all(t, n, kind == 0, pairs);
    size_t nb = split_text(n, pairs, np, b);
    for (size_t i = 0; i < nb; i++) { out[3 * i] = b[i].s; out[3 * i + 1] = b[i].e; out[3 * i + 2] = b[i].doProcess; }
    free(pairs);
    free(b);
    return nb;
}

/* ------------------------------------------------------------------------- */
/* cutNonZh (tokenizer.go:289-310)                                            */
/* ------------------------------------------------------------------------- */
static void cut_nonzh(const uint8_t *t, size_t n, size_t base, spans_t *o) {
    size_t *pairs = malloc(sizeof(size_t) * (2 * n + 2));
    size_t np = find_all(t, n, 0, pairs);
    if (np == 0) { free(pairs); return; } /* no alnum run: no tokens (Q6) */
    block_t *b = malloc(sizeof(block_t) * (2 * np + 2));
    size_t nb = split_text(n, pairs, np, b);
    for (size_t k = 0; k < nb; k++) {
        if (b[k].doProcess) { sp_push(o, base + b[k].s, base + b[k].e); continue; }
        size_t i = b[k].s;
        while (i < b[k].e) { /* for _, r := range b.text */
            uint32_t r;
            int w = go_decode(t + i, b[k].e - i, &r);
            if (!or_is_space(r)) sp_push(o, base + i, base + i + w);
            i += w;
        }
    }
    free(pairs);
    free(b);
}

OR_API long or_cut_nonzh(const uint8_t *t, size_t n, uint32_t *s, uint32_t *e, size_t cap) {
    spans_t o = {0};
    cut_nonzh(t, n, 0, &o);
    long r = (long)o.n;
    if (o.n > cap) r = -1;
    else { memcpy(s, o.s, o.n * 4); memcpy(e, o.e, o.n * 4); }
    free(o.s);
    free(o.e);
    return r;
}

/* ------------------------------------------------------------------------- */
/* DAG (tokenizer.go:462-578)                                                 */
/* ------------------------------------------------------------------------- */
typedef struct {
    int index;
    double proba;
} tail_t;

/* maxIndexProba (tokenizer.go:565-578) */
static tail_t max_index_proba(const tail_t *items, size_t n) {
    tail_t prev = {-1, minFloat}, best = {-1, minFloat};
    for (size_t k = 0; k < n; k++) {
        if (items[k].proba >= prev.proba) best = items[k];
        prev = items[k];
    }
    if (best.index == -1) return prev;
    return best;
}

OR_API void or_max_index_proba(const int *idx, const double *pr, size_t n, int *oi, double *op) {
    tail_t *it = malloc(sizeof(tail_t) * (n + 1));
    for (size_t k = 0; k < n; k++) { it[k].index = idx[k]; it[k].proba = pr[k]; }
    tail_t t = max_index_proba(it, n);
    *oi = t.index;
    *op = t.proba;
    free(it);
}

/* Encode runes[a:b] as a Go string. */
static size_t runes_str(const uint32_t *rs, size_t a, size_t b, uint8_t *buf) {
    size_t l = 0;
    for (size_t k = a; k < b; k++) l += go_encode(rs[k], buf + l);
    return l;
}

typedef struct {
    size_t *off; /* n+1 */
    int *ends;
} dag_t;

/* buildDag (tokenizer.go:462-497); dag[i] as CSR. */
static void build_dag(or_ctx *c, const uint32_t *rs, size_t n, dag_t *d, uint8_t *sbuf) {
    size_t cap = n * 4 + 16, ne = 0;
    d->off = malloc(sizeof(size_t) * (n + 1));
    d->ends = malloc(sizeof(int) * cap);
    for (size_t i = 0; i < n; i++) {
        d->off[i] = ne;
        int64_t count;
        size_t l = runes_str(rs, i, i + 1, sbuf);
        int found = smap_get(&c->tf, sbuf, l, &count);
        if (!found || count == 0) {
            if (ne == cap) { cap *= 2; d->ends = realloc(d->ends, sizeof(int) * cap); }
            d->ends[ne++] = (int)(i + 1);
            continue;
        }
        for (size_t j = 0; j < n - i; j++) {
            int64_t val;
            l = runes_str(rs, i, j + 1 + i, sbuf);
            if (!smap_get(&c->tf, sbuf, l, &val)) break;
            if (val > 0) {
                if (ne == cap) { cap *= 2; d->ends = realloc(d->ends, sizeof(int) * cap); }
                d->ends[ne++] = (int)(j + 1 + i);
            }
        }
    }
    d->off[n] = ne;
}

/* calcDagProba (tokenizer.go:502-548): dagProba[i] = list of (j, proba). */
static tail_t *calc_dag_proba(or_ctx *c, const uint32_t *rs, size_t n, const dag_t *d, uint8_t *sbuf) {
    double total = or_go_log((double)c->size);
    tail_t *dp = malloc(sizeof(tail_t) * (d->off[n] + 1));
    for (size_t ii = n; ii-- > 0;) {
        for (size_t k = d->off[ii]; k < d->off[ii + 1]; k++) {
            int j = d->ends[k];
            double tf = 1.0;
            int64_t val;
            size_t l = runes_str(rs, ii, (size_t)j, sbuf);
            if (smap_get(&c->tf, sbuf, l, &val)) tf = (double)val;
            double pieceFreq = or_go_log(tf) - total;
            tail_t nb;
            if ((size_t)j < n) nb = max_index_proba(dp + d->off[j], d->off[j + 1] - d->off[j]);
            else { tail_t sent = {j, 0.0}; nb = max_index_proba(&sent, 1); }
            dp[k].index = j;
            dp[k].proba = pieceFreq + nb.proba;
        }
    }
    return dp;
}

/* findDagPath (tokenizer.go:552-562). Returns number of pieces; a -1 tail
 * index makes cutDAG's slice panic (the caller reports it). */
static size_t find_dag_path(size_t n, const size_t *off, const tail_t *dp, int *pa, int *pb) {
    size_t np = 0;
    for (long i = 0; i < (long)n && i >= 0;) {
        tail_t t = max_index_proba(dp + off[i], off[i + 1] - off[i]);
        pa[np] = (int)i;
        pb[np] = t.index;
        np++;
        i = t.index;
    }
    return np;
}

OR_API long or_find_dag_path(size_t n, const size_t *off, const int *idx, const double *pr, int *pa, int *pb) {
    tail_t *dp = malloc(sizeof(tail_t) * (off[n] + 1));
    for (size_t k = 0; k < off[n]; k++) { dp[k].index = idx[k]; dp[k].proba = pr[k]; }
    long r = (long)find_dag_path(n, off, dp, pa, pb);
    free(dp);
    return r;
}

static size_t decode_runes(const uint8_t *t, size_t n, uint32_t *rs, size_t *pos) {
    size_t nr = 0, i = 0;
    while (i < n) {
        uint32_t r;
        int w = go_decode(t + i, n - i, &r);
        pos[nr] = i;
        rs[nr++] = r;
        i += w;
    }
    pos[nr] = n;
    return nr;
}

/* KAT entry: buildDag over text; ends written to out_ends, offsets to out_off. */
OR_API long or_build_dag(void *h, const uint8_t *t, size_t n, size_t *out_off, int *out_ends, size_t cap) {
    or_ctx *c = (or_ctx *)h;
    uint32_t *rs = malloc(sizeof(uint32_t) * (n + 1));
    size_t *pos = malloc(sizeof(size_t) * (n + 2));
    uint8_t *sbuf = malloc(n * 4 + 8);
    size_t nr = decode_runes(t, n, rs, pos);
    dag_t d;
    build_dag(c, rs, nr, &d, sbuf);
    long r = (long)nr;
    if (d.off[nr] > cap) r = -1;
    else {
        memcpy(out_off, d.off, sizeof(size_t) * (nr + 1));
        memcpy(out_ends, d.ends, sizeof(int) * d.off[nr]);
    }
    free(d.off);
    free(d.ends);
    free(rs);
    free(pos);
    free(sbuf);
    return r;
}

/* ------------------------------------------------------------------------- */
/* HMM Viterbi (tokenizer.go:668-756)                                         */
/* ------------------------------------------------------------------------- */
/* stateTransitionRoute (tokenizer.go:736-756); prev = hiddenStates[step-1]. */
static int state_transition_route(or_ctx *c, const double prev[4], int now, double *proba) {
    double routes[2];
    for (int k = 0; k < 2; k++) {
        int p = stateChange[now][k];
        routes[k] = prev[p] + transP(p, now);
    }
    int best = ST_NONE;
    double bp = minFloat;
    for (int k = 0; k < 2; k++) {
        if (routes[k] > bp) {
            best = stateChange[now][k];
            bp = routes[k];
        } else if (best != ST_NONE && routes[k] == bp && c) {
            __atomic_fetch_add(&c->ties, 1, __ATOMIC_RELAXED); /* Go map order decides (Q12) */
        }
    }
    *proba = bp;
    return best;
}

OR_API int or_state_transition_route(const double prev[4], int now, double *proba) {
    return state_transition_route(NULL, prev, now, proba);
}

/* viterbi (tokenizer.go:668-730) with the reference's literal per-state path
 * copying (:679-684, :703-718).  Writes the returned path's states (0..3) to
 * out and returns its length. */
static size_t viterbi_pathcopy(or_ctx *c, const uint32_t *rs, size_t m, int *out) {
    if (m == 1) { out[0] = ST_S; return 1; }
    double v[4], nv[4];
    int *full[4], *part[4];
    size_t flen[4], plen[4];
    for (int s = 0; s < 4; s++) {
        full[s] = malloc(sizeof(int) * (m + 1));
        part[s] = malloc(sizeof(int) * (m + 1));
        full[s][0] = s;
        flen[s] = 1;
        v[s] = startP(s) + emit_of(c, s, rs[0]);
    }
    for (size_t i = 1; i < m; i++) {
        for (int s = 0; s < 4; s++) {
            double rp;
            int from = state_transition_route(c, v, s, &rp);
            nv[s] = rp + emit_of(c, s, rs[i]);
            /* partialPath[s] = fullPath[route.from] ++ [s]; fullPath[""] is nil */
            plen[s] = 0;
            if (from != ST_NONE) { memcpy(part[s], full[from], sizeof(int) * flen[from]); plen[s] = flen[from]; }
            part[s][plen[s]++] = s;
        }
        for (int s = 0; s < 4; s++) {
            int *tmp = full[s]; full[s] = part[s]; part[s] = tmp;
            flen[s] = plen[s];
            v[s] = nv[s];
        }
    }
    int fin = v[ST_E] > v[ST_S] ? ST_E : ST_S;
    memcpy(out, full[fin], sizeof(int) * flen[fin]);
    size_t L = flen[fin];
    for (int s = 0; s < 4; s++) { free(full[s]); free(part[s]); }
    return L;
}

/* Same decisions with back-pointers + a NONE marker (O(m)); used for long runs
 * in property tests and checked against viterbi_pathcopy in tests. */
static size_t viterbi_backptr(or_ctx *c, const uint32_t *rs, size_t m, int *out) {
    if (m == 1) { out[0] = ST_S; return 1; }
    int8_t *bp = malloc(4 * m);
    double v[4], nv[4];
    for (int s = 0; s < 4; s++) v[s] = startP(s) + emit_of(c, s, rs[0]);
    for (size_t i = 1; i < m; i++) {
        for (int s = 0; s < 4; s++) {
            double rp;
            bp[4 * i + s] = (int8_t)state_transition_route(c, v, s, &rp);
            nv[s] = rp + emit_of(c, s, rs[i]);
        }
        memcpy(v, nv, sizeof v);
    }
    int st = v[ST_E] > v[ST_S] ? ST_E : ST_S;
    size_t t = m - 1;
    int *rev = malloc(sizeof(int) * m);
    size_t L = 0;
    for (;;) {
        rev[L++] = st;
        if (t == 0) break;
        int p = bp[4 * t + st];
        if (p == ST_NONE) break;
        st = p;
        t--;
    }
    for (size_t k = 0; k < L; k++) out[k] = rev[L - 1 - k];
    free(rev);
    free(bp);
    return L;
}

static int g_use_backptr = 0;
OR_API void or_set_viterbi_backptr(int on) { g_use_backptr = on; }

OR_API long or_viterbi(void *h, const uint8_t *t, size_t n, int *out, int backptr) {
    or_ctx *c = (or_ctx *)h;
    uint32_t *rs = malloc(sizeof(uint32_t) * (n + 1));
    size_t *pos = malloc(sizeof(size_t) * (n + 2));
    size_t m = decode_runes(t, n, rs, pos);
    long L = m ? (long)(backptr ? viterbi_backptr(c, rs, m, out) : viterbi_pathcopy(c, rs, m, out)) : 0;
    free(rs);
    free(pos);
    return L;
}

/* cutHMM (tokenizer.go:273-285): pieces runes[pieceStart:i+1] whenever
 * path[i] is E or S; indices count from the run's first rune. */
static void cut_hmm(const size_t *pos, const int *path, size_t L, size_t base, spans_t *o) {
    size_t pieceStart = 0;
    for (size_t i = 0; i < L; i++) {
        if (path[i] == ST_E || path[i] == ST_S) {
            sp_push(o, base + pos[pieceStart], base + pos[i + 1]);
            pieceStart = i + 1;
        }
    }
}

OR_API long or_cut_hmm(const uint8_t *t, size_t n, const int *path, size_t L, uint32_t *s, uint32_t *e) {
    uint32_t *rs = malloc(sizeof(uint32_t) * (n + 1));
    size_t *pos = malloc(sizeof(size_t) * (n + 2));
    decode_runes(t, n, rs, pos);
    spans_t o = {0};
    cut_hmm(pos, path, L, 0, &o);
    long r = (long)o.n;
    memcpy(s, o.s, o.n * 4);
    memcpy(e, o.e, o.n * 4);
    free(o.s); free(o.e); free(rs); free(pos);
    return r;
}

/* ------------------------------------------------------------------------- */
/* cutDAG / cutZh / Cut (tokenizer.go:151-162, 212-270)                       */
/* ------------------------------------------------------------------------- */
/* Emits cutZh(text, hmm) tokens for a Han block. Returns 0, or -5 when the
 * reference would panic in cutDAG (tail index -1). */
static int cut_zh(or_ctx *c, const uint8_t *t, size_t n, size_t base, int hmm, spans_t *o) {
    uint32_t *rs = malloc(sizeof(uint32_t) * (n + 1));
    size_t *pos = malloc(sizeof(size_t) * (n + 2));
    uint8_t *sbuf = malloc(n * 4 + 8);
    size_t nr = decode_runes(t, n, rs, pos);
    dag_t d;
    build_dag(c, rs, nr, &d, sbuf);
    tail_t *dp = calc_dag_proba(c, rs, nr, &d, sbuf);
    int *pa = malloc(sizeof(int) * (nr + 1)), *pb = malloc(sizeof(int) * (nr + 1));
    size_t np = find_dag_path(nr, d.off, dp, pa, pb);
    int rc = 0;
    for (size_t k = 0; k < np; k++) if (pb[k] < 0) rc = -5;
    if (!rc) {
        if (!hmm) {
            for (size_t k = 0; k < np; k++) sp_push(o, base + pos[pa[k]], base + pos[pb[k]]);
        } else {
            /* group maximal runs of single-rune pieces (tokenizer.go:228-253) */
            int *path = malloc(sizeof(int) * (nr + 1));
            size_t us = 0, ul = 0; /* uncut run: first rune index, length */
            for (size_t k = 0; k < np; k++) {
                if (pb[k] - pa[k] == 1) {
                    if (ul == 0) us = (size_t)pa[k];
                    ul++;
                    if (k + 1 >= np && ul) {
                        size_t L = g_use_backptr ? viterbi_backptr(c, rs + us, ul, path) : viterbi_pathcopy(c, rs + us, ul, path);
                        cut_hmm(pos + us, path, L, base, o);
                        ul = 0;
                    }
                } else {
                    if (ul) {
                        size_t L = g_use_backptr ? viterbi_backptr(c, rs + us, ul, path) : viterbi_pathcopy(c, rs + us, ul, path);
                        cut_hmm(pos + us, path, L, base, o);
                        ul = 0;
                    }
                    sp_push(o, base + pos[pa[k]], base + pos[pb[k]]);
                }
            }
            free(path);
        }
    }
    free(rs); free(pos); free(sbuf); free(d.off); free(d.ends); free(dp); free(pa); free(pb);
    return rc;
}

/* Cut (tokenizer.go:151-162) on one document; spans are offset by base. */
static int cut_doc(or_ctx *c, const uint8_t *t, size_t n, size_t base, int hmm, spans_t *o) {
    size_t *pairs = malloc(sizeof(size_t) * (2 * n + 2));
    block_t *b = malloc(sizeof(block_t) * (2 * n + 2));
    size_t np = find_all(t, n, 1, pairs);
    size_t nb = split_text(n, pairs, np, b);
    int rc = 0;
    for (size_t k = 0; k < nb && !rc; k++) {
        if (b[k].doProcess) rc = cut_zh(c, t + b[k].s, b[k].e - b[k].s, base + b[k].s, hmm, o);
        else cut_nonzh(t + b[k].s, b[k].e - b[k].s, base + b[k].s, o);
    }
    free(pairs);
    free(b);
    return rc;
}

/* One document. Returns #tokens, -1 if cap too small, -5 on reference panic. */
OR_API long or_cut(void *h, const uint8_t *t, size_t n, int hmm, uint32_t *s, uint32_t *e, size_t cap) {
    spans_t o = {0};
    int rc = cut_doc((or_ctx *)h, t, n, 0, hmm, &o);
    long r = rc ? rc : (long)o.n;
    if (!rc && o.n > cap) r = -1;
    else if (!rc) { memcpy(s, o.s, o.n * 4); memcpy(e, o.e, o.n * 4); }
    free(o.s);
    free(o.e);
    return r;
}

/* ---- batch over documents, optionally multi-threaded ---------------------- */
typedef struct {
    or_ctx *c;
    const uint8_t *t;
    const uint64_t *off;
    uint32_t d0, d1;
    int hmm, rc;
    spans_t o;
    uint64_t *doc_cnt;
} job_t;

static void *job_run(void *p) {
    job_t *j = (job_t *)p;
    for (uint32_t d = j->d0; d < j->d1 && !j->rc; d++) {
        size_t before = j->o.n;
        j->rc = cut_doc(j->c, j->t + j->off[d], j->off[d + 1] - j->off[d], j->off[d], j->hmm, &j->o);
        j->doc_cnt[d] = j->o.n - before;
    }
    return NULL;
}

/* Cut every document of a concatenated batch. Spans are absolute byte offsets;
 * tok_doc_off[d] is the first token of document d (ndocs+1 entries).
 * When s/e are NULL only the count is returned (spans discarded).
 * Returns total tokens, -1 if cap is too small, -5 on a reference panic. */
OR_API long long or_cut_batch(void *h, const uint8_t *t, const uint64_t *off, uint32_t ndocs, int hmm,
                              int nthreads, uint32_t *s, uint32_t *e, size_t cap, uint64_t *tok_doc_off) {
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > ndocs) nthreads = ndocs ? (int)ndocs : 1;
    job_t *jobs = calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t *cnt = calloc((size_t)ndocs + 1, sizeof(uint64_t));
    /* byte-balanced contiguous document ranges */
    uint64_t total = off[ndocs] - off[0];
    uint32_t d = 0;
    for (int k = 0; k < nthreads; k++) {
        uint64_t target = off[0] + total * (uint64_t)(k + 1) / (uint64_t)nthreads;
        uint32_t d1 = d;
        while (d1 < ndocs && (off[d1 + 1] <= target || d1 == d)) d1++;
        if (k == nthreads - 1) d1 = ndocs;
        jobs[k].c = (or_ctx *)h; jobs[k].t = t; jobs[k].off = off; jobs[k].d0 = d; jobs[k].d1 = d1;
        jobs[k].hmm = hmm; jobs[k].doc_cnt = cnt;
        d = d1;
    }
    for (int k = 0; k < nthreads; k++) pthread_create(&th[k], NULL, job_run, &jobs[k]);
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    long long n = 0;
    int rc = 0;
    for (int k = 0; k < nthreads; k++) { n += (long long)jobs[k].o.n; if (jobs[k].rc) rc = jobs[k].rc; }
    long long ret = rc ? rc : n;
    if (!rc && s && (size_t)n > cap) ret = -1;
    if (!rc && ret >= 0) {
        size_t w = 0;
        for (int k = 0; k < nthreads; k++) {
            if (s) { memcpy(s + w, jobs[k].o.s, jobs[k].o.n * 4); memcpy(e + w, jobs[k].o.e, jobs[k].o.n * 4); }
            w += jobs[k].o.n;
        }
        if (tok_doc_off) {
            uint64_t acc = 0;
            for (uint32_t q = 0; q < ndocs; q++) { tok_doc_off[q] = acc; acc += cnt[q]; }
            tok_doc_off[ndocs] = acc;
        }
    }
    for (int k = 0; k < nthreads; k++) { free(jobs[k].o.s); free(jobs[k].o.e); }
    free(jobs);
    free(th);
    free(cnt);
    return ret;
}
