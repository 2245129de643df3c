/*
 * c_abi_smoke.c — a plain C99 consumer of include/jiebahip.h, the way a cgo
 * preamble binds it: open as the Go binding does (build the
 * image, list its log keys, hand malloc'd logarithms to jb_open_image), Cut one
 * text, cut a batch, cut a batch into caller arrays, AddWord with suggestFreq,
 * Cut again, close.
 * Spans go to stdout, one line per call, for tests/test_gpu_parity.py to check
 * against the oracle.
 *
 *   c_abi_smoke DICT EMIT TEXTFILE WORD   (GPU)
 *   c_abi_smoke --expect-no-device        (no GPU: jb_open must fail with JB_EDEVICE)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jiebahip.h"

static int die(const char *what, int rc) {
    fprintf(stderr, "%s: rc=%d: %s\n", what, rc, jb_last_error());
    return 1;
}

static void print_spans(const char *tag, const uint64_t *s, const uint64_t *e, uint64_t n) {
    uint64_t k;
    printf("%s %llu", tag, (unsigned long long)n);
    for (k = 0; k < n; k++) printf(" %llu %llu", (unsigned long long)s[k], (unsigned long long)e[k]);
    printf("\n");
}

int main(int argc, char **argv) {
    jb_config cfg;
    jb_ctx *ctx = NULL;
    jb_spans sp;
    FILE *f;
    char *text;
    long len;
    int rc;
    int64_t freq = 0;
    uint64_t off[3], doc_tok[3], ntok = 0, cap, *st, *en;

    memset(&cfg, 0, sizeof cfg);
    cfg.ndevices = 1;
    if (argc == 2 && strcmp(argv[1], "--expect-no-device") == 0) {
        cfg.dict_buf = "\xe7\x94\xb2 3\n"; /* one key, 甲 */
        cfg.dict_len = strlen(cfg.dict_buf);
        cfg.emit_buf = "{}";
        cfg.emit_len = 2;
        rc = jb_open(&cfg, &ctx);
        if (rc != JB_EDEVICE) {
            fprintf(stderr, "jb_open without a device gave %d, want JB_EDEVICE\n", rc);
            return 1;
        }
        printf("no device: %s\n", jb_last_error());
        return 0;
    }
    if (argc != 5) {
        fprintf(stderr, "usage: %s DICT EMIT TEXTFILE WORD | --expect-no-device\n", argv[0]);
        return 2;
    }
    f = fopen(argv[3], "rb");
    if (!f) return die("open text", JB_EIO);
    fseek(f, 0, SEEK_END);
    len = ftell(f);
    fseek(f, 0, SEEK_SET);
    text = (char *)malloc((size_t)len * 2 + 1);
    if (!text || fread(text, 1, (size_t)len, f) != (size_t)len) return die("read text", JB_EIO);
    fclose(f);
    memcpy(text + len, text, (size_t)len); /* the batch: the text twice */

    cfg.dict_path = argv[1];
    cfg.dict_kind = JB_DICT_TXT;
    cfg.emit_path = argv[2];
    {
        /* jieba-go_amd/go/tokenizer.go open(): the image is built once; the log table
         * lives in C memory (cgo: no Go pointers inside a struct passed to C).  Go passes
         * math.Log; this C caller passes the library's restatement of it. */
        jb_image *img = NULL;
        size_t nk = 0, i;
        int64_t *keys;
        double *vals;
        if ((rc = jb_image_build(&cfg, &img))) return die("jb_image_build", rc);
        rc = jb_image_log_keys(img, NULL, 0, &nk);
        if (rc != JB_OK && rc != JB_ELIMIT) return die("jb_image_log_keys (count)", rc);
        keys = (int64_t *)malloc((nk + 1) * sizeof *keys);
        vals = (double *)malloc((nk + 1) * sizeof *vals);
        if (!keys || !vals) return die("malloc", JB_ENOMEM);
        if ((rc = jb_image_log_keys(img, keys, nk, &nk))) return die("jb_image_log_keys", rc);
        for (i = 0; i < nk; i++) vals[i] = jb_go_log((double)keys[i]);
        cfg.log_keys = keys;
        cfg.log_vals = vals;
        cfg.nlog = nk;
        rc = jb_open_image(img, &cfg, &ctx); /* consumes img */
        free(keys);
        free(vals);
        cfg.log_keys = NULL;
        cfg.log_vals = NULL;
        cfg.nlog = 0;
        if (rc) return die("jb_open_image", rc);
        printf("log keys %lu\n", (unsigned long)nk);
    }

    /* Tokenizer.Cut(text, true) */
    if ((rc = jb_cut(ctx, (const uint8_t *)text, (size_t)len, 1, &sp))) return die("jb_cut", rc);
    print_spans("cut", sp.start, sp.end, sp.ntokens);
    jb_spans_free(&sp);

    /* a batch of two documents, HMM off */
    off[0] = 0;
    off[1] = (uint64_t)len;
    off[2] = 2 * (uint64_t)len;
    if ((rc = jb_cut_batch(ctx, (const uint8_t *)text, off, 2, 0, &sp))) return die("jb_cut_batch", rc);
    print_spans("batch", sp.start, sp.end, sp.ntokens);
    printf("doc_tok %llu %llu %llu\n", (unsigned long long)sp.doc_tok[0], (unsigned long long)sp.doc_tok[1],
           (unsigned long long)sp.doc_tok[2]);
    jb_spans_free(&sp);

    /* the same into caller arrays, first too small (JB_ELIMIT and the count), then sized */
    cap = 1;
    st = (uint64_t *)malloc(sizeof(uint64_t));
    en = (uint64_t *)malloc(sizeof(uint64_t));
    rc = jb_cut_batch_into(ctx, (const uint8_t *)text, off, 2, 1, st, en, cap, doc_tok, &ntok);
    if (rc != JB_ELIMIT && !(rc == JB_OK && ntok <= 1)) return die("jb_cut_batch_into (small)", rc);
    free(st);
    free(en);
    cap = ntok;
    st = (uint64_t *)malloc((size_t)(cap ? cap : 1) * sizeof(uint64_t));
    en = (uint64_t *)malloc((size_t)(cap ? cap : 1) * sizeof(uint64_t));
    if ((rc = jb_cut_batch_into(ctx, (const uint8_t *)text, off, 2, 1, st, en, cap, doc_tok, &ntok)))
        return die("jb_cut_batch_into", rc);
    print_spans("into", st, en, ntok);
    free(st);
    free(en);

    /* the same as u32 offsets from the batch's first byte (what the Go binding calls) */
    {
        uint32_t *s32 = (uint32_t *)malloc((size_t)(cap ? cap : 1) * sizeof(uint32_t));
        uint32_t *e32 = (uint32_t *)malloc((size_t)(cap ? cap : 1) * sizeof(uint32_t));
        uint64_t k;
        if (!s32 || !e32) return die("malloc", -1);
        if ((rc = jb_cut_batch_into32(ctx, (const uint8_t *)text, off, 2, 1, s32, e32, cap, doc_tok, &ntok)))
            return die("jb_cut_batch_into32", rc);
        st = (uint64_t *)malloc((size_t)(ntok ? ntok : 1) * sizeof(uint64_t));
        en = (uint64_t *)malloc((size_t)(ntok ? ntok : 1) * sizeof(uint64_t));
        for (k = 0; k < ntok; k++) {
            st[k] = off[0] + s32[k];
            en[k] = off[0] + e32[k];
        }
        print_spans("into32", st, en, ntok);
        free(st);
        free(en);
        free(s32);
        free(e32);
    }

    /* AddWord(word, 0): suggestFreq's value, then Cut again */
    if ((rc = jb_suggest_freq(ctx, argv[4], strlen(argv[4]), &freq))) return die("jb_suggest_freq", rc);
    if ((rc = jb_add_word(ctx, argv[4], strlen(argv[4]), 0))) return die("jb_add_word", rc);
    if (jb_dict_get(ctx, argv[4], strlen(argv[4]), &freq) != 1) return die("jb_dict_get", -1);
    printf("freq %lld size %lld\n", (long long)freq, (long long)jb_dict_size(ctx));
    if ((rc = jb_cut(ctx, (const uint8_t *)text, (size_t)len, 1, &sp))) return die("jb_cut after AddWord", rc);
    print_spans("cut2", sp.start, sp.end, sp.ntokens);
    jb_spans_free(&sp);

    jb_close(ctx);
    free(text);
    return 0;
}
