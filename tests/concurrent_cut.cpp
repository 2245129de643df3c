// concurrent_cut.cpp — many threads calling jb_cut at once on one context, the
// way Go code calls Tokenizer.Cut from many goroutines (the reference takes only
// an RLock there, tokenizer.go:151-153).  Every result is checked against the
// spans the test computed with the oracle; prints the call rate of one thread and
// of all threads together.
//
//   concurrent_cut DICT EMIT SENTENCES EXPECTED THREADS CALLS [mixed]
// SENTENCES: one sentence per line; EXPECTED: per sentence "n s0 e0 s1 e1 ..."
// (byte offsets in the sentence), or "P" where the reference panics (JB_EPANIC
// expected).  With "mixed", EXPECTED has two lines per sentence (hmm on, then off)
// and the calls alternate hmm, so that coalesced batches mix both settings.
// Output: "serial ..." and "concurrent ..." lines.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "jiebahip.h"

struct Expect {
    bool panic = false;
    std::vector<uint64_t> s, e;
};

static int run(jb_ctx* ctx, const std::vector<std::string>& sent, const std::vector<Expect>& want, bool mixed,
               int nth, int calls, double* secs, uint64_t* bad) {
    std::atomic<uint64_t> mism{0}, errs{0};
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    auto body = [&](int t) {
        ready++;
        while (!go.load()) std::this_thread::yield();
        for (int i = 0; i < calls; i++) {
            const size_t k = ((size_t)t * 7919u + (size_t)i * 31u) % sent.size();
            const int hmm = mixed ? (int)((t + i) & 1) : 1;
            const Expect& w = want[mixed ? 2 * k + (hmm ? 0 : 1) : k];
            jb_spans sp;
            const int rc = jb_cut(ctx, (const uint8_t*)sent[k].data(), sent[k].size(), hmm, &sp);
            if (w.panic) {  // the reference panics here: JB_EPANIC for this call alone
                if (rc != JB_EPANIC) {
                    mism++;
                    if (rc == 0) jb_spans_free(&sp);
                }
                continue;
            }
            if (rc) {
                if (errs++ == 0) fprintf(stderr, "jb_cut rc=%d: %s\n", rc, jb_last_error());
                continue;
            }
            bool ok = sp.ntokens == w.s.size();
            for (uint64_t j = 0; ok && j < sp.ntokens; j++) ok = sp.start[j] == w.s[j] && sp.end[j] == w.e[j];
            if (!ok) mism++;
            jb_spans_free(&sp);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nth; t++) th.emplace_back(body, t);
    while (ready.load() < nth) std::this_thread::yield();
    const auto a = std::chrono::steady_clock::now();
    go = true;
    for (auto& x : th) x.join();
    *secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    *bad = mism.load() + errs.load();
    return errs.load() ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc != 7 && argc != 8) {
        fprintf(stderr, "usage: %s DICT EMIT SENTENCES EXPECTED THREADS CALLS [mixed]\n", argv[0]);
        return 2;
    }
    const bool mixed = argc == 8 && strcmp(argv[7], "mixed") == 0;
    const int nth = atoi(argv[5]), calls = atoi(argv[6]);
    std::vector<std::string> sent;
    {
        std::ifstream f(argv[3], std::ios::binary);
        std::string line;
        while (std::getline(f, line)) sent.push_back(line);
    }
    std::vector<Expect> want;
    {
        std::ifstream f(argv[4]);
        std::string line;
        while (std::getline(f, line)) {
            Expect x;
            if (!line.empty() && line[0] == 'P') {
                x.panic = true;
                want.push_back(x);
                continue;
            }
            std::istringstream is(line);
            size_t n;
            is >> n;
            x.s.resize(n);
            x.e.resize(n);
            for (size_t j = 0; j < n; j++) is >> x.s[j] >> x.e[j];
            want.push_back(x);
        }
    }
    if (sent.empty() || want.size() != sent.size() * (mixed ? 2u : 1u)) {
        fprintf(stderr, "%zu sentences, %zu expectations\n", sent.size(), want.size());
        return 2;
    }
    jb_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.dict_path = argv[1];
    cfg.emit_path = argv[2];
    cfg.ndevices = 1;
    jb_ctx* ctx = nullptr;
    int rc = jb_open(&cfg, &ctx);
    if (rc) {
        fprintf(stderr, "jb_open rc=%d: %s\n", rc, jb_last_error());
        return 1;
    }
    double s1 = 0, sn = 0;
    uint64_t b1 = 0, bn = 0;
    run(ctx, sent, want, mixed, 1, 200, &s1, &b1);  // warm-up
    rc = run(ctx, sent, want, mixed, 1, calls, &s1, &b1);
    printf("serial threads 1 calls %d mismatches %llu seconds %.4f calls_per_s %.0f\n", calls,
           (unsigned long long)b1, s1, calls / s1);
    rc |= run(ctx, sent, want, mixed, nth, calls, &sn, &bn);
    printf("concurrent threads %d calls %d mismatches %llu seconds %.4f calls_per_s %.0f\n", nth, nth * calls,
           (unsigned long long)bn, sn, (double)nth * calls / sn);
    jb_close(ctx);
    return rc || b1 || bn ? 1 : 0;
}
