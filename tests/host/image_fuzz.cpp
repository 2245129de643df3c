// image_fuzz.cpp — the host half of the library's loaders and image builder under AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_sanitizers.py builds it with jb_image.cpp and
// -fsanitize=address,undefined).  One full pass over real-sized inputs (dict.txt in both semantics, the
// emission JSON, a gob map, the image built, its hot rows, saved, loaded back and compared, lookups of
// every key), then bounded mutation rounds: truncations, byte flips and splices of each input fed to its
// parser or loader, which must return a code and never touch memory it does not own.
//   usage: image_fuzz dict.txt prob_emit.json dict.gob rounds seed
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "jb_image.h"
#include "jb_common.h"

using namespace jb;

static std::string slurp(const char* p) {
    FILE* f = fopen(p, "rb");
    if (!f) {
        perror(p);
        exit(2);
    }
    std::string s;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
    return s;
}

static void fail(const char* what, const std::string& err) {
    fprintf(stderr, "FAIL %s: %s\n", what, err.c_str());
    exit(1);
}

// A mutated copy: a truncation, a few byte flips, or a splice of the input into itself.
static std::string mutate(const std::string& s, std::mt19937_64& rng) {
    std::string m = s;
    if (m.empty()) return m;
    switch (rng() % 4) {
        case 0:
            m.resize(rng() % m.size());
            break;
        case 1:
            for (int k = 0, n = 1 + (int)(rng() % 8); k < n; k++) m[rng() % m.size()] = (char)(rng() & 0xFF);
            break;
        case 2: {
            const size_t a = rng() % m.size(), b = rng() % m.size(), n = rng() % 64;
            m.insert(a, s.substr(b, n));
            break;
        }
        default:
            m[rng() % m.size()] = "\n\t \"{}:,-0123456789"[rng() % 19];
            break;
    }
    return m;
}

int main(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s dict emit gob rounds seed\n", argv[0]);
        return 2;
    }
    const std::string dict = slurp(argv[1]), emit = slurp(argv[2]), gob = slurp(argv[3]);
    const int rounds = atoi(argv[4]);
    std::mt19937_64 rng(strtoull(argv[5], nullptr, 10));
    std::string err;

    // the full pass
    Emission em;
    if (parse_emission(emit.data(), emit.size(), &em, &err)) fail("emission", err);
    for (int kind = 0; kind < 2; kind++) {
        Dictionary d;
        if (parse_dictionary(dict.data(), dict.size(), kind, &d, &err)) fail("dictionary", err);
        Image img;
        if (build_image(d, em, &img, &err)) fail("build", err);
        std::vector<uint64_t> vals(JB_HOT_SLOTS);
        std::vector<uint16_t> tags(JB_HOT_SLOTS);
        build_hot_rows(img, vals.data(), tags.data());
        std::string saved;
        save_image(d, em, img, &saved);
        Dictionary d2;
        Emission e2;
        Image img2;
        if (load_image(saved.data(), saved.size(), &d2, &e2, &img2, &err)) fail("load", err);
        if (img2.cells != img.cells || img2.code != img.code || img2.wtab.size() != img.wtab.size() ||
            d2.term_freq != d.term_freq)
            fail("round trip", "the loaded image differs");
        if (!reweigh_image(d, &img2)) fail("reweigh", "weights moved");
        size_t hits = 0;
        for (const auto& kv : d.term_freq) {  // every key, walked as the kernels walk
            std::vector<uint32_t> r;
            for (size_t i = 0; i < kv.first.size();) {
                uint32_t x = 0, cp = 0;
                for (size_t k = 0; k < 4 && i + k < kv.first.size(); k++) x |= (uint32_t)(uint8_t)kv.first[i + k] << (8 * k);
                const uint32_t w = jb_decode(x, (uint32_t)std::min<size_t>(4, kv.first.size() - i), &cp);
                r.push_back(cp);
                i += w;
            }
            const Lookup lk = image_lookup(img, r.data(), r.size());
            hits += lk.found ? 1u : 0u;
        }
        if (hits == 0) fail("lookup", "no key found");
        // mutated saved images: load must refuse (checksum) or succeed, never fault
        for (int k = 0; k < rounds / 4; k++) {
            const std::string m = mutate(saved, rng);
            Dictionary dm;
            Emission emm;
            Image im;
            (void)load_image(m.data(), m.size(), &dm, &emm, &im, &err);
        }
    }
    {
        Dictionary dg;
        if (parse_gob_dictionary(gob.data(), gob.size(), &dg, &err)) fail("gob", err);
        if (dg.term_freq.empty()) fail("gob", "empty map");
    }
    // mutation rounds for the parsers; a small dictionary keeps the build in the loop cheap
    const std::string small = dict.substr(0, std::min<size_t>(dict.size(), 6000));
    for (int k = 0; k < rounds; k++) {
        {
            const std::string m = mutate(small, rng);
            Dictionary d;
            if (parse_dictionary(m.data(), m.size(), (int)(rng() & 1), &d, &err) == 0) {
                Image img;
                (void)build_image(d, em, &img, &err);
            }
        }
        {
            const std::string m = mutate(emit, rng);
            Emission e;
            (void)parse_emission(m.data(), m.size(), &e, &err);
        }
        {
            const std::string m = mutate(gob, rng);
            Dictionary d;
            (void)parse_gob_dictionary(m.data(), m.size(), &d, &err);
        }
    }
    printf("ok\n");
    return 0;
}
