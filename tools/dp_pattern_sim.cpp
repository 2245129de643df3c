// dp_pattern_sim.cpp — offline census of the DAG item lengths the long-block DP
// chain meets (diagnostic tool, not part of the product): builds the device image
// from a dictionary, walks every Han rune of a text file (buildDag's pieces,
// tokenizer.go:462-497) and prints how often a rune's items are (1), (1,2),
// (1,3), ... and how many aligned groups of G runes have only short forms, for
// sizing k_long_dp's per-group fast path.
//
//   g++ -O2 -std=c++17 -I include -I jieba-go_amd/csrc tools/dp_pattern_sim.cpp jieba-go_amd/csrc/jb_image.cpp -o /tmp/dp_pattern_sim
//   /tmp/dp_pattern_sim dict.txt prob_emit.json corpus.bin [kind] [size]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <cmath>
#include <string>
#include <vector>

#include "jb_image.h"
#include "jiebahip.h"

using namespace jb;

static std::string slurp(const char* p) {
    FILE* f = fopen(p, "rb");
    if (!f) {
        perror(p);
        exit(1);
    }
    std::string s;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
    return s;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s dict emit corpus [kind] [size]\n", argv[0]);
        return 2;
    }
    const int kind = argc > 4 ? atoi(argv[4]) : 1;
    const int64_t size = argc > 5 ? atoll(argv[5]) : 60101967;
    std::string d = slurp(argv[1]), e = slurp(argv[2]), text = slurp(argv[3]);
    Dictionary dict;
    Emission em;
    std::string err;
    if (parse_dictionary(d.data(), d.size(), kind, &dict, &err) || parse_emission(e.data(), e.size(), &em, &err)) {
        fprintf(stderr, "parse: %s\n", err.c_str());
        return 1;
    }
    if (size > 0) dict.size = size;
    Image img;
    if (build_image(dict, em, &img, &err)) {
        fprintf(stderr, "build: %s\n", err.c_str());
        return 1;
    }
    const uint16_t* pm = img.pagemap.data();
    std::map<std::string, uint64_t> pat;
    std::vector<uint8_t> cls;  // per rune: 0 = (1) or (1,2); 1 = (1,3) or (1,4); 2 = up to 4 items, L <= 4; 3 = other
    std::vector<uint32_t> run;
    uint64_t runes = 0;
    auto flush = [&]() {
        for (size_t i = 0; i < run.size(); i++) {
            runes++;
            std::vector<uint32_t> L;
            const uint32_t row = jb_row(pm, run[i]);
            uint32_t id = img.code[row];
            uint64_t c = img.cells[id];
            if (jb_cell_check(c) != JB_CHECK_ROOT) {
                L.push_back(1);
            } else {
                if (jb_cell_fc(c) == JB_FC_POS || jb_cell_fc(c) == JB_FC_ZERO) L.push_back(1);
                if (jb_cell_fc(c) != JB_FC_ZERO && jb_cell_hc(c))
                    for (size_t j = i + 1; j < run.size(); j++) {
                        const uint64_t t = (uint64_t)jb_cell_base(c) + img.code[jb_row(pm, run[j])];
                        const uint64_t ch = img.cells[t];
                        if (jb_cell_check(ch) != id + 1u) break;
                        if (jb_cell_fc(ch) == JB_FC_POS) L.push_back((uint32_t)(j - i + 1));
                        if (!jb_cell_hc(ch)) break;
                        id = (uint32_t)t;
                        c = ch;
                    }
            }
            std::string k;
            for (uint32_t x : L) k += std::to_string(x) + ",";
            if (L.size() > 4) k = ">4 items";
            pat[k]++;
            uint8_t cl = 3;
            const bool l1 = !L.empty() && L[0] == 1;
            if (l1 && (L.size() == 1 || (L.size() == 2 && L[1] == 2))) cl = 0;
            else if (l1 && L.size() == 2 && L[1] <= 4) cl = 1;
            else if (l1 && L.size() <= 4 && L.back() <= 4) cl = 2;
            cls.push_back(cl);
        }
        run.clear();
    };
    const uint8_t* p = (const uint8_t*)text.data();
    for (size_t i = 0; i < text.size();) {
        uint32_t x = 0;
        for (size_t k = 0; k < 4 && i + k < text.size(); k++) x |= (uint32_t)p[i + k] << (8 * k);
        uint32_t r;
        const uint32_t w = jb_decode(x, (uint32_t)std::min<size_t>(4, text.size() - i), &r);
        if (w >= 3 && jb_is_han(r)) run.push_back(r);
        else flush();
        i += w;
    }
    flush();
    std::vector<std::pair<uint64_t, std::string>> v;
    for (auto& kv : pat) v.push_back({kv.second, kv.first});
    std::sort(v.rbegin(), v.rend());
    printf("runes %llu; item lengths by share:\n", (unsigned long long)runes);
    for (size_t k = 0; k < v.size() && k < 16; k++) printf("  (%s) %.4f\n", v[k].second.c_str(), (double)v[k].first / runes);
    uint64_t cc[4] = {0};
    for (uint8_t c : cls) cc[c]++;
    printf("classes: short (1)/(1,2) %.4f, (1,3)/(1,4) %.4f, <=4 items all L<=4 %.4f, other %.4f\n",
           (double)cc[0] / runes, (double)cc[1] / runes, (double)cc[2] / runes, (double)cc[3] / runes);
    for (size_t G : {2, 4, 8}) {
        uint64_t g0 = 0, g1 = 0, g2 = 0, ng = 0;
        for (size_t a = 0; a + G <= cls.size(); a += G) {
            uint8_t m = 0;
            for (size_t k = 0; k < G; k++) m = std::max(m, cls[a + k]);
            ng++;
            g0 += m == 0;
            g1 += m <= 1;
            g2 += m <= 2;
        }
        printf("groups of %zu: all short %.4f, all class<=1 %.4f, all class<=2 %.4f\n", G, (double)g0 / ng,
               (double)g1 / ng, (double)g2 / ng);
    }
    return 0;
}
