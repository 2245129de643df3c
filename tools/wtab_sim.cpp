// wtab_sim.cpp — offline count of the DP's weight lookups by weight index
// (diagnostic tool, not part of the product): builds the device image from a
// dictionary, walks every Han rune of a text file as k_mark_walk does, and
// counts the weight index of every DAG edge (calcDagProba's pieceFreq,
// tokenizer.go:511-519).  Prints the share of lookups that fall past the H
// hottest weights (wtab is ordered by use) and, for k_zh's record fields, the
// chance that at least one of a wave's 64 lanes needs such a weight in a field.
//
//   g++ -O2 -std=c++17 -I include -I jieba-go_amd/csrc tools/wtab_sim.cpp jieba-go_amd/csrc/jb_image.cpp -o /tmp/wtab_sim
//   /tmp/wtab_sim dict.txt prob_emit.json corpus.bin [kind] [size]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
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
    std::vector<uint64_t> hits(img.wtab.size() + 1, 0);
    // per rune: the largest weight index among its (at most 4) record fields
    std::vector<uint32_t> rune_max;
    std::vector<uint32_t> run;
    uint64_t edges = 0, runes = 0, items_hist[9] = {0};
    auto flush = [&]() {
        for (size_t i = 0; i < run.size(); i++) {
            runes++;
            uint32_t mx = 0, nit = 0;
            auto edge = [&](uint32_t widx) {
                hits[widx]++;
                edges++;
                nit++;
                mx = std::max(mx, widx);
            };
            const uint32_t row = jb_row(pm, run[i]);
            uint32_t id = img.code[row];
            uint64_t c = img.cells[id];
            if (jb_cell_check(c) != JB_CHECK_ROOT) {
                edge(JB_WIDX_ABSENT);
                rune_max.push_back(mx);
                items_hist[1]++;
                continue;
            }
            edge(jb_cell_widx(c));  // (count 0 or a word: the L = 1 item)
            if (jb_cell_fc(c) != JB_FC_ZERO && jb_cell_hc(c))
                for (size_t j = i + 1; j < run.size(); j++) {
                    const uint64_t t = (uint64_t)jb_cell_base(c) + img.code[jb_row(pm, run[j])];
                    const uint64_t ch = img.cells[t];
                    if (jb_cell_check(ch) != id + 1u) break;
                    if (jb_cell_fc(ch) == JB_FC_POS) edge(jb_cell_widx(ch));
                    if (!jb_cell_hc(ch)) break;
                    id = (uint32_t)t;
                    c = ch;
                }
            rune_max.push_back(mx);
            items_hist[std::min(nit, 8u)]++;
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
    printf("distinct weights %zu, runes %llu, edges %llu (%.2f per rune)\n", img.wtab.size(),
           (unsigned long long)runes, (unsigned long long)edges, (double)edges / (double)runes);
    printf("DAG items per rune (1..7, 8+):");
    for (int k = 1; k <= 8; k++) printf(" %.4f", (double)items_hist[k] / (double)runes);
    printf("\n");
    for (uint32_t H : {64u, 128u, 256u, 512u, 1024u, 2048u, 4096u}) {
        uint64_t cold = 0;
        for (size_t k = H; k < hits.size(); k++) cold += hits[k];
        uint64_t rc = 0;
        for (uint32_t m : rune_max) rc += m >= H;
        const double pr = (double)rc / (double)runes;
        printf("H=%5u: lookups past H %.5f; runes with such an edge %.5f; P(some lane of 64 has one) %.3f\n", H,
               (double)cold / (double)edges, pr, 1.0 - std::pow(1.0 - pr, 64.0));
    }
    return 0;
}
