// trie_sim.cpp — offline model of k_mark_walk's trie probes (diagnostic tool,
// not part of the product): builds the device image from a dictionary, walks
// every Han rune of a text file the way the kernel does (level-1 row, then one
// double-array cell per further rune while the node has children and the Han
// run goes on), and replays the cell addresses through an LRU cache of one
// XCD's L2 (4 MB, 128-byte lines).  Used to compare cell layouts
// (JB_TRIE_LAYOUT) before spending GPU time on them.
//
//   g++ -O2 -std=c++17 -I include -I jieba-go_amd/csrc tools/trie_sim.cpp jieba-go_amd/csrc/jb_image.cpp -o /tmp/trie_sim
//   /tmp/trie_sim dict.txt prob_emit.json corpus.bin [kind] [size]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <list>
#include <string>
#include <unordered_map>
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

struct Lru {
    size_t cap;
    std::list<uint64_t> order;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> at;
    uint64_t hit = 0, miss = 0;
    explicit Lru(size_t lines) : cap(lines) {}
    void touch(uint64_t line) {
        auto it = at.find(line);
        if (it != at.end()) {
            hit++;
            order.splice(order.begin(), order, it->second);
            return;
        }
        miss++;
        order.push_front(line);
        at[line] = order.begin();
        if (order.size() > cap) {
            at.erase(order.back());
            order.pop_back();
        }
    }
};

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
    // Han runes of the text, 3-byte forms only (the synthetic corpus has no others), runs split at non-Han
    std::vector<uint32_t> run;
    Lru l2(4u << 20 >> 7), l2r(4u << 20 >> 7);
    std::vector<uint64_t> line_hits((img.cells.size() * 8 >> 7) + 1, 0);
    uint64_t probes = 0, runes = 0, walks = 0;
    // Child-code filters: per node with children, bit h(code) of each child's code for
    // B-bit filters (h = code mod B); a probe the filter rejects need not be made.
    constexpr int kFB[] = {1, 2, 3, 4, 5, 6, 8, 12, 16};
    constexpr int kNF = sizeof(kFB) / sizeof(kFB[0]);
    std::vector<uint32_t> filt(img.cells.size() * kNF, 0);
    for (size_t t = 0; t < img.cells.size(); t++) {
        const uint32_t ck = jb_cell_check(img.cells[t]);
        if (ck == 0 || ck == JB_CHECK_ROOT) continue;
        const uint32_t par = ck - 1u;
        const uint32_t code = (uint32_t)t - jb_cell_base(img.cells[par]);
        for (int f = 0; f < kNF; f++) filt[(size_t)par * kNF + f] |= 1u << (code % kFB[f]);
    }
    uint64_t miss_probes = 0, rejected[kNF] = {0};
    auto flush = [&]() {
        for (size_t i = 0; i < run.size(); i++) {
            runes++;
            const uint32_t row = jb_row(pm, run[i]);
            l2r.touch((uint64_t)row * 8 >> 7);  // the l1row load
            uint32_t id = img.code[row];
            uint64_t c = img.cells[id];
            if (jb_cell_check(c) != JB_CHECK_ROOT || !jb_cell_hc(c)) continue;
            walks++;
            for (size_t j = i + 1; j < run.size(); j++) {
                const uint64_t t = (uint64_t)jb_cell_base(c) + img.code[jb_row(pm, run[j])];
                probes++;
                l2.touch(t * 8 >> 7);
                line_hits[t * 8 >> 7]++;
                const uint64_t ch = img.cells[t];
                if (jb_cell_check(ch) != id + 1u) {
                    miss_probes++;
                    const uint32_t code = img.code[jb_row(pm, run[j])];
                    for (int f = 0; f < kNF; f++)
                        if (!((filt[(size_t)id * kNF + f] >> (code % kFB[f])) & 1u)) rejected[f]++;
                }
                if (jb_cell_check(ch) != id + 1u || !jb_cell_hc(ch)) break;
                id = (uint32_t)t;
                c = ch;
            }
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
    // how concentrated the probes are: bytes of the hottest lines covering 90/95/99 % of probes
    std::vector<uint64_t> h = line_hits;
    std::sort(h.begin(), h.end(), std::greater<uint64_t>());
    double acc = 0;
    size_t at90 = 0, at95 = 0, at99 = 0;
    for (size_t k = 0; k < h.size(); k++) {
        acc += (double)h[k];
        if (!at90 && acc >= 0.90 * probes) at90 = k + 1;
        if (!at95 && acc >= 0.95 * probes) at95 = k + 1;
        if (!at99 && acc >= 0.99 * probes) at99 = k + 1;
    }
    printf("cells %zu (%.1f MB) runes %llu walks %llu probes %llu (%.2f per rune)\n", img.cells.size(),
           img.cells.size() * 8 / 1e6, (unsigned long long)runes, (unsigned long long)walks,
           (unsigned long long)probes, (double)probes / (double)runes);
    printf("cell probes: LRU-4MB hit %.4f; hottest lines for 90/95/99%% of probes: %.2f / %.2f / %.2f MB\n",
           (double)l2.hit / (double)(l2.hit + l2.miss), at90 * 128 / 1e6, at95 * 128 / 1e6, at99 * 128 / 1e6);
    printf("l1row loads: LRU-4MB hit %.4f\n", (double)l2r.hit / (double)(l2r.hit + l2r.miss));
    printf("walk-ending misses %llu (%.3f of probes); rejected by a B-bit child-code filter:",
           (unsigned long long)miss_probes, (double)miss_probes / (double)probes);
    for (int f = 0; f < kNF; f++) printf(" B=%d %.3f", kFB[f], (double)rejected[f] / (double)probes);
    printf(" (of all probes)\n");
    return 0;
}
