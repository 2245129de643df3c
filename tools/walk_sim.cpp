// walk_sim.cpp — offline model of k_mark_walk's walk phase per 4 KiB tile (diagnostic
// tool, not part of the product).  It lists each tile's Han runes, puts the runes whose
// walk goes past level 1 on the walk list, splits the list in quarters over the four
// waves and runs every wave's lanes as the kernel does (one probe per active lane and
// trip, idle lanes refill from the wave's quarter).  Per trip it counts the distinct
// 128-byte lines the wave's probe gathers (what one gather asks of L2 when it misses
// the L1), for several orders of the walk list:
//   text   the list in text order (the kernel's atomicAdd order, roughly)
//   code1  sorted by the first rune's code
//   cell2  sorted by the first probe's cell (level-1 base + code of the next rune)
// It also counts the level-1 row gathers (one per lane slot and wave, hot rows excluded).
//
//   g++ -O2 -std=c++17 -I include -I jieba-go_amd/csrc tools/walk_sim.cpp jieba-go_amd/csrc/jb_image.cpp -o /tmp/walk_sim
//   /tmp/walk_sim dict.txt prob_emit.json corpus.bin [kind] [size]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_set>
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

struct Ent {
    uint32_t pos, row, code, run_next;  // run_next: index of the next rune of the run, or ~0
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
    std::vector<uint64_t> hv(JB_HOT_SLOTS);
    std::vector<uint16_t> ht(JB_HOT_SLOTS);
    build_hot_rows(img, hv.data(), ht.data());
    const uint16_t* pm = img.pagemap.data();
    // every rune of the text: Han runes as entries, others break runs
    std::vector<Ent> ents;
    const uint8_t* p = (const uint8_t*)text.data();
    bool prev_han = false;
    for (size_t i = 0; i < text.size();) {
        uint32_t x = 0;
        for (size_t k = 0; k < 4 && i + k < text.size(); k++) x |= (uint32_t)p[i + k] << (8 * k);
        uint32_t r;
        const uint32_t w = jb_decode(x, (uint32_t)std::min<size_t>(4, text.size() - i), &r);
        const bool h = w >= 3 && jb_is_han(r);
        if (h) {
            if (prev_han) ents.back().run_next = (uint32_t)ents.size();
            const uint32_t row = jb_row(pm, r);
            ents.push_back({(uint32_t)i, row, img.code[row], ~0u});
        }
        prev_han = h;
        i += w;
    }
    const size_t ntiles = (text.size() + 4095) / 4096;
    constexpr int NO = 6;
    const char* names[NO] = {"text", "code1", "cell2", "b128c1", "b128ln", "b64ln"};
    uint64_t lines[NO] = {0}, probes[NO] = {0}, trips[NO] = {0}, maxtrips[NO] = {0};
    uint64_t rng = 12345;
    uint64_t l1g_lines = 0, l1g_lanes = 0, l1_hot = 0, nent_all = 0, nwalk_all = 0;
    size_t e0 = 0;
    for (size_t t = 0; t < ntiles; t++) {
        const uint32_t t0 = (uint32_t)(t * 4096);
        size_t e1 = e0;
        while (e1 < ents.size() && ents[e1].pos < t0 + 4096) e1++;
        nent_all += e1 - e0;
        // level-1 gathers: wave = lane / 64, slot = the rune's index among the lane's Han starts
        {
            std::vector<std::unordered_set<uint32_t>> g(4 * 8);
            uint32_t lane_prev = ~0u, slot = 0;
            for (size_t k = e0; k < e1; k++) {
                const uint32_t lane = (ents[k].pos - t0) / 16;
                slot = lane == lane_prev ? slot + 1 : 0;
                lane_prev = lane;
                const uint32_t r = ents[k].row + 0x3300u;  // (U+3400..U+9FFF rows)
                if (ht[jb_hot_slot(r)] == r) {
                    l1_hot++;
                    continue;
                }
                l1g_lanes++;
                g[(lane / 64) * 8 + std::min(slot, 7u)].insert(ents[k].row * 8 / 128);
            }
            for (auto& s : g) l1g_lines += s.size();
        }
        // walk list: level-1 key with children, run goes on
        std::vector<uint32_t> wl;
        for (size_t k = e0; k < e1; k++) {
            const uint64_t c = img.cells[ents[k].code];
            if (ents[k].code == 0 || jb_cell_check(c) != JB_CHECK_ROOT || jb_cell_fc(c) == JB_FC_ZERO) continue;
            if (!jb_cell_hc(c) || ents[k].run_next == ~0u) continue;
            wl.push_back((uint32_t)k);
        }
        nwalk_all += wl.size();
        for (int ord = 0; ord < NO; ord++) {
            std::vector<uint32_t> L = wl;
            if (ord >= 3) {  // counting sort into B buckets; order within a bucket arbitrary (LDS atomics)
                const uint32_t B = ord == 5 ? 64u : 128u;
                auto bk = [&](uint32_t a) -> uint32_t {
                    if (ord == 3) return std::min(ents[a].code, B - 1u);
                    const uint64_t cell = (uint64_t)jb_cell_base(img.cells[ents[a].code]) + ents[ents[a].run_next].code;
                    return (uint32_t)(((cell >> 4) * 0x9E3779B1u) >> 7) % B;
                };
                std::vector<std::vector<uint32_t>> bb(B);
                for (uint32_t a : L) bb[bk(a)].push_back(a);
                L.clear();
                for (auto& v : bb) {
                    for (size_t q = v.size(); q > 1; q--) {  // shuffle (atomic order)
                        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
                        std::swap(v[q - 1], v[(rng >> 33) % q]);
                    }
                    L.insert(L.end(), v.begin(), v.end());
                }
            }
            if (ord == 1)
                std::stable_sort(L.begin(), L.end(), [&](uint32_t a, uint32_t b) { return ents[a].code < ents[b].code; });
            if (ord == 2) {
                auto key = [&](uint32_t a) {
                    return (uint64_t)jb_cell_base(img.cells[ents[a].code]) + ents[ents[a].run_next].code;
                };
                std::stable_sort(L.begin(), L.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
            }
            const uint32_t nwl = (uint32_t)L.size();
            uint32_t mt = 0;
            for (uint32_t wv = 0; wv < 4; wv++) {
                uint32_t head = nwl * wv / 4, hi = nwl * (wv + 1) / 4;
                struct W {
                    bool act = false;
                    uint32_t cur = 0, node = 0, len = 0;
                } ln[64];
                uint32_t tr = 0;
                for (;;) {
                    for (int l = 0; l < 64; l++)
                        if (!ln[l].act && head < hi) {
                            ln[l].act = true;
                            ln[l].cur = ents[L[head]].run_next;
                            ln[l].node = ents[L[head]].code;
                            ln[l].len = 1;
                            head++;
                        }
                    bool any = false;
                    std::unordered_set<uint64_t> s;
                    for (int l = 0; l < 64; l++) {
                        if (!ln[l].act) continue;
                        any = true;
                        const uint64_t c = img.cells[ln[l].node];
                        const uint32_t cell = jb_cell_base(c) + ents[ln[l].cur].code;
                        s.insert((uint64_t)cell * 8 / 128);
                        probes[ord]++;
                        const uint64_t ch = img.cells[cell];
                        const bool hit = jb_cell_check(ch) == ln[l].node + 1u;
                        ln[l].len++;
                        const uint32_t nx = ents[ln[l].cur].run_next;
                        // (walks stop 40 bytes past the tile in the kernel: about 13 runes)
                        const bool go = hit && jb_cell_hc(ch) && nx != ~0u && ents[nx].pos < t0 + 4096 + 40;
                        if (go) {
                            ln[l].node = cell;
                            ln[l].cur = nx;
                        } else {
                            ln[l].act = false;
                        }
                    }
                    if (!any) break;
                    tr++;
                    lines[ord] += s.size();
                }
                trips[ord] += tr;
                mt = std::max(mt, tr);
            }
            maxtrips[ord] += mt;
        }
        e0 = e1;
    }
    printf("tiles %zu Han runes %llu walks %llu (%.2f per tile)\n", ntiles, (unsigned long long)nent_all,
           (unsigned long long)nwalk_all, (double)nwalk_all / ntiles);
    printf("level-1: hot %.3f of runes; gathered lanes %.1f per tile -> %.1f lines per tile\n",
           (double)l1_hot / nent_all, (double)l1g_lanes / ntiles, (double)l1g_lines / ntiles);
    for (int ord = 0; ord < NO; ord++)
        printf("%-6s probes %.1f per tile, lines %.1f per tile (%.3f per probe), wave trips %.2f mean, %.2f max per tile\n",
               names[ord], (double)probes[ord] / ntiles, (double)lines[ord] / ntiles,
               (double)lines[ord] / probes[ord], (double)trips[ord] / ntiles / 4, (double)maxtrips[ord] / ntiles);
    return 0;
}
