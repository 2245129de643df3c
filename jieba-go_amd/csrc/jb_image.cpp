// jb_image.cpp — host loaders for the reference's model files and the builder
// of the device image (jb_common.h).  Host code only.
//
//   dict.txt          parse_dictionary  (tokenizer.go:389-437 and :340-366)
//   prob_emit.json    parse_emission    (tokenizer.go:653-661)
//   device image      build_image       (replaces termFreq/emitP map lookups,
//                                         tokenizer.go:468,475,516,689,708)
#include "jb_image.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <unordered_set>
#include <cstdlib>

#include "../../include/jiebahip.h"

namespace jb {

// Go 1.18 math.Log (src/math/log.go; the amd64 assembly performs the same
// operations in the same order).  Built with -ffp-contract=off so that no
// multiply-add is fused, as on Go/amd64.
double go_log(double x) {
    static const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                        L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                        L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                        L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                        L7 = 1.479819860511658591e-01;
    if (std::isnan(x) || x == INFINITY) return x;
    if (x < 0) return NAN;
    if (x == 0) return -INFINITY;
    int ki;
    double f1 = frexp(x, &ki);
    if (f1 < 0.70710678118654752440) {  // Sqrt2/2
        f1 *= 2;
        ki--;
    }
    const double f = f1 - 1;
    const double k = (double)ki;
    const double s = f / (2 + f);
    const double s2 = s * s;
    const double s4 = s2 * s2;
    const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    const double R = t1 + t2;
    const double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// ---------------------------------------------------------------------------
// UTF-8 helpers (Go semantics)
// ---------------------------------------------------------------------------
static uint32_t decode_at(const uint8_t* s, size_t n, uint32_t* r) {
    uint32_t x = 0;
    const size_t take = n < 4 ? n : 4;
    for (size_t k = 0; k < take; k++) x |= (uint32_t)s[k] << (8 * k);
    return jb_decode(x, (uint32_t)take, r);
}

static void append_utf8(std::string* o, uint32_t r) {
    if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = 0xFFFD;
    if (r < 0x80) o->push_back((char)r);
    else if (r < 0x800) { o->push_back((char)(0xC0 | (r >> 6))); o->push_back((char)(0x80 | (r & 0x3F))); }
    else if (r < 0x10000) {
        o->push_back((char)(0xE0 | (r >> 12)));
        o->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o->push_back((char)(0x80 | (r & 0x3F)));
    } else {
        o->push_back((char)(0xF0 | (r >> 18)));
        o->push_back((char)(0x80 | ((r >> 12) & 0x3F)));
        o->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o->push_back((char)(0x80 | (r & 0x3F)));
    }
}

// Runes of a key when every byte sequence is valid UTF-8; false otherwise.
static bool valid_runes(const std::string& k, std::vector<uint32_t>* out) {
    out->clear();
    const uint8_t* s = (const uint8_t*)k.data();
    size_t i = 0;
    while (i < k.size()) {
        uint32_t r;
        uint32_t w = decode_at(s + i, k.size() - i, &r);
        if (r == 0xFFFD && w == 1) return false;
        out->push_back(r);
        i += w;
    }
    return true;
}

// strconv.Atoi, base 10, 64-bit.
static bool atoi64(const char* s, size_t n, int64_t* v) {
    if (n == 0) return false;
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i == n) return false;
    unsigned __int128 acc = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        acc = acc * 10 + (unsigned)(s[i] - '0');
        if (acc > ((unsigned __int128)1 << 63)) return false;
    }
    if (!neg && acc > (unsigned __int128)INT64_MAX) return false;
    *v = neg ? (int64_t)(0 - (uint64_t)acc) : (int64_t)acc;
    return true;
}

int parse_dictionary(const char* buf, size_t len, int kind, Dictionary* out, std::string* err) {
    out->term_freq.clear();
    out->term_freq.reserve(len / (kind == JB_DICT_TXT ? 14 : 8) + 16);
    out->size = 0;
    int64_t total = 0;
    size_t pos = 0, lineno = 0;
    std::string piece;
    std::vector<uint32_t> runes;
    while (pos < len) {
        // bufio.ScanLines: split at '\n', drop one trailing '\r'
        size_t e = pos;
        while (e < len && buf[e] != '\n') e++;
        size_t l = e - pos;
        const char* line = buf + pos;
        pos = e < len ? e + 1 : e;
        lineno++;
        if (l > 0 && line[l - 1] == '\r') l--;
        if (l > 65535) break;  // bufio.Scanner stops at ErrTooLong; the reference ignores the error
        // strings.SplitN(line, " ", 3): parts[0] word, parts[1] count
        const char* sp = (const char*)memchr(line, ' ', l);
        if (!sp) {
            *err = "dictionary line " + std::to_string(lineno) + ": no count field (the reference panics)";
            return JB_EPARSE;
        }
        const size_t wl = (size_t)(sp - line);
        const char* c = sp + 1;
        const size_t rest = l - wl - 1;
        const char* sp2 = (const char*)memchr(c, ' ', rest);
        const size_t cl = sp2 ? (size_t)(sp2 - c) : rest;
        int64_t count;
        if (!atoi64(c, cl, &count)) {
            *err = "dictionary line " + std::to_string(lineno) + ": strconv.Atoi: invalid count";
            return JB_EPARSE;
        }
        std::string word(line, wl);
        if (kind == JB_DICT_TXT) {
            // first occurrence wins; size sums first occurrences (tokenizer.go:418-423)
            auto ins = out->term_freq.emplace(std::move(word), count);
            if (ins.second) out->size += count;
        } else {
            // last value wins, every line counted, prefixes added with 0 (tokenizer.go:343-362)
            total += count;
            if (word.empty()) {
                *err = "dictionary line " + std::to_string(lineno) + ": empty word (the reference panics)";
                return JB_EPARSE;
            }
            out->term_freq[word] = count;
            // prefix pieces are built rune by rune: invalid bytes become U+FFFD
            const uint8_t* s = (const uint8_t*)word.data();
            size_t i = 0;
            piece.clear();
            runes.clear();
            while (i < word.size()) {
                uint32_t r;
                i += decode_at(s + i, word.size() - i, &r);
                runes.push_back(r);
            }
            for (size_t k = 0; k + 1 < runes.size(); k++) {
                append_utf8(&piece, runes[k]);
                out->term_freq.emplace(piece, 0);  // only if absent
            }
        }
    }
    if (kind != JB_DICT_TXT) out->size = total;
    return JB_OK;
}

// ---------------------------------------------------------------------------
// prob_emit.json: encoding/json into map[string]map[string]float64
// ---------------------------------------------------------------------------
namespace {
struct Json {
    const char* s;
    size_t n, i = 0;
    void ws() {
        while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
    }
    bool lit(char c) {
        ws();
        if (i < n && s[i] == c) { i++; return true; }
        return false;
    }
    bool hex4(uint32_t* v) {
        if (i + 4 > n) return false;
        uint32_t x = 0;
        for (int k = 0; k < 4; k++) {
            const char c = s[i++];
            x <<= 4;
            if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
            else return false;
        }
        *v = x;
        return true;
    }
    bool str(std::string* o) {
        ws();
        o->clear();
        if (i >= n || s[i] != '"') return false;
        i++;
        while (i < n) {
            const uint8_t c = (uint8_t)s[i];
            if (c == '"') { i++; return true; }
            if (c == '\\') {
                if (++i >= n) return false;
                const char e = s[i++];
                switch (e) {
                    case '"': o->push_back('"'); break;
                    case '\\': o->push_back('\\'); break;
                    case '/': o->push_back('/'); break;
                    case 'b': o->push_back('\b'); break;
                    case 'f': o->push_back('\f'); break;
                    case 'n': o->push_back('\n'); break;
                    case 'r': o->push_back('\r'); break;
                    case 't': o->push_back('\t'); break;
                    case 'u': {
                        uint32_t r;
                        if (!hex4(&r)) return false;
                        if (r >= 0xD800 && r < 0xDC00) {
                            const size_t save = i;
                            uint32_t r2;
                            if (i + 1 < n && s[i] == '\\' && s[i + 1] == 'u') {
                                i += 2;
                                if (!hex4(&r2)) return false;
                                if (r2 >= 0xDC00 && r2 < 0xE000) r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
                                else { r = 0xFFFD; i = save; }
                            } else {
                                r = 0xFFFD;
                            }
                        } else if (r >= 0xDC00 && r < 0xE000) {
                            r = 0xFFFD;
                        }
                        append_utf8(o, r);
                        break;
                    }
                    default: return false;
                }
            } else if (c < 0x80) {
                o->push_back((char)c);
                i++;
            } else {
                uint32_t r;
                i += decode_at((const uint8_t*)s + i, n - i, &r);
                append_utf8(o, r);  // invalid UTF-8 becomes U+FFFD
            }
        }
        return false;
    }
    bool num(double* v) {
        ws();
        const size_t st = i;
        while (i < n && (strchr("+-.eE0123456789", s[i]) != nullptr) && s[i] != 0) i++;
        if (i == st || i - st > 120) return false;
        char tmp[128];
        memcpy(tmp, s + st, i - st);
        tmp[i - st] = 0;
        char* end;
        *v = strtod(tmp, &end);  // correctly rounded, as strconv.ParseFloat
        return *end == 0;
    }
    bool null() {
        ws();
        if (i + 4 <= n && memcmp(s + i, "null", 4) == 0) { i += 4; return true; }
        return false;
    }
};
}  // namespace

int parse_emission(const char* buf, size_t len, Emission* out, std::string* err) {
    for (auto& m : out->by_rune) m.clear();
    Json j{buf, len};
    std::string key, k2;
    auto fail = [&](const char* what) {
        *err = std::string("prob_emit.json: ") + what + " near byte " + std::to_string(j.i);
        return JB_EPARSE;
    };
    if (!j.lit('{')) return fail("expected object");
    if (j.lit('}')) return JB_OK;
    for (;;) {
        if (!j.str(&key)) return fail("expected key");
        if (!j.lit(':')) return fail("expected ':'");
        int st = -1;
        if (key == "B") st = JB_B;
        else if (key == "M") st = JB_M;
        else if (key == "E") st = JB_E;
        else if (key == "S") st = JB_S;
        // a repeated outer key decodes into a fresh inner map (last one wins)
        if (st >= 0) out->by_rune[st].clear();
        if (!j.null()) {
            if (!j.lit('{')) return fail("expected inner object");
            if (!j.lit('}')) {
                for (;;) {
                    if (!j.str(&k2)) return fail("expected inner key");
                    if (!j.lit(':')) return fail("expected ':'");
                    double v;
                    if (!j.num(&v)) return fail("expected number");
                    if (st >= 0) {
                        uint32_t r;
                        const uint32_t w = decode_at((const uint8_t*)k2.data(), k2.size(), &r);
                        if (!k2.empty() && w == k2.size()) out->by_rune[st][r] = v;
                    }
                    if (j.lit(',')) continue;
                    if (j.lit('}')) break;
                    return fail("expected ',' or '}'");
                }
            }
        }
        if (j.lit(',')) continue;
        if (j.lit('}')) break;
        return fail("expected ',' or '}'");
    }
    return JB_OK;
}

// ---------------------------------------------------------------------------
// Device image
// ---------------------------------------------------------------------------
static uint32_t jb_buckets_seed(uint32_t attempt) { return attempt * 0x7F4A7C15u + 0x2545F491u; }

static uint32_t freq_class(int64_t f) { return f > 0 ? JB_FC_POS : (f == 0 ? JB_FC_ZERO : JB_FC_NEG); }

int build_image(const Dictionary& d, const Emission& e, Image* img, std::string* err) {
    img->size = d.size;
    img->total = go_log((double)d.size);       // calcDagProba: total := math.Log(float64(pd.size))
    img->w_absent = go_log(1.0) - img->total;  // tf := 1.0 when the piece is absent (tokenizer.go:515)

    // Keys a walk can spell: valid UTF-8, every rune Han.
    struct Key { std::vector<uint32_t> r; int64_t f; };
    std::vector<Key> keys;
    keys.reserve(d.term_freq.size());
    std::vector<uint32_t> runes;
    for (const auto& kv : d.term_freq) {
        if (!valid_runes(kv.first, &runes) || runes.empty()) continue;
        bool han = true;
        for (uint32_t r : runes) han = han && jb_is_han(r);
        if (!han) continue;  // a Han run can never spell this key
        keys.push_back(Key{runes, kv.second});
    }
    std::sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) {
        if (a.r.size() != b.r.size()) return a.r.size() < b.r.size();
        return a.r < b.r;
    });

    // pages: single-rune keys and emission runes
    std::vector<uint8_t> page_used(JB_NPAGES_MAX, 0);
    for (const Key& k : keys)
        if (k.r.size() == 1) page_used[k.r[0] >> 8] = 1;
    for (int s = 0; s < 4; s++)
        for (const auto& kv : e.by_rune[s])
            if (kv.first < 0x110000u) page_used[kv.first >> 8] = 1;
    img->pagemap.assign(JB_NPAGES_MAX, 0);
    for (uint32_t p = 0; p < JB_DIRECT_PAGES; p++) img->pagemap[(JB_DIRECT_LO >> 8) + p] = (uint16_t)(p + 1);
    img->npages = 1 + JB_DIRECT_PAGES;  // page 0: the empty page; then the fixed U+3400..U+9FFF pages
    for (uint32_t p = 1; p < JB_NPAGES_MAX; p++)
        if (page_used[p] && img->pagemap[p] == 0) img->pagemap[p] = (uint16_t)img->npages++;
    if (page_used[0]) img->pagemap[0] = (uint16_t)img->npages++;
    img->nrows = img->npages * 256u;
    const uint16_t* pm = img->pagemap.data();

    // distinct weights: pieceFreq := math.Log(tf) - total (tokenizer.go:519).  Indices go to
    // the weights in order of how many keys use them (ties by value bits), so the
    // common ones get small indices (k_mark_walk packs 14-bit indices).
    img->wtab.assign(1, img->w_absent);
    std::unordered_map<uint64_t, uint32_t> widx_of;
    auto wbits = [&](int64_t f) -> uint64_t {
        const double w = go_log((double)f) - img->total;
        uint64_t bits;
        memcpy(&bits, &w, 8);
        return bits;
    };
    {
        std::unordered_map<uint64_t, uint64_t> uses;
        for (const Key& k : keys) uses[wbits(k.f)]++;
        std::vector<std::pair<uint64_t, uint64_t>> order(uses.begin(), uses.end());
        std::sort(order.begin(), order.end(), [](const std::pair<uint64_t, uint64_t>& a,
                                                 const std::pair<uint64_t, uint64_t>& b) {
            return a.second != b.second ? a.second > b.second : a.first < b.first;
        });
        for (const auto& o : order) {
            double w;
            memcpy(&w, &o.first, 8);
            widx_of.emplace(o.first, (uint32_t)img->wtab.size());
            img->wtab.push_back(w);
        }
    }
    auto widx = [&](int64_t f) -> uint32_t { return widx_of.at(wbits(f)); };

    size_t deep = 0;
    for (const Key& k : keys) deep += k.r.size() > 1;
    img->l1.assign(img->nrows, jb_l1_make(JB_FC_ABSENT, 0, JB_WIDX_ABSENT));
    img->maxlen = 0;
    img->nnodes = 0;
    for (const Key& k : keys) {  // level 1: the l1 rows
        if (k.r.size() != 1) continue;
        const uint32_t wi = widx(k.f);
        if (wi >= JB_MAX_WIDX) {
            *err = "more than " + std::to_string(JB_MAX_WIDX) + " distinct frequencies";
            return JB_ELIMIT;
        }
        img->l1[jb_row(pm, k.r[0])] = jb_l1_make(freq_class(k.f), 0, wi);
        img->nnodes++;
        img->maxlen = 1;
    }
    const std::vector<uint32_t> l1_base = img->l1;
    const uint64_t nnodes1 = img->nnodes;
    // Deeper levels: bucketed cuckoo hash, placed level by level.  A node's slot
    // is its id, so a placement may not move a node that is already a parent:
    // it moves leaves (keys no longer key extends) and nodes of the level being
    // placed.  Load <= 2/3; a placement that gets stuck retries with another
    // hash seed, and the table doubles after 16 seeds.
    std::unordered_set<std::string> internal;  // keys that a longer key extends by one rune
    auto rkey = [](const std::vector<uint32_t>& r, size_t n) {
        return std::string(reinterpret_cast<const char*>(r.data()), n * sizeof(uint32_t));
    };
    for (const Key& k : keys)
        if (k.r.size() >= 3) internal.insert(rkey(k.r, k.r.size() - 1));
    uint64_t cap = 1024;
    while (cap * 2 < deep * 3) cap <<= 1;  // load <= 2/3
    for (uint32_t attempt = 0;; attempt++) {
        if (attempt && attempt % 16 == 0) cap <<= 1;
        img->seed = attempt ? jb_buckets_seed(attempt) : 0u;
        if (img->nrows + cap >= JB_MAX_IDS - 1) {
            *err = "dictionary too large for the packed trie (" + std::to_string(deep) + " multi-rune keys)";
            return JB_ELIMIT;
        }
        img->nodes.assign(cap, JB_NODE_EMPTY);
        img->l1 = l1_base;
        img->nnodes = nnodes1;
        std::vector<uint8_t> lvl(cap, 0);  // level of the node in each slot; 0 = free to move
        const uint32_t bmask = (uint32_t)(cap / JB_BUCKET - 1);
        auto find = [&](uint32_t parent, uint32_t r) -> uint64_t {  // slot or ~0
            uint32_t b[2];
            jb_buckets(parent, r, bmask, img->seed, &b[0], &b[1]);
            for (int i = 0; i < 2 * JB_BUCKET; i++) {
                const uint64_t sl = (uint64_t)JB_BUCKET * b[i / JB_BUCKET] + (i % JB_BUCKET);
                if (jb_node_is(img->nodes[sl], parent, r)) return sl;
            }
            return ~0ull;
        };
        uint64_t rng = 0x9E3779B97F4A7C15ull;
        // level: the level being placed; a node is stored with its level, or 0 if it is a leaf
        auto place = [&](uint64_t node, uint8_t nlvl, uint8_t level) -> bool {
            for (int kick = 0; kick < 512; kick++) {
                uint32_t b[2];
                jb_buckets(jb_node_parent(node), jb_node_rune(node), bmask, img->seed, &b[0], &b[1]);
                // the emptier of the two buckets first (keeps buckets evenly filled)
                int fill[2] = {0, 0};
                for (int i = 0; i < 2 * JB_BUCKET; i++)
                    fill[i / JB_BUCKET] += img->nodes[(uint64_t)JB_BUCKET * b[i / JB_BUCKET] + (i % JB_BUCKET)] !=
                                           JB_NODE_EMPTY;
                const int first = fill[1] < fill[0] ? 1 : 0;
                uint64_t movable[2 * JB_BUCKET];
                int nm = 0;
                for (int i0 = 0; i0 < 2 * JB_BUCKET; i0++) {
                    const int i = (i0 + first * JB_BUCKET) % (2 * JB_BUCKET);
                    const uint64_t sl = (uint64_t)JB_BUCKET * b[i / JB_BUCKET] + (i % JB_BUCKET);
                    if (img->nodes[sl] == JB_NODE_EMPTY) {
                        img->nodes[sl] = node;
                        lvl[sl] = nlvl;
                        return true;
                    }
                    if (lvl[sl] == level || lvl[sl] == 0) movable[nm++] = sl;
                }
                if (nm == 0) {
                    if (getenv("JB_DEBUG_BUILD")) {
                        fprintf(stderr, "stuck kick %d:", kick);
                        for (int i = 0; i < 2 * JB_BUCKET; i++)
                            fprintf(stderr, " %u", (unsigned)lvl[(uint64_t)JB_BUCKET * b[i / JB_BUCKET] + (i % JB_BUCKET)]);
                        fprintf(stderr, " b=%u,%u\n", b[0], b[1]);
                    }
                    return false;
                }
                rng ^= rng << 13;
                rng ^= rng >> 7;
                rng ^= rng << 17;
                const uint64_t v = movable[rng % (uint64_t)nm];
                std::swap(node, img->nodes[v]);
                std::swap(nlvl, lvl[v]);
            }
            return false;
        };
        std::vector<uint32_t> parents;  // parent id of every stored deeper node
        bool ok_all = true;
        for (size_t i0 = 0; i0 < keys.size() && ok_all;) {
            const size_t n = keys[i0].r.size();
            size_t i1 = i0;
            while (i1 < keys.size() && keys[i1].r.size() == n) i1++;
            if (n >= 2) {
                for (size_t i = i0; i < i1 && ok_all; i++) {
                    const Key& k = keys[i];
                    // parent id: level-1 row, then nrows + slot for each deeper prefix
                    const uint32_t row0 = jb_row(pm, k.r[0]);
                    if ((img->l1[row0] & 3u) == JB_FC_ABSENT) continue;  // unreachable (tokenizer.go:475-478)
                    uint32_t parent = row0;
                    bool ok = true;
                    for (size_t j = 1; j + 1 < n && ok; j++) {
                        const uint64_t sl = find(parent, k.r[j]);
                        ok = sl != ~0ull;
                        if (ok) parent = img->nrows + (uint32_t)sl;
                    }
                    if (!ok) continue;
                    const uint32_t wi = widx(k.f);
                    if (wi >= JB_MAX_WIDX) {
                        *err = "more than " + std::to_string(JB_MAX_WIDX) + " distinct frequencies";
                        return JB_ELIMIT;
                    }
                    const uint8_t nl = internal.count(rkey(k.r, n)) ? (uint8_t)std::min<size_t>(n, 255) : 0;
                    if (!place(jb_node_make(parent, k.r.back(), freq_class(k.f), 0, wi), nl,
                               (uint8_t)std::min<size_t>(n, 255))) {
                        if (getenv("JB_DEBUG_BUILD")) fprintf(stderr, "cap %llu: placement failed at key %zu (len %zu) nnodes %llu\n", (unsigned long long)cap, i, n, (unsigned long long)img->nnodes);
                        ok_all = false;
                        break;
                    }
                    parents.push_back(parent);
                    img->nnodes++;
                    img->maxlen = std::max<uint32_t>(img->maxlen, (uint32_t)n);
                }
            }
            i0 = i1;
        }
        if (!ok_all) continue;  // another seed / a bigger table
        // has-children flags: a walk stops at a node without children, no probe
        for (uint32_t p : parents) {
            if (p < img->nrows) img->l1[p] |= 1u << 2;
            else img->nodes[p - img->nrows] |= 1ull << 23;
        }
        break;
    }
    img->emit.assign((size_t)img->npages * 256 * 4, JB_MIN_FLOAT);  // not found -> minFloat (tokenizer.go:690,710)
    for (int s = 0; s < 4; s++)
        for (const auto& kv : e.by_rune[s]) {
            if (kv.first >= 0x110000u) continue;
            img->emit[(size_t)jb_row(pm, kv.first) * 4 + s] = kv.second;
        }
    return JB_OK;
}

Lookup image_lookup(const Image& img, const uint32_t* runes, size_t n) {
    Lookup out;
    if (n == 0 || runes[0] >= 0x110000u) return out;
    const uint32_t row = jb_row(img.pagemap.data(), runes[0]);
    const uint32_t rec = img.l1[row];
    if ((rec & 3u) == JB_FC_ABSENT) return out;
    uint32_t id = row, fc = rec & 3u, wi = rec >> 3;
    const uint32_t bmask = (uint32_t)(img.nodes.size() / JB_BUCKET - 1);
    for (size_t i = 1; i < n; i++) {
        uint32_t b[2];
        jb_buckets(id, runes[i], bmask, img.seed, &b[0], &b[1]);
        uint64_t hit = ~0ull;
        for (int k = 0; k < 2 * JB_BUCKET && hit == ~0ull; k++) {
            const uint64_t sl = (uint64_t)JB_BUCKET * b[k / JB_BUCKET] + (k % JB_BUCKET);
            if (jb_node_is(img.nodes[sl], id, runes[i])) hit = sl;
        }
        if (hit == ~0ull) return Lookup{};
        const uint64_t nd = img.nodes[hit];
        id = img.nrows + (uint32_t)hit;
        fc = jb_node_fc(nd);
        wi = jb_node_widx(nd);
    }
    out.found = true;
    out.fc = fc;
    out.widx = wi;
    out.id = id;
    return out;
}

}  // namespace jb
