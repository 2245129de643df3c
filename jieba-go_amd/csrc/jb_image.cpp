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
#include <chrono>
#include <cstdio>
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
// prefix_dictionary.gob: encoding/gob stream of one map[string]int
// (newJiebaPrefixDictionary, tokenizer.go:439-458: decoder.Decode(&pd.termFreq)).
// Restated from the encoding/gob wire format of Go 1.18 (go.mod:3):
//   message  = uint(byte count) int(type id) payload
//   id < 0   : definition of type -id, payload = wireType struct
//   id > 0   : a value of type id; a non-struct value is preceded by the
//              singleton field delta, which is 0
//   uint     : < 0x80 one byte; else byte (256 - n) then n big-endian bytes
//   int      : uint u; u & 1 ? ^(u >> 1) : u >> 1
//   struct   : (uint field delta, field)* then delta 0
//   wireType : field 3 (MapT) = mapType{CommonType{Name, Id}, Key, Elem}
//   map      : uint count, then count x (key, elem)
//   string   : uint byte length, bytes (not checked as UTF-8)
// Predefined type ids: int = 2, string = 6.
// ---------------------------------------------------------------------------
namespace {
struct GobReader {
    const uint8_t* p;
    size_t n, i = 0;
    bool uint_(uint64_t* v) {
        if (i >= n) return false;
        const uint8_t b = p[i++];
        if (b < 0x80) { *v = b; return true; }
        const unsigned k = 256u - b;  // byte count
        if (k > 8 || n - i < k) return false;
        uint64_t x = 0;
        for (unsigned j = 0; j < k; j++) x = (x << 8) | p[i++];
        *v = x;
        return true;
    }
    bool int_(int64_t* v) {
        uint64_t u;
        if (!uint_(&u)) return false;
        *v = (u & 1) ? (int64_t)~(u >> 1) : (int64_t)(u >> 1);
        return true;
    }
};

constexpr int64_t kGobInt = 2, kGobString = 6;

// Skip a CommonType struct {Name string; Id typeId}; returns the Id.
bool gob_common_type(GobReader& r, int64_t* id) {
    int field = -1;
    for (;;) {
        uint64_t d;
        if (!r.uint_(&d)) return false;
        if (d == 0) return true;
        field += (int)d;
        if (field == 0) {  // Name
            uint64_t l;
            if (!r.uint_(&l) || r.n - r.i < l) return false;
            r.i += (size_t)l;
        } else if (field == 1) {  // Id
            if (!r.int_(id)) return false;
        } else {
            return false;
        }
    }
}
}  // namespace

int parse_gob_dictionary(const char* buf, size_t len, Dictionary* out, std::string* err) {
    out->term_freq.clear();
    out->size = 0;
    GobReader r{(const uint8_t*)buf, len};
    std::unordered_map<int64_t, std::pair<int64_t, int64_t>> maps;  // id -> (key, elem)
    for (;;) {
        uint64_t mlen;
        if (!r.uint_(&mlen) || mlen == 0 || r.n - r.i < mlen) {
            *err = r.i >= r.n ? "gob: no map value in stream (EOF)" : "gob: truncated message";
            return JB_EPARSE;
        }
        GobReader m{r.p + r.i, (size_t)mlen};
        r.i += (size_t)mlen;
        int64_t id;
        if (!m.int_(&id)) { *err = "gob: bad type id"; return JB_EPARSE; }
        if (id < 0) {
            // wireType: only MapT (field 3) can describe map[string]int
            uint64_t d;
            if (!m.uint_(&d) || d != 4) { *err = "gob: type definition is not a map (expected map[string]int)"; return JB_EPARSE; }
            int field = -1;
            int64_t tid = 0, key = 0, elem = 0;
            for (;;) {
                if (!m.uint_(&d)) { *err = "gob: truncated mapType"; return JB_EPARSE; }
                if (d == 0) break;
                field += (int)d;
                bool ok = false;
                if (field == 0) ok = gob_common_type(m, &tid);
                else if (field == 1) ok = m.int_(&key);
                else if (field == 2) ok = m.int_(&elem);
                if (!ok) { *err = "gob: bad mapType"; return JB_EPARSE; }
            }
            if (!m.uint_(&d) || d != 0) { *err = "gob: bad wireType end"; return JB_EPARSE; }
            if (tid != -id) { *err = "gob: type id mismatch in definition"; return JB_EPARSE; }
            maps[tid] = {key, elem};
            continue;
        }
        auto it = maps.find(id);
        if (it == maps.end() || it->second.first != kGobString || it->second.second != kGobInt) {
            *err = "gob: value is not a map[string]int (type " + std::to_string(id) + ")";
            return JB_EPARSE;
        }
        uint64_t d, cnt;
        if (!m.uint_(&d) || d != 0) { *err = "gob: corrupted data: non-zero delta for singleton"; return JB_EPARSE; }
        if (!m.uint_(&cnt) || cnt > m.n) { *err = "gob: bad map length"; return JB_EPARSE; }
        out->term_freq.reserve((size_t)cnt);
        for (uint64_t k = 0; k < cnt; k++) {
            uint64_t l;
            int64_t v;
            if (!m.uint_(&l) || m.n - m.i < l) { *err = "gob: truncated map key"; return JB_EPARSE; }
            std::string key((const char*)m.p + m.i, (size_t)l);
            m.i += (size_t)l;
            if (!m.int_(&v)) { *err = "gob: truncated map value"; return JB_EPARSE; }
            out->term_freq[std::move(key)] = v;  // reflect.Value.SetMapIndex: a repeated key overwrites
        }
        return JB_OK;  // Decode reads exactly one value; later messages are not read
    }
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
static uint32_t freq_class(int64_t f) { return f > 0 ? JB_FC_POS : (f == 0 ? JB_FC_ZERO : JB_FC_NEG); }

double dict_log(const Dictionary& d, int64_t x) {
    if (!d.log_of.empty()) {
        auto it = d.log_of.find(x);
        if (it != d.log_of.end()) return it->second;
    }
    return go_log((double)x);
}

std::vector<int64_t> weight_log_keys(const Dictionary& d) {
    std::vector<int64_t> out{1, d.size};
    std::vector<uint32_t> runes;
    for (const auto& kv : d.term_freq) {  // the keys build_image keeps
        if (!valid_runes(kv.first, &runes) || runes.empty()) continue;
        bool han = true;
        for (uint32_t r : runes) han = han && jb_is_han(r);
        if (han) out.push_back(kv.second);
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

int build_image(const Dictionary& d, const Emission& e, Image* img, std::string* err) {
    img->size = d.size;
    img->total = dict_log(d, d.size);         // calcDagProba: total := math.Log(float64(pd.size))
    img->w_absent = dict_log(d, 1) - img->total;  // tf := 1.0 when the piece is absent (tokenizer.go:515)

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
    // the weights in order of the summed frequency of the keys that use them (a key's
    // frequency is how often the reference's corpus saw it, so this is the order in
    // which text looks them up, so the hot weights share a few cache lines; ties by key
    // count, then value bits).  k_mark_walk packs 14-bit indices.
    img->wtab.assign(1, img->w_absent);
    std::unordered_map<uint64_t, uint32_t> widx_of;
    auto wbits = [&](int64_t f) -> uint64_t {
        const double w = dict_log(d, f) - img->total;
        uint64_t bits;
        memcpy(&bits, &w, 8);
        return bits;
    };
    {
        struct Use { uint64_t bits; double mass; uint64_t keys; };
        std::unordered_map<uint64_t, size_t> at;
        std::vector<Use> uses;
        for (const Key& k : keys) {
            const uint64_t b = wbits(k.f);
            auto it = at.find(b);
            if (it == at.end()) {
                at.emplace(b, uses.size());
                uses.push_back(Use{b, 0.0, 0});
                it = at.find(b);
            }
            Use& u = uses[it->second];
            u.mass += k.f > 0 ? (double)k.f : 0.0;
            u.keys++;
        }
        std::sort(uses.begin(), uses.end(), [](const Use& a, const Use& b) {
            if (a.mass != b.mass) return a.mass > b.mass;
            return a.keys != b.keys ? a.keys > b.keys : a.bits < b.bits;
        });
        for (const Use& u : uses) {
            double w;
            memcpy(&w, &u.bits, 8);
            widx_of.emplace(u.bits, (uint32_t)img->wtab.size());
            img->wtab.push_back(w);
        }
    }
    auto widx = [&](int64_t f) -> uint32_t { return widx_of.at(wbits(f)); };

    // ---- the trie as a double array over rune codes ----------------------------------
    // Codes are dense, in order of how often a rune occurs in the keys, so a
    // node's children sit close together.  Level-1 nodes are the cells at their
    // codes.  Every node with children then gets the first base at which base +
    // code(child) is free for all of them (a node's cell index is its id, which
    // its children's check holds), in order of access mass: the node's own
    // frequency plus its descendants', i.e. how often text walks through it.  The
    // hot nodes' child blocks, and the cells their walks probe, pack at the
    // front of the array, so the part of the 10.8 MB array that walks touch most
    // fits one XCD's 4 MB L2 better (modelled with tools/trie_sim.cpp: 90 % of
    // probes in 2.5 MB of lines instead of 2.9; k_mark_walk 3.87 -> 3.81 ms).
    // Parents come before their children (a child's mass is part of its parent's).
    {
        std::unordered_map<uint32_t, uint64_t> occ;
        for (const Key& k : keys)
            for (uint32_t r : k.r) occ[r]++;
        std::vector<std::pair<uint32_t, uint64_t>> ord(occ.begin(), occ.end());
        std::sort(ord.begin(), ord.end(), [](const auto& a, const auto& b) {
            return a.second != b.second ? a.second > b.second : a.first < b.first;
        });
        img->code.assign(img->nrows, 0u);
        for (size_t i = 0; i < ord.size(); i++) img->code[jb_row(pm, ord[i].first)] = (uint32_t)i + 1u;
        img->ncodes = (uint32_t)ord.size() + 1u;
        if (img->ncodes >= (1u << 17)) {  // k_mark_walk keeps 17-bit codes
            *err = "more than 131071 distinct runes in the dictionary keys";
            return JB_ELIMIT;
        }
    }
    auto code_of = [&](uint32_t r) { return img->code[jb_row(pm, r)]; };
    std::vector<uint64_t>& cells = img->cells;
    std::vector<uint64_t> used;  // bitmap of occupied cells (cell 0: the absent rune, never a node)
    auto is_used = [&](uint64_t i) { return i < used.size() * 64 && ((used[i >> 6] >> (i & 63)) & 1ull); };
    auto set_used = [&](uint64_t i) {
        if (i >= used.size() * 64) used.resize(i / 64 + 4096, 0ull);
        used[i >> 6] |= 1ull << (i & 63);
        if (i >= cells.size()) cells.resize(i + 4096, 0ull);
    };
    cells.assign(img->ncodes, 0ull);
    used.assign(img->ncodes / 64 + 4096, 0ull);
    set_used(0);
    img->maxlen = 0;
    img->nnodes = 0;
    std::unordered_map<std::string, uint32_t> id_of;  // key (runes) -> cell id
    auto rkey = [](const std::vector<uint32_t>& r, size_t n) {
        return std::string(reinterpret_cast<const char*>(r.data()), n * sizeof(uint32_t));
    };
    for (size_t i = 0; i < keys.size(); i++) {  // level 1: the cells at the codes
        const Key& k = keys[i];
        if (k.r.size() != 1) continue;
        const uint32_t wi = widx(k.f);
        if (wi >= JB_MAX_WIDX) {
            *err = "more than " + std::to_string(JB_MAX_WIDX) + " distinct frequencies";
            return JB_ELIMIT;
        }
        const uint32_t c = code_of(k.r[0]);
        cells[c] = jb_cell_make(JB_CHECK_ROOT, 0, freq_class(k.f), 0, wi);
        set_used(c);
        id_of.emplace(rkey(k.r, 1), c);
        img->nnodes++;
        img->maxlen = 1;
    }
    uint64_t first_free = 1;
    uint64_t probes = 0;
    // search start per child count: the base found last for that count (a node with
    // k children rarely fits below where the previous k-child node fitted)
    std::vector<uint64_t> start_k(65, 1);
    const auto tp0 = std::chrono::steady_clock::now();
    {
        // nodes with children in order of access mass (own + descendants' frequencies), parents first
        std::unordered_map<std::string, double> mass;
        for (const Key& k : keys)
            for (size_t n = 1; n <= k.r.size(); n++) mass[rkey(k.r, n)] += (double)std::max<int64_t>(k.f, 0) + 1e-9;
        std::unordered_map<std::string, std::vector<uint32_t>> kids;  // parent key -> child key indices
        for (size_t i = 0; i < keys.size(); i++)
            if (keys[i].r.size() >= 2) kids[rkey(keys[i].r, keys[i].r.size() - 1)].push_back((uint32_t)i);
        struct P { double m; uint32_t depth; std::string key; };
        std::vector<P> order;
        for (auto& kv : kids) order.push_back(P{mass[kv.first], (uint32_t)(kv.first.size() / 4), kv.first});
        std::sort(order.begin(), order.end(), [](const P& a, const P& b) {
            if (a.m != b.m) return a.m > b.m;
            if (a.depth != b.depth) return a.depth < b.depth;
            return a.key < b.key;
        });
        std::vector<uint32_t> cs, srt;
        for (size_t oi = 0; oi < order.size(); oi++) {
            auto pit = id_of.find(order[oi].key);
            if (pit == id_of.end()) continue;  // unreachable parent
            const uint32_t parent = pit->second;
            const auto& ch = kids[order[oi].key];
            const size_t n = order[oi].depth + 1;
            cs.clear();
            for (uint32_t ki : ch) cs.push_back(code_of(keys[ki].r[n - 1]));
            srt = cs;
            std::sort(srt.begin(), srt.end());
            while (is_used(first_free)) first_free++;
            const size_t kc = std::min<size_t>(srt.size(), 64);
            uint64_t f = std::max<uint64_t>(std::max<uint64_t>(first_free, start_k[kc]), (uint64_t)srt[0] + 1);
            uint64_t base = 0;
            for (;; f++) {
                if (is_used(f)) continue;
                probes++;
                base = f - srt[0];
                bool ok = true;
                for (size_t j = 1; j < srt.size() && ok; j++) ok = !is_used(base + srt[j]);
                if (ok) break;
            }
            start_k[kc] = f;
            if (base + srt.back() >= JB_MAX_CELLS) {
                *err = "dictionary too large for the double-array trie";
                return JB_ELIMIT;
            }
            cells[parent] |= jb_cell_make(0, (uint32_t)base, 0, 1, 0);
            for (size_t j = 0; j < ch.size(); j++) {
                const Key& k = keys[ch[j]];
                const uint32_t wi = widx(k.f);
                if (wi >= JB_MAX_WIDX) {
                    *err = "more than " + std::to_string(JB_MAX_WIDX) + " distinct frequencies";
                    return JB_ELIMIT;
                }
                const uint64_t c = base + cs[j];
                set_used(c);
                cells[c] = jb_cell_make(parent + 1u, 0, freq_class(k.f), 0, wi);
                id_of.emplace(rkey(k.r, n), (uint32_t)c);
                img->nnodes++;
                img->maxlen = std::max<uint32_t>(img->maxlen, (uint32_t)n);
            }
        }
    }
    if (getenv("JB_DEBUG_BUILD"))
        fprintf(stderr, "[jb] trie placement %.3f s, %llu candidate bases\n",
                std::chrono::duration<double>(std::chrono::steady_clock::now() - tp0).count(),
                (unsigned long long)probes);
    // room for base + code of any rune under any node: probes never leave the array
    uint64_t top = cells.size();
    while (top > img->ncodes && cells[top - 1] == 0ull) top--;
    cells.resize(top + img->ncodes + 1, 0ull);
    img->ncells = (uint32_t)cells.size();
    img->emit.assign((size_t)img->npages * 256 * 4, JB_MIN_FLOAT);  // not found -> minFloat (tokenizer.go:690,710)
    for (int s = 0; s < 4; s++)
        for (const auto& kv : e.by_rune[s]) {
            if (kv.first >= 0x110000u) continue;
            img->emit[(size_t)jb_row(pm, kv.first) * 4 + s] = kv.second;
        }
    return JB_OK;
}

bool reweigh_image(const Dictionary& d, Image* img) {
    // weight index -> the frequency whose weight it holds (from the cells the keys reach)
    std::vector<int64_t> freq_of(img->wtab.size(), 0);
    std::vector<uint8_t> seen(img->wtab.size(), 0);
    std::vector<uint32_t> runes;
    const double total = dict_log(d, d.size);
    auto weight = [&](int64_t f) { return dict_log(d, f) - total; };
    for (const auto& kv : d.term_freq) {
        if (!valid_runes(kv.first, &runes) || runes.empty()) continue;
        bool han = true;
        for (uint32_t r : runes) han = han && jb_is_han(r);
        if (!han) continue;
        const Lookup lk = image_lookup(*img, runes.data(), runes.size());
        if (!lk.found) continue;  // unreachable (a txt-semantics key without its prefixes): no cell
        if (lk.widx >= freq_of.size()) return false;  // not the image of these keys
        if (!seen[lk.widx]) {
            seen[lk.widx] = 1;
            freq_of[lk.widx] = kv.second;
        } else if (freq_of[lk.widx] != kv.second) {
            const double a = weight(freq_of[lk.widx]), b = weight(kv.second);
            if (memcmp(&a, &b, 8) != 0) return false;  // one index, two weights now
        }
    }
    img->size = d.size;
    img->total = total;
    img->w_absent = dict_log(d, 1) - total;  // tf := 1.0 when the piece is absent (tokenizer.go:515)
    img->wtab[0] = img->w_absent;
    for (size_t i = 1; i < img->wtab.size(); i++)
        if (seen[i]) img->wtab[i] = weight(freq_of[i]);
    return true;
}

Lookup image_lookup(const Image& img, const uint32_t* runes, size_t n) {
    Lookup out;
    if (n == 0 || runes[0] >= 0x110000u) return out;
    const uint16_t* pm = img.pagemap.data();
    uint32_t id = img.code[jb_row(pm, runes[0])];
    uint64_t c = img.cells[id];
    if (jb_cell_check(c) != JB_CHECK_ROOT) return out;
    for (size_t i = 1; i < n; i++) {
        if (runes[i] >= 0x110000u || !jb_cell_hc(c)) return Lookup{};
        const uint64_t t = (uint64_t)jb_cell_base(c) + img.code[jb_row(pm, runes[i])];
        if (t >= img.cells.size() || jb_cell_check(img.cells[t]) != id + 1u) return Lookup{};
        id = (uint32_t)t;
        c = img.cells[t];
    }
    out.found = true;
    out.fc = jb_cell_fc(c);
    out.widx = jb_cell_widx(c);
    out.id = id;
    return out;
}

}  // namespace jb

namespace jb {

// ---------------------------------------------------------------------------
// Serialized image (a fast-start cache, the role prefix_dictionary.gob plays
// for the reference's map, tokenizer.go:439-458): the host dictionary and
// emission maps that AddWord and suggestFreq need, plus the built device
// arrays, so that opening skips parsing and build_image.  Little-endian,
// versioned, checksummed; written and read only by this library.
// ---------------------------------------------------------------------------
namespace {
constexpr char kImgMagic[8] = {'J', 'B', 'I', 'M', 'A', 'G', 'E', '\0'};
constexpr uint32_t kImgVersion = 1;

uint64_t img_hash(const uint8_t* p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
    }
    for (; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h ^ (h >> 29);
}

struct Out {
    std::string* s;
    template <class T> void pod(const T& v) { s->append((const char*)&v, sizeof v); }
    template <class T> void vec(const std::vector<T>& v) {
        pod((uint64_t)v.size());
        s->append((const char*)v.data(), v.size() * sizeof(T));
    }
};

struct In {
    const uint8_t* p;
    size_t n, i = 0;
    template <class T> bool pod(T* v) {
        if (n - i < sizeof(T)) return false;
        memcpy(v, p + i, sizeof(T));
        i += sizeof(T);
        return true;
    }
    template <class T> bool vec(std::vector<T>* v, uint64_t max) {
        uint64_t c;
        if (!pod(&c) || c > max || (n - i) / sizeof(T) < c) return false;
        v->resize((size_t)c);
        memcpy(v->data(), p + i, (size_t)c * sizeof(T));
        i += (size_t)c * sizeof(T);
        return true;
    }
};
}  // namespace

void save_image(const Dictionary& d, const Emission& e, const Image& img, std::string* out) {
    std::string body;
    Out o{&body};
    o.pod(d.size);
    o.pod((uint64_t)d.term_freq.size());
    for (const auto& kv : d.term_freq) {
        o.pod((uint32_t)kv.first.size());
        body.append(kv.first);
        o.pod(kv.second);
    }
    for (int s = 0; s < 4; s++) {
        o.pod((uint64_t)e.by_rune[s].size());
        for (const auto& kv : e.by_rune[s]) {
            o.pod(kv.first);
            o.pod(kv.second);
        }
    }
    o.vec(img.pagemap);
    o.vec(img.emit);
    o.vec(img.code);
    o.vec(img.cells);
    o.vec(img.wtab);
    o.pod(img.npages); o.pod(img.nrows); o.pod(img.ncells); o.pod(img.ncodes); o.pod(img.maxlen);
    o.pod(img.nnodes); o.pod(img.total); o.pod(img.w_absent); o.pod(img.size);
    out->clear();
    out->append(kImgMagic, 8);
    Out h{out};
    h.pod(kImgVersion);
    h.pod((uint32_t)0);
    h.pod((uint64_t)body.size());
    h.pod(img_hash((const uint8_t*)body.data(), body.size()));
    out->append(body);
}

int load_image(const char* buf, size_t len, Dictionary* d, Emission* e, Image* img, std::string* err) {
    In h{(const uint8_t*)buf, len};
    uint32_t ver = 0, pad = 0;
    uint64_t blen = 0, hash = 0;
    if (len < 8 || memcmp(buf, kImgMagic, 8) != 0) { *err = "not a jiebahip image (bad magic)"; return JB_EPARSE; }
    h.i = 8;
    if (!h.pod(&ver) || !h.pod(&pad) || !h.pod(&blen) || !h.pod(&hash)) { *err = "image: truncated header"; return JB_EPARSE; }
    if (ver != kImgVersion) { *err = "image: version " + std::to_string(ver) + " (this library reads " +
                              std::to_string(kImgVersion) + "); rebuild it"; return JB_EPARSE; }
    if (len - h.i != blen) { *err = "image: truncated body"; return JB_EPARSE; }
    const uint8_t* body = h.p + h.i;
    if (img_hash(body, (size_t)blen) != hash) { *err = "image: checksum mismatch"; return JB_EPARSE; }
    In b{body, (size_t)blen};
    const char* bad = "image: corrupt body";
    uint64_t n;
    if (!b.pod(&d->size) || !b.pod(&n) || n > blen) { *err = bad; return JB_EPARSE; }
    d->term_freq.clear();
    d->term_freq.reserve((size_t)n);
    for (uint64_t k = 0; k < n; k++) {
        uint32_t l;
        int64_t f;
        if (!b.pod(&l) || b.n - b.i < l) { *err = bad; return JB_EPARSE; }
        std::string key((const char*)b.p + b.i, l);
        b.i += l;
        if (!b.pod(&f)) { *err = bad; return JB_EPARSE; }
        d->term_freq.emplace(std::move(key), f);
    }
    for (int s = 0; s < 4; s++) {
        e->by_rune[s].clear();
        if (!b.pod(&n) || n > blen) { *err = bad; return JB_EPARSE; }
        for (uint64_t k = 0; k < n; k++) {
            uint32_t r;
            double v;
            if (!b.pod(&r) || !b.pod(&v)) { *err = bad; return JB_EPARSE; }
            e->by_rune[s][r] = v;
        }
    }
    if (!b.vec(&img->pagemap, JB_NPAGES_MAX) || !b.vec(&img->emit, blen) || !b.vec(&img->code, blen) ||
        !b.vec(&img->cells, blen) || !b.vec(&img->wtab, blen) || !b.pod(&img->npages) || !b.pod(&img->nrows) ||
        !b.pod(&img->ncells) || !b.pod(&img->ncodes) || !b.pod(&img->maxlen) || !b.pod(&img->nnodes) ||
        !b.pod(&img->total) || !b.pod(&img->w_absent) || !b.pod(&img->size) || b.i != b.n) {
        *err = bad;
        return JB_EPARSE;
    }
    // the arrays must be the sizes the kernels index
    if (img->pagemap.size() != JB_NPAGES_MAX || img->code.size() != (size_t)img->npages * 256 ||
        img->emit.size() != (size_t)img->npages * 256 * 4 || img->cells.size() != img->ncells ||
        img->nrows != img->npages * 256 || img->wtab.empty() || img->wtab.size() > JB_MAX_WIDX) {
        *err = "image: inconsistent array sizes";
        return JB_EPARSE;
    }
    return JB_OK;
}

}  // namespace jb

namespace jb {
void build_hot_rows(const Image& img, uint64_t* vals, uint16_t* tags) {
    for (uint32_t k = 0; k < JB_HOT_SLOTS; k++) {
        vals[k] = 0;
        tags[k] = 0;
    }
    const size_t nc = img.cells.size();
    if (!nc) return;
    // summed frequency per code: every key (a cell with a positive count) adds its
    // frequency, exp(weight) up to the common factor size, to each rune on its path
    std::vector<double> score(img.ncodes + 1u, 0.0);
    for (size_t t = 0; t < nc; t++) {
        const uint64_t c = img.cells[t];
        const uint32_t ck = jb_cell_check(c);
        if (ck == 0u || jb_cell_fc(c) != JB_FC_POS) continue;
        const uint32_t wi = jb_cell_widx(c);
        if (wi >= img.wtab.size()) continue;
        const double f = exp(img.wtab[wi]);
        uint64_t node = t;
        for (uint32_t depth = 0; depth < 4096u; depth++) {  // (bounded: a walk up the trie)
            const uint32_t k = jb_cell_check(img.cells[node]);
            if (k == JB_CHECK_ROOT) {
                if (node < score.size()) score[node] += f;
                break;
            }
            if (k == 0u || k - 1u >= nc) break;
            const uint64_t parent = k - 1u;
            const uint64_t code = node - jb_cell_base(img.cells[parent]);
            if (code < score.size()) score[code] += f;
            node = parent;
        }
    }
    std::vector<std::pair<double, uint32_t>> rows;  // (score, row) of the direct rows
    for (uint32_t r = JB_DIRECT_LO; r < JB_DIRECT_LO + JB_DIRECT_N; r++) {
        const uint32_t row = r - 0x3300u;
        if (row >= img.code.size()) continue;
        const uint32_t cd = img.code[row];
        if (cd == 0u || cd >= score.size() || !(score[cd] > 0.0)) continue;
        rows.push_back({score[cd], row});
    }
    std::sort(rows.begin(), rows.end(), [](const auto& a, const auto& b) {
        return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    for (const auto& sr : rows) {
        const uint32_t r = sr.second + 0x3300u, slot = jb_hot_slot(r);
        if (tags[slot]) continue;
        const uint32_t cd = img.code[sr.second];
        tags[slot] = (uint16_t)r;
        vals[slot] = jb_l1row_make(cd, cd < nc ? img.cells[cd] : 0ull);
    }
}
}  // namespace jb
