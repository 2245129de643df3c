// jb_capi.cpp — the C ABI of libjiebahip.so (include/jiebahip.h).
//
// Host orchestration only: load the model files, build and upload the device
// image, size per-device workspaces, shard batches over devices, run the
// kernel pipeline (jb_kernels.hip) and hand spans back.  No segmentation
// happens on the CPU: without a usable HIP device every cut returns
// JB_EDEVICE.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <vector>

#include "../../include/jiebahip.h"
#include "jb_image.h"
#include "jb_kernels.h"

using namespace jb;

static thread_local std::string g_err = "";

static int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t _e = (x);                                                                   \
        if (_e != hipSuccess) return fail(JB_EDEVICE, "%s: %s", #x, hipGetErrorString(_e));   \
    } while (0)

struct jb_image {
    Dictionary dict;
    Emission emit;
    Image img;
    int dict_kind = 0;
};

namespace {

// Per-launch HIP events, recorded on the launch stream.
struct EventTimer final : KernelTimer {
    struct Rec { int id; hipEvent_t a, b; };
    std::vector<hipEvent_t> pool;
    std::vector<Rec> recs;
    size_t used = 0;
    hipEvent_t cur_a = nullptr;
    double ms[K_NUM] = {0};
    uint64_t launches[K_NUM] = {0};
    hipEvent_t take() {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
    void begin(int, hipStream_t s) override {
        cur_a = take();
        if (cur_a) (void)hipEventRecord(cur_a, s);
    }
    void end(int id, hipStream_t s) override {
        hipEvent_t b = take();
        if (b && cur_a) {
            (void)hipEventRecord(b, s);
            recs.push_back(Rec{id, cur_a, b});
        }
    }
    void harvest() {
        for (const Rec& r : recs) {
            (void)hipEventSynchronize(r.b);
            float t = 0;
            if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
                ms[r.id] += t;
                launches[r.id]++;
            }
        }
        recs.clear();
        used = 0;
    }
    void reset() {
        harvest();
        for (int k = 0; k < K_NUM; k++) { ms[k] = 0; launches[k] = 0; }
    }
    ~EventTimer() override {
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    }
};

// One device's copy of the image (jb_common.h layout).
struct ImageBufs {
    uint16_t* pagemap = nullptr;
    double* emit = nullptr;
    uint64_t* cells = nullptr;
    uint32_t* code = nullptr;
    double* wtab = nullptr;
    uint64_t* l1row = nullptr;
    uint64_t* hot = nullptr;  // hot level-1 rows: JB_HOT_SLOTS u64 values, then u16 tags
};

struct SmallReq;  // (cut_small)

struct Device {
    int ordinal = 0;
    std::mutex mu;  // one pipeline at a time per device workspace
    hipStream_t stream = nullptr;
    ImageBufs ib{};  // the device image
    DevImage dim{};
    // workspace
    Work w{};
    uint8_t* text = nullptr;   // staging for host batches (padded)
    uint64_t* doc_off = nullptr;
    uint64_t text_cap = 0;
    uint64_t doc_cap = 0;
    // pinned host staging for host batches (full-speed DMA both ways)
    uint8_t* h_text = nullptr;
    uint64_t h_text_cap = 0;
    uint64_t* h_misc = nullptr;  // piece-relative doc offsets (u64)
    uint64_t h_misc_cap = 0;
    // host-batch pipeline (cut_pieces): a batch is cut in pieces of whole documents;
    // piece k+1's text goes up on cstream while piece k runs on `stream` and the
    // spans / masks of earlier pieces come back on dstream
    hipStream_t cstream = nullptr, dstream = nullptr;
    std::vector<hipEvent_t> ev_h2d, ev_comp, ev_d2h;  // per piece
    static constexpr int kSets = 3;  // output sets in flight
    struct OutSet {
        uint32_t* ts = nullptr;  // device u32 spans and doc_tok of the piece
        uint32_t* te = nullptr;
        uint64_t* dt = nullptr;
        uint64_t cap_tok = 0;
        uint32_t cap_docs = 0;
        uint32_t* hs = nullptr;  // pinned: starts then ends
        uint64_t* hdt = nullptr; // pinned doc_tok
        uint64_t hcap_tok = 0;
        uint32_t hcap_docs = 0;
        // packed spans (span_pack): device u32 per token + block headers, side list; pinned copies
        uint16_t* pk = nullptr;
        uint32_t* phdr = nullptr;
        uint4* pside = nullptr;
        uint64_t cap_pk = 0, cap_phdr = 0, cap_pside = 0;
        uint16_t* hpk = nullptr;  // pinned copies
        uint32_t* hhdr = nullptr;
        uint4* hside = nullptr;
        uint64_t hcap_pk = 0, hcap_hdr = 0, hcap_side = 0;
    } outs[kSets];
    bool span_pack = true;  // host batches' spans come back packed, 2 B per token (JB_SPAN_PACK, default 1)
    uint32_t* h_pcnt = nullptr;  // mapped pinned: kSnapWords u32 per piece (k_snap writes them)
    uint32_t* d_pcnt = nullptr;  // its device address
    uint64_t h_pcnt_cap = 0;
    uint64_t* d_mask = nullptr;  // boundary masks of a range: starts then ends (u64 words)
    uint64_t* h_mask = nullptr;  // pinned copy
    uint64_t mask_cap = 0;       // u64 words of d_mask
    uint64_t mask_cap_h = 0;     // u64 words of h_mask
    uint8_t* h_zero = nullptr;   // 64 pinned zero bytes
    jb_stats acc{};              // counters summed over the pieces of the last host range
    bool acc_valid = false;      // the last run was such a range
    // k_small's pinned, mapped host buffers (coherent: the kernel reads and writes them directly)
    // per in-flight k_small batch (cut_small keeps up to kSmallSlots launched at once)
    struct SmallSlot {
        uint8_t* h_sin = nullptr;    // text (kSmallBytes + 128), then u64 doc offsets (kSmallDocs + 1)
        // header, spans, doc_tok (kSmallOutBytes), two of them: batches alternate, so the
        // slot's next batch runs while the callers of the last one get their spans
        uint32_t* h_sout[2] = {nullptr, nullptr};
        uint8_t* d_sin = nullptr;    // their device addresses
        uint32_t* d_sout[2] = {nullptr, nullptr};
        uint32_t ob = 0;             // the output buffer of the slot's current batch
        std::atomic<bool> reading[2] = {false, false};  // spans still being split out of h_sout[i]
        uint32_t seq = 0;            // the kernel writes this number last
        bool busy = false;
        hipStream_t st = nullptr;    // this slot's stream, masked to its own CU
    } slots[8];
    // jb_last_stats' view of the last batch: last_small, small_hdr and has_stats, under
    // stats_mu alone (a finished k_small batch publishes them without waiting for d->mu,
    // which a host-batch pipeline holds for its whole run; lock order: mu, then stats_mu)
    std::mutex stats_mu;
    bool last_small = false;     // the last batch took k_small (jb_last_stats reads small_hdr)
    // concurrent small calls, coalesced into shared k_small launches (cut_small)
    std::mutex small_mu;
    std::condition_variable small_cv;
    std::deque<SmallReq*> small_q;
    uint32_t small_sleepers = 0;         // callers asleep on small_cv (under small_mu)
    // JB_SMALL_TRACE=path (diagnostics): per batch its slot, calls, and the clocks (us) of
    // staging, launch return, completion word and split, written to path at jb_close
    std::vector<std::array<double, 6>> small_trace;
    uint32_t small_slots = 4;            // k_small batches in flight at most (JB_SMALL_SLOTS, 1..8)
    uint32_t small_hdr[kSmallHdr] = {0};
    uint32_t ncu = 0;
    uint64_t piece_bytes = 64ull << 20;  // host-batch pipeline piece (JB_PIECE_KIB)
    LaunchCfg lc{};  // launch shape, fixed at jb_open
    uint64_t last_nbytes = 0;  // batch size of the last pipeline run (jb_last_stats)
    bool has_stats = false;    // this device took part in the last cut (jb_last_stats skips it otherwise)
    // The workspace is shared by every stream a caller queues on (jb_cut_device): each
    // pipeline is recorded here, and a pipeline on another stream waits for it first.
    hipEvent_t ws_done = nullptr;
    hipStream_t ws_stream = nullptr;
    EventTimer timer;
    bool profile = false;
    // replay cache: the whole pipeline captured as one HIP graph for the last
    // (buffers, sizes, grids) it ran with; any change re-captures
    struct GraphKey {
        const void* text; uint64_t nbytes; const void* doc_off; uint32_t ndocs; bool hmm;
        uint64_t work_gen; hipStream_t stream; const void* out_s; const void* out_e; const void* out_d;
        bool operator==(const GraphKey& o) const {
            return text == o.text && nbytes == o.nbytes && doc_off == o.doc_off && ndocs == o.ndocs &&
                   hmm == o.hmm && work_gen == o.work_gen && stream == o.stream && out_s == o.out_s &&
                   out_e == o.out_e && out_d == o.out_d;
        }
    } gkey{};
    hipGraphExec_t gexec = nullptr;  // captured for gkey (null until the key repeats)
    uint64_t work_gen = 0;           // bumped whenever the workspace is reallocated
    // The workspace's document bitmap may hold set bits: a new workspace, or a pipeline
    // launch that failed part way.  Pipelines leave it all zeros (k_docbits, k_nonzh).
    bool docbits_dirty = true;
    uint64_t gkey_gen = 0;
};

void dfree(void* p) {
    if (p) (void)hipFree(p);
}
void hfree(void* p) {
    if (p) (void)hipHostFree(p);
}

// memcpy whose destination lines are written without being read first (non-temporal
// 16-byte stores; plain stores read every destination line before writing it): staging
// a batch into pinned memory, which the copy engine then reads.  Fenced at the end.
static void nt_copy(void* dst, const void* src, size_t n) {
    typedef long long v2i __attribute__((vector_size(16)));
    char* d = static_cast<char*>(dst);
    const char* s = static_cast<const char*>(src);
    const size_t head = std::min(n, (size_t)((16u - ((uintptr_t)d & 15u)) & 15u));
    memcpy(d, s, head);
    d += head;
    s += head;
    n -= head;
    for (; n >= 64; n -= 64, d += 64, s += 64) {
        v2i a, b, c, e;
        memcpy(&a, s, 16);
        memcpy(&b, s + 16, 16);
        memcpy(&c, s + 32, 16);
        memcpy(&e, s + 48, 16);
        __builtin_nontemporal_store(a, reinterpret_cast<v2i*>(d));
        __builtin_nontemporal_store(b, reinterpret_cast<v2i*>(d + 16));
        __builtin_nontemporal_store(c, reinterpret_cast<v2i*>(d + 32));
        __builtin_nontemporal_store(e, reinterpret_cast<v2i*>(d + 48));
    }
    memcpy(d, s, n);
    __builtin_ia32_sfence();
}

// memcpy with a few host threads for large copies (staging into pinned memory)
void par_copy(void* dst, const void* src, size_t n) {
    const size_t kMin = 8u << 20;
    const unsigned nt = (unsigned)std::min<size_t>(8, std::max<size_t>(1, n / kMin));
    if (nt <= 1) {
        memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + nt - 1) / nt;
    for (unsigned k = 0; k < nt; k++) {
        const size_t a = k * per, b = std::min(n, a + per);
        if (a < b) th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
    }
    for (auto& t : th) t.join();
}

// fn(0..n-1) on n threads (the caller's thread runs fn(0))
constexpr unsigned kCopyThreads = 8;
template <class F>
void run_threads(unsigned n, F& fn) {
    std::vector<std::thread> th;
    for (unsigned t = 1; t < n; t++) th.emplace_back([&fn, t] { fn(t); });
    fn(0);
    for (auto& x : th) x.join();
}

// out[k] = base + in[k] (u32 device spans -> u64 batch offsets), a few threads when large
void par_widen(uint64_t* out, const uint32_t* in, size_t n, uint64_t base) {
    const size_t kMin = 2u << 20;
    const unsigned nt = (unsigned)std::min<size_t>(8, std::max<size_t>(1, n / kMin));
    auto run = [=](size_t a, size_t b) {
        for (size_t k = a; k < b; k++) out[k] = base + in[k];
    };
    if (nt <= 1) {
        run(0, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + nt - 1) / nt;
    for (unsigned k = 0; k < nt; k++) {
        const size_t a = k * per, b = std::min(n, a + per);
        if (a < b) th.emplace_back(run, a, b);
    }
    for (auto& t : th) t.join();
}

// growable malloc'd span arrays (handed to the caller as jb_spans)
struct SpanBuf {
    uint64_t* s = nullptr;
    uint64_t* e = nullptr;
    // external u32 arrays instead (jb_cut_batch_into32): token k is s32[k] = start - b32
    uint32_t* s32 = nullptr;
    uint32_t* e32 = nullptr;
    uint64_t b32 = 0;
    size_t n = 0, cap = 0;
    bool external = false;          // caller-owned arrays of fixed capacity
    size_t needed = 0;              // tokens that did not fit an external buffer
    std::vector<uint64_t> per_doc;  // tokens per document
    bool reserve(size_t want) {
        if (want <= cap) return true;
        if (external) return false;
        const size_t nc = std::max(want, cap * 3 / 2 + 1024);
        uint64_t* ns = (uint64_t*)realloc(s, nc * 8);
        if (!ns) return false;
        s = ns;
        uint64_t* ne = (uint64_t*)realloc(e, nc * 8);
        if (!ne) return false;
        e = ne;
        cap = nc;
        return true;
    }
    void release() {
        if (!external) {
            free(s);
            free(e);
        }
        s = e = nullptr;
        n = cap = 0;
    }
};

}  // namespace

struct jb_ctx {
    std::unique_ptr<jb_image> im;
    std::vector<std::unique_ptr<Device>> devs;
    std::shared_mutex lock;  // prefixDictionary.lock: cuts share, AddWord excludes
};

// ---------------------------------------------------------------------------
// image
// ---------------------------------------------------------------------------
static int read_file(const char* path, std::string* out) {
    FILE* f = fopen(path, "rb");
    if (!f) return fail(JB_EIO, "open %s: %s", path, strerror(errno));
    std::string s;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    const bool err = ferror(f);
    fclose(f);
    if (err) return fail(JB_EIO, "read %s failed", path);
    *out = std::move(s);
    return JB_OK;
}

extern "C" int jb_image_build(const jb_config* cfg, jb_image** out) {
    if (!cfg || !out) return fail(JB_EINVAL, "jb_image_build: null argument");
    const int kind = cfg->dict_kind;
    if (kind != JB_DICT_TXT && kind != JB_DICT_PREFIX && kind != JB_DICT_GOB && kind != JB_DICT_IMAGE)
        return fail(JB_EINVAL, "unknown dict_kind %d", kind);
    std::string dbuf, ebuf;
    const char* d = cfg->dict_buf;
    size_t dl = cfg->dict_len;
    const char* e = cfg->emit_buf;
    size_t el = cfg->emit_len;
    int rc;
    if (cfg->dict_path) {
        if ((rc = read_file(cfg->dict_path, &dbuf))) return rc;
        d = dbuf.data();
        dl = dbuf.size();
    }
    if (!d && dl) return fail(JB_EINVAL, "no dictionary given");
    if (cfg->nlog && (!cfg->log_keys || !cfg->log_vals)) return fail(JB_EINVAL, "nlog > 0 without log_keys/log_vals");
    auto im = std::make_unique<jb_image>();
    im->dict_kind = kind;
    for (size_t i = 0; i < cfg->nlog; i++) im->dict.log_of[cfg->log_keys[i]] = cfg->log_vals[i];
    std::string err;
    if (kind == JB_DICT_IMAGE) {
        if ((rc = load_image(d ? d : "", dl, &im->dict, &im->emit, &im->img, &err))) return fail(rc, "%s", err.c_str());
        for (size_t i = 0; i < cfg->nlog; i++) im->dict.log_of[cfg->log_keys[i]] = cfg->log_vals[i];
        if ((cfg->size_override > 0 && cfg->size_override != im->dict.size) || cfg->nlog) {  // reweigh
            if (cfg->size_override > 0) im->dict.size = cfg->size_override;
            if (!reweigh_image(im->dict, &im->img) && (rc = build_image(im->dict, im->emit, &im->img, &err)))
                return fail(rc, "%s", err.c_str());
        }
        *out = im.release();
        return JB_OK;
    }
    if (cfg->emit_path) {
        if ((rc = read_file(cfg->emit_path, &ebuf))) return rc;
        e = ebuf.data();
        el = ebuf.size();
    }
    if (!e) return fail(JB_EINVAL, "no emission table given (prob_emit.json)");
    if (kind == JB_DICT_GOB) {
        // newJiebaPrefixDictionary (tokenizer.go:439-458): the gob map as stored, size hard-coded
        if ((rc = parse_gob_dictionary(d ? d : "", dl, &im->dict, &err))) return fail(rc, "%s", err.c_str());
        im->dict.size = JB_JIEBA_SIZE;
    } else if ((rc = parse_dictionary(d ? d : "", dl, kind, &im->dict, &err))) {
        return fail(rc, "%s", err.c_str());
    }
    if (cfg->size_override > 0) im->dict.size = cfg->size_override;
    if ((rc = parse_emission(e, el, &im->emit, &err))) return fail(rc, "%s", err.c_str());
    if ((rc = build_image(im->dict, im->emit, &im->img, &err))) return fail(rc, "%s", err.c_str());
    if (im->img.maxlen > 255) return fail(JB_ELIMIT, "dictionary word of %u runes (max 255)", im->img.maxlen);
    *out = im.release();
    return JB_OK;
}

static int write_file(const char* path, const std::string& data) {
    // write to a temporary name and rename, so a reader never sees half an image
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return fail(JB_EIO, "create %s: %s", tmp.c_str(), strerror(errno));
    const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
    if (fclose(f) != 0 || !ok) {
        remove(tmp.c_str());
        return fail(JB_EIO, "write %s failed", tmp.c_str());
    }
    if (rename(tmp.c_str(), path) != 0) {
        remove(tmp.c_str());
        return fail(JB_EIO, "rename to %s: %s", path, strerror(errno));
    }
    return JB_OK;
}

extern "C" int jb_image_save(const jb_image* img, const char* path) {
    if (!img || !path) return fail(JB_EINVAL, "jb_image_save: null argument");
    std::string data;
    save_image(img->dict, img->emit, img->img, &data);
    return write_file(path, data);
}

extern "C" int jb_image_dict_info(const jb_image* img, uint64_t* nentries, int64_t* size) {
    if (!img) return fail(JB_EINVAL, "jb_image_dict_info: null argument");
    if (nentries) *nentries = img->dict.term_freq.size();
    if (size) *size = img->dict.size;
    return JB_OK;
}

extern "C" void jb_image_free(jb_image* img) { delete img; }

extern "C" int jb_image_lookup(const jb_image* img, const char* word, size_t len, int64_t* freq, double* w) {
    if (!img || (!word && len)) return fail(JB_EINVAL, "jb_image_lookup: null argument");
    std::vector<uint32_t> runes;
    size_t i = 0;
    while (i < len) {
        uint32_t x = 0;
        for (size_t k = 0; k < 4 && i + k < len; k++) x |= (uint32_t)(uint8_t)word[i + k] << (8 * k);
        uint32_t r;
        const uint32_t wd = jb_decode(x, (uint32_t)std::min<size_t>(4, len - i), &r);
        runes.push_back(r);
        i += wd;
    }
    const Lookup lk = image_lookup(img->img, runes.data(), runes.size());
    if (!lk.found) return 0;
    if (freq) {
        auto it = img->dict.term_freq.find(std::string(word, len));
        *freq = it != img->dict.term_freq.end() ? it->second : (lk.fc == JB_FC_ZERO ? 0 : -1);
    }
    if (w) *w = img->img.wtab[lk.widx];
    return 1;
}

extern "C" int jb_image_stats(const jb_image* img, uint64_t* nodes, uint64_t* cap, uint32_t* npages,
                              uint32_t* maxlen, int64_t* size, double* w_absent) {
    if (!img) return fail(JB_EINVAL, "null image");
    if (nodes) *nodes = img->img.nnodes;
    if (cap) *cap = img->img.cells.size();
    if (npages) *npages = img->img.npages;
    if (maxlen) *maxlen = img->img.maxlen;
    if (size) *size = img->img.size;
    if (w_absent) *w_absent = img->img.w_absent;
    return JB_OK;
}

extern "C" double jb_image_emit(const jb_image* img, int state, uint32_t rune) {
    if (!img || state < 0 || state > 3 || rune >= 0x110000u) return JB_MIN_FLOAT;
    const Image& m = img->img;
    return m.emit[(size_t)jb_row(m.pagemap.data(), rune) * 4 + state];
}

extern "C" int jb_image_log_keys(const jb_image* img, int64_t* keys, size_t cap, size_t* n) {
    if (!img || !n || (cap && !keys)) return fail(JB_EINVAL, "jb_image_log_keys: null argument");
    const std::vector<int64_t> k = weight_log_keys(img->dict);
    *n = k.size();
    if (k.size() > cap) return cap ? fail(JB_ELIMIT, "%zu log keys do not fit %zu", k.size(), cap) : JB_ELIMIT;
    std::copy(k.begin(), k.end(), keys);
    return JB_OK;
}

extern "C" double jb_go_log(double x) { return go_log(x); }

// ---------------------------------------------------------------------------
// devices
// ---------------------------------------------------------------------------
template <class T>
static int upload(T** dst, const std::vector<T>& src) {
    *dst = nullptr;
    HIPCHK(hipMalloc(dst, std::max<size_t>(src.size(), 1) * sizeof(T)));
    if (!src.empty()) HIPCHK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return JB_OK;
}

static void free_image_bufs(ImageBufs* b) {
    dfree(b->pagemap); dfree(b->emit); dfree(b->cells); dfree(b->code); dfree(b->wtab); dfree(b->l1row);
    dfree(b->hot);
    *b = ImageBufs{};
}

// Copy an image into fresh buffers on `ordinal` (nothing of the device's current image
// changes; on failure nothing is left allocated).
static int stage_image(int ordinal, const Image& img, ImageBufs* b) {
    *b = ImageBufs{};
    HIPCHK(hipSetDevice(ordinal));
    // row-indexed level-1 table: code and level-1 cell of a rune in one 8-byte load
    std::vector<uint64_t> l1(img.code.size());
    for (size_t r = 0; r < l1.size(); r++) {
        const uint32_t cd = img.code[r];
        l1[r] = jb_l1row_make(cd, cd < img.cells.size() ? img.cells[cd] : 0ull);
    }
    // the weights behind one leading -Inf (DevImage::wtab1: record slots hold index + 1)
    std::vector<double> wt1(img.wtab.size() + 1);
    wt1[0] = -HUGE_VAL;
    std::copy(img.wtab.begin(), img.wtab.end(), wt1.begin() + 1);
    // hot level-1 rows (k_mark_walk keeps them in LDS)
    std::vector<uint64_t> hot(JB_HOT_SLOTS + JB_HOT_SLOTS / 4u, 0ull);
    build_hot_rows(img, hot.data(), reinterpret_cast<uint16_t*>(hot.data() + JB_HOT_SLOTS));
    int rc;
    if ((rc = upload(&b->pagemap, img.pagemap)) || (rc = upload(&b->emit, img.emit)) ||
        (rc = upload(&b->cells, img.cells)) || (rc = upload(&b->code, img.code)) ||
        (rc = upload(&b->wtab, wt1)) || (rc = upload(&b->l1row, l1)) || (rc = upload(&b->hot, hot))) {
        free_image_bufs(b);
        return rc;
    }
    return JB_OK;
}

// Make staged buffers the device's image (the old ones are freed).  The caller holds
// d->mu and nothing is queued on the device that reads the old image.
static int install_image(Device* d, ImageBufs* b, const Image& img) {
    free_image_bufs(&d->ib);
    d->ib = *b;
    *b = ImageBufs{};
    d->dim.l1row = d->ib.l1row;
    d->dim.hot = d->ib.hot;
    d->dim.pagemap = d->ib.pagemap;
    d->dim.emit = d->ib.emit;
    d->dim.cells = d->ib.cells;
    d->dim.code = d->ib.code;
    d->dim.wtab1 = d->ib.wtab;
    d->dim.wtab = d->ib.wtab + 1;
    d->dim.nrows = img.nrows;
    d->dim.nw1 = (uint32_t)std::min<size_t>(img.wtab.size() + 1, 0xFFFFFFFFu);
    d->dim.plainw = 1u;
    for (double w : img.wtab)
        if (std::isnan(w) || w == HUGE_VAL) d->dim.plainw = 0u;  // (a dictionary size <= 0)
    // a captured pipeline holds the old image pointers in its kernel arguments
    if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
    d->gexec = nullptr;
    d->gkey_gen = 0;
    return JB_OK;
}

static void free_work(Work* w) {
    dfree(w->docbits); dfree(w->tile_cnt);
    dfree(w->ttile_cnt); dfree(w->supt); dfree(w->alnum16); dfree(w->erec); dfree(w->lanemask);
    dfree(w->gbl); dfree(w->lsegb); dfree(w->lmap); dfree(w->lcx); dfree(w->lpath); dfree(w->lflag); dfree(w->lbp); dfree(w->gbest); dfree(w->tile4); dfree(w->longblk);
    dfree(w->tok_start); dfree(w->tok_end); dfree(w->doc_tok); dfree(w->counters); dfree(w->dbg); dfree(w->dbg_walk);
    *w = Work{};
}

// Grow-only workspace for nbytes of text and ndocs documents.
static int ensure_work(Device* d, uint64_t nbytes, uint32_t ndocs) {
    Work& w = d->w;
    if (nbytes <= w.cap_bytes && ndocs <= w.cap_docs && w.counters) return JB_OK;
    const uint64_t nb = std::max<uint64_t>(std::max(nbytes, w.cap_bytes), 4096);
    const uint32_t ndc = std::max(std::max(ndocs, w.cap_docs), 1024u);
    free_work(&w);
    if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
    d->gexec = nullptr;
    d->work_gen++;
    const uint64_t nwords = (nb + 31) / 32 + 8;
    const uint64_t ntiles = (nb + kTileBytes - 1) / kTileBytes + 1;
    const uint64_t nttiles = (nwords + kTokTileWords - 1) / kTokTileWords + 1;
    // docbits, sbits, ebits back to back so one memset clears all three
    HIPCHK(hipMalloc(&w.docbits, 3 * nwords * 4));
    w.sbits = w.docbits + nwords;
    w.ebits = w.docbits + 2 * nwords;
    w.bits_stride = nwords;
    HIPCHK(hipMalloc(&w.tile_cnt, ntiles * sizeof(uint2)));
    HIPCHK(hipMalloc(&w.ttile_cnt, nttiles * sizeof(uint2)));
    HIPCHK(hipMalloc(&w.alnum16, (nb / 1024 + 8) * 8));
    HIPCHK(hipMalloc(&w.erec, (nb / 3 + 8 + kErecPad) * 8));
    HIPCHK(hipMalloc(&w.lanemask, ntiles * 256 * 4));
    HIPCHK(hipMalloc(&w.gbl, nb / 3 + 8 + 512));
    HIPCHK(hipMalloc(&w.lflag, (nb / kZhLongMin + 2) * 4));
    HIPCHK(hipMalloc(&w.lsegb, (nb / kZhLongMin + 2) * 4));
    {
        const uint64_t nchunk = (nb / (3 * kSeg) + nb / kZhLongMin + 4) / kSeg + 2;  // 64-segment chunks
        HIPCHK(hipMalloc(&w.lmap, nchunk * 256));
        HIPCHK(hipMalloc(&w.lcx, nchunk));
        HIPCHK(hipMalloc(&w.lpath, nchunk * kSeg * sizeof(uint64_t)));  // per segment
    }
    HIPCHK(hipMalloc(&w.lbp, nb / 3 + 256));
    HIPCHK(hipMalloc(&w.tile4, ntiles * 4));
    HIPCHK(hipMalloc(&w.longblk, (nb / kZhLongMin + 2) * sizeof(uint2)));
    HIPCHK(hipMalloc(&w.gbest, (nb / 3 + 8) * sizeof(double)));

    HIPCHK(hipMalloc(&w.tok_start, (nb + 4) * 4));
    HIPCHK(hipMalloc(&w.tok_end, (nb + 4) * 4));
    HIPCHK(hipMalloc(&w.doc_tok, ((uint64_t)ndc + 2) * 8));
    HIPCHK(hipMalloc(&w.counters, 64 * 4));
    HIPCHK(hipMalloc(&w.supt, (nttiles / 256 + 2) * sizeof(uint2)));
    if (d->lc.diag & 0x100u) {
        HIPCHK(hipMalloc(&w.dbg, 65536 * 16 * 8));
        HIPCHK(hipMalloc(&w.dbg_walk, ntiles * 4 * 8 * 8));
        HIPCHK(hipMemset(w.dbg_walk, 0, ntiles * 4 * 8 * 8));
    }
    w.cap_bytes = nb;
    w.cap_docs = ndc;
    d->docbits_dirty = true;
    return JB_OK;
}

// grow-only device / pinned buffers (a call never has work in flight on them when it grows them)
template <class T>
static int grow_dev(T** p, uint64_t* cap, uint64_t want) {
    if (want <= *cap && *p) return JB_OK;
    dfree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t c = std::max<uint64_t>(want, 1);
    HIPCHK(hipMalloc(p, c * sizeof(T)));
    *cap = c;
    return JB_OK;
}
template <class T>
static int grow_pinned(T** p, uint64_t* cap, uint64_t want) {
    if (want <= *cap && *p) return JB_OK;
    const uint64_t c = std::max<uint64_t>(want, *cap * 3 / 2 + 1);
    hfree(*p);
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipHostMalloc(p, c * sizeof(T), hipHostMallocDefault));
    *cap = c;
    return JB_OK;
}

// grow-only mapped (device-visible), coherent pinned memory: kernels write it directly
template <class T>
static int grow_mapped(T** p, T** dp, uint64_t* cap, uint64_t want) {
    if (want <= *cap && *p) return JB_OK;
    const uint64_t c = std::max<uint64_t>(want, *cap * 3 / 2 + 1);
    hfree(*p);
    *p = *dp = nullptr;
    *cap = 0;
    HIPCHK(hipHostMalloc(p, c * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void**)dp, *p, 0));
    *cap = c;
    return JB_OK;
}

static void free_outs(Device* d) {
    for (auto& o : d->outs) {
        dfree(o.ts); dfree(o.te); dfree(o.dt); hfree(o.hs); hfree(o.hdt);
        dfree(o.pk); dfree(o.phdr); dfree(o.pside); hfree(o.hpk); hfree(o.hhdr); hfree(o.hside);
        o = Device::OutSet{};
    }
}

static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

static const uint64_t kMaxPiece = 1ull << 30;  // (a piece of several documents; device offsets are u32)

// The launch shape of a device, fixed at jb_open.  Tuning knobs come from the
// environment once, here (results do not depend on them):
//   JB_GRID_ZH   k_zh workgroups (default: resident workgroups per CU x CUs)
//   JB_ZH_GROUP  k_zh group bytes, a multiple of 32 in [kZhGroupSmall, kZhGroupBytes]
//                (default: by batch size, zh_group_for)
//   JB_PIECE_KIB host batches are cut in pieces of whole documents of at most this many KiB
//                (default 65536), pipelined over three streams (cut_range)
//   JB_SMALL     host batches up to this many bytes take k_small (0: never)
//   JB_STAMPS    (STAMPS=1 builds only) per-wave phase clocks to stderr
static int init_launch_cfg(Device* d) {
    LaunchCfg& lc = d->lc;
    lc.zh_waves = d->ncu * std::max(zh_waves_per_cu(true, false), zh_waves_per_cu(false, false));
    lc.zh_waves_wide = d->ncu * std::max(zh_waves_per_cu(true, true), zh_waves_per_cu(false, true));
    const int gz = env_int("JB_GRID_ZH", 0);  // (in 4-wave workgroups)
    if (gz > 0) lc.zh_waves = lc.zh_waves_wide = 4u * (uint32_t)gz;
    const int wide = env_int("JB_ZH_WIDE", -1);
    if (wide < -1 || wide > 1) return fail(JB_EINVAL, "JB_ZH_WIDE=%d: want -1 (by batch size), 0 or 1", wide);
    lc.zh_wide = wide;
    const int mws = env_int("JB_MW_SPLIT", -1);
    if (mws < -1 || mws > 3) return fail(JB_EINVAL, "JB_MW_SPLIT=%d: want -1 (by tile count) or 0-3", mws);
    lc.mw_split = mws;
    const int grp = env_int("JB_ZH_GROUP", 0);
    if (grp != 0) {
        if (grp < 256 || grp > (int)kZhGroupBytes || grp % 32 != 0)
            return fail(JB_EINVAL, "JB_ZH_GROUP=%d: want a multiple of 32 in [256, %u]", grp, kZhGroupBytes);
        lc.zh_group = (uint32_t)grp;
    }
    const int zt = env_int("JB_ZH_TAIL_KIB", 0), ztg = env_int("JB_ZH_TAIL_GROUP", 1024);
    if (zt < 0 || zt > (1 << 20) || ztg < (int)kZhGroupSmall || ztg > (int)kZhGroupBytes || ztg % 32 != 0)
        return fail(JB_EINVAL, "JB_ZH_TAIL_KIB=%d / JB_ZH_TAIL_GROUP=%d: want 0 .. 1048576 KiB, a multiple of 32 "
                    "in [%u, %u] bytes", zt, ztg, kZhGroupSmall, kZhGroupBytes);
    lc.zh_tail = (uint32_t)zt << 10;
    lc.zh_tail_group = (uint32_t)ztg;
#if JB_STAMPS
    lc.diag = (uint32_t)env_int("JB_STAMPS", 0) ? 0x100u : 0u;
#endif
    const int pk = env_int("JB_PIECE_KIB", 64 << 10);  // host-batch pipeline piece (KiB of whole documents)
    if (pk < 1 || (uint64_t)pk > kMaxPiece / 1024)
        return fail(JB_EINVAL, "JB_PIECE_KIB=%d: want 1 .. %llu", pk, (unsigned long long)(kMaxPiece / 1024));
    d->piece_bytes = (uint64_t)pk << 10;
    const int sm = env_int("JB_SMALL", (int)kSmallBytes);
    if (sm < 0 || sm > (int)kSmallBytes)
        return fail(JB_EINVAL, "JB_SMALL=%d: want 0 (off) .. %u bytes", sm, kSmallBytes);
    lc.small_max = (uint32_t)sm;
    const int ls = env_int("JB_LONG_SPEC", 1);
    if (ls < 0 || ls > 3) return fail(JB_EINVAL, "JB_LONG_SPEC=%d: want 0, 1, 3 (or 2: testing)", ls);
    lc.long_spec = (uint32_t)ls;
    const int lf = env_int("JB_LONG_FUSED", 1);
    if (lf < 0 || lf > 1) return fail(JB_EINVAL, "JB_LONG_FUSED=%d: want 0 or 1", lf);
    lc.long_fused = (uint32_t)lf;
    lc.ncu = std::max(1u, d->ncu);
    const int t1 = env_int("JB_TOK1", 1);
    if (t1 < 0 || t1 > 1) return fail(JB_EINVAL, "JB_TOK1=%d: want 0 or 1", t1);
    lc.tok1 = (uint32_t)t1;
    const int nzm = env_int("JB_NZ_FUSE_MIB", 4);
    if (nzm < 0 || nzm > 1024) return fail(JB_EINVAL, "JB_NZ_FUSE_MIB=%d: want 0 .. 1024", nzm);
    lc.nz_fuse_mib = (uint32_t)nzm;
    const int sp = env_int("JB_SPAN_PACK", 1);
    if (sp < 0 || sp > 1) return fail(JB_EINVAL, "JB_SPAN_PACK=%d: want 0 or 1", sp);
    d->span_pack = sp != 0;
    // k_long's phase waits give up after this long without progress (100 MHz ticks)
    const int lw = env_int("JB_LONG_WAIT_US", 20000000);
    if (lw < 1 || lw > 40000000) return fail(JB_EINVAL, "JB_LONG_WAIT_US=%d: want 1 .. 40000000", lw);
    lc.long_wait_ticks = (uint32_t)lw * 100u;
    const int ss = env_int("JB_SMALL_SLOTS", 4);
    if (ss < 1 || ss > 8) return fail(JB_EINVAL, "JB_SMALL_SLOTS=%d: want 1 .. 8", ss);
    d->small_slots = (uint32_t)ss;
    return JB_OK;
}

static int launch_pipeline_(Device* d, const Work& w, const uint8_t* d_text, uint64_t nbytes,
                            const uint64_t* d_doc_off, uint32_t ndocs, bool hmm, hipStream_t s, const MaskOut* mask);
static int launch_pipeline(Device* d, const Work& w, const uint8_t* d_text, uint64_t nbytes,
                           const uint64_t* d_doc_off, uint32_t ndocs, bool hmm, hipStream_t s, const MaskOut* mask) {
    if (d->docbits_dirty) {  // the whole bitmap, once (see Device::docbits_dirty)
        HIPCHK(run_zero(w.docbits, w.bits_stride * 4, s));
        d->docbits_dirty = false;
    }
    const int rc = launch_pipeline_(d, w, d_text, nbytes, d_doc_off, ndocs, hmm, s, mask);
    if (rc) d->docbits_dirty = true;
    return rc;
}
static int launch_pipeline_(Device* d, const Work& w, const uint8_t* d_text, uint64_t nbytes,
                            const uint64_t* d_doc_off, uint32_t ndocs, bool hmm, hipStream_t s, const MaskOut* mask) {
    static const bool dbg = getenv("JB_DEBUG") != nullptr;
    const LaunchCfg& lc = d->lc;
    d->last_nbytes = nbytes;
    {
        std::lock_guard<std::mutex> g(d->stats_mu);
        d->last_small = false;
    }
    if (dbg)
        fprintf(stderr, "[jb] nbytes=%llu ndocs=%u zh_waves=%u/%u wide=%d zh_group=%u\n", (unsigned long long)nbytes,
                ndocs, lc.zh_waves, lc.zh_waves_wide, lc.zh_wide, lc.zh_group ? lc.zh_group : zh_group_for(nbytes));
    static const bool use_graph = env_int("JB_GRAPH", 1) != 0;
    if (use_graph && !d->profile && lc.diag == 0 && s != nullptr && !mask) {
        const Device::GraphKey key{d_text, nbytes, d_doc_off, ndocs, hmm, d->work_gen, s, w.tok_start, w.tok_end, w.doc_tok};
        const bool repeat = d->gkey_gen != 0 && key == d->gkey;
        if (!repeat) {  // first call with this key: run directly, capture if it comes again
            if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
            d->gexec = nullptr;
            d->gkey = key;
            d->gkey_gen = 1;
            const hipError_t e = run_pipeline(d->dim, w, d_text, nbytes, d_doc_off, ndocs, hmm, lc, s, nullptr);
            if (e != hipSuccess) return fail(JB_EDEVICE, "pipeline launch: %s", hipGetErrorString(e));
            return JB_OK;
        }
        if (!d->gexec) {
            if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
            d->gexec = nullptr;
            hipGraph_t g = nullptr;
            HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            const hipError_t ec = run_pipeline(d->dim, w, d_text, nbytes, d_doc_off, ndocs, hmm, lc, s, nullptr);
            const hipError_t ee = hipStreamEndCapture(s, &g);
            if (ec != hipSuccess) return fail(JB_EDEVICE, "pipeline capture: %s", hipGetErrorString(ec));
            if (ee != hipSuccess) return fail(JB_EDEVICE, "pipeline capture end: %s", hipGetErrorString(ee));
            const hipError_t ei = hipGraphInstantiate(&d->gexec, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            if (ei != hipSuccess) {
                d->gexec = nullptr;
                return fail(JB_EDEVICE, "pipeline graph instantiate: %s", hipGetErrorString(ei));
            }
        }
        const hipError_t el = hipGraphLaunch(d->gexec, s);
        if (el != hipSuccess) return fail(JB_EDEVICE, "pipeline graph launch: %s", hipGetErrorString(el));
        return JB_OK;
    }
    const hipError_t e = run_pipeline(d->dim, w, d_text, nbytes, d_doc_off, ndocs, hmm, lc, s,
                                      d->profile ? &d->timer : nullptr, mask);
    if (e != hipSuccess) return fail(JB_EDEVICE, "pipeline launch: %s", hipGetErrorString(e));
    if ((lc.diag & 0x100u) && d->w.dbg) {  // diagnostic: per-wave clocks of k_zh (STAMPS builds)
        const uint32_t nwv = std::min<uint32_t>(std::max(lc.zh_waves, lc.zh_waves_wide), 16384u);
        std::vector<uint64_t> st((size_t)nwv * 16);
        HIPCHK(hipMemcpyAsync(st.data(), d->w.dbg, st.size() * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        double a[16] = {0};
        double n = 0;
        for (uint32_t i = 0; i < nwv; i++)
            if (st[i * 16 + 3]) {
                for (int k = 0; k < 16; k++) a[k] += (double)st[i * 16 + k];
                n++;
            }
        if (n == 0) n = 1;
        {  // the grid's tail: every wave starts with the kernel, so the spread of their totals is idle time
            std::vector<uint64_t> tot;
            for (uint32_t i = 0; i < nwv; i++)
                if (st[i * 16 + 3]) tot.push_back(st[i * 16 + 6]);
            if (!tot.empty()) {
                std::sort(tot.begin(), tot.end());
                fprintf(stderr, "[jb] k_zh wave totals: min %llu p10 %llu median %llu max %llu (waves %zu)\n",
                        (unsigned long long)tot.front(), (unsigned long long)tot[tot.size() / 10],
                        (unsigned long long)tot[tot.size() / 2], (unsigned long long)tot.back(), tot.size());
            }
        }
        fprintf(stderr, "[jb] k_zh clocks/wave: setup %.0f dp %.0f fwd walk %.0f viterbi fwd %.0f back+flush+rest %.0f "
                        "total %.0f; chunks/wave %.1f; lane DP steps %.0f vs 64*max %.0f (DP lane use %.2f); blocks past "
                        "the window per chunk %.3f; Viterbi lane use %.2f (longest lane %.1f runes per chunk)\n",
                a[0] / n, a[1] / n, a[8] / n, a[9] / n, a[2] / n, a[6] / n, a[3] / n, a[4] / n, 64.0 * a[5] / n,
                a[4] / (64.0 * a[5] + 1e-9), a[7] / (a[3] + 1e-9), a[10] / (64.0 * a[11] + 1e-9), a[11] / (a[3] + 1e-9));
        fprintf(stderr, "[jb] k_zh Viterbi forward half per chunk: longest lane %.2f runes, longest single run %.2f, "
                        "the wave's runes split evenly %.2f\n",
                a[11] / (a[3] + 1e-9), a[12] / (a[3] + 1e-9), a[13] / (a[3] + 1e-9));
        fprintf(stderr, "[jb] k_zh DP per chunk: longest lane %.2f runes, longest single block %.2f, the wave's runes "
                        "split evenly %.2f\n",
                a[5] / (a[3] + 1e-9), a[14] / (a[3] + 1e-9), a[4] / (64.0 * (a[3] + 1e-9)));
        HIPCHK(hipMemsetAsync(d->w.dbg, 0, (size_t)nwv * 128, s));
        const uint64_t nww = (nbytes + kTileBytes - 1) / kTileBytes * 4;
        std::vector<uint64_t> sw(nww * 8);
        HIPCHK(hipMemcpyAsync(sw.data(), d->w.dbg_walk, sw.size() * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        double b[8] = {0, 0, 0, 0, 0, 0, 0, 0}, m = 0;
        for (uint64_t i = 0; i < nww; i++)
            if (sw[i * 8 + 5] == 1) {
                for (int k = 0; k < 8; k++) b[k] += (double)sw[i * 8 + k];
                m++;
            }
        if (m == 0) m = 1;
        fprintf(stderr, "[jb] k_mark_walk clocks/wave: mark %.0f (staging %.0f) entries %.0f (loads %.0f) walk %.0f "
                        "tail %.0f; trips/wave %.2f\n",
                b[0] / m, b[6] / m, b[1] / m, b[7] / m, b[2] / m, b[3] / m, b[4] / m);
        std::vector<uint64_t> sl(64 * 32);
        HIPCHK(hipMemcpyAsync(sl.data(), d->w.dbg + 65536 * 4, sl.size() * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int i = 0; i < 64; i++) {  // per wave: run, barrier, windows, slow
            const uint64_t* o = sl.data() + i * 16;
            if (o[2])
                fprintf(stderr, "[jb] k_long_dp wg %d: chain run %llu bar %llu windows %llu slow %llu | "
                                "wave 1 run %llu bar %llu | wave 2 run %llu bar %llu (%llu) | wave 3 run %llu bar %llu\n", i,
                        (unsigned long long)o[0], (unsigned long long)o[1], (unsigned long long)o[2],
                        (unsigned long long)o[3], (unsigned long long)o[4], (unsigned long long)o[5],
                        (unsigned long long)o[8], (unsigned long long)o[9], (unsigned long long)o[11],
                        (unsigned long long)o[12], (unsigned long long)o[13]);
            const uint64_t* p = sl.data() + 64 * 16 + i * 16;
            if (o[2])
                fprintf(stderr, "[jb] k_long_dp wg %d sub-phases: w0 %llu %llu %llu %llu | w1 %llu %llu %llu %llu | "
                                "w2 %llu %llu %llu %llu | w3 %llu %llu %llu %llu\n", i,
                        (unsigned long long)p[0], (unsigned long long)p[1], (unsigned long long)p[2],
                        (unsigned long long)p[3], (unsigned long long)p[4], (unsigned long long)p[5],
                        (unsigned long long)p[6], (unsigned long long)p[7], (unsigned long long)p[8],
                        (unsigned long long)p[9], (unsigned long long)p[10], (unsigned long long)p[11],
                        (unsigned long long)p[12], (unsigned long long)p[13], (unsigned long long)p[14],
                        (unsigned long long)p[15]);
        }
        HIPCHK(hipMemsetAsync(d->w.dbg + 65536 * 4, 0, sl.size() * 8, s));
        if (const char* wo = getenv("JB_LDW_OUT")) {  // k_long_dp per-window records of block 0
            std::vector<uint64_t> wr(65536 * 2 * 4);
            HIPCHK(hipMemcpyAsync(wr.data(), d->w.dbg + 65536 * 8, wr.size() * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            if (FILE* f = fopen(wo, "wb")) {
                fwrite(wr.data(), 8, wr.size(), f);
                fclose(f);
            }
            HIPCHK(hipMemsetAsync(d->w.dbg + 65536 * 8, 0, wr.size() * 8, s));
        }
    }
    return JB_OK;
}

// Queue the pipeline on stream s.  The workspace is one per device: a pipeline waits
// for the previous one (on whatever stream it ran) before it starts.  `w` is the
// device's workspace, or a copy with caller-owned outputs (jb_cut_device_into).
static int launch(Device* d, const Work& w, const uint8_t* d_text, uint64_t nbytes, const uint64_t* d_doc_off,
                  uint32_t ndocs, bool hmm, hipStream_t s, const MaskOut* mask = nullptr) {
    if (!d->ws_done) HIPCHK(hipEventCreateWithFlags(&d->ws_done, hipEventDisableTiming));
    else HIPCHK(hipStreamWaitEvent(s, d->ws_done, 0));  // (free on the stream that recorded it)
    int rc = launch_pipeline(d, w, d_text, nbytes, d_doc_off, ndocs, hmm, s, mask);
    if (rc) return rc;
    HIPCHK(hipEventRecord(d->ws_done, s));
    d->ws_stream = s;
    {
        std::lock_guard<std::mutex> g(d->stats_mu);
        d->has_stats = true;
    }
    d->acc_valid = false;
    return JB_OK;
}

extern "C" void jb_close(jb_ctx* ctx);

// Streams, image and launch shape of one device of a new ctx.
static int open_device(Device* d, int ordinal, const Image& img) {
    d->ordinal = ordinal;
    int rc;
    HIPCHK(hipSetDevice(d->ordinal));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, d->ordinal));
    d->ncu = (uint32_t)prop.multiProcessorCount;
    HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&d->cstream, hipStreamNonBlocking));
    HIPCHK(hipHostMalloc(&d->h_zero, 64, hipHostMallocDefault));
    memset(d->h_zero, 0, 64);
    HIPCHK(hipStreamCreateWithFlags(&d->dstream, hipStreamNonBlocking));
    ImageBufs b;
    if ((rc = stage_image(d->ordinal, img, &b))) return rc;
    if ((rc = install_image(d, &b, img))) return rc;
    if ((rc = init_launch_cfg(d))) return rc;  // (sets small_slots)
    {
        // k_small runs one workgroup per batch, one stream per slot.  With JB_SMALL_CUMASK=1
        // (round 4's default) each slot's stream is masked to one CU (JB_SMALL_CU + slot x
        // JB_SMALL_CU_STRIDE), so that its batch finds the trie's hot lines in that XCD's L2;
        // round 5 measured plain streams faster (the sentence 21.8-22.2 -> 20.0-21.0 us per
        // call; concurrent calls the same at 4 slots and better at 8), so they are the default
        const int cu = env_int("JB_SMALL_CU", 0), cs = env_int("JB_SMALL_CU_STRIDE", 1);
        const int last = cu + ((int)d->small_slots - 1) * cs;  // (only the slots in use get a stream)
        if (cu < 0 || cs < 0 || last >= (int)d->ncu)
            return fail(JB_EINVAL,
                        "JB_SMALL_CU=%d, JB_SMALL_CU_STRIDE=%d, JB_SMALL_SLOTS=%u: slot k runs on CU "
                        "JB_SMALL_CU + k x JB_SMALL_CU_STRIDE, and the last one (%d) is past the device's %u CUs",
                        cu, cs, d->small_slots, last, d->ncu);
        const bool masked = env_int("JB_SMALL_CUMASK", 0) != 0;
        for (int k = 0; k < (int)d->small_slots; k++) {
            std::vector<uint32_t> mask((d->ncu + 31) / 32, 0u);
            const int c = cu + k * cs;
            mask[c / 32] = 1u << (c % 32);
            if (masked) HIPCHK(hipExtStreamCreateWithCUMask(&d->slots[k].st, (uint32_t)mask.size(), mask.data()));
            else HIPCHK(hipStreamCreateWithFlags(&d->slots[k].st, hipStreamNonBlocking));
        }
    }
    return JB_OK;
}

extern "C" int jb_open_image(jb_image* img, const jb_config* cfg, jb_ctx** out) {
    std::unique_ptr<jb_image> own(img);  // consumed on every path
    if (!img || !cfg || !out) return fail(JB_EINVAL, "jb_open_image: null argument");
    *out = nullptr;
    if (cfg->nlog && (!cfg->log_keys || !cfg->log_vals)) return fail(JB_EINVAL, "nlog > 0 without log_keys/log_vals");
    if (cfg->nlog) {  // the caller's logarithms: new weights, same trie
        for (size_t i = 0; i < cfg->nlog; i++) img->dict.log_of[cfg->log_keys[i]] = cfg->log_vals[i];
        if (!reweigh_image(img->dict, &img->img)) {
            std::string err;
            const int rc = build_image(img->dict, img->emit, &img->img, &err);
            if (rc) return fail(rc, "%s", err.c_str());
        }
    }
    auto ctx = std::make_unique<jb_ctx>();
    ctx->im = std::move(own);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(JB_EDEVICE, "no HIP device available");
    const int nuse = cfg->ndevices > 0 ? cfg->ndevices : 1;
    // JB_DEVICE_WRAP=1 (tests): device ordinals wrap around the devices present, so the
    // multi-device host path (one thread, stream and workspace per device) runs on one GPU
    const bool wrap = env_int("JB_DEVICE_WRAP", 0) != 0;
    if (cfg->device < 0 || (!wrap && cfg->device + nuse > ndev) || (wrap && cfg->device >= ndev))
        return fail(JB_EINVAL, "devices %d..%d requested, %d present", cfg->device, cfg->device + nuse - 1, ndev);
    int rc = JB_OK;
    for (int k = 0; k < nuse && rc == JB_OK; k++) {
        ctx->devs.push_back(std::make_unique<Device>());  // (jb_close releases a partial one)
        rc = open_device(ctx->devs.back().get(), (cfg->device + k) % ndev, ctx->im->img);
    }
    if (rc) {
        jb_close(ctx.release());
        return rc;
    }
    *out = ctx.release();
    return JB_OK;
}

extern "C" int jb_open(const jb_config* cfg, jb_ctx** out) {
    if (!cfg || !out) return fail(JB_EINVAL, "jb_open: null argument");
    *out = nullptr;
    jb_image* img = nullptr;
    int rc = jb_image_build(cfg, &img);
    if (rc) return rc;
    jb_config c = *cfg;
    c.nlog = 0;  // (jb_image_build applied the log table)
    return jb_open_image(img, &c, out);
}

extern "C" void jb_close(jb_ctx* ctx) {
    if (!ctx) return;
    for (auto& d : ctx->devs) {
        if (const char* tp = getenv("JB_SMALL_TRACE"); tp && !d->small_trace.empty())
            if (FILE* f = fopen(tp, "a")) {
                for (const auto& r : d->small_trace)
                    fprintf(f, "%g %g %.3f %.3f %.3f %.3f\n", r[0], r[1], r[2], r[3], r[4], r[5]);
                fclose(f);
            }
        (void)hipSetDevice(d->ordinal);
        (void)hipStreamSynchronize(d->stream);
        for (auto& sl : d->slots)
            if (sl.st) (void)hipStreamSynchronize(sl.st);
        d->timer.reset();
        // a jb_cut_device pipeline queued on a caller's stream may still use the workspace:
        // wait for its completion event before freeing anything (the caller's stream may be
        // gone by now, the event is ours)
        if (d->ws_done) (void)hipEventSynchronize(d->ws_done);
        if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
        d->gexec = nullptr;
        free_work(&d->w);
        dfree(d->text); dfree(d->doc_off);
        free_image_bufs(&d->ib);
        if (d->ws_done) (void)hipEventDestroy(d->ws_done);
        hfree(d->h_text); hfree(d->h_misc);
        for (auto& sl : d->slots) {
            hfree(sl.h_sin);
            hfree(sl.h_sout[0]);
            hfree(sl.h_sout[1]);
        }
        free_outs(d.get());
        hfree(d->h_pcnt); dfree(d->d_mask); hfree(d->h_mask); hfree(d->h_zero);
        for (auto* v : {&d->ev_h2d, &d->ev_comp, &d->ev_d2h})
            for (hipEvent_t e : *v) (void)hipEventDestroy(e);
        if (d->cstream) (void)hipStreamDestroy(d->cstream);
        if (d->dstream) (void)hipStreamDestroy(d->dstream);
        (void)hipStreamDestroy(d->stream);
        for (auto& sl : d->slots)
            if (sl.st) (void)hipStreamDestroy(sl.st);
    }
    delete ctx;
}

extern "C" const char* jb_last_error(void) { return g_err.c_str(); }

// ---------------------------------------------------------------------------
// cutting
// ---------------------------------------------------------------------------

// A batch of at most lc.small_max bytes and kSmallDocs documents (a single Cut
// call, BASELINE config 1) is one k_small launch that reads the text and offsets
// from mapped pinned host memory (or its kernel arguments) and writes the spans
// there.  Concurrent calls on a device are coalesced (the reference runs Cut calls
// side by side under RLock, tokenizer.go:151-153): each call queues a SmallReq.  A
// caller that finds a slot free (one of JB_SMALL_SLOTS pinned input/output buffer pairs,
// each with its own stream on its own CU) launches the queue's head requests (same hmm,
// up to the k_small limits together) as ONE k_small batch on it, their documents back to
// back, waits for that batch's completion word and hands each caller its own spans by its
// documents' doc_tok ranges.  The slot then goes straight to the caller of the next
// queued request, with the next batch: callers wait on their own request's state word,
// so a finished batch wakes the callers it served and the one it hands the slot to, not
// every waiting caller.  One caller alone: a batch of one.
namespace {
struct SmallReq {
    const uint8_t* text;
    const uint64_t* doc_off;  // doc_off[0..nd] absolute in text
    uint32_t nd;
    bool hmm;
    SpanBuf* out;
    int rc = JB_OK;
    std::string err;
    // kQueued, then kDone; or kLaunch first: this caller launches `batch` (its own request at
    // the head) on slot `sl`, which the caller that finished that slot's last batch handed over
    std::atomic<uint32_t> state{0};
    Device::SmallSlot* sl = nullptr;
    std::vector<SmallReq*> batch;
};
enum : uint32_t { kQueued = 0, kLaunch = 1, kDone = 2 };
}  // namespace

// One k_small launch over requests rq[0..n) (together within the limits) on the slot's
// next output buffer: stage, launch, wait for the completion word.  Returns the output
// (header, spans, doc_tok), or nullptr with each request's rc / err set.
static const uint32_t* small_launch(Device* d, Device::SmallSlot* sl, SmallReq* const* rq, uint32_t n) {
    auto fail_all = [&](int rc) {
        for (uint32_t i = 0; i < n; i++) {
            rq[i]->rc = rc;
            rq[i]->err = g_err;
        }
    };
    auto chk = [&](hipError_t e, const char* what) {
        if (e == hipSuccess) return true;
        fail_all(fail(e == hipErrorOutOfMemory ? JB_ENOMEM : JB_EDEVICE, "%s: %s", what, hipGetErrorString(e)));
        return false;
    };
    if (!chk(hipSetDevice(d->ordinal), "hipSetDevice")) return nullptr;
    if (!sl->h_sin || !sl->h_sout[0] || !sl->h_sout[1]) {
        // all three buffers or none: a failure part way frees what was allocated, so the
        // next call on the slot allocates again instead of using a null buffer
        auto drop = [&]() {
            for (void** p : {(void**)&sl->h_sin, (void**)&sl->h_sout[0], (void**)&sl->h_sout[1]})
                if (*p) {
                    (void)hipHostFree(*p);
                    *p = nullptr;
                }
            sl->d_sin = nullptr;
            sl->d_sout[0] = sl->d_sout[1] = nullptr;
        };
        drop();
        const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
        if (!chk(hipHostMalloc(&sl->h_sin, kSmallBytes + 128 + 8 * (kSmallDocs + 1), fl), "hipHostMalloc") ||
            !chk(hipHostGetDevicePointer((void**)&sl->d_sin, sl->h_sin, 0), "hipHostGetDevicePointer")) {
            drop();
            return nullptr;
        }
        for (int k = 0; k < 2; k++) {
            if (!chk(hipHostMalloc(&sl->h_sout[k], kSmallOutBytes, fl), "hipHostMalloc") ||
                !chk(hipHostGetDevicePointer((void**)&sl->d_sout[k], sl->h_sout[k], 0), "hipHostGetDevicePointer")) {
                drop();
                return nullptr;
            }
            sl->h_sout[k][SM_DONE] = 0;  // (recycled pinned memory may hold any value; seq starts at 1)
        }
    }
    // the other buffer: the last batch's callers may still be taking their spans from this one
    sl->ob ^= 1u;
    while (sl->reading[sl->ob].load(std::memory_order_acquire)) __builtin_ia32_pause();
    const bool hmm = rq[0]->hmm;
    uint64_t nbytes = 0;
    uint32_t nd = 0;
    for (uint32_t i = 0; i < n; i++) {
        nbytes += rq[i]->doc_off[rq[i]->nd] - rq[i]->doc_off[0];
        nd += rq[i]->nd;
    }
    const auto c0 = std::chrono::steady_clock::now();
    // a batch that fits the kernel arguments (96 bytes, 7 documents) travels in them (the kernel reads them from
    // the kernarg segment instead of host memory over PCIe); others go through h_sin
    const bool inl = nbytes <= kSmallInline && nd <= kSmallInlineDocs;
    SmallInline in;
    memset(&in, 0, sizeof in);
    uint8_t* const tx = inl ? in.txt : sl->h_sin;
    uint64_t* const hoff = reinterpret_cast<uint64_t*>(sl->h_sin + kSmallBytes + 128);
    uint64_t at = 0;
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++) {
        const SmallReq& r = *rq[i];
        const uint64_t base = r.doc_off[0], len = r.doc_off[r.nd] - base;
        if (len) memcpy(tx + at, r.text + base, len);
        for (uint32_t j = 0; j < r.nd; j++, k++) {
            if (inl) in.doff[k] = (uint16_t)(at + r.doc_off[j] - base);
            else hoff[k] = at + r.doc_off[j] - base;
        }
        at += len;
    }
    if (inl) in.doff[nd] = (uint16_t)nbytes;
    else {
        hoff[nd] = nbytes;
        memset(sl->h_sin + nbytes, 0, 16);
    }
    // the kernel writes the call's sequence number after everything else (system-scope
    // release); spinning on it returns as soon as the results are in host memory
    const uint32_t seq = ++sl->seq;
    volatile uint32_t* done = sl->h_sout[sl->ob] + SM_DONE;
    if (!chk(run_small(d->dim, inl ? nullptr : sl->d_sin, (uint32_t)nbytes,
                       inl ? nullptr : reinterpret_cast<const uint64_t*>(sl->d_sin + kSmallBytes + 128), nd, hmm,
                       sl->d_sout[sl->ob], seq, in, sl->st),
             "k_small launch"))
        return nullptr;
    const auto c1 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; *done != seq; spin++) {
        if ((spin & 1023u) != 1023u) continue;
        const hipError_t q = hipStreamQuery(sl->st);
        if (q == hipErrorNotReady) continue;
        if (!chk(q, "k_small")) return nullptr;
        if (*done != seq) {
            fail_all(fail(JB_EDEVICE, "k_small finished without its completion word"));
            return nullptr;
        }
        break;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    const auto c2 = std::chrono::steady_clock::now();
    static const bool trace = getenv("JB_SMALL_TRACE") != nullptr;
    if (trace) {
        auto us = [](std::chrono::steady_clock::time_point t) {
            return std::chrono::duration<double, std::micro>(t.time_since_epoch()).count();
        };
        std::lock_guard<std::mutex> g(d->stats_mu);
        d->small_trace.push_back({(double)(sl - d->slots), (double)n, us(c0), us(c1), us(c2),
                                  us(std::chrono::steady_clock::now())});
    }
    const uint32_t* h = sl->h_sout[sl->ob];
    {
        std::lock_guard<std::mutex> g(d->stats_mu);  // (jb_last_stats reads these; not d->mu: see Device)
        memcpy(d->small_hdr, h, sizeof d->small_hdr);
        d->last_small = true;
        d->has_stats = true;
    }
    static const bool dbg = getenv("JB_DEBUG") != nullptr;
    if (dbg) {  // k_small's phase clocks (10 ns ticks from its start)
        auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::micro>(b - a).count();
        };
        fprintf(stderr, "[jb] k_small %llu bytes, %u calls: stage+launch %.2f us, sync %.2f us; phases (us):",
                (unsigned long long)nbytes, n, us(c0, c1), us(c1, c2));
        for (int q = 0; q < 15; q++) fprintf(stderr, " %.2f", h[SM_CLK + q] * 0.01);
        fprintf(stderr, "; %u clocks (walk end %u, viterbi fwd %u, traceback %u; dp %u %u %u)", h[SM_CLK + 15],
                h[SM_CLK + 16], h[SM_CLK + 17], h[SM_CLK + 18], h[SM_CLK + 19], h[SM_CLK + 20], h[SM_CLK + 21]);
        fprintf(stderr, "\n");
    }
    return h;
}

// After a batch: its errors.  0 = spans to split; 1 = each request's rc / err set (a
// panic on one request of several: they were rerun one by one on the slot).
static void small_batch(Device* d, Device::SmallSlot* sl, SmallReq* const* rq, uint32_t n);
static int small_check(Device* d, Device::SmallSlot* sl, const uint32_t* h, SmallReq* const* rq, uint32_t n) {
    auto fail_all = [&](int rc) {
        for (uint32_t i = 0; i < n; i++) {
            rq[i]->rc = rc;
            rq[i]->err = g_err;
        }
    };
    if (h[SM_ERR]) {  // the reference panics on some document: find whose (each call alone)
        if (n > 1) {
            for (uint32_t i = 0; i < n; i++) small_batch(d, sl, rq + i, 1);
            return 1;
        }
        fail_all(fail(JB_EPANIC, "a Han block has no DAG path (the reference panics in cutDAG)"));
        return 1;
    }
    if (h[SM_NTOK] != h[SM_NTOKE]) {
        fail_all(fail(JB_EDEVICE, "internal: %u token starts vs %u ends", h[SM_NTOK], h[SM_NTOKE]));
        return 1;
    }
    return 0;
}

// Each request's spans out of a batch's output h (batch offsets -> the call's own text).
static void small_split(const uint32_t* h, SmallReq* const* rq, uint32_t n) {
    uint64_t at = 0;
    uint32_t k = 0;
    const uint32_t* hs = h + kSmallHdr;
    const uint32_t* he = hs + kSmallBytes;
    const uint64_t* dt = reinterpret_cast<const uint64_t*>(he + kSmallBytes);
    for (uint32_t i = 0; i < n; i++) {
        SmallReq& r = *rq[i];
        SpanBuf* out = r.out;
        const uint64_t base = r.doc_off[0];
        const uint64_t t0 = dt[k], t1 = dt[k + r.nd], nt = t1 - t0;
        const bool write = out->reserve(out->n + nt);
        if (!write && !out->external) {
            r.rc = fail(JB_ENOMEM, "out of host memory for %llu tokens", (unsigned long long)nt);
            r.err = g_err;
        } else {
            if (write && out->s32) {
                for (uint64_t t = 0; t < nt; t++) {  // (batch offsets -> this call's text, less b32)
                    out->s32[out->n + t] = (uint32_t)(base - out->b32 + hs[t0 + t] - at);
                    out->e32[out->n + t] = (uint32_t)(base - out->b32 + he[t0 + t] - at);
                }
            } else if (write) {
                for (uint64_t t = 0; t < nt; t++) {  // (batch offsets -> this call's text)
                    out->s[out->n + t] = base + hs[t0 + t] - at;
                    out->e[out->n + t] = base + he[t0 + t] - at;
                }
            } else {  // caller arrays too small: count the rest, write nothing more
                out->needed = out->n + nt;
                out->cap = 0;
            }
            out->n += nt;
            for (uint32_t j = 0; j < r.nd; j++) out->per_doc.push_back(dt[k + j + 1] - dt[k + j]);
        }
        at += r.doc_off[r.nd] - base;
        k += r.nd;
    }
}

// One whole batch, its callers' spans split before it returns (a lone rerun).
static void small_batch(Device* d, Device::SmallSlot* sl, SmallReq* const* rq, uint32_t n) {
    const uint32_t* h = small_launch(d, sl, rq, n);
    if (h && !small_check(d, sl, h, rq, n)) small_split(h, rq, n);
}

// The queue's head requests (same hmm as the head, together within the k_small limits),
// taken off the queue.  Under small_mu.
static std::vector<SmallReq*> take_batch(Device* d) {
    std::vector<SmallReq*> b;
    uint64_t bytes = 0;
    uint32_t docs = 0;
    const bool h = d->small_q.front()->hmm;
    for (auto it = d->small_q.begin(); it != d->small_q.end();) {
        SmallReq* q = *it;
        const uint64_t len = q->doc_off[q->nd] - q->doc_off[0];
        if (q->hmm != h || bytes + len > d->lc.small_max || docs + q->nd > kSmallDocs) {
            ++it;
            continue;
        }
        bytes += len;
        docs += q->nd;
        b.push_back(q);
        it = d->small_q.erase(it);
    }
    return b;
}

// Runs batch b on slot sl, completes its requests, and passes the slot on: the next batch
// from the queue goes to its head request's caller (which is waiting on its own state word,
// so a finished batch wakes one caller, not every waiting one), else the slot goes free.
static void small_run(Device* d, Device::SmallSlot* sl, std::vector<SmallReq*> b) {
    const uint32_t n = (uint32_t)b.size();
    const uint32_t* h = small_launch(d, sl, b.data(), n);
    const bool split = h && !small_check(d, sl, h, b.data(), n);
    const uint32_t ob = sl->ob;
    if (split) sl->reading[ob].store(true, std::memory_order_relaxed);  // (the slot is still ours)
    std::unique_lock<std::mutex> lk(d->small_mu);
    if (!d->small_q.empty()) {
        std::vector<SmallReq*> nb = take_batch(d);
        SmallReq* const next = nb[0];
        next->sl = sl;
        next->batch = std::move(nb);
        next->state.store(kLaunch, std::memory_order_release);
    } else {
        sl->busy = false;
    }
    const bool asleep = d->small_sleepers > 0;
    lk.unlock();
    if (asleep) d->small_cv.notify_all();  // (the caller handed the slot may be asleep)
    if (split) {  // (the slot's next batch writes the other buffer meanwhile)
        small_split(h, b.data(), n);
        sl->reading[ob].store(false, std::memory_order_release);
    }
    for (SmallReq* q : b) q->state.store(kDone, std::memory_order_release);  // (q may be gone after this)
    lk.lock();  // (a caller asleep on small_cv checked its state under small_mu)
    const bool wake = d->small_sleepers > 0;
    lk.unlock();
    if (wake) d->small_cv.notify_all();
}

static int cut_small(Device* d, const uint8_t* text, const uint64_t* doc_off, uint32_t nd, bool hmm,
                     SpanBuf* out) {
    SmallReq r{text, doc_off, nd, hmm, out};
    {
        std::unique_lock<std::mutex> lk(d->small_mu);
        d->small_q.push_back(&r);
        Device::SmallSlot* sl = nullptr;
        for (uint32_t k = 0; k < d->small_slots && !sl; k++)
            if (!d->slots[k].busy) sl = &d->slots[k];
        if (sl) {  // a free slot: launch the queue's head requests on it now
            sl->busy = true;
            std::vector<SmallReq*> b = take_batch(d);
            lk.unlock();
            small_run(d, sl, std::move(b));
        }
    }
    // wait on this request's own word: done by another caller's batch, or handed a slot to
    // launch on.  Spin up to ~100 us first (a batch takes 20-40 us; a sleeping caller's
    // wake-up costs about as much again), then yield the CPU between looks up to ~2 ms
    // (queued behind other batches), then sleep on small_cv.
    for (;;) {
        uint32_t st = r.state.load(std::memory_order_acquire);
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t i = 1; st == kQueued; i++) {
            if ((i & 63u) == 0) {
                const auto w = std::chrono::steady_clock::now() - t0;
                if (w > std::chrono::microseconds(2000)) break;
                if (w > std::chrono::microseconds(100)) std::this_thread::yield();
            }
            __builtin_ia32_pause();
            st = r.state.load(std::memory_order_acquire);
        }
        if (st == kQueued) {
            std::unique_lock<std::mutex> lk(d->small_mu);
            d->small_sleepers++;
            d->small_cv.wait(lk, [&] { return r.state.load(std::memory_order_acquire) != kQueued; });
            d->small_sleepers--;
            st = r.state.load(std::memory_order_acquire);
        }
        if (st == kDone) break;
        // kLaunch: this caller runs the batch it was handed (its own request among them)
        r.state.store(kQueued, std::memory_order_relaxed);
        small_run(d, r.sl, std::move(r.batch));
    }
    if (r.rc) g_err = r.err;
    return r.rc;
}

// Caller-owned boundary masks (jb_cut_batch_mask): bit i of s / e is byte batch0 + i.
struct MaskDst {
    uint64_t* s;
    uint64_t* e;
    uint64_t batch0;
};

// Words [lo, hi) of a range's masks (range word j = caller word rw + j, nw words in all)
// into the caller's arrays.  The range's first and last words may be shared with the
// neighbouring ranges of other devices: those are ORed (atomically) into words the
// caller zeroed first; the rest belong to this range alone and are stored.
static void put_mask_words(const MaskDst* m, uint64_t rw, uint64_t nw, uint64_t lo, uint64_t hi, const uint64_t* ms,
                           const uint64_t* me) {
    auto one = [&](uint64_t j) {
        if (j == 0 || j + 1 == nw) {
            __atomic_fetch_or(m->s + rw + j, ms[j], __ATOMIC_RELAXED);
            __atomic_fetch_or(m->e + rw + j, me[j], __ATOMIC_RELAXED);
        } else {
            m->s[rw + j] = ms[j];
            m->e[rw + j] = me[j];
        }
    };
    if (lo < hi && lo == 0) one(lo++);
    if (lo < hi && hi == nw) one(--hi);
    if (lo >= hi) return;
    const uint64_t n = hi - lo;
    const unsigned nth = n >= (1u << 18) ? kCopyThreads : 1u;
    auto work = [&](unsigned t) {
        const uint64_t a = lo + n * t / nth, b = lo + n * (t + 1) / nth;
        memcpy(m->s + rw + a, ms + a, (b - a) * 8);
        memcpy(m->e + rw + a, me + a, (b - a) * 8);
    };
    run_threads(nth, work);
}

// k_span_pack's packed spans of one piece back to u64 batch offsets (base = the piece's
// first byte in the batch): blocks of kPackBlock tokens decode independently from their
// header, a token at a time (start = previous end + gap, end = start + length), on
// kCopyThreads threads; an escaped token (0xFFFF) takes its span from the side list,
// sorted by token index first (on ordinary text it is empty or nearly so).
// One token of a packed piece: start = previous end + gap, end = start + length, or an
// escaped token's span from the sorted side list.  e: the previous token's end (batch offset).
static inline void unpack_one(uint32_t x, uint32_t i, const uint4* side, uint32_t nside, uint64_t base, uint64_t& s,
                              uint64_t& e) {
    if (x != 0xFFFFu) {
        s = e + (x & kPackGapEsc);
        e = s + (x >> kPackGapBits);
    } else {
        const uint4* q = std::lower_bound(side, side + nside, i, [](const uint4& a, uint32_t v) { return a.x < v; });
        s = base + q->y;
        e = base + q->z;
    }
}

// Tokens [i0, i1) of one block, eight at a time with AVX-512: the ends are a running sum
// of gap + length (an in-register scan: three shifted adds), the starts the ends minus
// the lengths; a group of eight with an escaped token goes through unpack_one.  T is the
// output word (u64 batch offsets, or u32 for jb_cut_batch_into32: base is then relative to
// the caller's first byte).  Stores are streaming where both outputs are aligned alike to
// the vector width (after a scalar head), plain otherwise.
template <class T>
__attribute__((target("avx512f"))) static void unpack_block_avx512(const uint16_t* pk, uint32_t i0, uint32_t i1,
                                                                  uint64_t e, const uint4* side, uint32_t nside,
                                                                  uint64_t base, T* os, T* oe) {
    constexpr uintptr_t kVec = 8u * sizeof(T) - 1u;  // (eight outputs: 64 or 32 bytes)
    uint32_t i = i0;
    const bool al = (((uintptr_t)(os + i) ^ (uintptr_t)(oe + i)) & kVec) == 0u;
    if (al)
        for (; i < i1 && ((uintptr_t)(os + i) & kVec); i++) {
            uint64_t s;
            unpack_one(pk[i], i, side, nside, base, s, e);
            __builtin_nontemporal_store((T)s, os + i);
            __builtin_nontemporal_store((T)e, oe + i);
        }
    const __m512i m6 = _mm512_set1_epi64(kPackGapEsc), z = _mm512_setzero_si512(), last = _mm512_set1_epi64(7);
    __m512i cv = _mm512_set1_epi64((long long)e);  // the previous token's end in every lane
    for (; i + 8u <= i1; i += 8u) {
        const __m128i raw = _mm_loadu_si128(reinterpret_cast<const __m128i*>(pk + i));
        if (_mm_movemask_epi8(_mm_cmpeq_epi16(raw, _mm_set1_epi16(-1)))) {  // an escaped token: one at a time
            e = (uint64_t)_mm_cvtsi128_si64(_mm512_castsi512_si128(cv));
            for (uint32_t k = i; k < i + 8u; k++) {
                uint64_t s;
                unpack_one(pk[k], k, side, nside, base, s, e);
                os[k] = (T)s;
                oe[k] = (T)e;
            }
            cv = _mm512_set1_epi64((long long)e);
            continue;
        }
        const __m512i x = _mm512_cvtepu16_epi64(raw);
        const __m512i l = _mm512_srli_epi64(x, kPackGapBits);
        __m512i t = _mm512_add_epi64(_mm512_and_si512(x, m6), l);  // gap + length
        t = _mm512_add_epi64(t, _mm512_alignr_epi64(t, z, 7));     // inclusive scan over 8 lanes
        t = _mm512_add_epi64(t, _mm512_alignr_epi64(t, z, 6));
        t = _mm512_add_epi64(t, _mm512_alignr_epi64(t, z, 4));
        const __m512i ev = _mm512_add_epi64(cv, t);
        const __m512i sv = _mm512_sub_epi64(ev, l);
        if constexpr (sizeof(T) == 8) {
            if (al) {
                _mm512_stream_si512(reinterpret_cast<__m512i*>(os + i), sv);
                _mm512_stream_si512(reinterpret_cast<__m512i*>(oe + i), ev);
            } else {
                _mm512_storeu_si512(os + i, sv);
                _mm512_storeu_si512(oe + i, ev);
            }
        } else {
            const __m256i s32 = _mm512_cvtepi64_epi32(sv), e32 = _mm512_cvtepi64_epi32(ev);
            if (al) {
                _mm256_stream_si256(reinterpret_cast<__m256i*>(os + i), s32);
                _mm256_stream_si256(reinterpret_cast<__m256i*>(oe + i), e32);
            } else {
                _mm256_storeu_si256(reinterpret_cast<__m256i*>(os + i), s32);
                _mm256_storeu_si256(reinterpret_cast<__m256i*>(oe + i), e32);
            }
        }
        cv = _mm512_permutexvar_epi64(last, ev);
    }
    e = (uint64_t)_mm_cvtsi128_si64(_mm512_castsi512_si128(cv));
    for (; i < i1; i++) {
        uint64_t s;
        unpack_one(pk[i], i, side, nside, base, s, e);
        os[i] = (T)s;
        oe[i] = (T)e;
    }
}

// k_span_pack's packed spans of one piece back to batch offsets (base = the piece's first
// byte in the batch, or relative to the caller's first byte for u32 outputs): blocks of
// kPackBlock tokens decode independently from their header, on kCopyThreads threads
// (eight tokens at a time with AVX-512 where the CPU has it); an escaped token (0xFFFF)
// takes its span from the side list, sorted by token index first (on ordinary text it is
// empty or nearly so).  The outputs are written without reading the caller's lines first
// (streaming stores), fenced before each thread ends.
template <class T>
static void unpack_spans(const uint16_t* pk, const uint32_t* hdr, uint4* side, uint32_t nside, uint32_t nt,
                         uint64_t base, T* os, T* oe) {
    if (nside > 1) std::sort(side, side + nside, [](const uint4& a, const uint4& b) { return a.x < b.x; });
    const uint32_t nb = (nt + kPackBlock - 1u) / kPackBlock;
    static const unsigned kDecodeThreads = (unsigned)std::min(32, std::max(1, env_int("JB_DECODE_THREADS", 8)));
    static const bool avx512 = __builtin_cpu_supports("avx512f") && env_int("JB_DECODE_AVX512", 1) != 0;
    const unsigned nth = nt >= (1u << 18) ? kDecodeThreads : 1u;
    auto work = [&](unsigned t) {
        const uint32_t b0 = (uint32_t)((uint64_t)nb * t / nth), b1 = (uint32_t)((uint64_t)nb * (t + 1) / nth);
        for (uint32_t b = b0; b < b1; b++) {
            const uint32_t i0 = b * kPackBlock, i1 = std::min(nt, i0 + kPackBlock);
            uint64_t e = base + hdr[b];
            if (avx512) {
                unpack_block_avx512<T>(pk, i0, i1, e, side, nside, base, os, oe);
                continue;
            }
            for (uint32_t i = i0; i < i1; i++) {
                uint64_t s;
                unpack_one(pk[i], i, side, nside, base, s, e);
                __builtin_nontemporal_store((T)s, os + i);
                __builtin_nontemporal_store((T)e, oe + i);
            }
        }
        __builtin_ia32_sfence();  // (the streaming stores are visible before the thread is joined)
    };
    run_threads(nth, work);
}

// Text already in pinned memory (jb_host_alloc): the pieces are copied to the device
// straight from it, without staging.
struct HostAlloc { uintptr_t a; size_t n; };
static std::mutex g_host_mu;
static std::vector<HostAlloc> g_host;  // jb_host_alloc allocations
static bool host_pinned(const void* p, uint64_t n) {
    const uintptr_t x = (uintptr_t)p;
    std::lock_guard<std::mutex> g(g_host_mu);
    for (const HostAlloc& h : g_host)
        if (x >= h.a && x + n <= h.a + h.n) return true;
    return false;
}


// Cut documents [d0, d1) of a host batch on one device: appends spans to `out`, or
// with `mask` writes the range's boundary bits into the caller's masks (out->n counts
// the tokens).  A range that fits k_small is one launch.  A larger one is cut in
// pieces of whole documents (JB_PIECE_MIB, default 64 MiB; a longer document is a
// piece of its own) as a three-stage pipeline over three streams: piece k+1's text is
// staged into pinned memory and copied up on cstream while piece k's kernels run on
// `stream` and piece k-1's spans (or final mask words) come back on dstream, then are
// widened to u64 batch offsets into `out` by kCopyThreads host threads.
static int cut_range(Device* d, const uint8_t* text, const uint64_t* doc_off, uint32_t d0, uint32_t d1, bool hmm,
                     SpanBuf* out, const MaskDst* mask) {
    if (d0 >= d1) return JB_OK;
    const uint64_t r0 = doc_off[d0], rbytes = doc_off[d1] - r0;
    const uint32_t ndr = d1 - d0;
    // mask geometry: range word j = caller word rw + j; the range's first bit is bit rsh of word 0
    const uint64_t rrel = mask ? r0 - mask->batch0 : 0, rw = rrel >> 6, rsh = rrel & 63u;
    const uint64_t nw = mask ? (rsh + rbytes + 63u) >> 6 : 0;
    int rc;
    // (small batches: k_small on its own stream and buffers, coalesced across callers, without
    // the device lock that the pipeline below holds)
    if (d->lc.small_max && rbytes <= d->lc.small_max && ndr <= kSmallDocs) {
        if (!mask) return cut_small(d, text, doc_off + d0, ndr, hmm, out);
        SpanBuf tmp;
        if ((rc = cut_small(d, text, doc_off + d0, ndr, hmm, &tmp))) {
            tmp.release();
            return rc;
        }
        std::vector<uint64_t> ws(2 * nw, 0ull);
        for (size_t k = 0; k < tmp.n; k++) {
            const uint64_t a = tmp.s[k] - r0 + rsh, b = tmp.e[k] - 1 - r0 + rsh;
            ws[a >> 6] |= 1ull << (a & 63u);
            ws[nw + (b >> 6)] |= 1ull << (b & 63u);
        }
        put_mask_words(mask, rw, nw, 0, nw, ws.data(), ws.data() + nw);
        out->n += tmp.n;
        tmp.release();
        return JB_OK;
    }
    std::lock_guard<std::mutex> g(d->mu);
    HIPCHK(hipSetDevice(d->ordinal));
    for (uint32_t k = d0; k < d1; k++)
        if (doc_off[k + 1] - doc_off[k] >= (1ull << 31))
            return fail(JB_ELIMIT, "document %u is %llu bytes (limit 2 GiB)", k,
                        (unsigned long long)(doc_off[k + 1] - doc_off[k]));
    const uint64_t kPiece = d->piece_bytes;
    struct Piece { uint32_t d0, d1; uint64_t off, slot; };  // documents, device text offset, offsets slot
    std::vector<Piece> pcs;
    uint64_t dev_bytes = 0, slots = 0, maxb = 0;
    uint32_t maxd = 0;
    for (uint32_t a = d0; a < d1;) {
        uint32_t b = a + 1;
        while (b < d1 && doc_off[b + 1] - doc_off[a] <= kPiece) b++;
        const uint64_t len = doc_off[b] - doc_off[a];
        pcs.push_back(Piece{a, b, dev_bytes, slots});
        dev_bytes += (len + 64 + 255) & ~255ull;  // 64 zero bytes after each piece, 256-byte aligned starts
        slots += b - a + 1;
        maxb = std::max(maxb, len);
        maxd = std::max(maxd, b - a);
        a = b;
    }
    const size_t np = pcs.size();
    const bool pinned_in = host_pinned(text + r0, rbytes);
    if ((rc = grow_dev(&d->text, &d->text_cap, dev_bytes)) || (rc = grow_dev(&d->doc_off, &d->doc_cap, slots)) ||
        (rc = grow_pinned(&d->h_misc, &d->h_misc_cap, slots)) ||
        (rc = grow_mapped(&d->h_pcnt, &d->d_pcnt, &d->h_pcnt_cap, (uint64_t)np * kSnapWords)) ||
        (!pinned_in && (rc = grow_pinned(&d->h_text, &d->h_text_cap, dev_bytes))) ||
        (rc = ensure_work(d, maxb, maxd)))
        return rc;
    for (auto* v : {&d->ev_h2d, &d->ev_comp, &d->ev_d2h})
        while (v->size() < np) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            v->push_back(e);
        }
    const bool pack = !mask && d->span_pack;
    const uint32_t side_cap = pack_side_cap(maxb);
    if (!mask) {
        for (auto& o : d->outs) {
            uint64_t ct = o.cap_tok, cd = o.cap_docs;
            if ((rc = grow_dev(&o.ts, &ct, maxb + 4)) || (rc = grow_dev(&o.te, &o.cap_tok, maxb + 4)) ||
                (rc = grow_dev(&o.dt, &cd, (uint64_t)maxd + 2)))
                return rc;
            o.cap_docs = (uint32_t)cd;
            if (pack && ((rc = grow_dev(&o.pk, &o.cap_pk, maxb + 4)) ||
                         (rc = grow_dev(&o.phdr, &o.cap_phdr, (maxb + 4) / kPackBlock + 2)) ||
                         (rc = grow_dev(&o.pside, &o.cap_pside, side_cap))))
                return rc;
        }
    } else {
        if ((rc = grow_dev(&d->d_mask, &d->mask_cap, 2 * nw)) || (rc = grow_pinned(&d->h_mask, &d->mask_cap_h, 2 * nw)))
            return rc;
        HIPCHK(run_zero(d->d_mask, 2 * nw * 8, d->stream));
    }
    {
        std::lock_guard<std::mutex> g(d->stats_mu);
        d->last_small = false;
    }
    jb_stats acc{};
    auto drain = [&](int code) {  // an error with work in flight: let the streams finish first
        (void)hipStreamSynchronize(d->cstream);
        (void)hipStreamSynchronize(d->stream);
        (void)hipStreamSynchronize(d->dstream);
        return code;
    };
    std::vector<uint32_t> ntok(np, 0);
    std::vector<std::pair<uint64_t, uint64_t>> words(np);  // mask words each piece copies back
    static const bool tdbg2 = env_int("JB_DEBUG", 0) >= 2;  // per-piece event clocks
    std::vector<hipEvent_t> tev;  // t0, then per piece: H2D done, kernels done, results back
    auto tmark = [&](size_t i, hipStream_t st) {
        if (tdbg2 && i < tev.size()) (void)hipEventRecord(tev[i], st);
    };
    if (tdbg2) {
        tev.resize(1 + 3 * np);
        for (auto& e : tev) (void)hipEventCreate(&e);
        (void)hipEventRecord(tev[0], d->stream);
    }
    uint64_t mask_done = 0;

    static const bool nt_stage = env_int("JB_NT_STAGE", 1) != 0;  // (A/B switch)
    auto stage = [&](size_t k) -> int {
        const Piece& p = pcs[k];
        const uint64_t pb = doc_off[p.d0], len = doc_off[p.d1] - pb;
        for (uint32_t j = 0; j <= p.d1 - p.d0; j++) d->h_misc[p.slot + j] = doc_off[p.d0 + j] - pb;
        HIPCHK(hipMemcpyAsync(d->doc_off + p.slot, d->h_misc + p.slot, (uint64_t)(p.d1 - p.d0 + 1) * 8,
                              hipMemcpyHostToDevice, d->cstream));
        if (pinned_in) {
            // (the 64 zero bytes after the piece come from pinned zeros: a memset would be a
            // kernel, queued behind the persistent k_zh for CUs, and the copies behind it)
            if (len) HIPCHK(hipMemcpyAsync(d->text + p.off, text + pb, len, hipMemcpyHostToDevice, d->cstream));
            HIPCHK(hipMemcpyAsync(d->text + p.off + len, d->h_zero, 64, hipMemcpyHostToDevice, d->cstream));
        } else {
            // kCopyThreads threads stage their share in 4 MiB sub-pieces and queue each one's copy at once
            const uint64_t total = len + 64, kSub = 4ull << 20;
            memset(d->h_text + p.off + len, 0, 64);
            const unsigned nth = total >= (16ull << 20) ? kCopyThreads : 1u;
            const uint64_t share = ((total + nth - 1) / nth + 4095) & ~4095ull;
            std::atomic<int> err{0};
            auto work = [&](unsigned t) {
                if (hipSetDevice(d->ordinal) != hipSuccess) err = 1;
                const uint64_t lo = std::min(total, t * share), hi = std::min(total, lo + share);
                for (uint64_t o = lo; o < hi; o += kSub) {
                    const uint64_t l = std::min(kSub, hi - o);
                    if (o < len) {
                        if (nt_stage) nt_copy(d->h_text + p.off + o, text + pb + o, std::min(l, len - o));
                        else memcpy(d->h_text + p.off + o, text + pb + o, std::min(l, len - o));
                    }
                    if (hipMemcpyAsync(d->text + p.off + o, d->h_text + p.off + o, l, hipMemcpyHostToDevice,
                                       d->cstream) != hipSuccess)
                        err = 1;
                }
            };
            run_threads(nth, work);
            if (err) return fail(JB_EDEVICE, "H2D copy failed");
        }
        HIPCHK(hipEventRecord(d->ev_h2d[k], d->cstream));
        tmark(1 + 3 * k, d->cstream);
        return JB_OK;
    };
    auto compute = [&](size_t k) -> int {
        const Piece& p = pcs[k];
        const uint64_t pb = doc_off[p.d0], len = doc_off[p.d1] - pb;
        HIPCHK(hipStreamWaitEvent(d->stream, d->ev_h2d[k], 0));
        Work w = d->w;
        MaskOut mo{nullptr, nullptr, 0};
        if (mask) {
            mo = MaskOut{d->d_mask, d->d_mask + nw, rsh + (pb - r0)};
        } else {
            if (k >= (size_t)Device::kSets) HIPCHK(hipStreamWaitEvent(d->stream, d->ev_d2h[k - Device::kSets], 0));
            const Device::OutSet& o = d->outs[k % Device::kSets];
            w.tok_start = o.ts;
            w.tok_end = o.te;
            w.doc_tok = o.dt;
        }
        int r;
        if ((r = launch(d, w, d->text + p.off, len, d->doc_off + p.slot, p.d1 - p.d0, hmm, d->stream,
                        mask ? &mo : nullptr)))
            return r;
        d->last_nbytes = len;
        if (pack) {  // the spans packed for the trip back: 4 B per token (k_span_pack)
            const Device::OutSet& o = d->outs[k % Device::kSets];
            const hipError_t ep = run_span_pack(o.ts, o.te, d->w.counters, o.pk, o.phdr, o.pside, side_cap,
                                                len + 1, d->stream);
            if (ep != hipSuccess) return fail(JB_EDEVICE, "k_span_pack: %s", hipGetErrorString(ep));
        }
        // counters and block counts by a kernel into mapped memory: a copy-engine transfer here
        // would queue behind the bulk copies of later pieces and hold up this stream
        const hipError_t es = run_snap(d->w, len, d->d_pcnt + k * kSnapWords, d->stream);
        if (es != hipSuccess) return fail(JB_EDEVICE, "k_snap: %s", hipGetErrorString(es));
        HIPCHK(hipEventRecord(d->ev_comp[k], d->stream));
        tmark(2 + 3 * k, d->stream);
        return JB_OK;
    };
    auto collect = [&](size_t k) -> int {  // piece k's kernels are done: queue its results' copy back
        const Piece& p = pcs[k];
        HIPCHK(hipEventSynchronize(d->ev_comp[k]));
        const volatile uint32_t* c = d->h_pcnt + k * kSnapWords;
        if (c[CNT_ERR] & 2u) return fail(JB_EDEVICE, "k_long: a phase wait gave up (no progress for JB_LONG_WAIT_US)");
        if (c[CNT_ERR] & 4u) return fail(JB_EDEVICE, "internal: k_span_pack's side list overflowed");
        if (c[CNT_ERR]) return fail(JB_EPANIC, "a Han block has no DAG path (the reference panics in cutDAG)");
        if (c[CNT_NTOK] != c[CNT_NTOKE])
            return fail(JB_EDEVICE, "internal: %u token starts vs %u ends", c[CNT_NTOK], c[CNT_NTOKE]);
        const uint32_t nt = ntok[k] = c[CNT_NTOK];
        HIPCHK(hipStreamWaitEvent(d->dstream, d->ev_comp[k], 0));
        if (!mask) {
            Device::OutSet& o = d->outs[k % Device::kSets];
            uint64_t hd = o.hcap_docs;
            int r;
            if ((!pack && (r = grow_pinned(&o.hs, &o.hcap_tok, 2ull * nt + 2))) ||
                (r = grow_pinned(&o.hdt, &hd, (uint64_t)(p.d1 - p.d0) + 2)))
                return r;
            o.hcap_docs = (uint32_t)hd;
            if (pack) {
                const uint32_t nside = c[CNT_SIDE], nb = (nt + kPackBlock - 1u) / kPackBlock;
                if ((r = grow_pinned(&o.hpk, &o.hcap_pk, (uint64_t)nt + 1)) ||
                    (r = grow_pinned(&o.hhdr, &o.hcap_hdr, (uint64_t)nb + 1)) ||
                    (r = grow_pinned(&o.hside, &o.hcap_side, (uint64_t)nside + 1)))
                    return r;
                if (nt) {
                    HIPCHK(hipMemcpyAsync(o.hpk, o.pk, (uint64_t)nt * 2, hipMemcpyDeviceToHost, d->dstream));
                    HIPCHK(hipMemcpyAsync(o.hhdr, o.phdr, (uint64_t)nb * 4, hipMemcpyDeviceToHost, d->dstream));
                }
                if (nside)
                    HIPCHK(hipMemcpyAsync(o.hside, o.pside, (uint64_t)nside * 16, hipMemcpyDeviceToHost, d->dstream));
            } else if (nt) {
                HIPCHK(hipMemcpyAsync(o.hs, o.ts, (uint64_t)nt * 4, hipMemcpyDeviceToHost, d->dstream));
                HIPCHK(hipMemcpyAsync(o.hs + nt, o.te, (uint64_t)nt * 4, hipMemcpyDeviceToHost, d->dstream));
            }
            HIPCHK(hipMemcpyAsync(o.hdt, o.dt, (uint64_t)(p.d1 - p.d0 + 1) * 8, hipMemcpyDeviceToHost, d->dstream));
        } else {
            // final words: those before the word that holds the next piece's first bit
            const uint64_t hi = k + 1 < np ? (rsh + (doc_off[pcs[k + 1].d0] - r0)) >> 6 : nw;
            const uint64_t lo = mask_done;
            if (hi > lo) {
                HIPCHK(hipMemcpyAsync(d->h_mask + lo, d->d_mask + lo, (hi - lo) * 8, hipMemcpyDeviceToHost,
                                      d->dstream));
                HIPCHK(hipMemcpyAsync(d->h_mask + nw + lo, d->d_mask + nw + lo, (hi - lo) * 8,
                                      hipMemcpyDeviceToHost, d->dstream));
                mask_done = hi;
            }
            words[k] = {lo, std::max(lo, hi)};
        }
        HIPCHK(hipEventRecord(d->ev_d2h[k], d->dstream));
        tmark(3 + 3 * k, d->dstream);
        return JB_OK;
    };
    auto finish = [&](size_t k) -> int {  // piece k's results have landed: into the caller's arrays
        const Piece& p = pcs[k];
        HIPCHK(hipEventSynchronize(d->ev_d2h[k]));
        const uint32_t nt = ntok[k];
        {
            const volatile uint32_t* c = d->h_pcnt + k * kSnapWords;
            acc.tokens += nt;
            acc.long_blocks += c[CNT_NLONG];
            acc.viterbi_ties += c[CNT_TIES];
            acc.blocks += (uint64_t)c[CNT_CLEAR] | (uint64_t)c[CNT_CLEAR + 1] << 32;
            acc.zh_blocks += (uint64_t)c[CNT_CLEAR + 2] | (uint64_t)c[CNT_CLEAR + 3] << 32;
        }
        if (mask) {
            put_mask_words(mask, rw, nw, words[k].first, words[k].second, d->h_mask, d->h_mask + nw);
            out->n += nt;
            return JB_OK;
        }
        const Device::OutSet& o = d->outs[k % Device::kSets];
        const bool write = out->reserve(out->n + nt);
        if (!write && !out->external) return fail(JB_ENOMEM, "out of host memory for %u tokens", nt);
        if (write && pack) {
            const uint32_t nside = d->h_pcnt[k * kSnapWords + CNT_SIDE];
            if (out->s32)
                unpack_spans(o.hpk, o.hhdr, o.hside, nside, nt, doc_off[p.d0] - out->b32, out->s32 + out->n,
                             out->e32 + out->n);
            else
                unpack_spans(o.hpk, o.hhdr, o.hside, nside, nt, doc_off[p.d0], out->s + out->n, out->e + out->n);
        } else if (write && out->s32) {
            const uint32_t b = (uint32_t)(doc_off[p.d0] - out->b32);
            uint32_t* const os = out->s32 + out->n;
            uint32_t* const oe = out->e32 + out->n;
            const uint32_t* const hs = o.hs;
            const unsigned nth = nt >= (1u << 20) ? kCopyThreads : 1u;
            auto work = [&](unsigned t) {
                const uint64_t a = (uint64_t)nt * t / nth, c = (uint64_t)nt * (t + 1) / nth;
                for (uint64_t i = a; i < c; i++) os[i] = b + hs[i];
                for (uint64_t i = a; i < c; i++) oe[i] = b + hs[nt + i];
            };
            run_threads(nth, work);
        } else if (write) {
            const uint64_t base = doc_off[p.d0];
            uint64_t* const os = out->s + out->n;
            uint64_t* const oe = out->e + out->n;
            const uint32_t* const hs = o.hs;
            const unsigned nth = nt >= (1u << 20) ? kCopyThreads : 1u;
            auto work = [&](unsigned t) {
                const uint64_t a = (uint64_t)nt * t / nth, b = (uint64_t)nt * (t + 1) / nth;
                for (uint64_t i = a; i < b; i++) os[i] = base + hs[i];
                for (uint64_t i = a; i < b; i++) oe[i] = base + hs[nt + i];
            };
            run_threads(nth, work);
        } else {  // caller arrays too small: count the rest, write nothing more
            out->needed = out->n + nt;
            out->cap = 0;
        }
        out->n += nt;
        for (uint32_t j = 0; j < p.d1 - p.d0; j++) out->per_doc.push_back(o.hdt[j + 1] - o.hdt[j]);
        return JB_OK;
    };
    static const bool tdbg = getenv("JB_DEBUG") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto c0 = now();
    // Three threads: the stager stages piece after piece (every piece has its own pinned
    // and device text region); the launcher queues piece k's kernels once its copy is
    // queued (and, for spans, once the output set it reuses has been copied back); this
    // thread hands results back in order.  Each publishes its progress under `pm`.
    std::mutex pm;
    std::condition_variable pcv;
    size_t staged = 0, launched = 0, collected = 0;
    int prc = JB_OK;
    std::string perr;
    bool stop = false;
    double t_stage = 0, t_launch = 0;
    auto publish = [&](size_t* ctr, size_t v, int r) {
        std::lock_guard<std::mutex> l(pm);
        if (r && prc == JB_OK) {
            prc = r;
            perr = g_err;
        }
        if (!r) *ctr = v;
        pcv.notify_all();
    };
    auto wait_for = [&](const size_t* ctr, size_t v) -> bool {  // false: an error or stop
        std::unique_lock<std::mutex> l(pm);
        pcv.wait(l, [&] { return *ctr >= v || prc != JB_OK || stop; });
        return *ctr >= v;
    };
    constexpr size_t kAhead = 3;
    std::thread stager([&] {
        const auto a = now();
        if (hipSetDevice(d->ordinal) != hipSuccess) {
            publish(&staged, 0, fail(JB_EDEVICE, "hipSetDevice(%d) failed", d->ordinal));
            return;
        }
        for (size_t k = 0; k < np; k++) {
            {
                std::lock_guard<std::mutex> l(pm);
                if (stop || prc) break;
            }
            // at most kAhead pieces' copies queued beyond the last piece whose kernels are done: a
            // deeper queue of bulk copies (pinned input queues all of them at once) delayed the
            // first pieces' kernels by 13 ms, everything on the device waiting behind the copies
            if (k >= kAhead && !wait_for(&collected, k - kAhead + 1)) break;
            const int r = stage(k);
            publish(&staged, k + 1, r);
            if (r) break;
        }
        t_stage = ms(a, now());
    });
    std::thread launcher([&] {
        const auto a = now();
        if (hipSetDevice(d->ordinal) != hipSuccess) {
            publish(&launched, 0, fail(JB_EDEVICE, "hipSetDevice(%d) failed", d->ordinal));
            return;
        }
        for (size_t k = 0; k < np; k++) {
            if (!wait_for(&staged, k + 1)) break;
            if (!mask && k >= (size_t)Device::kSets && !wait_for(&collected, k - Device::kSets + 1)) break;
            const int r = compute(k);
            publish(&launched, k + 1, r);
            if (r) break;
        }
        t_launch = ms(a, now());
    });
    auto stop_threads = [&] {
        {
            std::lock_guard<std::mutex> l(pm);
            stop = true;
        }
        pcv.notify_all();
        stager.join();
        launcher.join();
    };
    auto bail = [&](int code, const std::string& msg) {  // stop the other threads, drain, keep the message
        stop_threads();
        drain(code);
        g_err = msg;
        return code;
    };
    double t_wait = 0, t_collect = 0, t_finish = 0;
    auto timed = [&](double& accm, auto&& fn) {
        const auto a = now();
        const int r = fn();
        accm += ms(a, now());
        return r;
    };
    for (size_t k = 0; k < np; k++) {
        {
            const auto a = now();
            const bool ok = wait_for(&launched, k + 1);
            t_wait += ms(a, now());
            if (!ok) {
                int code;
                std::string msg;
                {
                    std::lock_guard<std::mutex> l(pm);
                    code = prc ? prc : JB_EDEVICE;
                    msg = prc ? perr : "host pipeline stopped";
                }
                return bail(code, msg);
            }
        }
        if ((rc = timed(t_collect, [&] { return collect(k); }))) return bail(rc, g_err);
        publish(&collected, k + 1, JB_OK);
        if (k >= 1 && (rc = timed(t_finish, [&] { return finish(k - 1); }))) return bail(rc, g_err);
    }
    stop_threads();
    if ((rc = finish(np - 1))) return drain(rc);
    d->acc = acc;
    d->acc_valid = true;
    if (tdbg2) {
        (void)hipDeviceSynchronize();
        fprintf(stderr, "[jb] piece: H2D done / kernels done / results back (ms from the start)\n");
        for (size_t k = 0; k < np; k++) {
            float a = 0, b = 0, c = 0;
            (void)hipEventElapsedTime(&a, tev[0], tev[1 + 3 * k]);
            (void)hipEventElapsedTime(&b, tev[0], tev[2 + 3 * k]);
            (void)hipEventElapsedTime(&c, tev[0], tev[3 + 3 * k]);
            fprintf(stderr, "[jb]   %2zu: %7.2f %7.2f %7.2f\n", k, a, b, c);
        }
        for (auto& e : tev) (void)hipEventDestroy(e);
    }
    if (tdbg)
        fprintf(stderr, "[jb] host range %.1f MiB (%s%s) in %zu pieces: %.2f ms (stager %.2f, launcher %.2f; here: "
                        "waits for launches %.2f, kernels %.2f, results %.2f)\n", rbytes / 1048576.0,
                mask ? "masks" : "spans", pinned_in ? ", pinned input" : "", np, ms(c0, now()), t_stage, t_launch,
                t_wait, t_collect, t_finish);
    return JB_OK;
}

// Contiguous byte-balanced document ranges: part k owns
// documents [cut[k], cut[k+1]); cut[0] = 0, cut[nparts] = ndocs.  The cut
// before part k is the first document that does not end at or before byte
// total * k / nparts (jieba-go_amd/python/shard.py restates the rule for
// bench.py's one-process-per-GPU runs).
extern "C" int jb_shard_bounds(const uint64_t* doc_off, uint32_t ndocs, uint32_t nparts, uint32_t* cut) {
    if (!cut || nparts == 0 || (!doc_off && ndocs)) return fail(JB_EINVAL, "jb_shard_bounds: bad argument");
    for (uint32_t k = 0; k < ndocs; k++)
        if (doc_off[k + 1] < doc_off[k]) return fail(JB_EINVAL, "doc_off not monotonic at %u", k);
    for (uint32_t k = 0; k <= nparts; k++) cut[k] = ndocs;
    cut[0] = 0;
    const uint64_t total = ndocs ? doc_off[ndocs] - doc_off[0] : 0;
    for (uint32_t k = 1; k < nparts; k++) {
        // (total * k fits u64: total < 2^56 for any batch a host holds)
        const uint64_t target = (ndocs ? doc_off[0] : 0) + total * k / nparts;
        uint32_t lo = cut[k - 1];
        while (lo < ndocs && doc_off[lo + 1] <= target) lo++;
        cut[k] = lo;
    }
    return JB_OK;
}

// The first Han-run start of the document [lo, hi) at or after pos (and after lo):
// a position q where a Han rune begins (Go's DecodeRune over the document) and the
// rune before it is not Han; hi if there is none.  Cutting a document there is
// exact: splitText's blocks (tokenizer.go:165-210) are the same in both parts, and
// blocks are cut independently (tokenizer.go:158-160).  Decoding from lo lands on
// every lead byte of a valid sequence (a continuation byte is never a lead byte), so
// the rune before q is the valid 2-4 byte sequence that ends at q if there is one,
// else the single byte q-1.
static uint64_t han_run_start(const uint8_t* t, uint64_t lo, uint64_t hi, uint64_t pos) {
    auto dec = [&](uint64_t q, uint32_t* r) -> uint32_t {
        const uint64_t lim = std::min<uint64_t>(4, hi - q);
        uint32_t x = 0;
        for (uint64_t k = 0; k < lim; k++) x |= (uint32_t)t[q + k] << (8 * k);
        return jb_decode(x, (uint32_t)lim, r);
    };
    for (uint64_t q = std::max(pos, lo + 1); q < hi; q++) {
        if (t[q] < 0xE0u) continue;  // Han runes are 3 or 4 bytes long
        uint32_t r;
        if (dec(q, &r) < 3 || !jb_is_han(r)) continue;
        bool prev_han = false;
        if (t[q - 1] >= 0x80u)
            for (uint32_t k = 2; k <= 4; k++) {
                uint32_t pr;
                if (q >= lo + k && dec(q - k, &pr) == k) {
                    prev_han = jb_is_han(pr);
                    break;
                }
            }
        if (!prev_han) return q;
    }
    return hi;
}

extern "C" int jb_split_points(const uint8_t* text, const uint64_t* doc_off, uint32_t ndocs, uint32_t nparts,
                               uint64_t* cut) {
    if (!cut || nparts == 0 || (!doc_off && ndocs)) return fail(JB_EINVAL, "jb_split_points: bad argument");
    for (uint32_t k = 0; k < ndocs; k++)
        if (doc_off[k + 1] < doc_off[k]) return fail(JB_EINVAL, "doc_off not monotonic at %u", k);
    const uint64_t b0 = ndocs ? doc_off[0] : 0, total = ndocs ? doc_off[ndocs] - b0 : 0;
    if (total && !text) return fail(JB_EINVAL, "jb_split_points: null text");
    cut[0] = b0;
    cut[nparts] = b0 + total;
    uint32_t j = 0;
    uint64_t known = 0, known_q = 0;  // in document j: the first Han-run start at or after `known` is known_q
    bool have = false;
    for (uint32_t k = 1; k < nparts; k++) {
        const uint64_t target = std::max(b0 + total * k / nparts, cut[k - 1]);
        const uint32_t j0 = j;
        while (j < ndocs && doc_off[j + 1] <= target) j++;
        if (j != j0) have = false;
        if (j >= ndocs) {
            cut[k] = b0 + total;
            continue;
        }
        if (doc_off[j] >= target) {
            cut[k] = doc_off[j];
            continue;
        }
        if (!have || target < known || target > known_q) {
            known = target;
            known_q = han_run_start(text, doc_off[j], doc_off[j + 1], target);
            have = true;
        }
        cut[k] = known_q;  // (the next document's start when the rest of this one has none)
    }
    return JB_OK;
}

// Cut units: documents, or parts of documents cut at Han-run starts (han_run_start),
// so that one large document spreads over several devices and over
// several pipeline pieces within a device.  Unit u is bytes [off[u], off[u+1]) of
// document doc[u]; device k owns units [dev[k], dev[k+1]).
struct Units {
    std::vector<uint64_t> off;
    std::vector<uint32_t> doc;
    std::vector<uint32_t> dev;
};

// Shard the batch over the devices and cut, one host thread per device.  With one
// device and no document longer than its pipeline piece the units are the
// documents; otherwise the device ranges are byte-balanced (jb_split_points) and
// documents longer than a piece are cut into units at Han-run starts.  sb[k]
// receives device k's spans and tokens per unit; *unit_doc (left empty when units
// are documents) maps units to documents.  The caller holds ctx->lock (shared for
// cuts, exclusive inside jb_add_word).
static int cut_sharded(jb_ctx* ctx, const uint8_t* text, const uint64_t* doc_off, uint32_t ndocs, int hmm,
                       std::vector<SpanBuf>* sbp, const MaskDst* mask = nullptr,
                       std::vector<uint32_t>* unit_doc = nullptr) {
    if (ndocs && !text && doc_off[ndocs] > doc_off[0]) return fail(JB_EINVAL, "null text");
    for (uint32_t k = 0; k < ndocs; k++)
        if (doc_off[k + 1] < doc_off[k]) return fail(JB_EINVAL, "doc_off not monotonic at %u", k);
    std::vector<SpanBuf>& sb = *sbp;
    const size_t nd = ctx->devs.size();
    const uint64_t b0 = ndocs ? doc_off[0] : 0, b1 = ndocs ? doc_off[ndocs] : 0;
    bool split = nd > 1;
    for (uint32_t j = 0; j < ndocs && !split; j++)
        split = doc_off[j + 1] - doc_off[j] > ctx->devs[0]->piece_bytes;
    Units un;
    std::vector<uint64_t> cutb(nd + 1, b0);
    cutb[nd] = b1;
    if (split) {
        int rc0 = jb_split_points(text, doc_off, ndocs, (uint32_t)nd, cutb.data());
        if (rc0) return rc0;
        un.off.reserve((size_t)ndocs + 2 * nd + 1);
        un.doc.reserve((size_t)ndocs + 2 * nd);
        un.dev.assign(nd + 1, 0);
        size_t k = 0;
        auto dev_of = [&](uint64_t pos) {  // the last device whose range starts at or before pos
            while (k + 1 < nd && cutb[k + 1] <= pos && (cutb[k + 1] < b1 || pos >= b1)) {
                k++;
                un.dev[k] = (uint32_t)un.doc.size();
            }
        };
        for (uint32_t j = 0; j < ndocs; j++) {
            uint64_t pos = doc_off[j];
            const uint64_t de = doc_off[j + 1];
            for (;;) {
                dev_of(pos);
                const uint64_t end = std::min(de, k + 1 < nd && cutb[k + 1] > pos ? cutb[k + 1] : de);
                const uint64_t pb = ctx->devs[k]->piece_bytes;
                uint64_t u = pos;
                while (end - u > pb) {  // a longer part: pipeline pieces at Han-run starts
                    const uint64_t q = han_run_start(text, doc_off[j], de, u + pb);
                    if (q >= end) break;
                    un.off.push_back(u);
                    un.doc.push_back(j);
                    u = q;
                }
                un.off.push_back(u);
                un.doc.push_back(j);
                if (end >= de) break;
                pos = end;
            }
        }
        un.off.push_back(b1);
        for (size_t q = k + 1; q <= nd; q++) un.dev[q] = (uint32_t)un.doc.size();
        if (un.doc.size() > 0xFFFFFFFFull) return fail(JB_ELIMIT, "too many cut units");
    }
    const uint64_t* uoff = split ? un.off.data() : doc_off;
    if (unit_doc) {
        unit_doc->clear();
        if (split) *unit_doc = un.doc;
    }
    for (auto& d : ctx->devs) {  // jb_last_stats: only the devices this batch reaches
        std::lock_guard<std::mutex> g(d->stats_mu);
        d->has_stats = false;
    }
    if (mask)  // the words a device range shares with its neighbours are ORed into: clear them first
        for (size_t k = 0; k < nd; k++)
            if (cutb[k] < cutb[k + 1]) {
                mask->s[(cutb[k] - mask->batch0) >> 6] = 0;
                mask->e[(cutb[k] - mask->batch0) >> 6] = 0;
                mask->s[(cutb[k + 1] - 1 - mask->batch0) >> 6] = 0;
                mask->e[(cutb[k + 1] - 1 - mask->batch0) >> 6] = 0;
            }
    std::vector<int> rcs(nd, JB_OK);
    std::vector<std::string> errs(nd);
    auto work = [&](size_t k) {
        const uint32_t u0 = split ? un.dev[k] : (k == 0 ? 0u : ndocs), u1 = split ? un.dev[k + 1] : ndocs;
        if (u0 < u1) {
            rcs[k] = cut_range(ctx->devs[k].get(), text, uoff, u0, u1, hmm != 0, &sb[k], mask);
            if (rcs[k]) errs[k] = g_err;
        }
    };
    if (nd == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 0; k < nd; k++) th.emplace_back(work, k);
        for (auto& t : th) t.join();
    }
    for (size_t k = 0; k < nd; k++)
        if (rcs[k]) return fail(rcs[k], "%s", errs[k].c_str());
    return JB_OK;
}

// doc_tok from the tokens per unit (in unit order over the devices' buffers)
static void fill_doc_tok(const std::vector<SpanBuf>& sb, uint32_t ndocs, uint64_t* doc_tok,
                         const std::vector<uint32_t>& unit_doc) {
    for (uint32_t d = 0; d <= ndocs; d++) doc_tok[d] = 0;
    size_t u = 0;
    for (const auto& b : sb)
        for (uint64_t c : b.per_doc) {
            const uint32_t d = unit_doc.empty() ? (uint32_t)u : unit_doc[u];
            doc_tok[d + 1] += c;
            u++;
        }
    for (uint32_t d = 0; d < ndocs; d++) doc_tok[d + 1] += doc_tok[d];
}

// jb_cut_batch with ctx->lock already held by the caller.
static int cut_batch_locked(jb_ctx* ctx, const uint8_t* text, const uint64_t* doc_off, uint32_t ndocs, int hmm,
                            jb_spans* out) {
    const size_t nd = ctx->devs.size();
    std::vector<SpanBuf> sb(nd);
    auto release_all = [&] {
        for (auto& b : sb) b.release();
    };
    std::vector<uint32_t> unit_doc;
    int rc = cut_sharded(ctx, text, doc_off, ndocs, hmm, &sb, nullptr, &unit_doc);
    if (rc) {
        release_all();
        return rc;
    }
    uint64_t nt = 0;
    for (size_t k = 0; k < nd; k++) nt += sb[k].n;
    out->ntokens = nt;
    out->ndocs = ndocs;
    out->doc_tok = (uint64_t*)malloc(((uint64_t)ndocs + 1) * 8);
    if (nd == 1 || nt == sb[0].n) {  // one device's buffers are the result
        out->start = sb[0].s ? sb[0].s : (uint64_t*)malloc(8);
        out->end = sb[0].e ? sb[0].e : (uint64_t*)malloc(8);
        sb[0].s = sb[0].e = nullptr;
    } else {
        out->start = (uint64_t*)malloc(std::max<uint64_t>(nt, 1) * 8);
        out->end = (uint64_t*)malloc(std::max<uint64_t>(nt, 1) * 8);
        if (out->start && out->end) {
            uint64_t w = 0;
            for (size_t k = 0; k < nd; k++) {
                if (sb[k].n) {
                    memcpy(out->start + w, sb[k].s, sb[k].n * 8);
                    memcpy(out->end + w, sb[k].e, sb[k].n * 8);
                }
                w += sb[k].n;
            }
        }
    }
    if (!out->start || !out->end || !out->doc_tok) {
        release_all();
        jb_spans_free(out);
        return fail(JB_ENOMEM, "out of host memory for %llu tokens", (unsigned long long)nt);
    }
    fill_doc_tok(sb, ndocs, out->doc_tok, unit_doc);
    release_all();
    return JB_OK;
}

extern "C" int jb_cut_batch(jb_ctx* ctx, const uint8_t* text, const uint64_t* doc_off, uint32_t ndocs, int hmm,
                            jb_spans* out) {
    if (!ctx || !out || (!doc_off && ndocs)) return fail(JB_EINVAL, "jb_cut_batch: null argument");
    memset(out, 0, sizeof *out);
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    return cut_batch_locked(ctx, text, doc_off, ndocs, hmm, out);
}

extern "C" int jb_cut_batch_into(jb_ctx* ctx, const uint8_t* text, const uint64_t* doc_off, uint32_t ndocs,
                                 int hmm, uint64_t* start, uint64_t* end, uint64_t cap, uint64_t* doc_tok,
                                 uint64_t* ntokens) {
    if (!ctx || !ntokens || !doc_tok || (!doc_off && ndocs) || (cap && (!start || !end)))
        return fail(JB_EINVAL, "jb_cut_batch_into: null argument");
    *ntokens = 0;
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    const size_t nd = ctx->devs.size();
    std::vector<SpanBuf> sb(nd);
    if (nd == 1) {  // the device writes straight into the caller's arrays
        sb[0].s = start;
        sb[0].e = end;
        sb[0].cap = cap;
        sb[0].external = true;
    }
    auto release_all = [&] {
        for (auto& b : sb) b.release();
    };
    std::vector<uint32_t> unit_doc;
    int rc = cut_sharded(ctx, text, doc_off, ndocs, hmm, &sb, nullptr, &unit_doc);
    if (rc) {
        release_all();
        return rc;
    }
    uint64_t nt = 0;
    for (size_t k = 0; k < nd; k++) nt += sb[k].n;
    *ntokens = nt;
    if (nt > cap) {
        release_all();
        return fail(JB_ELIMIT, "%llu tokens do not fit the %llu-token output arrays", (unsigned long long)nt,
                    (unsigned long long)cap);
    }
    if (nd > 1) {
        uint64_t w = 0;
        for (size_t k = 0; k < nd; k++) {
            if (sb[k].n) {
                memcpy(start + w, sb[k].s, sb[k].n * 8);
                memcpy(end + w, sb[k].e, sb[k].n * 8);
            }
            w += sb[k].n;
        }
    }
    fill_doc_tok(sb, ndocs, doc_tok, unit_doc);
    release_all();
    return JB_OK;
}

extern "C" int jb_cut_batch_into32(jb_ctx* ctx, const uint8_t* text, const uint64_t* doc_off, uint32_t ndocs,
                                   int hmm, uint32_t* start, uint32_t* end, uint64_t cap, uint64_t* doc_tok,
                                   uint64_t* ntokens) {
    if (!ctx || !ntokens || !doc_tok || (!doc_off && ndocs) || (cap && (!start || !end)))
        return fail(JB_EINVAL, "jb_cut_batch_into32: null argument");
    *ntokens = 0;
    const uint64_t b0 = ndocs ? doc_off[0] : 0;
    if (ndocs && doc_off[ndocs] - b0 > 0xFFFFFFFFull)
        return fail(JB_ELIMIT, "jb_cut_batch_into32: a batch of %llu bytes (u32 offsets: under 4 GiB)",
                    (unsigned long long)(doc_off[ndocs] - b0));
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    const size_t nd = ctx->devs.size();
    std::vector<SpanBuf> sb(nd);
    if (nd == 1) {  // the pieces' spans are decoded straight into the caller's arrays
        sb[0].s32 = start;
        sb[0].e32 = end;
        sb[0].b32 = b0;
        sb[0].cap = cap;
        sb[0].external = true;
    }
    auto release_all = [&] {
        for (auto& b : sb) b.release();
    };
    std::vector<uint32_t> unit_doc;
    int rc = cut_sharded(ctx, text, doc_off, ndocs, hmm, &sb, nullptr, &unit_doc);
    if (rc) {
        release_all();
        return rc;
    }
    uint64_t nt = 0;
    for (size_t k = 0; k < nd; k++) nt += sb[k].n;
    *ntokens = nt;
    if (nt > cap) {
        release_all();
        return fail(JB_ELIMIT, "%llu tokens do not fit the %llu-token output arrays", (unsigned long long)nt,
                    (unsigned long long)cap);
    }
    if (nd > 1) {  // (several devices: each one's u64 spans, narrowed here)
        uint64_t w = 0;
        for (size_t k = 0; k < nd; k++) {
            for (uint64_t i = 0; i < sb[k].n; i++) {
                start[w + i] = (uint32_t)(sb[k].s[i] - b0);
                end[w + i] = (uint32_t)(sb[k].e[i] - b0);
            }
            w += sb[k].n;
        }
    }
    fill_doc_tok(sb, ndocs, doc_tok, unit_doc);
    release_all();
    return JB_OK;
}

extern "C" int jb_cut_batch_mask(jb_ctx* ctx, const uint8_t* text, const uint64_t* doc_off, uint32_t ndocs,
                                 int hmm, uint64_t* starts, uint64_t* ends, uint64_t nwords, uint64_t* ntokens) {
    if (!ctx || !ntokens || (!doc_off && ndocs)) return fail(JB_EINVAL, "jb_cut_batch_mask: null argument");
    *ntokens = 0;
    const uint64_t nbytes = ndocs ? doc_off[ndocs] - doc_off[0] : 0;
    const uint64_t need = (nbytes + 63) / 64;
    if (nwords < need) return fail(JB_EINVAL, "jb_cut_batch_mask: %llu words for %llu bytes (want %llu)",
                                   (unsigned long long)nwords, (unsigned long long)nbytes, (unsigned long long)need);
    if (need && (!starts || !ends)) return fail(JB_EINVAL, "jb_cut_batch_mask: null mask");
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    const size_t nd = ctx->devs.size();
    std::vector<SpanBuf> sb(nd);
    const MaskDst m{starts, ends, ndocs ? doc_off[0] : 0};
    int rc = cut_sharded(ctx, text, doc_off, ndocs, hmm, &sb, &m);
    uint64_t nt = 0;
    for (auto& b : sb) {
        nt += b.n;
        b.release();
    }
    if (rc) return rc;
    if (nwords > need) {  // the header promises every word: clear the caller's tail past the batch
        memset(starts + need, 0, (nwords - need) * 8);
        memset(ends + need, 0, (nwords - need) * 8);
    }
    *ntokens = nt;
    return JB_OK;
}

extern "C" int jb_host_alloc(size_t n, void** p) {
    if (!p) return fail(JB_EINVAL, "jb_host_alloc: null argument");
    *p = nullptr;
    const hipError_t e = hipHostMalloc(p, std::max<size_t>(n, 1), hipHostMallocPortable);
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(e == hipErrorOutOfMemory ? JB_ENOMEM : JB_EDEVICE, "hipHostMalloc(%zu): %s", n,
                    hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host.push_back(HostAlloc{(uintptr_t)*p, n});
    return JB_OK;
}

extern "C" void jb_host_free(void* p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        for (size_t i = 0; i < g_host.size(); i++)
            if (g_host[i].a == (uintptr_t)p) {
                g_host.erase(g_host.begin() + (long)i);
                break;
            }
    }
    (void)hipHostFree(p);
}

extern "C" int jb_cut(jb_ctx* ctx, const uint8_t* text, size_t len, int hmm, jb_spans* out) {
    const uint64_t off[2] = {0, (uint64_t)len};
    static const uint8_t empty[1] = {0};
    return jb_cut_batch(ctx, text ? text : empty, off, 1, hmm, out);
}

extern "C" void jb_spans_free(jb_spans* s) {
    if (!s) return;
    free(s->start);
    free(s->end);
    free(s->doc_tok);
    memset(s, 0, sizeof *s);
}

static int cut_device(jb_ctx* ctx, const uint8_t* d_text, uint64_t nbytes, const uint64_t* d_doc_off,
                      uint32_t ndocs, int hmm, void* stream, uint32_t* o_start, uint32_t* o_end, uint64_t* o_doc_tok,
                      uint64_t* o_ntok, uint32_t** d_start, uint32_t** d_end, uint64_t** d_doc_tok, uint64_t** d_ntok) {
    if (!ctx || (!d_text && nbytes) || !d_doc_off) return fail(JB_EINVAL, "jb_cut_device: null argument");
    if (nbytes >= (1ull << 31)) return fail(JB_ELIMIT, "device batch of %llu bytes (limit 2 GiB)",
                                            (unsigned long long)nbytes);
    if (((uintptr_t)d_text & 15u) != 0) return fail(JB_EINVAL, "d_text must be 16-byte aligned");
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    for (size_t k = 1; k < ctx->devs.size(); k++) {
        std::lock_guard<std::mutex> g(ctx->devs[k]->stats_mu);
        ctx->devs[k]->has_stats = false;
    }
    Device* d = ctx->devs[0].get();
    std::lock_guard<std::mutex> g(d->mu);
    HIPCHK(hipSetDevice(d->ordinal));
    int rc;
    if ((rc = ensure_work(d, nbytes, ndocs))) return rc;
    const hipStream_t s = (hipStream_t)stream;
    if (o_start) {  // caller-owned outputs: the pipeline writes its spans and offsets there
        Work w = d->w;
        w.tok_start = o_start;
        w.tok_end = o_end;
        w.doc_tok = o_doc_tok;
        if ((rc = launch(d, w, d_text, nbytes, d_doc_off, ndocs, hmm != 0, s))) return rc;
        HIPCHK(hipMemcpyAsync(o_ntok, d->w.counters + CNT_NWORDS, 8, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipEventRecord(d->ws_done, s));  // (the counters are workspace too)
        return JB_OK;
    }
    if ((rc = launch(d, d->w, d_text, nbytes, d_doc_off, ndocs, hmm != 0, s))) return rc;
    if (d_start) *d_start = d->w.tok_start;
    if (d_end) *d_end = d->w.tok_end;
    if (d_doc_tok) *d_doc_tok = d->w.doc_tok;
    if (d_ntok) *d_ntok = reinterpret_cast<uint64_t*>(d->w.counters + CNT_NWORDS);
    return JB_OK;
}

extern "C" int jb_cut_device(jb_ctx* ctx, const uint8_t* d_text, uint64_t nbytes, const uint64_t* d_doc_off,
                             uint32_t ndocs, int hmm, void* stream, uint32_t** d_start, uint32_t** d_end,
                             uint64_t** d_doc_tok, uint64_t** d_ntok) {
    return cut_device(ctx, d_text, nbytes, d_doc_off, ndocs, hmm, stream, nullptr, nullptr, nullptr, nullptr, d_start,
                      d_end, d_doc_tok, d_ntok);
}

extern "C" int jb_cut_device_into(jb_ctx* ctx, const uint8_t* d_text, uint64_t nbytes, const uint64_t* d_doc_off,
                                  uint32_t ndocs, int hmm, void* stream, uint32_t* d_start, uint32_t* d_end,
                                  uint64_t cap, uint64_t* d_doc_tok, uint64_t* d_ntok) {
    if (!d_start || !d_end || !d_doc_tok || !d_ntok) return fail(JB_EINVAL, "jb_cut_device_into: null output");
    if (cap < nbytes) return fail(JB_EINVAL, "jb_cut_device_into: cap %llu < nbytes %llu (a batch of n bytes "
                                  "has up to n tokens)", (unsigned long long)cap, (unsigned long long)nbytes);
    return cut_device(ctx, d_text, nbytes, d_doc_off, ndocs, hmm, stream, d_start, d_end, d_doc_tok, d_ntok, nullptr,
                      nullptr, nullptr, nullptr);
}

// ---------------------------------------------------------------------------
// dictionary mutation / introspection
// ---------------------------------------------------------------------------
extern "C" int jb_dict_get(jb_ctx* ctx, const char* word, size_t len, int64_t* freq) {
    if (!ctx || (!word && len)) return fail(JB_EINVAL, "jb_dict_get: null argument");
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    auto it = ctx->im->dict.term_freq.find(std::string(word ? word : "", len));
    if (it == ctx->im->dict.term_freq.end()) return 0;
    if (freq) *freq = it->second;
    return 1;
}

extern "C" int64_t jb_dict_size(jb_ctx* ctx) {
    if (!ctx) return 0;
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    return ctx->im->dict.size;
}

// suggestFreq (tokenizer.go:589-614); the caller holds ctx->lock
static int suggest_freq(jb_ctx* ctx, const char* word, size_t len, int64_t* out) {
    const Dictionary& dict = ctx->im->dict;
    double dsize = (double)dict.size;
    if (dsize < 1.0) dsize = 1.0;
    double freq = 1.0;
    jb_spans sp;
    memset(&sp, 0, sizeof sp);
    static const uint8_t empty[1] = {0};
    const uint64_t off[2] = {0, (uint64_t)len};
    int rc = cut_batch_locked(ctx, word ? (const uint8_t*)word : empty, off, 1, 0, &sp);
    if (rc) return rc;
    for (uint64_t k = 0; k < sp.ntokens; k++) {
        std::string piece;
        if (sp.end[k] - sp.start[k] == 1 && (uint8_t)word[sp.start[k]] >= 0x80) piece = "\xEF\xBF\xBD";
        else piece.assign(word + sp.start[k], sp.end[k] - sp.start[k]);
        auto it = dict.term_freq.find(piece);
        const int64_t pf = it != dict.term_freq.end() ? it->second : 1;
        freq *= (double)pf / dsize;
    }
    jb_spans_free(&sp);
    const int64_t a = (int64_t)(freq * dsize) + 1;
    int64_t b = 1;
    auto it = dict.term_freq.find(std::string(word, len));
    if (it != dict.term_freq.end()) b = it->second;
    *out = a > b ? a : b;
    return JB_OK;
}

extern "C" int jb_suggest_freq(jb_ctx* ctx, const char* word, size_t len, int64_t* freq) {
    if (!ctx || !freq || (!word && len)) return fail(JB_EINVAL, "jb_suggest_freq: null argument");
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    return suggest_freq(ctx, word ? word : "", len, freq);
}

extern "C" int jb_add_log(jb_ctx* ctx, const int64_t* keys, const double* vals, size_t n) {
    if (!ctx || (n && (!keys || !vals))) return fail(JB_EINVAL, "jb_add_log: null argument");
    std::unique_lock<std::shared_mutex> wl(ctx->lock);
    for (size_t i = 0; i < n; i++) ctx->im->dict.log_of[keys[i]] = vals[i];
    return JB_OK;
}

extern "C" int jb_add_word(jb_ctx* ctx, const char* word, size_t len, int64_t freq) {
    if (!ctx || (!word && len)) return fail(JB_EINVAL, "jb_add_word: null argument");
    int rc;
    std::unique_lock<std::shared_mutex> wl(ctx->lock);  // (the reference deadlocks here: :376 + :581)
    if (freq < 1 && (rc = suggest_freq(ctx, word, len, &freq))) return rc;
    // addTerm (tokenizer.go:580-585): no prefix entries are added.  The new dictionary and
    // image are built aside and staged on every device; ctx changes only once all of that
    // worked, so a failure (JB_ELIMIT, JB_EDEVICE, JB_ENOMEM) leaves it as it was.
    try {
        Dictionary nd = ctx->im->dict;
        nd.term_freq[std::string(word, len)] = freq;
        nd.size += freq;
        Image ni;
        std::string err;
        if ((rc = build_image(nd, ctx->im->emit, &ni, &err))) return fail(rc, "%s", err.c_str());
        if (ni.maxlen > 255) return fail(JB_ELIMIT, "dictionary word of %u runes (max 255)", ni.maxlen);
        std::vector<ImageBufs> staged(ctx->devs.size());
        for (size_t k = 0; k < ctx->devs.size() && rc == JB_OK; k++)
            rc = stage_image(ctx->devs[k]->ordinal, ni, &staged[k]);
        if (rc) {
            for (auto& b : staged) {
                (void)hipSetDevice(ctx->devs[&b - staged.data()]->ordinal);
                free_image_bufs(&b);
            }
            return rc;
        }
        for (size_t k = 0; k < ctx->devs.size(); k++) {  // commit
            Device* d = ctx->devs[k].get();
            std::lock_guard<std::mutex> g(d->mu);
            (void)hipSetDevice(d->ordinal);
            (void)hipStreamSynchronize(d->stream);
            if (d->ws_done) (void)hipEventSynchronize(d->ws_done);  // (a jb_cut_device pipeline)
            (void)install_image(d, &staged[k], ni);
        }
        ctx->im->dict = std::move(nd);
        ctx->im->img = std::move(ni);
    } catch (const std::bad_alloc&) {
        return fail(JB_ENOMEM, "out of host memory rebuilding the dictionary");
    }
    return JB_OK;
}

extern "C" int jb_save(jb_ctx* ctx, const char* path) {
    if (!ctx || !path) return fail(JB_EINVAL, "jb_save: null argument");
    std::string data;
    {
        std::shared_lock<std::shared_mutex> rl(ctx->lock);
        save_image(ctx->im->dict, ctx->im->emit, ctx->im->img, &data);
    }
    return write_file(path, data);
}

extern "C" int jb_last_stats(jb_ctx* ctx, jb_stats* out) {
    if (!ctx || !out) return fail(JB_EINVAL, "jb_last_stats: null argument");
    memset(out, 0, sizeof *out);
    uint32_t err = 0;  // CNT_ERR of a device pipeline (jb_cut_device*)
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    for (auto& d : ctx->devs) {
        {
            std::lock_guard<std::mutex> sg(d->stats_mu);
            if (!d->has_stats) continue;  // not reached by the last batch (its counters are older)
            if (d->last_small) {  // k_small's counters came back with its spans (no device lock needed)
                out->tokens += d->small_hdr[SM_NTOK];
                out->blocks += d->small_hdr[SM_BLOCKS];
                out->zh_blocks += d->small_hdr[SM_ZHBLOCKS];
                out->viterbi_ties += d->small_hdr[SM_TIES];
                continue;
            }
        }
        std::lock_guard<std::mutex> g(d->mu);
        if (d->acc_valid) {  // a host range cut in pieces: summed as they came back
            out->tokens += d->acc.tokens;
            out->blocks += d->acc.blocks;
            out->zh_blocks += d->acc.zh_blocks;
            out->long_blocks += d->acc.long_blocks;
            out->viterbi_ties += d->acc.viterbi_ties;
            continue;
        }
        if (!d->w.counters) continue;
        HIPCHK(hipSetDevice(d->ordinal));
        HIPCHK(hipDeviceSynchronize());  // (jb_cut_device may have queued on a caller's stream)
        uint32_t c[CNT_CLEAR];
        HIPCHK(hipMemcpy(c, d->w.counters, sizeof c, hipMemcpyDeviceToHost));
        uint64_t ntok;
        memcpy(&ntok, c + CNT_NWORDS, 8);
        out->tokens += ntok;
        // blocks: the per-tile counts k_mark_walk left in the workspace
        const uint64_t ntiles = (d->last_nbytes + kTileBytes - 1) / kTileBytes;
        if (ntiles) {
            std::vector<uint2> tc(ntiles);
            HIPCHK(hipMemcpy(tc.data(), d->w.tile_cnt, ntiles * sizeof(uint2), hipMemcpyDeviceToHost));
            for (const uint2& t : tc) {
                out->blocks += t.x;
                out->zh_blocks += t.y;
            }
        }
        out->long_blocks += c[CNT_NLONG];
        out->viterbi_ties += c[CNT_TIES];
        err |= c[CNT_ERR];
    }
    // (a host batch already returned these from its own call; a device pipeline reports them here)
    if (err & 2u) return fail(JB_EDEVICE, "k_long: a phase wait gave up (no progress for JB_LONG_WAIT_US)");
    if (err) return fail(JB_EPANIC, "a Han block has no DAG path (the reference panics in cutDAG)");
    return JB_OK;
}

extern "C" int jb_device_status(jb_ctx* ctx, void* stream) {
    if (!ctx) return fail(JB_EINVAL, "jb_device_status: null ctx");
    std::shared_lock<std::shared_mutex> rl(ctx->lock);
    Device* d = ctx->devs[0].get();
    std::lock_guard<std::mutex> g(d->mu);
    if (!d->w.counters) return JB_OK;  // no device pipeline has run
    HIPCHK(hipSetDevice(d->ordinal));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    if (d->ws_done) HIPCHK(hipEventSynchronize(d->ws_done));
    uint32_t e = 0;
    HIPCHK(hipMemcpy(&e, d->w.counters + CNT_ERR, sizeof e, hipMemcpyDeviceToHost));
    if (e & 2u) return fail(JB_EDEVICE, "k_long: a phase wait gave up (no progress for JB_LONG_WAIT_US)");
    if (e) return fail(JB_EPANIC, "a Han block has no DAG path (the reference panics in cutDAG)");
    return JB_OK;
}

// ---------------------------------------------------------------------------
// profiling
// ---------------------------------------------------------------------------
extern "C" int jb_profile_enable(jb_ctx* ctx, int on) {
    if (!ctx) return fail(JB_EINVAL, "null ctx");
    for (auto& d : ctx->devs) d->profile = on != 0;
    return JB_OK;
}

extern "C" int jb_profile_reset(jb_ctx* ctx) {
    if (!ctx) return fail(JB_EINVAL, "null ctx");
    for (auto& d : ctx->devs) {
        (void)hipSetDevice(d->ordinal);
        d->timer.reset();
    }
    return JB_OK;
}

extern "C" int jb_profile_read(jb_ctx* ctx, const char** names, double* ms, uint64_t* launches, int cap) {
    if (!ctx) return fail(JB_EINVAL, "null ctx");
    double tot_ms[K_NUM] = {0};
    uint64_t tot_n[K_NUM] = {0};
    for (auto& d : ctx->devs) {
        (void)hipSetDevice(d->ordinal);
        d->timer.harvest();
        for (int k = 0; k < K_NUM; k++) {
            tot_ms[k] += d->timer.ms[k];
            tot_n[k] += d->timer.launches[k];
        }
    }
    int n = 0;
    for (int k = 0; k < K_NUM && n < cap; k++, n++) {
        if (names) names[n] = kKernelNames[k];
        if (ms) ms[n] = tot_ms[k];
        if (launches) launches[n] = tot_n[k];
    }
    return n;
}
