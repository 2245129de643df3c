// tokenizer.cpp — C++ mirror of jieba-go's Tokenizer over the C ABI.
#include "tokenizer.hpp"

#include <cstring>

namespace jiebago {

static void check(int rc) {
    if (rc != JB_OK) throw Error(rc, jb_last_error());
}

std::unique_ptr<Tokenizer> Tokenizer::Open(const jb_config& cfg) {
    jb_ctx* c = nullptr;
    check(jb_open(&cfg, &c));
    return std::unique_ptr<Tokenizer>(new Tokenizer(c));
}

std::unique_ptr<Tokenizer> Tokenizer::NewTokenizer(const std::string& dictionaryFile, int device) {
    jb_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.dict_path = dictionaryFile.c_str();
    cfg.dict_kind = JB_DICT_TXT;
    cfg.emit_path = "prob_emit.json";
    cfg.device = device;
    cfg.ndevices = 1;
    return Open(cfg);
}

std::unique_ptr<Tokenizer> Tokenizer::NewJiebaTokenizer(int device) {
    jb_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.dict_path = "prefix_dictionary.gob";
    cfg.dict_kind = JB_DICT_GOB;  // size 60,101,967 (tokenizer.go:454)
    cfg.emit_path = "prob_emit.json";
    cfg.device = device;
    cfg.ndevices = 1;
    return Open(cfg);
}

std::unique_ptr<Tokenizer> Tokenizer::FromImage(const std::string& path, int device) {
    jb_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.dict_path = path.c_str();
    cfg.dict_kind = JB_DICT_IMAGE;
    cfg.device = device;
    cfg.ndevices = 1;
    return Open(cfg);
}

Tokenizer::~Tokenizer() { jb_close(ctx_); }

static std::string token_at(const std::string& text, uint64_t s, uint64_t e) {
    // an invalid UTF-8 byte is emitted as "�" by the reference's range loop
    if (e - s == 1 && (unsigned char)text[s] >= 0x80) return "\xEF\xBF\xBD";
    return text.substr(s, e - s);
}

std::vector<std::string> Tokenizer::Cut(const std::string& text, bool useHmm) {
    jb_spans sp;
    check(jb_cut(ctx_, (const uint8_t*)text.data(), text.size(), useHmm ? 1 : 0, &sp));
    std::vector<std::string> out;
    out.reserve(sp.ntokens);
    for (uint64_t k = 0; k < sp.ntokens; k++) out.push_back(token_at(text, sp.start[k], sp.end[k]));
    jb_spans_free(&sp);
    return out;
}

std::vector<std::string> Tokenizer::CutParallel(const std::string& text, bool hmm, int, bool) {
    return Cut(text, hmm);
}

std::vector<std::vector<std::string>> Tokenizer::CutBatch(const std::vector<std::string>& docs, bool hmm) {
    std::string all;
    std::vector<uint64_t> off(1, 0);
    for (const auto& d : docs) {
        all += d;
        off.push_back(all.size());
    }
    jb_spans sp;
    check(jb_cut_batch(ctx_, (const uint8_t*)all.data(), off.data(), (uint32_t)docs.size(), hmm ? 1 : 0, &sp));
    std::vector<std::vector<std::string>> out(docs.size());
    for (size_t d = 0; d < docs.size(); d++)
        for (uint64_t k = sp.doc_tok[d]; k < sp.doc_tok[d + 1]; k++)
            out[d].push_back(token_at(all, sp.start[k], sp.end[k]));
    jb_spans_free(&sp);
    return out;
}

void Tokenizer::AddWord(const std::string& word, int freq) {
    check(jb_add_word(ctx_, word.data(), word.size(), freq));
}

void Tokenizer::AddWord(const std::string& word, int freq, const std::function<double(double)>& log) {
    int64_t f = freq;
    if (freq < 1) check(jb_suggest_freq(ctx_, word.data(), word.size(), &f));  // (tokenizer.go:373-375)
    const int64_t keys[2] = {f, jb_dict_size(ctx_) + f};
    const double vals[2] = {log((double)keys[0]), log((double)keys[1])};
    check(jb_add_log(ctx_, keys, vals, 2));
    check(jb_add_word(ctx_, word.data(), word.size(), f));
}

void Tokenizer::Save(const std::string& path) { check(jb_save(ctx_, path.c_str())); }

}  // namespace jiebago
