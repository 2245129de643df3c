// cpp_tok_smoke.cpp — a consumer of the C++ mirror of jieba-go's Tokenizer
// (jieba-go_amd/host/tokenizer.hpp, libjbtok.so): NewTokenizer from the working
// directory's prob_emit.json, Cut, CutParallel, CutBatch, AddWord, Save and
// FromImage.  Each call prints one line of tokens joined by '|', which
// tests/test_gpu_parity.py compares with the oracle.
//
//   cpp_tok_smoke DICT TEXTFILE WORD IMAGE   (GPU; run in the directory of prob_emit.json)
//   cpp_tok_smoke --expect-no-device         (no GPU: construction throws JB_EDEVICE)
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "tokenizer.hpp"

static void line(const char* tag, const std::vector<std::string>& toks) {
    std::printf("%s", tag);
    for (const auto& t : toks) std::printf("|%s", t.c_str());
    std::printf("\n");
}

int main(int argc, char** argv) {
    if (argc == 2 && std::strcmp(argv[1], "--expect-no-device") == 0) {
        jb_config cfg;
        std::memset(&cfg, 0, sizeof cfg);
        cfg.dict_buf = "\xe7\x94\xb2 3\n";
        cfg.dict_len = std::strlen(cfg.dict_buf);
        cfg.emit_buf = "{}";
        cfg.emit_len = 2;
        cfg.ndevices = 1;
        try {
            auto tk = jiebago::Tokenizer::Open(cfg);
        } catch (const jiebago::Error& e) {
            if (e.code == JB_EDEVICE) {
                std::printf("no device: %s\n", e.what());
                return 0;
            }
            std::fprintf(stderr, "unexpected error %d: %s\n", e.code, e.what());
            return 1;
        }
        std::fprintf(stderr, "opened without a device\n");
        return 1;
    }
    if (argc != 5) {
        std::fprintf(stderr, "usage: %s DICT TEXTFILE WORD IMAGE | --expect-no-device\n", argv[0]);
        return 2;
    }
    std::ifstream f(argv[2], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    try {
        auto tk = jiebago::Tokenizer::NewTokenizer(argv[1]);
        line("cut_hmm", tk->Cut(text, true));
        line("cut_nohmm", tk->Cut(text, false));
        line("cut_parallel", tk->CutParallel(text, true, 4, false));
        const auto docs = tk->CutBatch({text, "", text}, true);
        for (const auto& d : docs) line("batch_doc", d);
        tk->AddWord(argv[3], 0);
        line("cut_added", tk->Cut(text, true));
        // the caller-log overload, as a Go AddWord passes math.Log (here the library's restatement)
        tk->AddWord("\xe8\xa8\x8e\xe8\xab\x96\xe9\x87\x8f\xe5\xad\x90", 7, [](double x) { return jb_go_log(x); });
        line("cut_added_log", tk->Cut(text, true));
        tk->Save(argv[4]);
        auto img = jiebago::Tokenizer::FromImage(argv[4]);
        line("cut_image", img->Cut(text, true));
    } catch (const jiebago::Error& e) {
        std::fprintf(stderr, "error %d: %s\n", e.code, e.what());
        return 1;
    }
    return 0;
}
