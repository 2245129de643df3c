// tokenizer.hpp — C++ mirror of jieba-go's public Tokenizer API
// (/root/reference/tokenizer.go:52-162, 372-379) over libjiebahip.so.
//
// The Go toolchain is absent from this image, so the host side above the C ABI
// is written in C++ (the reference is compiled code); the cgo binding a Go
// maintainer would add instead is jieba-go_amd/go/tokenizer.go.
//
// Same names and argument meaning as the reference.  Where the reference calls
// log.Fatal / panic (constructor load errors, tokenizer.go:397-416,443,452,656,660;
// the cutDAG slice panic), this mirror throws jiebago::Error.
#pragma once
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "jiebahip.h"

namespace jiebago {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

class Tokenizer {
public:
    // NewTokenizer(dictionaryFile) (tokenizer.go:61): dict.txt semantics, HMM from
    // "prob_emit.json" in the working directory (tokenizer.go:654).
    static std::unique_ptr<Tokenizer> NewTokenizer(const std::string& dictionaryFile, int device = 0);
    // NewJiebaTokenizer() (tokenizer.go:69): decodes "prefix_dictionary.gob" from
    // the working directory (newJiebaPrefixDictionary, tokenizer.go:439-458), size
    // 60_101_967 (tokenizer.go:454).
    static std::unique_ptr<Tokenizer> NewJiebaTokenizer(int device = 0);
    // A serialized image written by Save (no parsing or trie build at start).
    static std::unique_ptr<Tokenizer> FromImage(const std::string& path, int device = 0);
    // Full control (paths, semantics, size override, devices).
    static std::unique_ptr<Tokenizer> Open(const jb_config& cfg);

    ~Tokenizer();
    Tokenizer(const Tokenizer&) = delete;
    Tokenizer& operator=(const Tokenizer&) = delete;

    // Cut (tokenizer.go:151)
    std::vector<std::string> Cut(const std::string& text, bool useHmm);
    // CutParallel (tokenizer.go:81).  Blocks are segmented in parallel on the
    // GPU; numWorkers is accepted for API compatibility.  Output is always in
    // text order (ordered=false in the reference is a block permutation).
    std::vector<std::string> CutParallel(const std::string& text, bool hmm, int numWorkers, bool ordered);
    // Many documents in one device pass (what CutParallel is used for).
    std::vector<std::vector<std::string>> CutBatch(const std::vector<std::string>& docs, bool hmm);
    // AddWord (tokenizer.go:372) without the reference's self-deadlock.  The new
    // weights use the library's restatement of Go's math.Log (jb_go_log).
    void AddWord(const std::string& word, int freq);
    // The same with the caller's logarithm (the Go binding passes math.Log): log(f) of
    // the new frequency and log(size + f) of the new pd.size (addTerm, tokenizer.go:580-585)
    // go to jb_add_log first, so the rebuilt weights use exactly those values.
    void AddWord(const std::string& word, int freq, const std::function<double(double)>& log);
    // Write the current image (AddWord changes included) for FromImage.
    void Save(const std::string& path);

    jb_ctx* handle() { return ctx_; }

private:
    explicit Tokenizer(jb_ctx* c) : ctx_(c) {}
    jb_ctx* ctx_;
};

}  // namespace jiebago
