// jb_image.h — host-side model tables and the device image built from them.
#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "jb_common.h"

namespace jb {

// prefixDictionary (tokenizer.go:381-387) as loaded on the host: the whole
// termFreq map (reachable or not) and size.  Kept for AddWord / suggestFreq
// and for rebuilding the device image.
struct Dictionary {
    std::unordered_map<std::string, int64_t> term_freq;
    int64_t size = 0;
};

// emitP (tokenizer.go:619) restricted to the 4 states the Viterbi reads:
// single-rune keys only (viterbi looks up string(rune), tokenizer.go:689,708).
struct Emission {
    std::unordered_map<uint32_t, double> by_rune[4];  // B, M, E, S
};

// Flat arrays uploaded to every device (layout: jb_common.h).
struct Image {
    std::vector<uint16_t> pagemap;  // JB_NPAGES_MAX
    std::vector<jb_l1> l1;          // npages * 256
    std::vector<double> emit;       // npages * 256 * 4
    std::vector<jb_node> nodes;     // hash capacity (power of two)
    uint32_t npages = 0;
    uint32_t maxlen = 0;            // longest reachable key, runes
    uint64_t nnodes = 0;
    double total = 0;               // math.Log(float64(size))
    double w_absent = 0;            // math.Log(1.0) - total
    int64_t size = 0;
};

double go_log(double x);

// Parse dict.txt-format text with the two reference semantics
// (kind 0: newPrefixDictionaryFromFile, kind 1: buildPrefixDictionary).
// Returns 0 or a negative JB_E* code; err receives a message.
int parse_dictionary(const char* buf, size_t len, int kind, Dictionary* out, std::string* err);
int parse_emission(const char* buf, size_t len, Emission* out, std::string* err);
void build_image(const Dictionary& d, const Emission& e, Image* img);

// Walk the image like the kernel does: returns node id or JB_EMPTY.
uint32_t image_lookup(const Image& img, const uint32_t* runes, size_t n);

}  // namespace jb
