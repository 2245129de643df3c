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
    // Caller-supplied math.Log(float64(x)) values (jb_config.log_keys/log_vals,
    // jb_add_log): the weights use them instead of go_log for these x.
    std::unordered_map<int64_t, double> log_of;
};

// math.Log(float64(x)) for the weights (tokenizer.go:503,515-519): the caller's
// value when it gave one for x, else the restatement go_log.
double dict_log(const Dictionary& d, int64_t x);
// The x whose logarithm build_image takes: frequencies of Han-spellable keys, 1, size.
std::vector<int64_t> weight_log_keys(const Dictionary& d);

// emitP (tokenizer.go:619) restricted to the 4 states the Viterbi reads:
// single-rune keys only (viterbi looks up string(rune), tokenizer.go:689,708).
struct Emission {
    std::unordered_map<uint32_t, double> by_rune[4];  // B, M, E, S
};

// Flat arrays uploaded to every device (layout: jb_common.h).
struct Image {
    std::vector<uint16_t> pagemap;  // JB_NPAGES_MAX

    std::vector<double> emit;       // npages * 256 * 4
    std::vector<uint32_t> code;     // npages * 256: dense rune code (0: in no key), by key occurrence
    std::vector<uint64_t> cells;    // double-array trie over codes (level-1 nodes at their codes)
    std::vector<double> wtab;       // distinct weights; [0] = w_absent
    uint32_t npages = 0;
    uint32_t nrows = 0;             // npages * 256: ids of level-1 nodes are their rows
    uint32_t ncells = 0;
    uint32_t ncodes = 0;
    uint32_t maxlen = 0;            // longest reachable key, runes
    uint64_t nnodes = 0;            // reachable keys (all levels)
    double total = 0;               // math.Log(float64(size))
    double w_absent = 0;            // math.Log(1.0) - total
    int64_t size = 0;
};

struct Lookup {
    bool found = false;
    uint32_t fc = JB_FC_ABSENT;
    uint32_t widx = 0;
    uint32_t id = JB_EMPTY;
};

double go_log(double x);

// The hot-row table of an image (JB_HOT_SLOTS values, then JB_HOT_SLOTS u16 tags):
// runes of U+3400..U+9FFF ranked by the summed frequency of the keys that hold them
// (each key's frequency from its weight), placed in descending rank at their slot
// jb_hot_slot(rune) when it is still free.  The value is the rune's l1row entry.
void build_hot_rows(const Image& img, uint64_t* vals, uint16_t* tags);

// Parse dict.txt-format text with the two reference semantics
// (kind 0: newPrefixDictionaryFromFile, kind 1: buildPrefixDictionary).
// Returns 0 or a negative JB_E* code; err receives a message.
int parse_dictionary(const char* buf, size_t len, int kind, Dictionary* out, std::string* err);
// prefix_dictionary.gob (tokenizer.go:439-458): a gob-encoded map[string]int;
// size is left 0 (the caller applies the reference's hard-coded 60,101,967).
int parse_gob_dictionary(const char* buf, size_t len, Dictionary* out, std::string* err);
int parse_emission(const char* buf, size_t len, Emission* out, std::string* err);
// Returns 0 or JB_ELIMIT (too many trie nodes / distinct weights for the packed layout).
int build_image(const Dictionary& d, const Emission& e, Image* img, std::string* err);
// Recompute an image's weights (total, w_absent, wtab) from d's size and logarithms
// (dict_log) without placing the trie again; img must have been built from d's keys
// and frequencies.  Returns false when two frequencies that share a weight index get
// different weights (the caller then runs build_image).
bool reweigh_image(const Dictionary& d, Image* img);

// Serialized image: dictionary + emission maps + device arrays (fast start).
void save_image(const Dictionary& d, const Emission& e, const Image& img, std::string* out);
int load_image(const char* buf, size_t len, Dictionary* d, Emission* e, Image* img, std::string* err);

// Walk the image like the kernels do.
Lookup image_lookup(const Image& img, const uint32_t* runes, size_t n);

}  // namespace jb
