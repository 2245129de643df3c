// Package jiebahip is the drop-in Go front end of the MI355X segmentation path:
// the API of github.com/ericlingit/jieba-go's Tokenizer (tokenizer.go:52-162,
// 372-379) over the C ABI of libjiebahip.so (include/jiebahip.h).
//
// Not built in the development image (no Go toolchain there); see
// INTEGRATION.md for how a maintainer wires it into the reference module.
package jiebahip

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../lib -ljiebahip -Wl,-rpath,${SRCDIR}/../lib
#include <stdlib.h>
#include "jiebahip.h"
*/
import "C"

import (
	"errors"
	"log"
	"math"
	"runtime"
	"sync"
	"unsafe"
)

// JiebaSize is the total count NewJiebaTokenizer uses (tokenizer.go:454).
const JiebaSize = 60101967

// Tokenizer mirrors the reference's Tokenizer: safe for concurrent Cut calls,
// AddWord takes the exclusive lock (tokenizer.go:82-83,152-153,376).
type Tokenizer struct {
	mu  sync.RWMutex
	ctx *C.jb_ctx
}

func lastError() string { return C.GoString(C.jb_last_error()) }

func open(dictPath, emitPath string, kind C.int, size int64) *Tokenizer {
	cd := C.CString(dictPath)
	ce := C.CString(emitPath)
	defer C.free(unsafe.Pointer(cd))
	defer C.free(unsafe.Pointer(ce))
	// cfg is Go memory passed to C by address, so every pointer it holds is C memory
	// (cgo pointer rules: no Go pointer to memory that holds Go pointers).
	var cfg C.jb_config
	cfg.dict_path = cd
	cfg.emit_path = ce
	cfg.dict_kind = kind
	cfg.size_override = C.int64_t(size)
	cfg.device = 0
	cfg.ndevices = 1
	// calcDagProba's weights are math.Log(tf) - math.Log(pd.size) (tokenizer.go:503,
	// 515-519): build the image once, list the values its weights need, take Go's own
	// math.Log of each and open the device context from that image with the table
	// (jb_open_image reweighs it; the trie is not placed again).
	var img *C.jb_image
	if rc := C.jb_image_build(&cfg, &img); rc != C.JB_OK {
		log.Fatal("jiebahip: ", lastError())
	}
	var n C.size_t
	if rc := C.jb_image_log_keys(img, nil, 0, &n); rc != C.JB_OK && rc != C.JB_ELIMIT {
		C.jb_image_free(img)
		log.Fatal("jiebahip: ", lastError())
	}
	cnt := int(n) + 1
	ckeys := (*C.int64_t)(C.malloc(C.size_t(cnt) * C.size_t(unsafe.Sizeof(C.int64_t(0)))))
	cvals := (*C.double)(C.malloc(C.size_t(cnt) * C.size_t(unsafe.Sizeof(C.double(0)))))
	defer C.free(unsafe.Pointer(ckeys))
	defer C.free(unsafe.Pointer(cvals))
	if rc := C.jb_image_log_keys(img, ckeys, n, &n); rc != C.JB_OK {
		C.jb_image_free(img)
		log.Fatal("jiebahip: ", lastError())
	}
	keys := unsafe.Slice(ckeys, cnt)
	vals := unsafe.Slice(cvals, cnt)
	for i := 0; i < int(n); i++ {
		vals[i] = C.double(math.Log(float64(keys[i])))
	}
	cfg.log_keys = ckeys
	cfg.log_vals = cvals
	cfg.nlog = n
	var ctx *C.jb_ctx
	if rc := C.jb_open_image(img, &cfg, &ctx); rc != C.JB_OK { // consumes img
		// the reference stops the process on load errors (tokenizer.go:397,443,656)
		log.Fatal("jiebahip: ", lastError())
	}
	t := &Tokenizer{ctx: ctx}
	runtime.SetFinalizer(t, (*Tokenizer).Close)
	return t
}

// NewTokenizer loads a dict.txt-format dictionary (tokenizer.go:61).
func NewTokenizer(dictionaryFile string) *Tokenizer {
	return open(dictionaryFile, "prob_emit.json", C.JB_DICT_TXT, 0)
}

// NewJiebaTokenizer is the reference's default tokenizer (tokenizer.go:69):
// it decodes prefix_dictionary.gob (tokenizer.go:439-458) with size 60,101,967.
func NewJiebaTokenizer() *Tokenizer {
	return open("prefix_dictionary.gob", "prob_emit.json", C.JB_DICT_GOB, 0)
}

// NewTokenizerFromImage opens an image written by Save: no parsing, no trie build.
func NewTokenizerFromImage(path string) *Tokenizer {
	return open(path, "", C.JB_DICT_IMAGE, 0)
}

// Save writes the current dictionary (AddWord changes included) as an image.
func (t *Tokenizer) Save(path string) error {
	t.mu.RLock()
	defer t.mu.RUnlock()
	cp := C.CString(path)
	defer C.free(unsafe.Pointer(cp))
	if rc := C.jb_save(t.ctx, cp); rc != C.JB_OK {
		return errors.New("jiebahip: " + lastError())
	}
	return nil
}

// Close releases the device context.
func (t *Tokenizer) Close() {
	t.mu.Lock()
	defer t.mu.Unlock()
	if t.ctx != nil {
		C.jb_close(t.ctx)
		t.ctx = nil
	}
}

func spansToTokens(text string, s *C.jb_spans, doc int) []string {
	n := int(s.ntokens)
	starts := unsafe.Slice((*uint64)(unsafe.Pointer(s.start)), n)
	ends := unsafe.Slice((*uint64)(unsafe.Pointer(s.end)), n)
	docTok := unsafe.Slice((*uint64)(unsafe.Pointer(s.doc_tok)), int(s.ndocs)+1)
	a, b := int(docTok[doc]), int(docTok[doc+1])
	out := make([]string, 0, b-a)
	for k := a; k < b; k++ {
		st, en := int(starts[k]), int(ends[k])
		if en-st == 1 && text[st] >= 0x80 {
			out = append(out, "�") // invalid UTF-8 byte (tokenizer.go:301-306)
		} else {
			out = append(out, text[st:en])
		}
	}
	return out
}

// cut32 cuts a batch held in buf (documents [off[d], off[d+1]), off[0] == 0) into u32
// spans (jb_cut_batch_into32) in Go slices: half the bytes the library writes for u64
// spans, which bound a host batch's host side.  A first try has room for one token per
// three bytes; on JB_ELIMIT a second one has the count the library returned.  The slices
// hold no Go pointers, so cgo lets C write them during the call (it keeps none).
func (t *Tokenizer) cut32(buf []byte, off []uint64, hmm C.int) (starts, ends []uint32, docTok []uint64) {
	n := len(off) - 1
	total := int(off[n] - off[0])
	docTok = make([]uint64, n+1)
	capTok := total/3 + 64
	for try := 0; try < 2; try++ {
		starts = make([]uint32, capTok)
		ends = make([]uint32, capTok)
		var nt C.uint64_t
		rc := C.jb_cut_batch_into32(t.ctx, (*C.uint8_t)(unsafe.Pointer(&buf[0])), (*C.uint64_t)(unsafe.Pointer(&off[0])),
			C.uint32_t(n), hmm, (*C.uint32_t)(unsafe.Pointer(&starts[0])), (*C.uint32_t)(unsafe.Pointer(&ends[0])),
			C.uint64_t(capTok), (*C.uint64_t)(unsafe.Pointer(&docTok[0])), &nt)
		if rc == C.JB_OK {
			return starts[:int(nt)], ends[:int(nt)], docTok
		}
		if rc == C.JB_ELIMIT && int(nt) > capTok {
			capTok = int(nt)
			continue
		}
		// JB_EPANIC: the reference panics on this input (cutDAG slice with tail -1)
		panic("jiebahip: " + lastError())
	}
	panic("jiebahip: " + lastError())
}

// tokens [a, b) of u32 spans over text (offsets from text's first byte) as strings.
func tokens32(text string, starts, ends []uint32, a, b int) []string {
	out := make([]string, 0, b-a)
	for k := a; k < b; k++ {
		st, en := int(starts[k]), int(ends[k])
		if en-st == 1 && text[st] >= 0x80 {
			out = append(out, "�") // invalid UTF-8 byte (tokenizer.go:301-306)
		} else {
			out = append(out, text[st:en])
		}
	}
	return out
}

// Cut segments one text (tokenizer.go:151).  Never returns nil.
func (t *Tokenizer) Cut(text string, useHmm bool) []string {
	t.mu.RLock()
	defer t.mu.RUnlock()
	if len(text) == 0 {
		return []string{}
	}
	b := []byte(text)
	hmm := C.int(0)
	if useHmm {
		hmm = 1
	}
	if uint64(len(b)) < 1<<32 { // u32 spans (jb_cut_batch_into32)
		starts, ends, _ := t.cut32(b, []uint64{0, uint64(len(b))}, hmm)
		return tokens32(text, starts, ends, 0, len(starts))
	}
	var s C.jb_spans
	if rc := C.jb_cut(t.ctx, (*C.uint8_t)(unsafe.Pointer(&b[0])), C.size_t(len(b)), hmm, &s); rc != C.JB_OK {
		// JB_EPANIC: the reference panics on this input (cutDAG slice with tail -1)
		panic("jiebahip: " + lastError())
	}
	defer C.jb_spans_free(&s)
	return spansToTokens(text, &s, 0)
}

// CutParallel (tokenizer.go:81) returns the tokens of Cut in document order.
// The library splits the work itself: the text goes to the device in pieces cut
// at Han-run starts (jb_split_points), and over every device of a multi-device
// context; numWorkers is accepted for API parity.  ordered=false allows any block
// order in the reference; this order is one of them.
func (t *Tokenizer) CutParallel(text string, hmm bool, numWorkers int, ordered bool) []string {
	return t.Cut(text, hmm)
}

// CutBatch segments many documents in one device call (the batched form of Cut).
func (t *Tokenizer) CutBatch(docs []string, useHmm bool) [][]string {
	t.mu.RLock()
	defer t.mu.RUnlock()
	total := 0
	for _, d := range docs {
		total += len(d)
	}
	buf := make([]byte, 0, total+1)
	off := make([]uint64, len(docs)+1)
	for i, d := range docs {
		buf = append(buf, d...)
		off[i+1] = uint64(len(buf))
	}
	buf = append(buf, 0)
	hmm := C.int(0)
	if useHmm {
		hmm = 1
	}
	all := string(buf[:total])
	out := make([][]string, len(docs))
	if uint64(total) < 1<<32 { // u32 spans (jb_cut_batch_into32); tokens share one copy of the batch text
		starts, ends, docTok := t.cut32(buf, off, hmm)
		for i := range docs {
			out[i] = tokens32(all, starts, ends, int(docTok[i]), int(docTok[i+1]))
		}
		return out
	}
	var s C.jb_spans
	if rc := C.jb_cut_batch(t.ctx, (*C.uint8_t)(unsafe.Pointer(&buf[0])), (*C.uint64_t)(unsafe.Pointer(&off[0])),
		C.uint32_t(len(docs)), hmm, &s); rc != C.JB_OK {
		panic("jiebahip: " + lastError())
	}
	defer C.jb_spans_free(&s)
	for i := range docs {
		out[i] = spansToTokens(all, &s, i)
	}
	return out
}

// AddWord adds or updates a word (tokenizer.go:372).  freq < 1 takes
// suggestFreq's value (tokenizer.go:589-614).  Unlike the reference it does
// not deadlock.
func (t *Tokenizer) AddWord(word string, freq int) {
	t.mu.Lock()
	defer t.mu.Unlock()
	cw := C.CString(word)
	defer C.free(unsafe.Pointer(cw))
	f := C.int64_t(freq)
	if freq < 1 {
		if rc := C.jb_suggest_freq(t.ctx, cw, C.size_t(len(word)), &f); rc != C.JB_OK {
			log.Fatal("jiebahip: ", lastError())
		}
	}
	// Go's math.Log of the new frequency and of the new pd.size for the rebuild
	// (addTerm adds freq to pd.size even when the word was present, tokenizer.go:580-585)
	size := int64(C.jb_dict_size(t.ctx))
	keys := []int64{int64(f), size + int64(f)} // (Go memory without Go pointers: may be passed to C)
	vals := []float64{math.Log(float64(keys[0])), math.Log(float64(keys[1]))}
	if rc := C.jb_add_log(t.ctx, (*C.int64_t)(unsafe.Pointer(&keys[0])), (*C.double)(unsafe.Pointer(&vals[0])), 2); rc != C.JB_OK {
		log.Fatal("jiebahip: ", lastError())
	}
	// atomic: on an error the dictionary and the device image are unchanged
	if rc := C.jb_add_word(t.ctx, cw, C.size_t(len(word)), f); rc != C.JB_OK {
		log.Fatal("jiebahip: ", lastError())
	}
}
