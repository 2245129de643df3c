"""ctypes wrapper over gen/_build/libsynth.so (synthetic D_syn / E_syn / C_syn).

Test and bench infrastructure: deterministic seeded data shaped like the
jieba data files, which are absent from the reference (Git-LFS pointers).
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libsynth.so")
_lib = None

DICT_SEED = 1
EMIT_SEED = 2
KIND_DOCS, KIND_SENTENCES, KIND_LONG_PUNCT, KIND_LONG_OOV = 0, 1, 2, 3


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.syn_new.restype = C.c_void_p
        L.syn_new.argtypes = [C.c_uint64, C.c_uint32]
        L.syn_free.argtypes = [C.c_void_p]
        L.syn_nwords.restype = C.c_uint32
        L.syn_nwords.argtypes = [C.c_void_p]
        L.syn_maxlen.restype = C.c_uint32
        L.syn_maxlen.argtypes = [C.c_void_p]
        L.syn_write_dict.restype = C.c_long
        L.syn_write_dict.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p]
        L.syn_write_emit.restype = C.c_long
        L.syn_write_emit.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p]
        L.syn_corpus.restype = C.c_longlong
        L.syn_corpus.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                 C.c_void_p, C.c_uint64, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


class Synth:
    def __init__(self, nwords=350_000, seed=DICT_SEED):
        self.h = lib().syn_new(seed, nwords)
        self.nwords = lib().syn_nwords(self.h)
        self.maxlen = lib().syn_maxlen(self.h)

    def close(self):
        if self.h:
            lib().syn_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def write_files(self, outdir, emit_seed=EMIT_SEED):
        os.makedirs(outdir, exist_ok=True)
        dpath = os.path.join(outdir, "dict.txt")
        epath = os.path.join(outdir, "prob_emit.json")
        if lib().syn_write_dict(self.h, DICT_SEED, dpath.encode()) < 0:
            raise OSError(dpath)
        if lib().syn_write_emit(self.h, emit_seed, epath.encode()) < 0:
            raise OSError(epath)
        return dpath, epath

    def corpus(self, kind=KIND_DOCS, doc0=0, max_docs=1 << 62, target_bytes=1 << 20, target_runes=0,
               pad=64):
        """Returns (buf uint8 with `pad` trailing zero bytes, doc_off uint64[ndocs+1], nrunes)."""
        if kind in (KIND_LONG_PUNCT, KIND_LONG_OOV):
            cap = target_runes * 4 + 4096
            max_off = 2
        else:
            cap = target_bytes + (1 << 16) if max_docs >= 1 << 40 else min(target_bytes, max_docs * 4096) + (1 << 16)
            if kind == KIND_SENTENCES:
                cap = min(cap, max_docs * 512 + 4096)
            max_off = min(max_docs, target_bytes // 16 + 2) + 2
        buf = np.zeros(cap + pad, np.uint8)
        off = np.zeros(max_off + 1, np.uint64)
        nd, nr = C.c_uint64(), C.c_uint64()
        n = lib().syn_corpus(self.h, kind, doc0, max_docs, target_bytes, target_runes, buf.ctypes.data, cap,
                             off.ctypes.data, C.byref(nd), C.byref(nr))
        out = np.zeros(n + pad, np.uint8)
        out[:n] = buf[:n]
        return out, off[: nd.value + 1].copy(), int(nr.value)

    def _docs_range(self, kind, doc0, count, cap_per_doc=48 << 10):
        """Documents doc0 .. doc0+count-1 (each from its own seed 3 + index,
        gen/synth.c), concatenated: (bytes, doc lengths, runes)."""
        parts, lens, runes = [], [], 0
        done = 0
        while done < count:
            want = count - done
            cap = want * cap_per_doc + (1 << 20)
            buf = np.empty(cap, np.uint8)
            off = np.zeros(want + 1, np.uint64)
            nd, nr = C.c_uint64(), C.c_uint64()
            n = lib().syn_corpus(self.h, kind, doc0 + done, want, 1 << 62, 0, buf.ctypes.data, cap,
                                 off.ctypes.data, C.byref(nd), C.byref(nr))
            if nd.value == 0:
                raise RuntimeError("document larger than the generator buffer")
            parts.append(buf[:n].copy())
            lens.append(np.diff(off[: nd.value + 1]))
            runes += int(nr.value)
            done += int(nd.value)
        return np.concatenate(parts), np.concatenate(lens), runes

    def corpus_parallel(self, kind=KIND_DOCS, doc0=0, target_bytes=1 << 30, threads=8, chunk_docs=2048, pad=64):
        """The same corpus as corpus(kind, doc0, target_bytes=...) (documents
        doc0, doc0+1, ... up to the first one that reaches target_bytes),
        generated chunk by chunk on `threads` threads (the C generator releases
        the GIL).  Returns (buf with `pad` zero bytes, doc_off, nrunes)."""
        from concurrent.futures import ThreadPoolExecutor
        assert kind in (KIND_DOCS, KIND_SENTENCES)
        chunks, total, k = [], 0, 0
        with ThreadPoolExecutor(threads) as ex:
            while total < target_bytes:
                futs = [ex.submit(self._docs_range, kind, doc0 + (k + i) * chunk_docs, chunk_docs)
                        for i in range(threads)]
                for f in futs:
                    b, l, r = f.result()
                    chunks.append((b, l, r))
                    total += len(b)
                k += threads
        lens = np.concatenate([c[1] for c in chunks])
        off = np.zeros(len(lens) + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        nd = int(np.searchsorted(off, target_bytes, side="left"))  # first doc count reaching the target
        nd = max(1, min(nd, len(lens)))
        n = int(off[nd])
        out = np.zeros(n + pad, np.uint8)
        pos = 0
        for b, _, _ in chunks:
            if pos >= n:
                break
            m = min(len(b), n - pos)
            out[pos : pos + m] = b[:m]
            pos += m
        nrunes = int(np.count_nonzero((out[:n] & 0xC0) != 0x80))
        return out, off[: nd + 1].copy(), nrunes

