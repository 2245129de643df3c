"""ctypes wrapper over oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of /root/reference/tokenizer.go (see
jieba_oracle.c).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker or the
timed CPU baseline; the product library never touches it.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

ST = "BMES"  # state ids 0..3, tokenizer.go:685 HMMstates order


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_open.restype = C.c_void_p
        L.or_open.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_longlong, C.c_char_p, C.c_size_t,
                              C.POINTER(C.c_int)]
        L.or_close.argtypes = [C.c_void_p]
        L.or_go_log.restype = C.c_double
        L.or_go_log.argtypes = [C.c_double]
        L.or_is_han.argtypes = [C.c_uint32]
        L.or_is_space.argtypes = [C.c_uint32]
        L.or_dict_size.restype = C.c_longlong
        L.or_dict_size.argtypes = [C.c_void_p]
        L.or_dict_count.restype = C.c_longlong
        L.or_dict_count.argtypes = [C.c_void_p]
        L.or_dict_get.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_longlong)]
        L.or_dict_iter.restype = C.c_long
        L.or_dict_iter.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_longlong)]
        L.or_dict_cap.restype = C.c_size_t
        L.or_dict_cap.argtypes = [C.c_void_p]
        L.or_add_term.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_longlong]
        L.or_ties.restype = C.c_longlong
        L.or_ties.argtypes = [C.c_void_p]
        L.or_emit.restype = C.c_double
        L.or_emit.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(C.c_int)]
        L.or_split_text.restype = C.c_size_t
        L.or_split_text.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_void_p]
        L.or_cut_nonzh.restype = C.c_long
        L.or_cut_nonzh.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t]
        L.or_max_index_proba.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_int),
                                         C.POINTER(C.c_double)]
        L.or_find_dag_path.restype = C.c_long
        L.or_find_dag_path.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_build_dag.restype = C.c_long
        L.or_build_dag.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t]
        L.or_state_transition_route.restype = C.c_int
        L.or_state_transition_route.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        L.or_viterbi.restype = C.c_long
        L.or_viterbi.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p, C.c_int]
        L.or_cut_hmm.restype = C.c_long
        L.or_cut_hmm.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
        L.or_cut.restype = C.c_long
        L.or_cut.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]
        L.or_cut_batch.restype = C.c_longlong
        L.or_cut_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.c_int,
                                   C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.or_set_viterbi_backptr.argtypes = [C.c_int]
        _lib = L
    return _lib


def _b(s):
    return s.encode("utf-8") if isinstance(s, str) else bytes(s)


def go_log(x):
    return lib().or_go_log(float(x))


def split_text(text, kind=0):
    """splitText(text, zh|alnum FindAllIndex) -> [(substring bytes, doProcess)]."""
    t = _b(text)
    out = np.zeros(3 * (2 * len(t) + 2), dtype=np.uint64)
    n = lib().or_split_text(t, len(t), kind, out.ctypes.data)
    return [(t[int(out[3 * i]):int(out[3 * i + 1])], bool(out[3 * i + 2])) for i in range(n)]


def cut_nonzh(text):
    t = _b(text)
    s = np.zeros(len(t) + 1, np.uint32)
    e = np.zeros(len(t) + 1, np.uint32)
    n = lib().or_cut_nonzh(t, len(t), s.ctypes.data, e.ctypes.data, len(t) + 1)
    return spans_to_tokens(t, s[:n], e[:n])


def max_index_proba(items):
    idx = np.array([i for i, _ in items] or [0], dtype=np.int32)
    pr = np.array([p for _, p in items] or [0.0], dtype=np.float64)
    oi, op = C.c_int(), C.c_double()
    lib().or_max_index_proba(idx.ctypes.data, pr.ctypes.data, len(items), C.byref(oi), C.byref(op))
    return oi.value, op.value


def find_dag_path(n, dag_proba):
    """dag_proba: {i: [(j, proba), ...]} for i in range(n) -> [(i, j), ...]"""
    off = np.zeros(n + 1, np.uint64)
    idx, pr = [], []
    for i in range(n):
        off[i] = len(idx)
        for j, p in dag_proba.get(i, []):
            idx.append(j)
            pr.append(p)
    off[n] = len(idx)
    idx = np.array(idx + [0], np.int32)
    pr = np.array(pr + [0.0], np.float64)
    pa = np.zeros(n + 2, np.int32)
    pb = np.zeros(n + 2, np.int32)
    k = lib().or_find_dag_path(n, off.ctypes.data, idx.ctypes.data, pr.ctypes.data, pa.ctypes.data, pb.ctypes.data)
    return [(int(pa[i]), int(pb[i])) for i in range(k)]


def state_transition_route(prev, now):
    """prev: 4 floats (B,M,E,S) of hiddenStates[step-1]; now: 'B'..'S' -> (from or '', proba)."""
    arr = (C.c_double * 4)(*prev)
    p = C.c_double()
    r = lib().or_state_transition_route(arr, ST.index(now), C.byref(p))
    return ("" if r < 0 else ST[r]), p.value


def cut_hmm(text, path):
    t = _b(text)
    p = np.array([ST.index(x) for x in path], np.int32)
    s = np.zeros(len(t) + 1, np.uint32)
    e = np.zeros(len(t) + 1, np.uint32)
    n = lib().or_cut_hmm(t, len(t), p.ctypes.data, len(p), s.ctypes.data, e.ctypes.data)
    return spans_to_tokens(t, s[:n], e[:n])


def spans_to_tokens(text, s, e):
    """Span -> Go string: a 1-byte span holding a byte >= 0x80 is an invalid
    UTF-8 byte that Go's range loop turns into "\\uFFFD" (tokenizer.go:301-306)."""
    t = _b(text)
    out = []
    for a, b in zip(s.tolist(), e.tolist()):
        if b - a == 1 and t[a] >= 0x80:
            out.append("�")
        else:
            out.append(t[a:b].decode("utf-8"))
    return out


class Oracle:
    """A restated jieba-go Tokenizer on the CPU (kind 0: NewTokenizer(dict.txt)
    semantics; kind 1: buildPrefixDictionary / prefix_dictionary.gob)."""

    def __init__(self, dict_bytes, emit_bytes, kind=0, size_override=0):
        err = C.c_int(0)
        d, e = _b(dict_bytes), _b(emit_bytes)
        self.h = lib().or_open(d, len(d), kind, size_override, e, len(e), C.byref(err))
        if not self.h:
            raise ValueError(f"oracle open failed: {err.value}")

    @classmethod
    def from_files(cls, dict_path, emit_path, kind=0, size_override=0):
        with open(dict_path, "rb") as f:
            d = f.read()
        with open(emit_path, "rb") as f:
            e = f.read()
        return cls(d, e, kind, size_override)

    def close(self):
        if self.h:
            lib().or_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def size(self):
        return lib().or_dict_size(self.h)

    @property
    def ties(self):
        return lib().or_ties(self.h)

    def get(self, key):
        k = _b(key)
        v = C.c_longlong()
        return v.value if lib().or_dict_get(self.h, k, len(k), C.byref(v)) else None

    def items(self):
        cap = lib().or_dict_cap(self.h)
        buf = C.create_string_buffer(1 << 16)
        v = C.c_longlong()
        out = {}
        for i in range(cap):
            n = lib().or_dict_iter(self.h, i, buf, len(buf), C.byref(v))
            if n >= 0:
                out[buf.raw[:n].decode("utf-8", "surrogateescape")] = v.value
        return out

    def add_term(self, key, freq):
        k = _b(key)
        lib().or_add_term(self.h, k, len(k), freq)

    def emit(self, state, ch):
        f = C.c_int()
        v = lib().or_emit(self.h, ST.index(state), ord(ch), C.byref(f))
        return v if f.value else None

    def build_dag(self, text):
        t = _b(text)
        cap = 64 * len(t) + 64
        off = np.zeros(len(t) + 2, np.uint64)
        ends = np.zeros(cap, np.int32)
        n = lib().or_build_dag(self.h, t, len(t), off.ctypes.data, ends.ctypes.data, cap)
        return {i: ends[int(off[i]):int(off[i + 1])].tolist() for i in range(n)}

    def viterbi(self, text, backptr=False):
        t = _b(text)
        out = np.zeros(len(t) + 2, np.int32)
        L = lib().or_viterbi(self.h, t, len(t), out.ctypes.data, int(backptr))
        return [ST[x] for x in out[:L]]

    def cut_spans(self, text, hmm):
        t = _b(text)
        s = np.zeros(len(t) + 1, np.uint32)
        e = np.zeros(len(t) + 1, np.uint32)
        n = lib().or_cut(self.h, t, len(t), int(hmm), s.ctypes.data, e.ctypes.data, len(t) + 1)
        if n < 0:
            raise RuntimeError(f"oracle cut failed ({n}): the reference panics on this input")
        return s[:n].copy(), e[:n].copy()

    def cut(self, text, hmm):
        """Tokenizer.Cut (tokenizer.go:151) -> list of str."""
        s, e = self.cut_spans(text, hmm)
        return spans_to_tokens(text, s, e)

    def cut_batch(self, buf, doc_off, hmm, nthreads=1, want_spans=True):
        """Cut every document of a concatenated uint8 buffer.
        Returns (starts, ends, tok_doc_off) as numpy arrays (absolute offsets)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        ndocs = len(doc_off) - 1
        cap = int(doc_off[-1] - doc_off[0]) + 1 if want_spans else 0
        s = np.zeros(max(cap, 1), np.uint32)
        e = np.zeros(max(cap, 1), np.uint32)
        tdo = np.zeros(ndocs + 1, np.uint64)
        n = lib().or_cut_batch(self.h, buf.ctypes.data, doc_off.ctypes.data, ndocs, int(hmm), nthreads,
                               s.ctypes.data if want_spans else None, e.ctypes.data if want_spans else None,
                               cap, tdo.ctypes.data)
        if n < 0:
            raise RuntimeError(f"oracle cut_batch failed ({n})")
        return s[:n], e[:n], tdo


def set_viterbi_backptr(on):
    lib().or_set_viterbi_backptr(int(on))
