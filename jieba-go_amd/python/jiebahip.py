"""ctypes binding of libjiebahip.so (include/jiebahip.h).

A thin Python view of the same C ABI the Go cgo wrapper binds
(jieba-go_amd/go/tokenizer.go): used by tests/, bench.py and
__graft_entry__.py.  `Tokenizer` mirrors jieba-go's API (tokenizer.go:52-162,
372-379): NewTokenizer / NewJiebaTokenizer / Cut / CutParallel / AddWord.

The library is loaded from jieba-go_amd/lib/ (built in-tree by
`make -C jieba-go_amd`); a missing or unloadable library raises — there is no
CPU fallback.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
# JB_LIB: another in-tree build of the same library (diagnostic variants, e.g. make STAMPS=1 OUT=var/stamps)
LIB_PATH = os.environ.get("JB_LIB") or os.path.join(PKG_DIR, "lib", "libjiebahip.so")

JB_OK, JB_EINVAL, JB_EIO, JB_EPARSE, JB_EDEVICE, JB_ENOMEM, JB_EPANIC, JB_ELIMIT = 0, -1, -2, -3, -4, -5, -6, -7
JB_DICT_TXT, JB_DICT_PREFIX, JB_DICT_GOB, JB_DICT_IMAGE = 0, 1, 2, 3
JIEBA_SIZE = 60_101_967  # tokenizer.go:454

# Every symbol include/jiebahip.h declares.
EXPORTS = [
    "jb_open", "jb_close", "jb_last_error", "jb_cut", "jb_cut_batch", "jb_cut_batch_into", "jb_spans_free",
    "jb_cut_device", "jb_cut_device_into", "jb_open_image", "jb_cut_batch_mask", "jb_host_alloc", "jb_host_free",
    "jb_split_points",
    "jb_add_word", "jb_dict_get", "jb_dict_size", "jb_save", "jb_profile_enable", "jb_profile_read",
    "jb_profile_reset", "jb_image_build", "jb_image_free", "jb_image_save", "jb_image_dict_info", "jb_image_lookup",
    "jb_image_stats", "jb_image_emit", "jb_go_log", "jb_shard_bounds", "jb_last_stats",
    "jb_suggest_freq", "jb_add_log", "jb_image_log_keys", "jb_device_status", "jb_cut_batch_into32",
]


class JbError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class jb_config(C.Structure):
    _fields_ = [
        ("dict_path", C.c_char_p), ("dict_buf", C.c_char_p), ("dict_len", C.c_size_t), ("dict_kind", C.c_int),
        ("size_override", C.c_int64), ("emit_path", C.c_char_p), ("emit_buf", C.c_char_p), ("emit_len", C.c_size_t),
        ("device", C.c_int), ("ndevices", C.c_int),
        ("log_keys", C.POINTER(C.c_int64)), ("log_vals", C.POINTER(C.c_double)), ("nlog", C.c_size_t),
    ]


class jb_stats(C.Structure):
    _fields_ = [("tokens", C.c_uint64), ("blocks", C.c_uint64), ("zh_blocks", C.c_uint64),
                ("long_blocks", C.c_uint64), ("viterbi_ties", C.c_uint64)]


class jb_spans(C.Structure):
    _fields_ = [
        ("ntokens", C.c_uint64), ("start", C.POINTER(C.c_uint64)), ("end", C.POINTER(C.c_uint64)),
        ("doc_tok", C.POINTER(C.c_uint64)), ("ndocs", C.c_uint32),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise JbError(JB_EIO, f"{LIB_PATH} not built: run `make -C jieba-go_amd` (no CPU fallback exists)")
        # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7
        # (ROCm 7.0) under torch/lib.  Loading torch first makes the dynamic
        # linker bind libjiebahip.so's libamdhip64.so.7 dependency to that same
        # runtime, so torch tensors and this library share device pointers,
        # streams and one HSA context.  (Loading the system ROCm 7.2 runtime and
        # torch's side by side in one process left torch with "No HIP GPUs are
        # available".)  Outside Python (Go / C++ callers) the system runtime is used.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        vp, cp = C.c_void_p, C.c_char_p
        L.jb_open.argtypes = [C.POINTER(jb_config), C.POINTER(vp)]
        L.jb_close.argtypes = [vp]
        L.jb_close.restype = None
        L.jb_last_error.restype = cp
        L.jb_cut.argtypes = [vp, vp, C.c_size_t, C.c_int, C.POINTER(jb_spans)]
        L.jb_cut_batch.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, C.POINTER(jb_spans)]
        L.jb_cut_batch_into.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, vp, vp, C.c_uint64, vp,
                                        C.POINTER(C.c_uint64)]
        L.jb_spans_free.argtypes = [C.POINTER(jb_spans)]
        L.jb_spans_free.restype = None
        L.jb_cut_device.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, C.c_int, vp, C.POINTER(vp), C.POINTER(vp),
                                    C.POINTER(vp), C.POINTER(vp)]
        L.jb_cut_device_into.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, C.c_int, vp, vp, vp, C.c_uint64, vp,
                                         vp]
        L.jb_open_image.argtypes = [vp, C.POINTER(jb_config), C.POINTER(vp)]
        L.jb_cut_batch_mask.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]
        L.jb_host_alloc.argtypes = [C.c_size_t, C.POINTER(vp)]
        L.jb_host_free.argtypes = [vp]
        L.jb_host_free.restype = None
        L.jb_add_word.argtypes = [vp, cp, C.c_size_t, C.c_int64]
        L.jb_dict_get.argtypes = [vp, cp, C.c_size_t, C.POINTER(C.c_int64)]
        L.jb_dict_size.argtypes = [vp]
        L.jb_dict_size.restype = C.c_int64
        L.jb_save.argtypes = [vp, cp]
        L.jb_image_save.argtypes = [vp, cp]
        L.jb_image_dict_info.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_int64)]
        L.jb_profile_enable.argtypes = [vp, C.c_int]
        L.jb_profile_reset.argtypes = [vp]
        L.jb_profile_read.argtypes = [vp, C.POINTER(cp), C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]
        L.jb_image_build.argtypes = [C.POINTER(jb_config), C.POINTER(vp)]
        L.jb_image_free.argtypes = [vp]
        L.jb_image_free.restype = None
        L.jb_image_lookup.argtypes = [vp, cp, C.c_size_t, C.POINTER(C.c_int64), C.POINTER(C.c_double)]
        L.jb_image_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_int64), C.POINTER(C.c_double)]
        L.jb_image_emit.argtypes = [vp, C.c_int, C.c_uint32]
        L.jb_image_emit.restype = C.c_double
        L.jb_go_log.argtypes = [C.c_double]
        L.jb_go_log.restype = C.c_double
        L.jb_shard_bounds.argtypes = [vp, C.c_uint32, C.c_uint32, vp]
        L.jb_split_points.argtypes = [vp, vp, C.c_uint32, C.c_uint32, vp]
        L.jb_image_log_keys.argtypes = [vp, vp, C.c_size_t, C.POINTER(C.c_size_t)]
        L.jb_suggest_freq.argtypes = [vp, cp, C.c_size_t, C.POINTER(C.c_int64)]
        L.jb_add_log.argtypes = [vp, vp, vp, C.c_size_t]
        L.jb_last_stats.argtypes = [vp, C.POINTER(jb_stats)]
        L.jb_device_status.argtypes = [vp, vp]
        L.jb_cut_batch_into32.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, vp, vp, C.c_uint64, vp,
                                          C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


def _check(rc):
    if rc < 0:
        raise JbError(rc, lib().jb_last_error().decode("utf-8", "replace"))
    return rc


def _b(s):
    return s.encode("utf-8") if isinstance(s, str) else bytes(s)


def make_config(dict_path=None, emit_path=None, dict_bytes=None, emit_bytes=None, kind=JB_DICT_TXT,
                size_override=0, device=0, ndevices=1, logs=None):
    """logs: optional {x: math.Log(float64(x))} the caller computed (jb_config.log_keys/log_vals)."""
    cfg = jb_config()
    keep = []
    if logs:
        ks = np.ascontiguousarray(list(logs.keys()), np.int64)
        vs = np.ascontiguousarray([logs[k] for k in logs.keys()], np.float64)
        keep += [ks, vs]
        cfg.log_keys = ks.ctypes.data_as(C.POINTER(C.c_int64))
        cfg.log_vals = vs.ctypes.data_as(C.POINTER(C.c_double))
        cfg.nlog = len(ks)
    if dict_path is not None:
        cfg.dict_path = os.fsencode(dict_path)
    else:
        d = _b(dict_bytes or b"")
        keep.append(d)
        cfg.dict_buf, cfg.dict_len = d, len(d)
    if emit_path is not None:
        cfg.emit_path = os.fsencode(emit_path)
    else:
        e = _b(emit_bytes or b"{}")
        keep.append(e)
        cfg.emit_buf, cfg.emit_len = e, len(e)
    cfg.dict_kind = kind
    cfg.size_override = size_override
    cfg.device = device
    cfg.ndevices = ndevices
    cfg._keep = keep
    return cfg


def spans_to_tokens(text, starts, ends):
    """(start, end) byte spans -> Go strings; an invalid UTF-8 byte becomes "�"."""
    t = _b(text)
    out = []
    for a, b in zip(starts, ends):
        if b - a == 1 and t[a] >= 0x80:
            out.append("�")
        else:
            out.append(t[a:b].decode("utf-8"))
    return out


class Image:
    """Host-only device image (no GPU needed): loader + table builder."""

    def __init__(self, cfg):
        h = C.c_void_p()
        _check(lib().jb_image_build(C.byref(cfg), C.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().jb_image_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def lookup(self, word):
        w = _b(word)
        f, x = C.c_int64(), C.c_double()
        r = _check(lib().jb_image_lookup(self.h, w, len(w), C.byref(f), C.byref(x)))
        return (f.value, x.value) if r else None

    def stats(self):
        n, cap, sz = C.c_uint64(), C.c_uint64(), C.c_int64()
        npg, ml = C.c_uint32(), C.c_uint32()
        wa = C.c_double()
        _check(lib().jb_image_stats(self.h, C.byref(n), C.byref(cap), C.byref(npg), C.byref(ml), C.byref(sz),
                                    C.byref(wa)))
        return dict(nodes=n.value, cap=cap.value, npages=npg.value, maxlen=ml.value, size=sz.value,
                    w_absent=wa.value)

    def emit(self, state, ch):
        return lib().jb_image_emit(self.h, "BMES".index(state), ord(ch))

    def save(self, path):
        _check(lib().jb_image_save(self.h, os.fsencode(path)))

    def log_keys(self):
        """jb_image_log_keys: the x whose math.Log the weights use."""
        n = C.c_size_t()
        lib().jb_image_log_keys(self.h, None, 0, C.byref(n))
        out = np.zeros(max(n.value, 1), np.int64)
        _check(lib().jb_image_log_keys(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out[:n.value]

    def dict_info(self):
        n, sz = C.c_uint64(), C.c_int64()
        _check(lib().jb_image_dict_info(self.h, C.byref(n), C.byref(sz)))
        return n.value, sz.value


class Tokenizer:
    """jieba-go Tokenizer over the MI355X path."""

    def __init__(self, cfg):
        h = C.c_void_p()
        _check(lib().jb_open(C.byref(cfg), C.byref(h)))
        self.h = h

    @classmethod
    def from_image(cls, image, device=0, ndevices=1, logs=None):
        """jb_open_image: a ctx from an Image built by jb_image_build (the trie is placed
        once), optionally reweighed with the caller's {x: math.Log(x)}.  Consumes `image`."""
        cfg = make_config(dict_bytes=b"", device=device, ndevices=ndevices, logs=logs)
        h, img = C.c_void_p(), image.h
        image.h = None  # jb_open_image owns it from here, success or not
        _check(lib().jb_open_image(img, C.byref(cfg), C.byref(h)))
        self = cls.__new__(cls)
        self.h = h
        return self

    @classmethod
    def NewTokenizer(cls, dictionaryFile, emit_path="prob_emit.json", device=0):
        """tokenizer.go:61 — dict.txt semantics."""
        return cls(make_config(dict_path=dictionaryFile, emit_path=emit_path, kind=JB_DICT_TXT, device=device))

    @classmethod
    def NewJiebaTokenizer(cls, dict_path="prefix_dictionary.gob", emit_path="prob_emit.json", device=0):
        """tokenizer.go:69 — decodes prefix_dictionary.gob (tokenizer.go:439-458), size 60,101,967.
        A path ending in .txt is read with buildPrefixDictionary semantics instead (the map the gob holds)."""
        if str(dict_path).endswith(".txt"):
            return cls(make_config(dict_path=dict_path, emit_path=emit_path, kind=JB_DICT_PREFIX,
                                   size_override=JIEBA_SIZE, device=device))
        return cls(make_config(dict_path=dict_path, emit_path=emit_path, kind=JB_DICT_GOB, device=device))

    @classmethod
    def FromImage(cls, image_path, device=0, ndevices=1):
        """Open a serialized image written by save() (no parsing, no trie build)."""
        return cls(make_config(dict_path=image_path, kind=JB_DICT_IMAGE, device=device, ndevices=ndevices))

    def save(self, path):
        """Write the current image (including AddWord changes) for FromImage."""
        _check(lib().jb_save(self.h, os.fsencode(path)))

    def close(self):
        if self.h:
            lib().jb_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- cutting ---------------------------------------------------------
    def cut_spans(self, text, hmm):
        t = _b(text)
        sp = jb_spans()
        _check(lib().jb_cut(self.h, t, len(t), int(hmm), C.byref(sp)))
        try:
            n = sp.ntokens
            s = np.ctypeslib.as_array(sp.start, (max(n, 1),))[:n].copy()
            e = np.ctypeslib.as_array(sp.end, (max(n, 1),))[:n].copy()
        finally:
            lib().jb_spans_free(C.byref(sp))
        return s, e

    def Cut(self, text, useHmm):
        """Tokenizer.Cut (tokenizer.go:151)."""
        s, e = self.cut_spans(text, useHmm)
        return spans_to_tokens(text, s.tolist(), e.tolist())

    def CutParallel(self, text, hmm, numWorkers=1, ordered=True):
        """Tokenizer.CutParallel (tokenizer.go:81): always in text order."""
        return self.Cut(text, hmm)

    def cut_batch(self, buf, doc_off, hmm):
        """Host batch -> (starts u64, ends u64, doc_tok u64[ndocs+1])."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        nd = len(doc_off) - 1
        sp = jb_spans()
        _check(lib().jb_cut_batch(self.h, buf.ctypes.data, doc_off.ctypes.data, nd, int(hmm), C.byref(sp)))
        try:
            n = sp.ntokens
            s = np.ctypeslib.as_array(sp.start, (max(n, 1),))[:n].copy()
            e = np.ctypeslib.as_array(sp.end, (max(n, 1),))[:n].copy()
            d = np.ctypeslib.as_array(sp.doc_tok, (nd + 1,)).copy()
        finally:
            lib().jb_spans_free(C.byref(sp))
        return s, e, d

    def cut_batch_into(self, buf, doc_off, hmm, out=None):
        """Host batch into caller-owned arrays (jb_cut_batch_into).  `out` =
        (starts u64, ends u64, doc_tok u64[ndocs+1]) to reuse; grown when too
        small.  Returns (starts[:n], ends[:n], doc_tok, out)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        nd = len(doc_off) - 1
        if out is None or len(out[2]) != nd + 1:
            cap = max(1024, int(doc_off[-1] - doc_off[0]) // 2)
            out = (np.empty(cap, np.uint64), np.empty(cap, np.uint64), np.empty(nd + 1, np.uint64))
        n = C.c_uint64()
        for _ in range(2):
            rc = lib().jb_cut_batch_into(self.h, buf.ctypes.data, doc_off.ctypes.data, nd, int(hmm),
                                         out[0].ctypes.data, out[1].ctypes.data, len(out[0]), out[2].ctypes.data,
                                         C.byref(n))
            if rc == JB_ELIMIT and n.value > len(out[0]):
                out = (np.empty(n.value, np.uint64), np.empty(n.value, np.uint64), out[2])
                continue
            _check(rc)
            break
        k = n.value
        return out[0][:k], out[1][:k], out[2], out

    def cut_batch_into32(self, buf, doc_off, hmm, out=None):
        """jb_cut_batch_into32: u32 spans relative to doc_off[0] in caller-owned arrays.
        `out` = (starts u32, ends u32, doc_tok u64[ndocs+1]) to reuse; grown when too
        small.  Returns (starts[:n], ends[:n], doc_tok, out)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        nd = len(doc_off) - 1
        if out is None or len(out[2]) != nd + 1:
            cap = max(1024, int(doc_off[-1] - doc_off[0]) // 2)
            out = (np.empty(cap, np.uint32), np.empty(cap, np.uint32), np.empty(nd + 1, np.uint64))
        n = C.c_uint64()
        for _ in range(2):
            rc = lib().jb_cut_batch_into32(self.h, buf.ctypes.data, doc_off.ctypes.data, nd, int(hmm),
                                           out[0].ctypes.data, out[1].ctypes.data, len(out[0]), out[2].ctypes.data,
                                           C.byref(n))
            if rc == JB_ELIMIT and n.value > len(out[0]):
                out = (np.empty(n.value, np.uint32), np.empty(n.value, np.uint32), out[2])
                continue
            _check(rc)
            break
        k = n.value
        return out[0][:k], out[1][:k], out[2], out

    def cut_batch_mask(self, buf, doc_off, hmm, out=None):
        """jb_cut_batch_mask: (starts u64 words, ends u64 words, ntokens); `out` = the
        two arrays to reuse."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)  # (a HostBuffer's .array stays where it is)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        nd = len(doc_off) - 1
        nw = (int(doc_off[-1] - doc_off[0]) + 63) // 64 if nd else 0
        if out is None or len(out[0]) < nw:
            out = (np.empty(max(nw, 1), np.uint64), np.empty(max(nw, 1), np.uint64))
        n = C.c_uint64()
        _check(lib().jb_cut_batch_mask(self.h, buf.ctypes.data, doc_off.ctypes.data, nd, int(hmm), out[0].ctypes.data,
                                       out[1].ctypes.data, len(out[0]), C.byref(n)))
        return out[0][:nw], out[1][:nw], n.value

    def cut_device(self, d_text_ptr, nbytes, d_doc_off_ptr, ndocs, hmm, stream_ptr=0):
        """Device-resident cut; returns device pointers (start, end, doc_tok, ntok)."""
        a, b, c, d = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        _check(lib().jb_cut_device(self.h, C.c_void_p(d_text_ptr), nbytes, C.c_void_p(d_doc_off_ptr), ndocs,
                                   int(hmm), C.c_void_p(stream_ptr), C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return a.value, b.value, c.value, d.value

    def cut_device_into(self, d_text_ptr, nbytes, d_doc_off_ptr, ndocs, hmm, d_start, d_end, cap, d_doc_tok, d_ntok,
                        stream_ptr=0):
        """jb_cut_device_into: caller-owned device outputs (raw pointers)."""
        _check(lib().jb_cut_device_into(self.h, C.c_void_p(d_text_ptr), nbytes, C.c_void_p(d_doc_off_ptr), ndocs,
                                        int(hmm), C.c_void_p(stream_ptr), C.c_void_p(d_start), C.c_void_p(d_end),
                                        cap, C.c_void_p(d_doc_tok), C.c_void_p(d_ntok)))

    def device_status(self, stream_ptr=0):
        """jb_device_status: raises JbError when the last device pipeline hit an error."""
        _check(lib().jb_device_status(self.h, C.c_void_p(stream_ptr)))

    def last_stats(self):
        """Counters of the last pipeline run (jb_last_stats); synchronises."""
        st = jb_stats()
        _check(lib().jb_last_stats(self.h, C.byref(st)))
        return {k: getattr(st, k) for k, _ in jb_stats._fields_}

    def last_ties(self):
        return self.last_stats()["viterbi_ties"]

    # -- dictionary ------------------------------------------------------
    def AddWord(self, word, freq):
        """Tokenizer.AddWord (tokenizer.go:372) without the reference's deadlock."""
        w = _b(word)
        _check(lib().jb_add_word(self.h, w, len(w), freq))

    def suggest_freq(self, word):
        """suggestFreq (tokenizer.go:589-614)."""
        w = _b(word)
        f = C.c_int64()
        _check(lib().jb_suggest_freq(self.h, w, len(w), C.byref(f)))
        return f.value

    def add_log(self, logs):
        """jb_add_log: caller-computed {x: math.Log(float64(x))} for the next image build."""
        ks = np.ascontiguousarray(list(logs.keys()), np.int64)
        vs = np.ascontiguousarray([logs[k] for k in logs.keys()], np.float64)
        _check(lib().jb_add_log(self.h, ks.ctypes.data, vs.ctypes.data, len(ks)))

    def dict_get(self, word):
        w = _b(word)
        f = C.c_int64()
        return f.value if _check(lib().jb_dict_get(self.h, w, len(w), C.byref(f))) else None

    @property
    def size(self):
        return lib().jb_dict_size(self.h)

    # -- profiling -------------------------------------------------------
    def profile(self, on=True):
        _check(lib().jb_profile_enable(self.h, int(on)))

    def profile_reset(self):
        _check(lib().jb_profile_reset(self.h))

    def profile_read(self):
        names = (C.c_char_p * 32)()
        ms = (C.c_double * 32)()
        n = (C.c_uint64 * 32)()
        k = _check(lib().jb_profile_read(self.h, names, ms, n, 32))
        return {names[i].decode(): (ms[i], n[i]) for i in range(k)}


class HostBuffer:
    """jb_host_alloc'd pinned memory as a numpy uint8 array (`.array`); batches cut
    from that array skip the library's staging copy."""

    def __init__(self, n):
        p = C.c_void_p()
        _check(lib().jb_host_alloc(n, C.byref(p)))
        self.p = p
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(n, 1)).from_address(p.value))[:n]

    def free(self):
        if self.p:
            self.array = None
            lib().jb_host_free(self.p)
            self.p = None


def mask_to_spans(ms, me, nbytes, base=0):
    """Boundary masks -> (starts, ends) byte spans (start bit k pairs with end bit k)."""
    nw = (nbytes + 63) // 64
    sb = np.unpackbits(np.asarray(ms[:nw]).view(np.uint8), bitorder="little")[:nbytes]
    eb = np.unpackbits(np.asarray(me[:nw]).view(np.uint8), bitorder="little")[:nbytes]
    return (np.flatnonzero(sb).astype(np.uint64) + np.uint64(base),
            np.flatnonzero(eb).astype(np.uint64) + np.uint64(base + 1))


_hip = None


def dev_to_host(ptr, nbytes, dtype):
    """Copy nbytes of device memory at a raw pointer into a numpy array."""
    global _hip
    if _hip is None:
        lib()
        _hip = C.CDLL("libamdhip64.so.7")  # the runtime libjiebahip.so is bound to
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype)
    if nbytes:
        rc = _hip.hipMemcpy(out.ctypes.data, C.c_void_p(ptr), nbytes, 2)  # hipMemcpyDeviceToHost
        if rc != 0:
            raise JbError(JB_EDEVICE, f"hipMemcpy failed: {rc}")
    return out


def loaded_runtime():
    """Paths of the HIP runtime and of libjiebahip.so mapped into this process."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for l in f:
                if "libamdhip64" in l or "libjiebahip" in l:
                    out.add(l.split()[-1])
    except OSError:
        pass
    return sorted(out)


def shard_bounds(doc_off, nparts):
    """jb_shard_bounds: the document ranges jb_cut_batch gives each device."""
    doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
    cut = np.zeros(nparts + 1, np.uint32)
    _check(lib().jb_shard_bounds(doc_off.ctypes.data, len(doc_off) - 1, nparts, cut.ctypes.data))
    return [int(x) for x in cut]


def split_points(buf, doc_off, nparts):
    """jb_split_points: byte cuts at document starts or Han-run starts."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    doc_off = np.ascontiguousarray(doc_off, dtype=np.uint64)
    cut = np.zeros(nparts + 1, np.uint64)
    _check(lib().jb_split_points(buf.ctypes.data, doc_off.ctypes.data, len(doc_off) - 1, nparts, cut.ctypes.data))
    return [int(x) for x in cut]


def go_log(x):
    return lib().jb_go_log(float(x))
