"""GPU parity: the MI355X path (through the C ABI) against the oracle,
bit-exact token boundaries.  Every test here runs kernels and needs the GPU."""
import os
import random

import numpy as np
import pytest

import jiebahip as J
import oracle as O
import synth

pytestmark = pytest.mark.gpu


def _pair(dp, ep, kind=J.JB_DICT_TXT, size_override=0):
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, kind=kind, size_override=size_override))
    o = O.Oracle.from_files(dp, ep, kind, size_override)
    return tk, o


def _pair_env(dp, ep, env, **kw):
    with pytest.MonkeyPatch.context() as mp:
        for k, v in env.items():
            mp.setenv(k, v)
        return _pair(dp, ep, **kw)


# k_zh's two forms: 4-wave workgroups with the weights gathered from HBM (what batches
# under 16 MiB get), and 16-wave workgroups with the weight table in LDS (the headline
# batches' form), forced with JB_ZH_WIDE=1 on these small ones; and k_nonzh as a launch of
# its own (JB_NZ_FUSE_MIB=0), where batches under 4 MiB otherwise run its work inside k_long
ZH_FORMS = {"auto": {}, "wide": {"JB_ZH_WIDE": "1"}, "nzapart": {"JB_NZ_FUSE_MIB": "0"}}


@pytest.fixture(scope="module", params=list(ZH_FORMS))
def small(syn_small, request):
    dp, ep, s = syn_small
    tk, o = _pair_env(dp, ep, ZH_FORMS[request.param])
    yield tk, o, s
    tk.close()


@pytest.fixture(scope="module", params=list(ZH_FORMS))
def full(syn_full, request):
    dp, ep, s = syn_full
    tk, o = _pair_env(dp, ep, ZH_FORMS[request.param])
    yield tk, o, s
    tk.close()


def _cmp_batch(tk, o, buf, off, hmm, label=""):
    gs, ge, gd = tk.cut_batch(buf, off, hmm)
    os_, oe, od = o.cut_batch(buf, off, hmm, nthreads=8)
    if not (np.array_equal(gs, os_) and np.array_equal(ge, oe)):
        n = min(len(gs), len(os_))
        bad = int(np.argmax((gs[:n] != os_[:n]) | (ge[:n] != oe[:n]))) if n else 0
        lo = int(min(gs[bad] if len(gs) > bad else 0, os_[bad] if len(os_) > bad else 0))
        ctx = bytes(np.asarray(buf)[max(0, lo - 30):lo + 60]).decode("utf-8", "replace")
        raise AssertionError(f"{label}: {len(gs)} vs {len(os_)} tokens; first diff #{bad} near byte {lo}: {ctx!r}; "
                             f"gpu={list(zip(gs[bad:bad+5], ge[bad:bad+5]))} ref={list(zip(os_[bad:bad+5], oe[bad:bad+5]))}")
    assert np.array_equal(gd, od), label


def _batch_of(texts):
    bs = [t.encode("utf-8") if isinstance(t, str) else t for t in texts]
    off = np.zeros(len(bs) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    buf = np.frombuffer(b"".join(bs) + b"\0" * 16, np.uint8)
    return buf, off


def test_reference_kats_mini_dict(kats, mini_paths):
    for kind in (J.JB_DICT_TXT, J.JB_DICT_PREFIX):
        tk = J.Tokenizer(J.make_config(dict_path=mini_paths[0], emit_path=mini_paths[1], kind=kind))
        o = O.Oracle.from_files(*mini_paths, kind=kind)
        cases = {c["name"]: c for c in kats["cut_real_data"]["cases"]}
        for name in ("cut 8", "cut 10", "cut 4", "cut 5", "cut 6", "cut 7"):
            c = cases[name]
            assert tk.Cut(c["text"], c["hmm"]) == c["want"], name
        for c in kats["cut_real_data"]["cases"] + [{"text": x["text"], "hmm": h} for x in kats["split_text"]["cases"]
                                                   for h in (False, True)]:
            assert tk.Cut(c["text"], c["hmm"]) == o.cut(c["text"], c["hmm"]), c["text"]
        for c in kats["cut_nonzh"]["cases"]:
            assert tk.Cut(c["text"], False) == c["want"]
        tk.close()


EDGE_TEXTS = [
    "", " ", "\t\n", "a", "中", "中文", "，", "。。。", "abc", "abc 中文 def", "中文abc中文",
    "english번역『하다』今天天氣很好，ステーションabc1231+1=2我昨天去上海*important*去",
    "　全角空格　中文　abc x\u0085y z",
    "𠀀𠀁𠀂中𪜀文",          # 4-byte Han (Ext-B/C)
    "㐀㐁㐂一二三㐃",        # Ext-A: absent from dict and emissions
    "丁" * 300,
    "一㐀丁" * 50,
    b"\xff\xfe" + "中文".encode() + b"\x80abc\xe4\xb8",
    "中文".encode() + b"\xed\xa0\x80\xc0\xaf\xf4\x90\x80\x80" + "文".encode() + b"\xe0\x80\xaf",
    "⺀⺙⺛⻳⼀⿕々〇〡〩〸〻豈鶴侮頻𖿰𖿱",  # every Han range edge
    "〆ゝ中ー文",
    "a1+1=2 中文 x　y",
    "丁" * 2719, "丁" * 2720, "丁" * 2721, "一丁" * 1400, "𠀀" * 2041,   # around the k_zh window limit
    ("中文。" * 900) + "丁" * 3000 + ("，中文" * 900),                   # long block between short ones
    # k_zh groups are 6144-byte spans with a 7168-byte window: blocks that start
    # at or just before a group edge, and ones that end at / just past the window
    "a" * 6141 + "丁" * 342, "a" * 6141 + "丁" * 343, "a" * 6144 + "丁" * 341 + "，" + "丁" * 5,
    "a" * 6143 + "丁" * 400, "中，" * 3072 + "丁" * 700, "a" * 6140 + "𠀀" * 300 + "丁" * 30,
    "，".join(["中文"] * 4000),                                           # many short blocks per group
    # k_zh_long (blocks of >= 8 KiB): all-3-byte ones by the whole-wave path, across its
    # 1024-rune windows; one with a 4-byte Han rune by the one-lane path
    "丁" * 2731, "一丁㐀中文" * 700, "中文" * 1500 + "𠀀" + "中文" * 1500,
    "a" * 6000 + "一丁㐀中文" * 900 + "。" + "中" * 10,
]


@pytest.mark.parametrize("hmm", [False, True])
def test_edge_cases(small, hmm):
    tk, o, s = small
    for t in EDGE_TEXTS:
        b = t.encode("utf-8") if isinstance(t, str) else t
        gs, ge = tk.cut_spans(b, hmm)
        os_, oe = o.cut_spans(b, hmm)
        assert np.array_equal(gs, os_) and np.array_equal(ge, oe), repr(t)


def test_invalid_utf8_and_doc_boundaries(small):
    """Multi-byte sequences cut by a document boundary decode as invalid bytes
    (each document is its own Go string)."""
    tk, o, s = small
    rng = random.Random(1)
    pieces = [x.encode() for x in ("中", "文", "a", " ", "　", "𠀀", "，")] + [b"\xe4", b"\xb8\xad", b"\xf0\x9f",
                                                                            b"\x80", b"\xc2", b"\xff"]
    texts = [b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 12))) for _ in range(400)]
    # split a valid string at arbitrary byte positions
    whole = "中文字符串测试abc中文𠀀𠀁".encode("utf-8")
    for cut in range(1, len(whole)):
        texts += [whole[:cut], whole[cut:]]
    buf, off = _batch_of(texts)
    for hmm in (0, 1):
        _cmp_batch(tk, o, buf, off, hmm, "invalid/boundaries")


def test_random_mixed_script(small):
    tk, o, s = small
    rng = random.Random(2)
    alphabet = [chr(c) for c in range(0x4E00, 0x4E00 + 3000, 3)] + ["㐀", "㒐", "a", "Z", "9", " ", "，", "。",
                                                                    "　", "ス", "한", " ", "\n", "𠀀"]
    texts = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 80))) for _ in range(2000)]
    buf, off = _batch_of(texts)
    for hmm in (0, 1):
        _cmp_batch(tk, o, buf, off, hmm, "mixed")


@pytest.mark.parametrize("hmm", [False, True])
def test_s10k_sentences(full, hmm):
    """Configs 2/3: 10k synthetic sentences (10-40 runes), HMM off/on."""
    tk, o, s = full
    buf, off, nr = s.corpus(synth.KIND_SENTENCES, 0, max_docs=10_000, target_bytes=1 << 30)
    assert len(off) - 1 == 10_000
    _cmp_batch(tk, o, buf, off, hmm, f"s10k hmm={hmm}")


@pytest.mark.parametrize("hmm", [False, True])
def test_docs_corpus(full, hmm):
    tk, o, s = full
    buf, off, nr = s.corpus(synth.KIND_DOCS, 1000, target_bytes=8 << 20)
    _cmp_batch(tk, o, buf, off, hmm, f"docs hmm={hmm}")


# JB_TEST_ZH_GROUPS: the groups to force, e.g. "12288" with a library built by
# `make ZH_GROUP=12288 OUT=../var/g12 OBJ=../var/g12o` and loaded through JB_LIB
ZH_GROUPS = [int(x) for x in os.environ.get("JB_TEST_ZH_GROUPS", "1024,3072,6144").split(",")]


@pytest.mark.parametrize("group", ZH_GROUPS)
def test_docs_corpus_zh_groups(syn_full, group, monkeypatch):
    """k_zh picks its group size by batch size (1 KiB under 16 MiB, 6 KiB at the
    headline's size); JB_ZH_GROUP (read at jb_open) forces one, so the large-batch
    group runs here on a small batch, both HMM settings, bit-exact."""
    dp, ep, s = syn_full
    monkeypatch.setenv("JB_ZH_GROUP", str(group))
    tk, o = _pair(dp, ep)
    monkeypatch.delenv("JB_ZH_GROUP")
    buf, off, nr = s.corpus(synth.KIND_DOCS, 2000 + group, target_bytes=6 << 20)
    for hmm in (False, True):
        _cmp_batch(tk, o, buf, off, hmm, f"docs group={group} hmm={hmm}")
    sbuf, soff, _ = s.corpus(synth.KIND_SENTENCES, 50, max_docs=3000, target_bytes=1 << 30)
    _cmp_batch(tk, o, sbuf, soff, True, f"sentences group={group}")
    tk.close()


@pytest.mark.parametrize("tail_group", [1024, 2048])
def test_docs_corpus_zh_tail_groups(syn_full, tail_group, monkeypatch):
    """JB_ZH_TAIL_KIB / JB_ZH_TAIL_GROUP (off by default): the last KiB of a batch in
    smaller k_zh groups (groups start at tail0 + (g - g1) * sgrp).  With the 6 KiB
    body group forced and a 1 MiB tail, a 6 MiB batch has both geometries; bit-exact
    with HMM on and off."""
    dp, ep, s = syn_full
    monkeypatch.setenv("JB_ZH_GROUP", "6144")
    monkeypatch.setenv("JB_ZH_TAIL_KIB", "1024")
    monkeypatch.setenv("JB_ZH_TAIL_GROUP", str(tail_group))
    tk, o = _pair(dp, ep)
    for k in ("JB_ZH_GROUP", "JB_ZH_TAIL_KIB", "JB_ZH_TAIL_GROUP"):
        monkeypatch.delenv(k)
    buf, off, nr = s.corpus(synth.KIND_DOCS, 2100 + tail_group, target_bytes=6 << 20)
    for hmm in (False, True):
        _cmp_batch(tk, o, buf, off, hmm, f"docs tail group={tail_group} hmm={hmm}")
    tk.close()


def test_graph_replay_after_add_word(syn_small):
    """A batch cut twice is replayed from a captured HIP graph; AddWord re-uploads
    the image (new device buffers), so the next cut must not replay the old graph."""
    dp, ep, s = syn_small
    tk, o = _pair(dp, ep)
    buf, off, nr = s.corpus(synth.KIND_DOCS, 31, target_bytes=1 << 20)
    for _ in range(3):  # direct, captured, replayed
        _cmp_batch(tk, o, buf, off, True, "before AddWord")
    text = bytes(np.asarray(buf)[: int(off[1])]).decode("utf-8")
    import re
    # two adjacent Han runes whose first is a word (AddWord adds no prefixes, so the
    # walk reaches the new word only through a key, tokenizer.go:475-478,580-585)
    word = next(m.group(0) for m in re.finditer("(?=([\u4e00-\u9fa5]{2}))", text)
                for m in [re.match(".*", m.group(1))] if (o.get(m.group(0)[0]) or 0) > 0 and o.get(m.group(0)) is None)
    tk.AddWord(word, 10_000_000)
    o.add_term(word, 10_000_000)
    for _ in range(3):
        _cmp_batch(tk, o, buf, off, True, "after AddWord")
    gs, ge, _ = tk.cut_batch(buf, off, True)
    assert any(bytes(np.asarray(buf)[a:b]).decode("utf-8") == word for a, b in zip(gs[:5000], ge[:5000]))
    tk.close()


@pytest.mark.parametrize("kind", [synth.KIND_LONG_PUNCT, synth.KIND_LONG_OOV])
def test_long_document(full, kind):
    """Config 5: one 1M-rune document (5a punctuated, 5b long OOV runs)."""
    tk, o, s = full
    buf, off, nr = s.corpus(kind, 77, target_runes=1_000_000)
    O.set_viterbi_backptr(True)  # same decisions as path copying (test_oracle_kats), O(m)
    try:
        for hmm in (0, 1):
            _cmp_batch(tk, o, buf, off, hmm, f"long kind={kind} hmm={hmm}")
    finally:
        O.set_viterbi_backptr(False)


def test_prefix_semantics_and_size_override(syn_small):
    dp, ep, s = syn_small
    tk, o = _pair(dp, ep, J.JB_DICT_PREFIX, J.JIEBA_SIZE)
    buf, off, nr = s.corpus(synth.KIND_DOCS, 5, target_bytes=1 << 20)
    for hmm in (0, 1):
        _cmp_batch(tk, o, buf, off, hmm, "prefix dict")
    tk.close()


def test_gob_dictionary_and_saved_image(syn_small, tmp_path):
    """NewJiebaTokenizer's gob loader (tokenizer.go:439-458) on a gob-encoded
    prefix map, then the same tokenizer saved and reopened from its image, and
    after AddWord: every form cuts as the oracle does on the same map."""
    import gobenc
    dp, ep, s = syn_small
    m = {}
    with open(dp, "rb") as f:
        for line in f.read().splitlines():
            w, c = line.split(b" ")[:2]
            m[w] = int(c)
            t = w.decode("utf-8")
            for i in range(1, len(t)):
                m.setdefault(t[:i].encode("utf-8"), 0)
    gp = str(tmp_path / "prefix_dictionary.gob")
    with open(gp, "wb") as f:
        f.write(gobenc.encode_map(m.items()))
    tk = J.Tokenizer.NewJiebaTokenizer(gp, ep)
    o = O.Oracle(gobenc.map_to_dict_lines(m).decode(), open(ep, encoding="utf-8").read(), 0,
                 size_override=J.JIEBA_SIZE)
    buf, off, nr = s.corpus(synth.KIND_DOCS, 6, target_bytes=1 << 20)
    for hmm in (0, 1):
        _cmp_batch(tk, o, buf, off, hmm, "gob dict")
    ip = str(tmp_path / "syn.jbimg")
    tk.save(ip)
    tk2 = J.Tokenizer.FromImage(ip)
    for hmm in (0, 1):
        _cmp_batch(tk2, o, buf, off, hmm, "image")
    word = "天氣很好"
    tk2.AddWord(word, 777)
    o.add_term(word, 777)
    tk2.save(ip)
    tk3 = J.Tokenizer.FromImage(ip)
    assert tk3.dict_get(word) == 777 and tk3.size == o.size
    text = "今天天氣很好，" + bytes(np.asarray(buf)[:4000]).decode("utf-8", "ignore")
    for hmm in (False, True):
        assert tk3.Cut(text, hmm) == o.cut(text, hmm)
    for t in (tk, tk2, tk3):
        t.close()


def test_add_word(mini_paths):
    tk = J.Tokenizer(J.make_config(dict_path=mini_paths[0], emit_path=mini_paths[1]))
    o = O.Oracle.from_files(*mini_paths, kind=0)
    text = "今天天氣很好，我昨天去上海"
    assert tk.Cut(text, False) == o.cut(text, False)
    tk.AddWord("天氣", 500)
    o.add_term("天氣", 500)
    assert tk.dict_get("天氣") == 500 and tk.size == o.size
    assert tk.Cut(text, False) == o.cut(text, False)
    assert "天氣" in tk.Cut(text, False)
    # freq < 1: suggestFreq (tokenizer.go:589-614)
    pieces = o.cut("很好", False)
    dsize = float(o.size)
    f = 1.0
    for p in pieces:
        v = o.get(p)
        f *= float(v if v is not None else 1) / dsize
    want = max(int(f * dsize) + 1, o.get("很好") or 1)
    tk.AddWord("很好", 0)
    o.add_term("很好", want)
    assert tk.dict_get("很好") == want
    assert tk.Cut(text, True) == o.cut(text, True)
    tk.close()


def test_add_word_atomic(syn_small, tmp_path):
    """AddWord that fails (a reachable word of 256 runes: JB_ELIMIT) changes nothing:
    not the dictionary, not pd.size, not the device image (tokenizer.go:372-379,580-585)."""
    dp, ep, s = syn_small
    d2 = str(tmp_path / "dict255.txt")
    with open(dp, encoding="utf-8") as f:
        base = f.read()
    with open(d2, "w", encoding="utf-8") as f:  # every prefix of the long word is a key, so it is reachable
        f.write(base + "".join(f"{'丁' * k} 3\n" for k in range(1, 256)))
    tk, o = _pair(d2, ep)
    text = "丁" * 300 + "，" + "中文" * 20
    buf, off, _ = s.corpus(synth.KIND_DOCS, 17, target_bytes=1 << 20)
    before = tk.cut_batch(buf, off, True)
    size0 = tk.size
    with pytest.raises(J.JbError) as e:
        tk.AddWord("丁" * 256, 5)
    assert e.value.code == J.JB_ELIMIT
    assert tk.dict_get("丁" * 256) is None and tk.size == size0 == o.size
    assert tk.Cut(text, True) == o.cut(text, True)
    after = tk.cut_batch(buf, off, True)
    assert all(np.array_equal(a, b) for a, b in zip(before, after))
    tk.AddWord("丁" * 255, 9)  # the limit itself still works
    o.add_term("丁" * 255, 9)
    assert tk.Cut(text, True) == o.cut(text, True)
    tk.close()


def test_open_image_with_log_table(syn_small):
    """The Go binding's constructor path: jb_image_build, jb_image_log_keys, math.Log
    of each key, jb_open_image (the trie placed once, the weights recomputed from the
    table).  An identity table keeps bit parity; a perturbed table cuts exactly as
    jb_open with the same table does."""
    import math
    dp, ep, s = syn_small
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus(synth.KIND_DOCS, 12, target_bytes=1 << 20)
    img = J.Image(J.make_config(dict_path=dp, emit_path=ep))
    keys = [int(x) for x in img.log_keys()]
    tk = J.Tokenizer.from_image(img, logs={k: J.go_log(k) for k in keys})
    for hmm in (False, True):
        _cmp_batch(tk, o, buf, off, hmm, "jb_open_image, identity table")
    tk.close()
    bump = {k: math.nextafter(J.go_log(k), math.inf if i % 2 else -math.inf) for i, k in enumerate(keys)}
    a = J.Tokenizer.from_image(J.Image(J.make_config(dict_path=dp, emit_path=ep)), logs=bump)
    b = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, logs=bump))
    ra, rb = a.cut_batch(buf, off, True), b.cut_batch(buf, off, True)
    assert all(np.array_equal(x, y) for x, y in zip(ra, rb))
    a.close()
    b.close()


def test_empty_batch_and_docs(small):
    tk, o, s = small
    buf, off = _batch_of(["", "", "中文", "", "abc", ""])
    gs, ge, gd = tk.cut_batch(buf, off, True)
    os_, oe, od = o.cut_batch(buf, off, True)
    assert np.array_equal(gs, os_) and np.array_equal(ge, oe) and np.array_equal(gd, od)
    buf, off = _batch_of([])
    gs, ge, gd = tk.cut_batch(buf, off, True)
    assert len(gs) == 0 and list(gd) == [0]


def test_device_api_and_profile(small):
    """jb_cut_device on torch-owned HBM buffers (the bench path) equals the
    host-batch path; per-kernel event timing records every launch."""
    import torch
    tk, o, s = small
    buf, off, nr = s.corpus(synth.KIND_DOCS, 9, target_bytes=2 << 20)
    dev = torch.device("cuda:0")
    d_text = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    tk.profile(True)
    tk.profile_reset()
    stream = torch.cuda.current_stream().cuda_stream
    ps, pe, pd, pn = tk.cut_device(d_text.data_ptr(), int(off[-1]), d_off.data_ptr(), len(off) - 1, True, stream)
    torch.cuda.synchronize()
    prof = tk.profile_read()
    tk.profile(False)
    assert prof["k_zh"][1] == 1 and prof["k_zh"][0] > 0
    n = int(J.dev_to_host(pn, 8, np.uint64)[0])
    gs = J.dev_to_host(ps, 4 * n, np.uint32)
    ge = J.dev_to_host(pe, 4 * n, np.uint32)
    gd = J.dev_to_host(pd, 8 * len(off), np.uint64)
    hs, he, hd = tk.cut_batch(buf, off, True)
    assert np.array_equal(gs, hs) and np.array_equal(ge, he) and np.array_equal(gd, hd)


@pytest.mark.parametrize("nfill", [20000, 3000])
@pytest.mark.parametrize("kind", [J.JB_DICT_TXT, J.JB_DICT_PREFIX])
def test_record_overflow_paths(tmp_path, syn_small, kind, nfill):
    """Dictionaries that push k_walk's packed records past their limits: runes
    with more than 4 edges, edges longer than 8 runes (k_zh's redo with the
    global best array) and more than 2^14 distinct weights (14-bit indices;
    nfill 20000).  With 3000 fill words the weight table fits k_zh's LDS copy, and
    JB_ZH_WIDE=1 runs the wide form on the same overflow records."""
    _, ep, _ = syn_small
    rng = random.Random(11)
    pool = [chr(c) for c in range(0x4E00, 0x4E00 + 600)]
    lines, seqs = [], []
    f = 7
    for _ in range(40):  # nested chains: every prefix of a 6..24-rune string is a word
        s = "".join(rng.choice(pool) for _ in range(rng.randint(6, 24)))
        seqs.append(s)
        for k in range(1, len(s) + 1):
            if rng.random() < 0.8:
                f += rng.randint(1, 5)
                lines.append(f"{s[:k]} {f}")
    fill = []
    for i in range(nfill):  # distinct frequencies (20000: > 2^14 weights)
        w = rng.choice(pool) + rng.choice(pool) + (rng.choice(pool) if i % 3 == 0 else "")
        fill.append(w)
        lines.append(f"{w} {1000 + 3 * i}")
    dp = tmp_path / "dict.txt"
    dp.write_text("\n".join(lines) + "\n", encoding="utf-8")
    tk, o = _pair_env(str(dp), ep, ZH_FORMS["wide"], kind=kind,
                      size_override=60101967 if kind == J.JB_DICT_PREFIX else 0)
    try:
        texts = []
        for _ in range(400):
            parts = []
            for _ in range(rng.randint(1, 12)):
                r = rng.random()
                if r < 0.35:
                    s = rng.choice(seqs)
                    parts.append(s[: rng.randint(1, len(s))])
                elif r < 0.7:
                    parts.append(rng.choice(fill))
                elif r < 0.9:
                    parts.append("".join(rng.choice(pool) for _ in range(rng.randint(1, 6))))
                else:
                    parts.append(rng.choice(["，", "。", " ab12 ", "\n"]))
            texts.append("".join(parts))
        texts.append("".join(seqs))  # one block through every chain
        texts.append("".join(seqs) * 6)  # the same as a long block (k_zh_long's overflow walks)
        buf, off = _batch_of(texts)
        for hmm in (False, True):
            _cmp_batch(tk, o, buf, off, hmm, f"overflow kind={kind} hmm={hmm}")
        # the same texts in batches of at most 4 KiB (k_small: its DP walks runes
        # with more than 4 edges again, edges up to the longest key)
        for i, docs in enumerate(_small_batches(texts)):
            bufs, offs = _batch_of(docs)
            for hmm in (False, True):
                _cmp_batch(tk, o, bufs, offs, hmm, f"overflow small batch {i} kind={kind} hmm={hmm}")
    finally:
        tk.close()


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("spec", ["1", "0", "2", "3"])
@pytest.mark.parametrize("kind", [J.JB_DICT_TXT, J.JB_DICT_PREFIX])
def test_long_blocks_many(tmp_path, syn_small, kind, spec, fused, monkeypatch):
    """The k_long_* kernels: several long blocks in one batch, sharing path-bitmap
    words across a 1-byte gap and across a document boundary; edges longer than
    a 64-rune segment (a piece spans whole segments); runes with more than 4
    items (the chain's side list) and windows whose items overflow it (the chain
    walks the trie itself).  With the speculative choices and the path chain
    (JB_LONG_SPEC=1, the default), with the decided chain (3), with the exact chain
    alone (0), and with wrong choices planted (2: the verification must send every
    block to the exact chain).  The long-block kernels as one launch (k_long, JB_LONG_FUSED=1,
    the default: phases whose items are claimed in phase order, each phase ending in a
    counted wait that needs no grid residency) and as separate launches (0)."""
    monkeypatch.setenv("JB_LONG_SPEC", spec)
    monkeypatch.setenv("JB_LONG_FUSED", fused)
    _, ep, _ = syn_small
    rng = random.Random(5)
    pool = [chr(c) for c in range(0x4E00, 0x4E00 + 300)]
    lines = [f"{'丁' * k} {10 + k}" for k in range(1, 21)]  # every 丁 starts up to 20 items
    longw = []
    for _ in range(30):  # 65..200-rune words; every prefix is a key, the word itself the likeliest
        w = "".join(rng.choice(pool) for _ in range(rng.randint(65, 200)))
        longw.append(w)
        lines += [f"{w[:k]} {rng.randint(1, 3) if k < len(w) else 10 ** 6}" for k in range(1, len(w) + 1)]
    dp = tmp_path / "dict.txt"
    dp.write_text("\n".join(lines) + "\n", encoding="utf-8")
    tk, o = _pair(str(dp), ep, kind=kind, size_override=60101967 if kind == J.JB_DICT_PREFIX else 0)
    try:
        a = "".join(rng.choice(longw) for _ in range(40))
        b = "丁" * 3000
        c = "".join(rng.choice([rng.choice(longw), "丁" * rng.randint(1, 30),
                                "".join(rng.choice(pool) for _ in range(rng.randint(1, 40)))]) for _ in range(300))
        texts = [a + "x" + c, b, c + "。" + a, "短文本，中文", b[:2800] + a[:3000], "丁乙" * 1500]
        buf, off = _batch_of(texts)
        for hmm in (False, True):
            _cmp_batch(tk, o, buf, off, hmm, f"long blocks kind={kind} hmm={hmm}")
            assert tk.last_stats()["long_blocks"] >= 6
    finally:
        tk.close()


def test_long_wait_bound(tmp_path, syn_small, monkeypatch):
    """k_long's phase waits give up after JB_LONG_WAIT_US without progress (VERDICT r05
    item 6): with a debug-small bound (20 us) a long block, whose k_long_dp
    item alone takes milliseconds, makes the waiting workgroups give up; the kernel
    drains (every workgroup leaves once CNT_ERR bit 1 is set) and the call returns
    JB_EDEVICE, from a host batch and, through jb_device_status, from the device path.
    The same context then cuts the next batch bit-exact, and with the default bound the
    long block is bit-exact too."""
    import torch
    dp, ep, _ = syn_small
    rng = random.Random(17)
    pool = [chr(c) for c in range(0x4E00, 0x4E00 + 3000)]
    longdoc = "".join(rng.choice(pool) for _ in range(300_000))  # one unpunctuated Han run
    buf, off = _batch_of([longdoc, "短文本，中文"])
    monkeypatch.setenv("JB_LONG_WAIT_US", "20")
    tk, o = _pair(dp, ep)
    try:
        with pytest.raises(J.JbError) as ei:
            tk.cut_batch(buf, off, True)
        assert ei.value.code == J.JB_EDEVICE, ei.value
        nbytes = int(off[-1])
        d_text = torch.from_numpy(np.concatenate([buf[:nbytes], np.zeros(64, np.uint8)])).cuda()
        d_off = torch.from_numpy(np.asarray(off, np.int64)).cuda()
        stream = torch.cuda.current_stream().cuda_stream
        tk.cut_device(d_text.data_ptr(), nbytes, d_off.data_ptr(), len(off) - 1, True, stream)
        with pytest.raises(J.JbError) as ei:
            tk.device_status(stream)
        assert ei.value.code == J.JB_EDEVICE, ei.value
        sb, soff = _batch_of(["短文本，中文", "我们在这里" * 20])  # no long block: unaffected
        _cmp_batch(tk, o, sb, soff, True, "after a given-up wait")
        s_text = torch.from_numpy(np.concatenate([sb[: int(soff[-1])], np.zeros(64, np.uint8)])).cuda()
        s_off = torch.from_numpy(np.asarray(soff, np.int64)).cuda()
        tk.cut_device(s_text.data_ptr(), int(soff[-1]), s_off.data_ptr(), len(soff) - 1, True, stream)
        tk.device_status(stream)  # (the next device pipeline starts with a clear error word)
    finally:
        tk.close()
    monkeypatch.delenv("JB_LONG_WAIT_US")
    tk, o = _pair(dp, ep)
    try:
        _cmp_batch(tk, o, buf, off, True, "long block, default wait bound")
    finally:
        tk.close()


def test_long_block_4byte_rune_after_junk(tmp_path, syn_small, monkeypatch):
    """A long block with a 4-byte Han rune, cut in a workspace that the batch before
    filled with DAG records: its stride-3 slots past the 4-byte rune are
    not rune starts, so k_long_spec must leave such a block alone (k_long_dp takes it
    on its general path) instead of reading the stale records there."""
    monkeypatch.setenv("JB_LONG_SPEC", "1")
    dp, ep, _ = syn_small
    tk, o = _pair(dp, ep)
    try:
        rng = random.Random(11)
        pool = [chr(c) for c in range(0x4E00, 0x4E00 + 2000)]
        han = "".join(rng.choice(pool) for _ in range(12000))
        junk = [han[:6000], han[6000:]]  # every slot of both blocks gets a record
        with4 = [han[:1500] + "\U00020000" + han[1502:6000], "\U00020000" + han[6002:12000]]
        assert sum(len(t.encode()) for t in with4) <= sum(len(t.encode()) for t in junk)
        for hmm in (False, True):
            for texts in (junk, with4):
                buf, off = _batch_of(texts)
                _cmp_batch(tk, o, buf, off, hmm, f"4-byte rune after junk hmm={hmm}")
    finally:
        tk.close()


def test_synthetic_golden_vectors(syn_golden):
    """The GPU path reproduces the committed golden vectors (oracle output frozen in tests/golden)."""
    g, docs, dp, ep = syn_golden
    buf, off = _batch_of(docs)
    for kind, size in ((J.JB_DICT_TXT, 0), (J.JB_DICT_PREFIX, 60101967)):
        tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, kind=kind, size_override=size))
        try:
            for hmm in (False, True):
                gs, ge, gd = tk.cut_batch(buf, off, hmm)
                for c in g["cases"]:
                    if c["kind"] != kind or c["hmm"] != hmm:
                        continue
                    d = c["doc"]
                    a, b = int(gd[d]), int(gd[d + 1])
                    base = int(off[d])
                    assert (gs[a:b] - base).tolist() == c["starts"], (kind, hmm, d)
                    assert (ge[a:b] - base).tolist() == c["ends"], (kind, hmm, d)
        finally:
            tk.close()


@pytest.mark.parametrize("split", ["-1", "0", "1", "2"])
def test_repeat_runs_identical(syn_small, split):
    """The same batch cut several times gives the same tokens every time (and the oracle's):
    k_mark_walk with 1, 2 or 4 workgroups per tile (JB_MW_SPLIT; -1 = 2 for a batch of at most
    one tile per CU, as here), whose entries are shared out by index.  A split by walk-list
    position, whose order comes from LDS atomics, once walked some entries twice and some never,
    which only showed as two runs of one batch disagreeing."""
    dp, ep, s = syn_small
    tk, o = _pair_env(dp, ep, {"JB_MW_SPLIT": split})
    try:
        buf, off, _ = s.corpus(synth.KIND_SENTENCES, 51, max_docs=3000, target_bytes=512 << 10)
        for hmm in (False, True):
            _cmp_batch(tk, o, buf, off, hmm, f"split {split} hmm {hmm}")
            first = tk.cut_batch(buf, off, hmm)
            for _ in range(3):
                again = tk.cut_batch(buf, off, hmm)
                assert all(np.array_equal(a, b) for a, b in zip(first, again)), f"split {split} hmm {hmm}"
    finally:
        tk.close()


def test_cut_batch_into_caller_arrays(small):
    """jb_cut_batch_into: same spans as jb_cut_batch; too-small arrays give
    JB_ELIMIT with the needed count, and the binding retries."""
    tk, o, s = small
    buf, off, _ = s.corpus(synth.KIND_SENTENCES, 40, max_docs=300, target_bytes=1 << 20)
    for hmm in (False, True):
        gs, ge, gd = tk.cut_batch(buf, off, hmm)
        tiny = (np.empty(3, np.uint64), np.empty(3, np.uint64), np.empty(len(off), np.uint64))
        ts, te, td, out = tk.cut_batch_into(buf, off, hmm, tiny)
        assert len(out[0]) >= len(gs)
        assert np.array_equal(ts, gs) and np.array_equal(te, ge) and np.array_equal(td, gd)
        ts2, te2, td2, _ = tk.cut_batch_into(buf, off, hmm, out)  # reuse
        assert np.array_equal(ts2, gs) and np.array_equal(td2, gd)


@pytest.mark.parametrize("pack", ["1", "0"])
def test_cut_batch_into32(syn_small, pack, monkeypatch):
    """jb_cut_batch_into32 (u32 spans relative to doc_off[0], what the Go binding slices its
    strings with) gives jb_cut_batch_into's spans less doc_off[0]: a batch that does not
    start at byte 0 of its buffer, cut in several pieces (JB_PIECE_KIB=256), over two
    devices (JB_DEVICE_WRAP), as a k_small batch (<= 4 KiB), with arrays too small (the
    binding retries with the count the library returns); packed spans on and off."""
    monkeypatch.setenv("JB_SPAN_PACK", pack)
    monkeypatch.setenv("JB_PIECE_KIB", "256")
    dp, ep, s = syn_small
    buf, off, _ = s.corpus(synth.KIND_SENTENCES, 41, max_docs=4000, target_bytes=1 << 20)
    off = np.asarray(off, np.uint64)
    lo = 37  # documents 37.. : the batch starts inside the buffer
    sub = off[lo:]
    small = off[lo:lo + 12]
    for ndev, wrap in ((1, None), (2, "1")):
        if wrap:
            monkeypatch.setenv("JB_DEVICE_WRAP", wrap)
        tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, ndevices=ndev))
        try:
            for hmm in (False, True):
                for o_ in (sub, small):
                    ws, we, wd, _ = tk.cut_batch_into(buf, o_, hmm)
                    b0 = int(o_[0])
                    tiny = (np.empty(2, np.uint32), np.empty(2, np.uint32), np.empty(len(o_), np.uint64))
                    for out in (None, tiny):
                        gs, ge, gd, _ = tk.cut_batch_into32(buf, o_, hmm, out)
                        assert gs.dtype == np.uint32 and len(gs) == len(ws), (ndev, hmm, len(o_))
                        assert np.array_equal(gs.astype(np.uint64) + b0, ws) and np.array_equal(ge.astype(np.uint64) + b0, we)
                        assert np.array_equal(gd, wd)
        finally:
            tk.close()


@pytest.mark.parametrize("pack", ["1", "0"])
def test_packed_spans_escapes(syn_small, pack, monkeypatch):
    """Host batches' spans come back packed (JB_SPAN_PACK=1, the default: k_span_pack's
    u16 gap | length << 6 per token, decoded on the host by blocks of 4,096 tokens) or as
    u32 spans (0).  Escapes (gap >= 63 or length >= 1,023): long gaps (a non-Han block
    without an alnum byte has no tokens, tokenizer.go:290-293), long tokens (an alnum run
    is one token, :296-300), gaps of exactly 62 / 63 bytes and tokens of exactly 1,022 /
    1,023 bytes, thousands of escapes in a row (an unsorted side list), blocks of 4,096
    tokens that start right after an escape; several pieces (JB_PIECE_KIB=256) and two
    devices (JB_DEVICE_WRAP): every span and doc_tok against the oracle, through
    jb_cut_batch and jb_cut_batch_into."""
    monkeypatch.setenv("JB_SPAN_PACK", pack)
    monkeypatch.setenv("JB_PIECE_KIB", "256")
    dp, ep, _ = syn_small
    rng = random.Random(23)
    pool = [chr(c) for c in range(0x4E00, 0x4E00 + 3000)]
    han = lambda n: "".join(rng.choice(pool) for _ in range(n))  # noqa: E731
    texts = [
        han(50) + "，" * 30000 + han(20),          # 90 KB without a token
        "a" * 70000 + han(30),                       # one 70,000-byte token
        han(10) + "；" * 21 + han(5) + "；" * 20 + "é" + han(5),  # gaps of exactly 63 (escaped) and 62 bytes
        "b" * 1023 + " " + "c" * 1022 + " " + "d" * 1024 + han(8),  # tokens of 1,023 / 1,024 (escaped) and 1,022
        "".join("e" * 1100 + "，" * 30 for _ in range(3000)),  # 6,000 escapes in a row
        han(4096 * 3) + "x" * 66000 + han(4096),       # escapes in the middle of 4,096-token blocks
        "".join(han(rng.randint(1, 30)) + rng.choice(["，", "。", " ab1 ", "ーー"]) for _ in range(3000)),
    ]
    buf, off = _batch_of(texts)
    for ndev, wrap in ((1, None), (2, "1")):
        if wrap:
            monkeypatch.setenv("JB_DEVICE_WRAP", wrap)
        tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, ndevices=ndev))
        o = O.Oracle.from_files(dp, ep, 0, 0)
        try:
            for hmm in (False, True):
                _cmp_batch(tk, o, buf, off, hmm, f"packed={pack} ndev={ndev} hmm={hmm}")
                os_, oe, od = o.cut_batch(buf, off, hmm, nthreads=8)
                ts, te, td, _ = tk.cut_batch_into(buf, off, hmm)
                assert np.array_equal(ts, os_) and np.array_equal(te, oe) and np.array_equal(td, od)
                t32, e32, d32, _ = tk.cut_batch_into32(buf, off, hmm)
                assert np.array_equal(t32.astype(np.uint64), os_) and np.array_equal(e32.astype(np.uint64), oe)
                assert np.array_equal(d32, od)
        finally:
            tk.close()


def _tie_emissions():
    """Emissions under which the 3-rune HMM run 甲乙丙 has an exact route tie
    vE + T_EB == vS + T_SB > minFloat at its third rune (state B, Q12), found by
    stepping eS(乙) one ulp at a time (float64 adds as in tokenizer.go:686-716)."""
    import math
    START_B, START_S = -0.26268660809250016, -1.4652633398537678  # tokenizer.go:629-632
    T_BE, T_SS, T_EB, T_SB = -0.51082562376599, -0.6658631448798212, -0.5897149736854513, -0.7211965654669841
    eB0, eS0, eE1 = -3.0, -4.0, -5.0
    vE1 = ((START_B + eB0) + T_BE) + eE1
    a = vE1 + T_EB
    pS = (START_S + eS0) + T_SS
    x = (a - T_SB) - pS
    for _ in range(4096):
        if (pS + x) + T_SB == a:
            break
        x = math.nextafter(x, -math.inf if (pS + x) + T_SB > a else math.inf)
    else:
        raise AssertionError("no exact tie found")
    return {"B": {"甲": eB0, "乙": -6.0, "丙": -2.5, "词": -3.0}, "E": {"乙": eE1, "丙": -2.0, "语": -3.0},
            "M": {"乙": -7.0}, "S": {"甲": eS0, "乙": x, "丙": -3.5}}


def test_viterbi_ties_counted(tmp_path):
    """Exact stateTransitionRoute ties (tokenizer.go:748-753, resolved in Go map
    order) are counted on the GPU (jb_last_stats) exactly as the oracle counts
    them, in each Viterbi code path: k_zh's deferred runs (all-3-byte window),
    its general path (a 4-byte Han rune in the window) and k_zh_long (a block
    of >= 8 KiB); the cut itself is bit-exact."""
    import json
    dp, ep = tmp_path / "d.txt", tmp_path / "e.json"
    dp.write_text("词 5\n词语 1000\n", encoding="utf-8")
    ep.write_text(json.dumps(_tie_emissions(), ensure_ascii=False), encoding="utf-8")
    texts = ["甲乙丙", "x，甲乙丙。", "\U00020000，甲乙丙", "词语" * 1400 + "甲乙丙"]
    for t in texts:
        tk, o = _pair(str(dp), str(ep))
        buf, off = _batch_of([t])
        _cmp_batch(tk, o, buf, off, True, t[:8])
        st = tk.last_stats()
        assert o.ties >= 1, t[:8]
        assert st["viterbi_ties"] == o.ties, (t[:8], st, o.ties)
        if len(t) > 4000:
            assert st["long_blocks"] == 1
        tk.close()


from conftest import ROOT, real_data_dir  # noqa: E402

SENTENCE = "我昨天去上海交通大學與老師討論量子力學"  # tokenizer_test.go:531


def _spans_line(line):
    parts = line.split()
    n = int(parts[1])
    v = list(map(int, parts[2:]))
    assert len(v) == 2 * n
    return v[0::2], v[1::2]


def test_c_abi_smoke_program(syn_small, tmp_path):
    """A C99 program bound to include/jiebahip.h (what cgo sees): open as the Go binding
    does (jb_image_build, jb_image_log_keys, jb_open_image), Cut, a batch,
    a batch into caller arrays, AddWord with suggestFreq, Cut again — every span
    against the oracle."""
    import subprocess
    dp, ep, s = syn_small
    exe = str(tmp_path / "c_abi_smoke")
    lib = os.path.join(ROOT, "jieba-go_amd", "lib")
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I",
                           os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c_abi_smoke.c"), "-L", lib,
                           "-ljiebahip", "-Wl,-rpath," + lib, "-o", exe])
    buf, off, _ = s.corpus(synth.KIND_DOCS, 3, target_bytes=20_000)
    text = SENTENCE.encode() + b" abc 12 " + bytes(buf[:int(off[1])]) + "㐀㐁一二".encode()
    tf = tmp_path / "text.txt"
    tf.write_bytes(text)
    word = "量子力學"
    r = subprocess.run([exe, dp, ep, str(tf), word], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = {ln.split()[0]: ln for ln in r.stdout.splitlines()}
    assert int(out["log"].split()[2]) > 2  # opened through jb_image_build + jb_open_image with a log table
    o = O.Oracle.from_files(dp, ep, 0)
    s1, e1 = o.cut_spans(text, True)
    assert _spans_line(out["cut"]) == (s1.tolist(), e1.tolist())
    n = len(text)
    both = np.frombuffer(text + text + b"\0" * 16, np.uint8)
    off2 = np.array([0, n, 2 * n], np.uint64)
    bs, be, bd = o.cut_batch(both, off2, False)
    assert _spans_line(out["batch"]) == (bs.tolist(), be.tolist())
    assert list(map(int, out["doc_tok"].split()[1:])) == bd.tolist()
    hs, he, _ = o.cut_batch(both, off2, True)
    assert _spans_line(out["into"]) == (hs.tolist(), he.tolist())
    assert _spans_line(out["into32"]) == (hs.tolist(), he.tolist())
    freq = int(out["freq"].split()[1])
    o.add_term(word, freq)
    assert int(out["freq"].split()[3]) == o.size
    s2, e2 = o.cut_spans(text, True)
    assert _spans_line(out["cut2"]) == (s2.tolist(), e2.tolist())


def test_cpp_tokenizer_mirror(syn_small, tmp_path):
    """The C++ mirror of the Go Tokenizer API (libjbtok.so): NewTokenizer, Cut,
    CutParallel, CutBatch, AddWord, Save/FromImage — tokens against the oracle."""
    import subprocess
    dp, ep, s = syn_small
    exe = str(tmp_path / "cpp_tok_smoke")
    lib = os.path.join(ROOT, "jieba-go_amd", "lib")
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "jieba-go_amd", "host"),
                           os.path.join(ROOT, "tests", "cpp_tok_smoke.cpp"), "-L", lib, "-ljbtok", "-ljiebahip",
                           "-Wl,-rpath," + lib, "-o", exe])
    buf, off, _ = s.corpus(synth.KIND_DOCS, 5, target_bytes=8_000)
    text = (SENTENCE + " x1 ").encode() + bytes(buf[:int(off[1])])
    tf = tmp_path / "text.txt"
    tf.write_bytes(text)
    word = "交通大學與"
    r = subprocess.run([exe, dp, str(tf), word, str(tmp_path / "img.jbi")], capture_output=True, timeout=120,
                       cwd=os.path.dirname(ep))
    assert r.returncode == 0, r.stderr
    got = {}
    for ln in r.stdout.decode("utf-8").splitlines():
        tag, *toks = ln.split("|")
        got.setdefault(tag, []).append(toks)
    o = O.Oracle.from_files(dp, ep, 0)
    t = text.decode("utf-8")
    assert got["cut_hmm"][0] == o.cut(t, True)
    assert got["cut_nohmm"][0] == o.cut(t, False)
    assert got["cut_parallel"][0] == o.cut(t, True)
    assert got["batch_doc"] == [o.cut(t, True), [], o.cut(t, True)]
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
    f = tk.suggest_freq(word)
    tk.close()
    o.add_term(word, f)
    assert got["cut_added"][0] == o.cut(t, True)
    o.add_term("討論量子", 7)  # (AddWord with the caller's log function)
    assert got["cut_added_log"][0] == o.cut(t, True)
    assert got["cut_image"][0] == o.cut(t, True)


def test_caller_log_table_gpu(syn_small):
    """Identity jb_config log table (math.Log values for every key the image uses)
    keeps bit parity on the GPU; a perturbed table reopens and cuts (CPU tests pin
    its weights)."""
    dp, ep, s = syn_small
    img = J.Image(J.make_config(dict_path=dp, emit_path=ep))
    keys = [int(x) for x in img.log_keys()]
    img.close()
    logs = {k: J.go_log(k) for k in keys}
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, logs=logs))
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus(synth.KIND_DOCS, 11, target_bytes=1 << 20)
    for hmm in (False, True):
        _cmp_batch(tk, o, buf, off, hmm, "identity log table")
    # AddWord with caller logs for the new frequency and size
    w = "量子力學"
    f = 77
    tk.add_log({f: J.go_log(f), tk.size + f: J.go_log(tk.size + f)})
    tk.AddWord(w, f)
    o.add_term(w, f)
    _cmp_batch(tk, o, buf, off, True, "identity log table after AddWord")
    tk.close()


@pytest.mark.skipif(real_data_dir() is None, reason="real jieba data (LFS objects) not present; set JIEBA_DATA_DIR")
def test_gpu_real_data_kats(kats):
    """TestCut "cut 1..10" (tokenizer_test.go:28-59) through the HIP path on the
    genuine dictionary and emission table (sha256-checked), both as
    NewJiebaTokenizer's map (dict.txt with prefix semantics, size 60,101,967) and,
    when present, prefix_dictionary.gob itself."""
    d = real_data_dir()
    ep = os.path.join(d, "prob_emit.json")
    tks = [J.Tokenizer(J.make_config(dict_path=os.path.join(d, "dict.txt"), emit_path=ep, kind=J.JB_DICT_PREFIX,
                                     size_override=J.JIEBA_SIZE))]
    gp = os.path.join(d, "prefix_dictionary.gob")
    if os.path.exists(gp):
        tks.append(J.Tokenizer(J.make_config(dict_path=gp, emit_path=ep, kind=J.JB_DICT_GOB)))
    for tk in tks:
        for c in kats["cut_real_data"]["cases"]:
            assert tk.Cut(c["text"], c["hmm"]) == c["want"], c["name"]
        tk.close()


def test_nonzh_blocks_across_chunks_and_tiles(small):
    """cutNonZh (tokenizer.go:289-310) where k_nonzh's block bounds come from the
    lane masks: alnum bytes at 16-byte chunk edges, non-Han blocks longer than a
    4 KiB tile with their first alnum byte far from the block start, blocks with
    no alnum at all (no tokens), several blocks in one chunk, and document
    boundaries inside non-Han runs."""
    tk, o, s = small
    rng = random.Random(77)
    pieces = ["。", "，", " ", "\t", "…", "abc", "Z9", "1", "中文", "世界", "é", "—", "!!", "x y", "　"]
    docs = []
    for n in range(60):
        k = rng.choice([1, 3, 15, 16, 17, 31, 33, 200, 5000, 9000])
        parts = []
        while sum(len(p.encode()) for p in parts) < k:
            parts.append(rng.choice(pieces))
        docs.append("".join(parts))
    # a long punctuation-only run with one alnum byte at its very end, across tiles
    docs.append("，" * 3000 + "a")
    docs.append("a" + "，" * 3000)
    docs.append("。" * 2000)  # no alnum: no tokens
    docs.append(" " * 4095 + "q" + "中" + " " * 20 + "7")
    docs.append("x" * 10000)  # one alnum run over several tiles
    for pad in range(0, 33):  # an alnum run starting at every offset of a chunk
        docs.append("，" * (pad // 3) + " " * (pad % 3) + "ab12" + "字")
    buf, off = _batch_of(docs)
    for hmm in (False, True):
        _cmp_batch(tk, o, buf, off, hmm, "nonzh edges")
    # the same texts as one document (blocks spanning the former boundaries)
    buf1, off1 = _batch_of(["".join(docs)])
    _cmp_batch(tk, o, buf1, off1, True, "nonzh one document")


def test_nonzh_mask_tokenizer_rune_classes(small):
    """k_nonzh tokenizes a block that fits one round of four 16-byte loads from bit
    masks (nonzh_masks) and decodes only its bytes >= 0x80 rune by rune; longer
    blocks take the per-byte path.  cutNonZh's rules (tokenizer.go:289-310) over
    every class the masks separate: alnum runs, ASCII punctuation, all six ASCII
    spaces, the non-ASCII spaces of unicode.IsSpace (U+0085, U+00A0, U+1680, U+2000,
    U+200A, U+2028, U+2029, U+202F, U+205F, U+3000), 2/3/4-byte runes, invalid and
    truncated sequences, at every start offset of a chunk and with block lengths
    around the 48/64-byte edges of the mask path, between Han runs."""
    tk, o, s = small
    rng = random.Random(4242)
    spaces = [" ", "\t", "\n", "\v", "\f", "\r", "\u0085", " ", " ", " ", " ",
              " ", " ", " ", " ", "　"]
    others = ["a", "Zq", "09", "x1y2", "!", "#", "-", ".", "，", "é", "ß", "—", "😀", "Ω", "ｱ", "k"]
    bad = [b"\x80", b"\xff", b"\xc3", b"\xe4\xb8", b"\xf0\x9f\x98", b"\xc0\xaf", b"\xed\xa0\x80", b"\xf4\x90\x80\x80"]
    docs = []
    for n in range(400):
        parts = [b"\xe4\xb8\xad" * rng.randint(0, 20)]  # Han before the block: every start offset
        k = rng.choice([1, 2, 5, 15, 16, 17, 31, 32, 33, 46, 47, 48, 49, 50, 63, 64, 65, 70, 100])
        blk = b""
        while len(blk) < k:
            r = rng.random()
            if r < 0.3:
                blk += rng.choice(spaces).encode()
            elif r < 0.9:
                blk += rng.choice(others).encode()
            else:
                blk += rng.choice(bad)
        if not any(ch in b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789" for ch in blk):
            blk += b"7"  # (a block without alnum has no tokens at all)
        parts.append(blk)
        parts.append("国".encode() * rng.randint(0, 3))
        docs.append(b"".join(parts))
    buf, off = _batch_of(docs)
    for hmm in (False, True):
        _cmp_batch(tk, o, buf, off, hmm, "nonzh rune classes")
    buf1, off1 = _batch_of([b"".join(docs)])
    _cmp_batch(tk, o, buf1, off1, True, "nonzh rune classes, one document")


@pytest.mark.parametrize("group", [1024, 6144])
def test_zh_blocks_from_lane_masks(syn_small, group, monkeypatch):
    """k_zh takes its groups' Han blocks from k_mark_walk's lane masks: groups with
    more Han blocks than one chunk (single-rune blocks between commas), blocks that
    end past the lookahead round but inside the window (1-7 KiB Han runs), blocks
    that end exactly at group and batch ends, and documents that end inside a run."""
    monkeypatch.setenv("JB_ZH_GROUP", str(group))
    dp, ep, s = syn_small
    tk, o = _pair(dp, ep)
    rng = random.Random(group)
    han = "的一是在不了有和人这中大为上个国我以要他时来用们生到作地于出就分对成会可主发年动同工也能下过子说产种面而方后多定行学法所民得经十三之进着等部度家电力里如水化高自二理起小物现实加量都两体制机当使点从业本去把性好应开它合还因由其些然前外天政四日那社义事平形相全表间样与关各重新线内数正心反你明看原又么利比或但质气第向道命此变条只没结解问意建月公无系军很情者最立代想已通并提直题党程展五果料象员革位入常文总次品式活设及管特件长求老头基资边流路级少图山统接知较将组见计别她手角期根论运农指几九区强放决西被干做必战先回则任取据处队南给色光门即保治北造百规热领七海口东导器压志世金增争济阶油思术极交受联什认六共权收证改清己美再采转更单风切打白教速花带安场身车例真务具万每目至达走积示议声报斗完类八离华名确才科张信马节话米整空元况今集温传土许步群广石记需段研界拉林律叫且究观越织装影算低持音众书布复容儿须际商非验连断深难近矿千周委素技备半办青省列习响约支般史感劳便团往酸历市克何除消构府称太准精值号率族维划选标写存候毛亲快效斯院查江型眼王按格养易置派层片始却专状育厂京识适属圆包火住调满县局照参红细引听该铁价严"
    docs = []
    # dense: single-rune Han blocks between commas (more blocks than one chunk per group)
    docs.append("，".join(rng.choice(han) for _ in range(6000)))
    # long runs of 300..2500 runes (0.9-7.5 KiB) at varied offsets, punctuation between
    for k in range(12):
        pad = "a" * rng.randrange(0, 40)
        docs.append(pad + "".join(rng.choice(han) for _ in range(rng.randrange(300, 2500))) + "。")
    # runs ending exactly at group boundaries (3-byte runes: group/3 runes, with offsets)
    for off in (0, 1, 2, 32):
        docs.append("x" * off + "".join(rng.choice(han) for _ in range(group // 3)) + "，" + "".join(
            rng.choice(han) for _ in range(50)))
    # a document that ends inside a Han run (the next document starts Han as well)
    docs.append("".join(rng.choice(han) for _ in range(700)))
    docs.append("".join(rng.choice(han) for _ in range(40)))
    buf, off = _batch_of(docs)
    for hmm in (False, True):
        _cmp_batch(tk, o, buf, off, hmm, f"lane-mask blocks group={group}")
    # the same as one batch padded to a multiple of the group size
    tail = (-int(off[-1])) % group
    buf2, off2 = _batch_of(docs + ["中" * (tail // 3) + "a" * (tail % 3)])
    _cmp_batch(tk, o, buf2, off2, True, f"lane-mask blocks group={group}, batch end at a group end")
    tk.close()


def _small_batches(texts, limit=4096, max_docs=4096):
    """Group texts (in order) into batches of at most `limit` bytes and `max_docs`
    documents: the batches a one-workgroup k_small launch takes whole."""
    out, cur, size = [], [], 0
    for t in texts:
        b = t.encode("utf-8") if isinstance(t, str) else t
        if len(b) > limit:
            continue
        if cur and (size + len(b) > limit or len(cur) >= max_docs):
            out.append(cur)
            cur, size = [], 0
        cur.append(b)
        size += len(b)
    if cur:
        out.append(cur)
    return out


def test_small_batches_one_workgroup(syn_small, monkeypatch):
    """Batches of at most 4 KiB (a single Cut call, BASELINE config 1) take k_small:
    one workgroup, text and offsets read from mapped pinned host memory, the whole
    Cut path in LDS.  Against the oracle and against the eleven-kernel pipeline
    (JB_SMALL=0, read at jb_open), bit-exact, with the same block, Han-block, token
    and Viterbi-tie counts: edge texts, invalid UTF-8 split by documents, random
    mixed scripts, empty documents, dense Han up to the 4096-byte limit, 4-byte Han
    runes, and batches just past the limits (which take the pipeline)."""
    dp, ep, s = syn_small
    tk, o = _pair(dp, ep)
    monkeypatch.setenv("JB_SMALL", "0")
    tp = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
    monkeypatch.delenv("JB_SMALL")
    rng = random.Random(4096)
    texts = list(EDGE_TEXTS)
    pieces = [x.encode() for x in ("中", "文", "a", " ", "　", "𠀀", "，", "ab12", "é")] + \
        [b"\xe4", b"\xb8\xad", b"\xf0\x9f", b"\x80", b"\xc2", b"\xff", b"\xed\xa0\x80"]
    texts += [b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 16))) for _ in range(600)]
    alphabet = [chr(c) for c in range(0x4E00, 0x4E00 + 3000, 3)] + ["㐀", "㒐", "a", "Z", "9", " ", "，", "。",
                                                                    "　", "ス", "한", "\n", "𠀀", "々"]
    texts += ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 300))) for _ in range(300)]
    batches = _small_batches(texts)
    # batches of at most 96 bytes and 7 documents travel in the kernel arguments
    short = [t for t in texts[len(EDGE_TEXTS):] if len(t if isinstance(t, bytes) else t.encode()) <= 30]
    batches += [short[i:i + 3] for i in range(0, 90, 3)] + _small_batches(short[:300], limit=96, max_docs=7)
    batches += [[("中" * 32).encode()], [("中" * 31).encode() + b"abc"], [b"x" * 97]]  # 96, 96 and 97 bytes
    batches += [[("丁" * 1365).encode()], [("一丁" * 682).encode() + b"ab"], [("𠀀" * 1024).encode()],
                [b""] * 4096, [b""] * 100 + ["中文".encode()] + [b""] * 100, [b"x" * 4096],
                [("中" * 1365 + "a").encode()],                      # 4097 bytes: pipeline
                [b""] * 4097]                                          # 4097 documents: pipeline
    n_small = 0
    for i, docs in enumerate(batches):
        buf, off = _batch_of(docs)
        small = int(off[-1]) <= 4096 and len(docs) <= 4096
        n_small += small
        for hmm in (False, True):
            _cmp_batch(tk, o, buf, off, hmm, f"small batch {i} hmm={hmm}")
            st = tk.last_stats()
            _cmp_batch(tp, o, buf, off, hmm, f"pipeline batch {i} hmm={hmm}")
            sp = tp.last_stats()
            if int(off[-1]):
                for k in ("tokens", "blocks", "zh_blocks", "viterbi_ties"):
                    assert st[k] == sp[k], (i, hmm, k, st, sp)
    assert n_small >= 20
    # the reference's benchmark sentence through Cut
    assert tk.Cut(SENTENCE, True) == o.cut(SENTENCE, True) == tp.Cut(SENTENCE, True)
    tk.close()
    tp.close()


@pytest.mark.parametrize("entries", [
    [("中", 0), ("文", 0), ("中文", 0), ("上海", 0)],          # size 0: Log(0) - Log(0) = NaN, Log(1) - Log(0) = +Inf
    [("中", 5), ("文", 1), ("中文", -20), ("天氣", 2)],         # size < 0: every weight NaN
    [("中", 5), ("文", -9), ("中文", 1), ("天氣", 2)],          # ... and a lone 文 has no DAG edge: panic
])
def test_degenerate_dictionary_weights(tmp_path, mini_paths, entries, monkeypatch):
    """A dictionary whose size is <= 0 makes pieceFreq +Inf or NaN (tokenizer.go:503,515-519).
    k_zh's record fold assumes finite or -Inf weights (DevImage::plainw); here k_mark_walk
    writes only overflow records and every rune is folded by maxIndexProba's literal rule.
    Both the pipeline (JB_SMALL=0) and k_small, against the oracle's IEEE arithmetic."""
    dp = str(tmp_path / "dict.txt")
    with open(dp, "w", encoding="utf-8") as f:
        for w, c in entries:
            f.write(f"{w} {c}\n")
    texts = ["中文", "中文上海天氣很好", "我昨天去上海交通大學與老師討論量子力學", "中" * 40 + "，" + "文中" * 30,
             "abc 中文 def", "一丁㐀中文" * 20]
    buf, off = _batch_of(texts * 3)
    for small in ("0", None):
        if small is None:
            monkeypatch.delenv("JB_SMALL", raising=False)
        else:
            monkeypatch.setenv("JB_SMALL", small)
        tk, o = _pair(dp, mini_paths[1])

        def outcome(fn, t, hmm):  # the tokens, or "panic" where the reference panics (cutDAG, JB_EPANIC)
            try:
                return fn(t, hmm)
            except (J.JbError, RuntimeError, ValueError):
                return "panic"
        for hmm in (False, True):
            for t in texts:
                assert outcome(tk.Cut, t, hmm) == outcome(o.cut, t, hmm), (small, hmm, t)
            if all(outcome(o.cut, t, hmm) != "panic" for t in texts):
                _cmp_batch(tk, o, buf, off, hmm, f"degenerate dict JB_SMALL={small}")
        tk.close()


def test_document_bitmap_between_runs(small):
    """The document-start bitmap is not cleared by a pass of its own: k_nonzh clears
    the words a run set.  The same bytes cut under different document layouts, one
    after another on one context (pipeline sizes, past k_small), must each match the
    oracle: a start left over from an earlier run would split a Han run."""
    tk, o, s = small
    rng = random.Random(7)
    text = "".join(rng.choice(["中文", "文字", "测试", "丁", "，", "abc", " ", "𠀀"]) for _ in range(40000)).encode()
    n = len(text)
    buf = np.frombuffer(text + b"\0" * 16, np.uint8)
    layouts = []
    for k in range(3):  # random cut points (a cut may fall inside a rune: invalid bytes, as Go strings)
        cuts = sorted(set(rng.randrange(1, n) for _ in range(200 * (k + 1))))
        layouts.append(np.array([0] + cuts + [n], np.uint64))
    layouts.append(np.array([0, n], np.uint64))
    for hmm in (0, 1):
        for rep in range(2):
            for i, off in enumerate(layouts):
                _cmp_batch(tk, o, buf, off, hmm, f"layout {i} rep {rep}")


@pytest.mark.parametrize("slots", [1, 2, 4, 8])
def test_concurrent_cut_calls(syn_small, tmp_path, slots):
    """16 threads x 1,000 jb_cut calls at once on one context (Go code calling Cut
    from many goroutines; the reference takes only an RLock, tokenizer.go:151-153):
    every result equals the oracle's, and the calls are coalesced into shared
    k_small launches (tests/concurrent_cut.cpp prints both rates), with 1, 2, 4 or 8
    batches in flight (JB_SMALL_SLOTS)."""
    import subprocess
    dp, ep, s = syn_small
    exe = str(tmp_path / "concurrent_cut")
    lib = os.path.join(ROOT, "jieba-go_amd", "lib")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "concurrent_cut.cpp"), "-L", lib, "-ljiebahip",
                           "-Wl,-rpath," + lib, "-o", exe])
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus(synth.KIND_SENTENCES, 77, max_docs=300, target_bytes=1 << 30)
    sents = [bytes(np.asarray(buf)[int(off[i]):int(off[i + 1])]) for i in range(len(off) - 1)]
    sents = [x for x in sents if b"\n" not in x] + [SENTENCE.encode(), "abc 中文 x".encode(), b""]
    with open(tmp_path / "sent.txt", "wb") as f:
        f.write(b"\n".join(sents) + b"\n")
    with open(tmp_path / "want.txt", "w") as f:
        for x in sents:
            a, b = o.cut_spans(x, True)
            f.write(" ".join([str(len(a))] + [f"{int(p)} {int(q)}" for p, q in zip(a, b)]) + "\n")
    env = dict(os.environ, JB_SMALL_SLOTS=str(slots))
    if os.environ.get("JB_CONC_LOG"):  # (diagnostics: the per-batch clocks, JB_SMALL_TRACE)
        env["JB_SMALL_TRACE"] = f"{os.environ['JB_CONC_LOG']}.trace{slots}.txt"
    r = subprocess.run([exe, dp, ep, str(tmp_path / "sent.txt"), str(tmp_path / "want.txt"), "16", "1000"],
                       capture_output=True, text=True, timeout=300, env=env)
    print(f"JB_SMALL_SLOTS={slots}")
    print(r.stdout)
    if os.environ.get("JB_CONC_LOG"):  # (diagnostics: JB_DEBUG's per-batch lines)
        with open(f"{os.environ['JB_CONC_LOG']}.slots{slots}.txt", "w") as f:
            f.write(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    # the rates are evidence, printed above, not a correctness condition: a loaded box
    # may run the concurrent pass no faster
    rates = {ln.split()[0]: float(ln.split()[-1]) for ln in r.stdout.splitlines() if ln.strip()}
    print(f"concurrent/serial = {rates.get('concurrent', 0.0) / max(rates.get('serial', 1.0), 1e-9):.2f}")


def test_concurrent_cut_mixed_hmm_and_panics(tmp_path, mini_paths):
    """The coalescing paths the test above leaves out: calls with hmm on and
    off at once (a batch takes only the queue head's setting, the others wait for the
    next), and calls whose text makes the reference panic (cutDAG: a lone 文 has no DAG
    edge under this dictionary) coalesced with good ones (the batch reruns its requests
    one by one, so JB_EPANIC reaches only the caller whose text caused it)."""
    import subprocess
    dp = str(tmp_path / "dict.txt")
    with open(dp, "w", encoding="utf-8") as f:
        for w, c in [("中", 5), ("文", -9), ("中文", 1), ("天氣", 2), ("上海", 3), ("很好", 4)]:
            f.write(f"{w} {c}\n")
    exe = str(tmp_path / "concurrent_cut")
    lib = os.path.join(ROOT, "jieba-go_amd", "lib")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "concurrent_cut.cpp"), "-L", lib, "-ljiebahip",
                           "-Wl,-rpath," + lib, "-o", exe])
    o = O.Oracle.from_files(dp, mini_paths[1], 0)
    sents = ["中文", "中文上海天氣很好", "上海很好", "文", "天氣文", "abc 中文 def", "中文上海", "很好中文天氣", "",
             "上海 天氣 中文"]
    with open(tmp_path / "sent.txt", "wb") as f:
        f.write(b"\n".join(x.encode() for x in sents) + b"\n")
    npanic = 0
    with open(tmp_path / "want.txt", "w") as f:
        for x in sents:
            for hmm in (True, False):
                try:
                    a, b = o.cut_spans(x.encode(), hmm)
                    f.write(" ".join([str(len(a))] + [f"{int(p)} {int(q)}" for p, q in zip(a, b)]) + "\n")
                except (RuntimeError, ValueError):
                    f.write("P\n")
                    npanic += 1
    assert npanic >= 2  # (the texts with a lone 文)
    r = subprocess.run([exe, dp, mini_paths[1], str(tmp_path / "sent.txt"), str(tmp_path / "want.txt"), "16", "300",
                        "mixed"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
