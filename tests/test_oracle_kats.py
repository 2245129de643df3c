"""CPU: pin the oracle (oracle/jieba_oracle.c) to the reference's own
known-answer tests (tokenizer_test.go), restated in tests/golden/."""
import math
import random
import struct

import numpy as np
import pytest

import oracle as O
from conftest import real_data_dir


def test_split_text(kats):
    for c in kats["split_text"]["cases"]:
        got = [(t.decode("utf-8"), p) for t, p in O.split_text(c["text"], 0)]
        assert got == [tuple(x) for x in c["want"]], c["text"]


def test_max_index_proba(kats):
    for c in kats["max_index_proba"]["cases"]:
        i, p = O.max_index_proba([tuple(x) for x in c["candidates"]])
        assert i == c["want_idx"] and p == c["want_proba"]


def test_max_index_proba_quirks():
    # Appendix A Q1: not an argmax
    assert O.max_index_proba([(1, -5.0), (2, -20.0), (3, -10.0)]) == (3, -10.0)
    assert O.max_index_proba([]) == (-1, -3.14e100)
    inf = float("-inf")
    assert O.max_index_proba([(4, inf), (5, inf)]) == (5, inf)
    assert O.max_index_proba([(4, inf)]) == (4, inf)


def test_find_dag_path(kats):
    for c in kats["find_dag_path"]["cases"]:
        n = len(c["text"])
        dp = {int(k): [tuple(x) for x in v] for k, v in c["dag_proba"].items()}
        assert O.find_dag_path(n, dp) == [tuple(x) for x in c["want"]], c["text"]


def test_state_transition_route(kats):
    k = kats["state_transition_route"]
    prev = [k["prev"][s] for s in "BMES"]
    for c in k["cases"]:
        frm, _ = O.state_transition_route(prev, c["now"])
        assert frm == c["want_from"]


def test_state_transition_route_threshold():
    # Q11: no candidate strictly above minFloat -> "" route with proba minFloat
    frm, p = O.state_transition_route([-3.14e100] * 4, "B")
    assert frm == "" and p == -3.14e100


def test_cut_hmm(kats):
    for c in kats["cut_hmm"]["cases"]:
        assert O.cut_hmm(c["text"], c["path"]) == c["want"]


def test_cut_nonzh(kats):
    for c in kats["cut_nonzh"]["cases"]:
        assert O.cut_nonzh(c["text"]) == c["want"]


def test_build_prefix_dict(kats):
    k = kats["build_prefix_dict"]
    o = O.Oracle("\n".join(k["lines"]) + "\n", "{}", kind=1)
    assert o.items() == k["want"]
    assert o.size == sum(int(l.split(" ")[1]) for l in k["lines"])


def test_add_word(kats):
    k = kats["add_word"]
    o = O.Oracle("", "{}", kind=0)
    for t, f in k["terms"].items():
        o.add_term(t, f)
    for t, f in k["terms"].items():
        assert o.get(t) == f
    assert o.size == k["want_size"]


@pytest.mark.parametrize("kind", [0, 1])
def test_build_dag_structure_on_mini_dict(kats, mini_paths, kind):
    """The mini dictionary reproduces TestBuildDAG's expected edges in both
    dictionary semantics (撙 is a freq-0 entry, tokenizer_test.go:126)."""
    o = O.Oracle.from_files(*mini_paths, kind=kind)
    for c in kats["build_dag_structure"]["cases"]:
        got = o.build_dag(c["text"])
        want = {int(k): v for k, v in c["want"].items()}
        assert got == want, c["text"]


@pytest.mark.parametrize("kind", [0, 1])
def test_cut8_cut10_pinned(kats, mini_paths, kind):
    """TestCut "cut 8"/"cut 10" depend only on the DAG structure: every route
    through the freq-0 rune is -Inf (Q4) and maxIndexProba's last-wins rule (Q1)
    picks the pieces, whatever the positive frequencies."""
    o = O.Oracle.from_files(*mini_paths, kind=kind)
    cases = {c["name"]: c for c in kats["cut_real_data"]["cases"]}
    for name in ("cut 8", "cut 10", "cut 4", "cut 5", "cut 6", "cut 7"):
        c = cases[name]
        assert o.cut(c["text"], c["hmm"]) == c["want"], name


def test_go_log_close_to_libm():
    """Go's math.Log is within 1 ulp of the correctly rounded value; the
    restatement must be too (its bit pattern is what the weights use)."""
    rng = random.Random(7)
    xs = [1.0, 2.0, 3.0, 10.0, 60101967.0, 60101964.0, 0.5, 1e-300, 1e300] + \
         [float(rng.randint(1, 10 ** 9)) for _ in range(3000)] + [rng.uniform(1e-5, 1e5) for _ in range(3000)]
    for x in xs:
        a, b = O.go_log(x), math.log(x)
        ua = struct.unpack("<q", struct.pack("<d", a))[0]
        ub = struct.unpack("<q", struct.pack("<d", b))[0]
        assert abs(ua - ub) <= 1, (x, a, b)
    assert O.go_log(1.0) == 0.0
    assert O.go_log(0.0) == float("-inf")
    assert math.isnan(O.go_log(-1.0))
    assert O.go_log(float("inf")) == float("inf")


HAN_RANGES = [(0x2E80, 0x2E99), (0x2E9B, 0x2EF3), (0x2F00, 0x2FD5), (0x3005, 0x3005), (0x3007, 0x3007),
              (0x3021, 0x3029), (0x3038, 0x303B), (0x3400, 0x4DBF), (0x4E00, 0x9FFC), (0xF900, 0xFA6D),
              (0xFA70, 0xFAD9), (0x16FF0, 0x16FF1), (0x20000, 0x2A6DD), (0x2A700, 0x2B734), (0x2B740, 0x2B81D),
              (0x2B820, 0x2CEA1), (0x2CEB0, 0x2EBE0), (0x2F800, 0x2FA1D), (0x30000, 0x3134A)]


def test_han_table_size():
    # Unicode 13.0 Script=Han: 94,204 code points
    L = O.lib()
    assert sum(b - a + 1 for a, b in HAN_RANGES) == 94204
    for a, b in HAN_RANGES:
        assert L.or_is_han(a) and L.or_is_han(b) and not L.or_is_han(a - 1) and not L.or_is_han(b + 1)
    for cp in (0x3001, 0x3002, 0xFF0C, 0x300E, 0x300F, 0xAC00, 0x30B9, 0x9FFD, 0x9FFF, 0x31350):
        assert not L.or_is_han(cp)


def test_is_space():
    L = O.lib()
    spaces = [9, 10, 11, 12, 13, 32, 0x85, 0xA0, 0x1680] + list(range(0x2000, 0x200B)) + \
             [0x2028, 0x2029, 0x202F, 0x205F, 0x3000]
    for cp in range(0, 0x3100):
        assert bool(L.or_is_space(cp)) == (cp in spaces), hex(cp)


def test_viterbi_backptr_equals_pathcopy(syn_small):
    """The O(m) back-pointer Viterbi (used for very long runs) takes the
    reference's decisions: identical paths on random runs, incl. OOV runes."""
    dp, ep, s = syn_small
    o = O.Oracle.from_files(dp, ep, 0)
    rng = random.Random(3)
    han = [0x4E00 + i for i in range(0, 20902, 7)]
    oov = [0x3400 + i for i in range(0, 6000, 13)]
    for _ in range(600):
        m = rng.randint(1, 40)
        runes = [rng.choice(oov) if rng.random() < 0.2 else rng.choice(han) for _ in range(m)]
        t = "".join(map(chr, runes))
        assert o.viterbi(t, False) == o.viterbi(t, True), t


def test_viterbi_collapse_drops_runes(syn_small):
    """Q11: an emission-less rune inside a run makes every state's route ""
    (path restarts), so cutHMM labels only the first runes."""
    dp, ep, s = syn_small
    o = O.Oracle.from_files(dp, ep, 0)
    t = "一㐀丁"  # middle rune has no emission in E_syn
    p = o.viterbi(t)
    assert len(p) < 3


@pytest.mark.skipif(real_data_dir() is None, reason="real jieba data (LFS objects) not present; set JIEBA_DATA_DIR")
def test_real_data_kats(kats):
    import os
    d = real_data_dir()
    o = O.Oracle.from_files(os.path.join(d, "dict.txt"), os.path.join(d, "prob_emit.json"), kind=1,
                            size_override=60_101_967)
    for c in kats["cut_real_data"]["cases"]:
        assert o.cut(c["text"], c["hmm"]) == c["want"], c["name"]
    for c in kats["viterbi_real_data"]["cases"]:
        assert o.viterbi(c["text"]) == c["want"]
    for s, v in kats["load_hmm_real_data"]["want"].items():
        assert o.emit(s, kats["load_hmm_real_data"]["char"]) == v
    # NewJiebaTokenizer proper: the genuine prefix_dictionary.gob (sha256-checked),
    # decoded by the test-side gob restatement and loaded with txt semantics
    import hashlib

    import gobenc
    gp = os.path.join(d, "prefix_dictionary.gob")
    if os.path.exists(gp):
        data = open(gp, "rb").read()
        assert hashlib.sha256(data).hexdigest() == kats["real_data_sha256"]["prefix_dictionary.gob"]
        m = gobenc.decode_map(data)
        og = O.Oracle(gobenc.map_to_dict_lines(m),
                      open(os.path.join(d, "prob_emit.json"), encoding="utf-8").read(), 0, size_override=60_101_967)
        for c in kats["cut_real_data"]["cases"]:
            assert og.cut(c["text"], c["hmm"]) == c["want"], c["name"]


def test_batch_equals_per_doc(syn_small):
    import synth
    dp, ep, s = syn_small
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, nr = s.corpus(synth.KIND_DOCS, 0, target_bytes=200_000)
    for hmm in (0, 1):
        st, en, tdo = o.cut_batch(buf, off, hmm, nthreads=3)
        for d in range(len(off) - 1):
            a, b = int(off[d]), int(off[d + 1])
            s1, e1 = o.cut_spans(bytes(buf[a:b]), hmm)
            k0, k1 = int(tdo[d]), int(tdo[d + 1])
            assert np.array_equal(st[k0:k1], s1 + a) and np.array_equal(en[k0:k1], e1 + a)


def test_oracle_reproduces_synthetic_golden(syn_golden):
    """The oracle still produces the committed golden spans (tests/golden/make_golden.py)."""
    g, docs, dp, ep = syn_golden
    oracles = {}
    for c in g["cases"]:
        key = (c["kind"], c["size"])
        if key not in oracles:
            oracles[key] = O.Oracle.from_files(dp, ep, c["kind"], c["size"])
        s, e = oracles[key].cut_spans(docs[c["doc"]], c["hmm"])
        assert s.tolist() == c["starts"] and e.tolist() == c["ends"], (c["kind"], c["hmm"], c["doc"])
