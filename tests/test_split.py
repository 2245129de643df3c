"""jb_split_points (host only): byte-balanced cuts that may fall inside a document,
only where a Han run begins, so that one large document spreads over several
devices.  Checked against the oracle: every cut is a document start
or the start of a zh block of splitText (tokenizer.go:165-210), and cutting the
parts as separate documents gives the whole documents' tokens (blocks are cut
independently, tokenizer.go:158-160)."""
import random

import numpy as np
import pytest

import jiebahip as J
import oracle as O


def _zh_starts(doc):
    """Byte offsets where splitText's zh blocks begin (the oracle's split_text)."""
    out, pos = set(), 0
    for sub, zh in O.split_text(doc):
        if zh and pos > 0:
            out.add(pos)
        pos += len(sub)
    assert pos == len(doc)
    return out


PIECES = [x.encode() for x in ("中文", "天氣很好", "丁", "𠀀", "𪜀中", "㐀", "，", "。", "　", "a", "abc1", " ", "\n",
                               "ス", "한", "〇", "々")] + [b"\xe4\xb8", b"\x80", b"\xff", b"\xed\xa0\x80", b"\xf0\x9f",
                                                         b"\xe4", b"\xb8\xad"]


def _corpus(rng, ndocs, maxlen):
    docs = [b"".join(rng.choice(PIECES) for _ in range(rng.randint(0, maxlen))) for _ in range(ndocs)]
    off = np.zeros(ndocs + 1, np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    buf = np.frombuffer(b"".join(docs) + b"\0" * 64, np.uint8)
    return docs, buf, off


@pytest.mark.parametrize("seed", range(6))
def test_split_points_at_han_run_starts(syn_small, seed):
    dp, ep, _ = syn_small
    o = O.Oracle.from_files(dp, ep, 0)
    rng = random.Random(seed)
    docs, buf, off = _corpus(rng, rng.choice([1, 2, 5, 40]), rng.choice([30, 400, 3000]))
    total = int(off[-1])
    starts = {int(x) for x in off}
    zh = set()
    for d, a in zip(docs, off[:-1]):
        zh |= {int(a) + q for q in _zh_starts(d)}
    for nparts in (1, 2, 3, 4, 7, 8, 64):
        cut = J.split_points(buf, off, nparts)
        assert cut[0] == 0 and cut[-1] == total and cut == sorted(cut)
        for k in range(1, nparts):
            c = cut[k]
            assert c in starts or c in zh, (nparts, k, c)
            t = total * k // nparts
            assert c >= t  # the first eligible point at or after the target
            assert not any(t <= x < c for x in starts | zh), (nparts, k, c, t)
        # the parts (documents cut at the points) give the whole documents' tokens
        pts = sorted(set(int(x) for x in off) | set(cut))
        poff = np.array(pts, np.uint64)
        for hmm in (False, True):
            ws, we, _ = o.cut_batch(buf, off, hmm)
            ps, pe, _ = o.cut_batch(buf, poff, hmm)
            assert np.array_equal(ws, ps) and np.array_equal(we, pe), (seed, nparts, hmm)


def test_split_points_one_large_document(syn_small):
    """One punctuated document split 8 ways: the parts are near equal."""
    dp, ep, s = syn_small
    import synth
    buf, off, _ = s.corpus(synth.KIND_LONG_PUNCT, 3, target_runes=200_000)
    cut = J.split_points(buf, off, 8)
    total = int(off[-1])
    sizes = np.diff(cut)
    assert len(off) == 2 and sizes.min() > 0.95 * total / 8, sizes
    o = O.Oracle.from_files(dp, ep, 0)
    ws, we, _ = o.cut_batch(buf, off, True)
    ps, pe, _ = o.cut_batch(buf, np.array(cut, np.uint64), True)
    assert np.array_equal(ws, ps) and np.array_equal(we, pe)


def test_split_points_no_han_run():
    """No Han-run start after the target: the cut moves to the next document start."""
    docs = ["中文" + "a" * 1000, "b" * 10, "中" * 100]
    bs = [d.encode() for d in docs]
    off = np.array([0, len(bs[0]), len(bs[0]) + len(bs[1]), sum(map(len, bs))], np.uint64)
    buf = np.frombuffer(b"".join(bs) + b"\0" * 64, np.uint8)
    cut = J.split_points(buf, off, 2)
    assert cut[1] == int(off[1])
    # one Han run only: it starts at byte 0, so it cannot be cut
    b = ("中" * 500).encode()
    cut = J.split_points(np.frombuffer(b + b"\0" * 8, np.uint8), np.array([0, len(b)], np.uint64), 4)
    assert cut == [0, len(b), len(b), len(b), len(b)]
