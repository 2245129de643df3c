"""The closed form k_long_dp's chain folds a rune with (jb_kernels.hip, the
chain's comment): for items in length order with L1 = 1, sums p1..pm and NaN
for the absent p(m+1)..p4,
    P = p4 if p4 >= p3, else p3 if p3 >= p2, else max(p1, p2)
(v_max_f64 drops a NaN operand).  Checked against the oracle's maxIndexProba
(tokenizer.go:565-578, oracle/jieba_oracle.c) on 1-4 items with ties and -Inf
(count-0 weights).  The chain keeps only the taken item's value (k_long_seg
recomputes the lengths), so the value is what must match, bit for bit.  The GPU
parity tests run the kernel itself."""
import itertools
import math
import random

import pytest

import oracle as O

NAN = float("nan")
INF = float("inf")


def vmax(a, b):  # v_max_f64: IEEE maxNum (a NaN operand gives the other one)
    if math.isnan(a):
        return b
    if math.isnan(b):
        return a
    return a if a >= b else b


def chain_fold(p):
    """The chain's fold of sums p (1-4 items, in length order)."""
    p1, p2, p3, p4 = (list(p) + [NAN] * 4)[:4]
    k3, k4 = p3 >= p2, p4 >= p3
    return (p4 if k4 else p3) if (k3 or k4) else vmax(p1, p2)


def reference(p):
    return O.max_index_proba(list(enumerate(p)))[1]


def _same(a, b):
    return a == b or (math.isinf(a) and math.isinf(b) and (a > 0) == (b > 0))


def test_chain_fold_random():
    rng = random.Random(1)
    pool = [-1.0, -2.0, -3.0, -0.5, -7.25, -INF]
    bad = []
    for _ in range(40000):
        m = rng.randint(1, 4)
        p = [rng.choice(pool + [rng.uniform(-80.0, 0.0)]) for _ in range(m)]
        want, got = reference(p), chain_fold(p)
        if not _same(want, got):
            bad.append((p, want, got))
    assert not bad, bad[:3]


@pytest.mark.parametrize("m", [1, 2, 3, 4])
def test_chain_fold_every_order(m):
    """Every order of the items' sums, ties and -Inf included."""
    for p in itertools.product([-4.0, -3.0, -2.0, -1.0, -INF], repeat=m):
        assert _same(reference(list(p)), chain_fold(p)), p


def small_fold(p):
    """k_small's branch-free step (plainw weights): the chosen item's index by nested
    selects, p3 if p3 >= p2, else p2 if p2 >= p1, else p1 if p1 >= p0, else p0."""
    p0, p1, p2, p3 = (list(p) + [NAN] * 4)[:4]
    return 3 if p3 >= p2 else (2 if p2 >= p1 else (1 if p1 >= p0 else 0))


@pytest.mark.parametrize("m", [1, 2, 3, 4])
def test_small_fold_every_order(m):
    """k_small's step picks the reference's item (index, hence length and value) on every
    order of 1-4 finite or -Inf sums."""
    for p in itertools.product([-4.0, -3.0, -2.0, -1.0, -INF], repeat=m):
        assert O.max_index_proba(list(enumerate(p)))[0] == small_fold(p), p


def test_small_fold_needs_plain_weights():
    """With NaN sums (a dictionary of size <= 0) no item qualifies and the reference
    takes the last one, which the nested form does not: k_small keeps the literal fold
    for !plainw (jb_kernels.hip)."""
    p = [NAN, NAN]
    assert O.max_index_proba(list(enumerate(p)))[0] == 1 and small_fold(p) == 0


def _dag(rng, n):
    """Per rune, items (L, weight) in length order; L = 1 always present (plainw)."""
    dag = []
    for i in range(n):
        its = [(1, -rng.uniform(5.0, 15.0))]
        for L in range(2, min(9, n - i + 1)):
            if rng.random() < 0.3:
                its.append((L, -rng.uniform(5.0, 20.0)))
        dag.append(its)
    return dag


def _fold(items, best, n):
    """maxIndexProba over pieceProba = w + best(i + L) (tokenizer.go:519-578), as the
    oracle does: the chosen (L, w)."""
    pr = [(L, w + (0.0 if L == 0 else best[L])) for L, w in items]
    k, _ = O.max_index_proba([(j, p) for j, (_, p) in enumerate(pr)])
    return items[k]


def _exact(dag, n):
    best = [0.0] * (n + 1)
    for i in range(n - 1, -1, -1):
        L, w = _fold(dag[i], {L: best[i + L] for L, _ in dag[i]}, n)
        best[i] = w + best[i + L]
    return best


def _spec(dag, n, seg, over):
    """k_long_spec: per segment, the DP from `over` runes past it with best = 0.0 there."""
    ch = [None] * n
    for a in range(0, n, seg):
        lim, top = min(a + seg, n), min(a + seg + over, n)
        b = {top: 0.0}
        for i in range(top - 1, a - 1, -1):
            L, w = _fold(dag[i], {L: (0.0 if i + L >= top else b[i + L]) for L, _ in dag[i]}, n)
            b[i] = w + (0.0 if i + L >= top else b[i + L])
            if i < lim:
                ch[i] = (L, w)
    return ch


def _decided(dag, ch, n):
    """k_long_dp's decided chain (one add per rune), then the helpers' verification:
    every rune's choice by the rule over the chain's values."""
    best = [0.0] * (n + 1)
    for i in range(n - 1, -1, -1):
        L, w = ch[i]
        best[i] = w + best[i + L]
    ok = all(_fold(dag[i], {L: best[i + L] for L, _ in dag[i]}, n)[0] == ch[i][0] for i in range(n))
    return best, ok


@pytest.mark.parametrize("over", [0, 4, 64])
def test_decided_chain_is_exact_when_verified(over):
    """Decide-add-verify (k_long_spec + k_long_dp's decided chain): when every choice
    passes the rule over the added values, the values are the exact DP's bit for bit
    (same adds, same operands); a wrong choice never passes.  With a short overlap the
    guesses go wrong and the block takes the exact chain."""
    rng = random.Random(7 + over)
    seen_ok = seen_bad = 0
    for _ in range(6):
        n = rng.randint(50, 400)
        dag = _dag(rng, n)
        exact = _exact(dag, n)
        ch = _spec(dag, n, 16, over)
        best, ok = _decided(dag, ch, n)
        right = all(ch[i][0] == _fold(dag[i], {L: exact[i + L] for L, _ in dag[i]}, n)[0] for i in range(n))
        assert ok == right
        if ok:
            assert best == exact
            seen_ok += 1
        else:
            seen_bad += 1
    if over == 64:
        assert seen_ok
    if over == 0:
        assert seen_bad
