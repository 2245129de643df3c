#!/usr/bin/env python3
"""Regenerate tests/golden/syn_golden.json: seeded synthetic inputs and the
token spans of the oracle (oracle/jieba_oracle.c, the C restatement of
tokenizer.go) for them.  The dictionary and emission table are the
deterministic generator's (gen/synth.c, 20k words, seeds 1/2); their sha256
values are stored so a generator change is caught.  Run from the repo root:

    python tests/golden/make_golden.py
"""
import base64
import hashlib
import json
import os
import random
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for sub in ("oracle", "gen"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
import synth  # noqa: E402

NWORDS = 20_000


def inputs(s):
    """Documents: synthetic sentences and documents, long singleton runs, and hand-made edge texts."""
    docs = []
    buf, off, _ = s.corpus(synth.KIND_SENTENCES, 0, max_docs=120, target_bytes=1 << 20)
    docs += [bytes(buf[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    buf, off, _ = s.corpus(synth.KIND_DOCS, 1000, max_docs=3, target_bytes=24 << 10)
    docs += [bytes(buf[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    for kind in (synth.KIND_LONG_PUNCT, synth.KIND_LONG_OOV):
        buf, off, _ = s.corpus(kind, 0, target_runes=3000)
        docs.append(bytes(buf[off[0]:off[1]]))
    rng = random.Random(5)
    han = [chr(c) for c in range(0x4E00, 0x4E00 + 400)] + [chr(c) for c in range(0x3400, 0x3410)]
    for _ in range(40):
        parts = []
        for _ in range(rng.randint(1, 10)):
            r = rng.random()
            if r < 0.6:
                parts.append("".join(rng.choice(han) for _ in range(rng.randint(1, 12))))
            elif r < 0.75:
                parts.append(rng.choice(["，", "。", "！", "、", "　", " ", "\n", "\t"]))
            elif r < 0.9:
                parts.append(rng.choice(["abc", "x1", "2024", "Go1.18", "é", "ü"]))
            else:
                parts.append(rng.choice(["々", "〇", "〻", "⺀", "\U00020000", "\U0002a700"]))
        docs.append("".join(parts).encode("utf-8"))
    docs += [b"", b" ", b"\xff\xfe", b"\xe4\xb8", "中".encode() + b"\x80" + "文".encode(), b"\xf0\x9f\x98\x80a"]
    return docs


def main():
    s = synth.Synth(nwords=NWORDS)
    tmp = tempfile.mkdtemp(prefix="jb_golden_")
    dp, ep = s.write_files(tmp)
    sha = {}
    for name, p in (("dict.txt", dp), ("prob_emit.json", ep)):
        with open(p, "rb") as f:
            sha[name] = hashlib.sha256(f.read()).hexdigest()
    docs = inputs(s)
    out = {"_source": "oracle/jieba_oracle.c on gen/synth.c data; made by tests/golden/make_golden.py",
           "nwords": NWORDS, "sha256": sha, "cases": []}
    for kind, size in ((0, 0), (1, 60101967)):
        o = O.Oracle.from_files(dp, ep, kind, size)
        for hmm in (False, True):
            for i, d in enumerate(docs):
                st, en = o.cut_spans(d, hmm)
                out["cases"].append({"kind": kind, "size": size, "hmm": hmm, "doc": i,
                                     "starts": st.tolist(), "ends": en.tolist()})
        o.close()
    out["docs_b64"] = [base64.b64encode(d).decode() for d in docs]
    with open(os.path.join(ROOT, "tests", "golden", "syn_golden.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(len(docs), "docs,", len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
