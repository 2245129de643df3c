"""Document sharding for multi-GPU runs.

Documents are independent units (Cut per document; blocks never cross a
document, tokenizer.go:158-160), so a batch splits into contiguous,
byte-balanced document ranges, one per rank / device, with no data exchange.
Rank r's tokens are the tokens of its documents; concatenating rank outputs
in rank order gives document order.  The same rule is implemented in C++ for
in-process multi-device contexts (jb_cut_batch in csrc/jb_capi.cpp).
"""
import numpy as np


def shard_bounds(doc_off, world):
    """Contiguous byte-balanced document ranges: returns cut[0..world], rank r
    owns documents [cut[r], cut[r+1])."""
    doc_off = np.asarray(doc_off, dtype=np.uint64)
    ndocs = len(doc_off) - 1
    cut = [0] * (world + 1)
    cut[world] = ndocs
    total = int(doc_off[-1] - doc_off[0]) if ndocs else 0
    lo = 0
    for k in range(1, world):
        target = int(doc_off[0]) + total * k // world
        while lo < ndocs and int(doc_off[lo + 1]) <= target:
            lo += 1
        cut[k] = lo
    return cut


def shard_of(buf, doc_off, world, rank):
    """(sub-buffer, rebased doc offsets, first doc index, base byte) of rank's shard."""
    cut = shard_bounds(doc_off, world)
    d0, d1 = cut[rank], cut[rank + 1]
    base = int(doc_off[d0])
    end = int(doc_off[d1])
    sub = np.zeros(end - base + 16, np.uint8)
    sub[: end - base] = np.asarray(buf)[base:end]
    off = np.asarray(doc_off[d0 : d1 + 1], dtype=np.uint64) - np.uint64(base)
    return sub, off, d0, base


def merge(parts):
    """Concatenate per-rank (starts, ends, doc_tok, base) in rank order into
    batch-absolute spans and document token offsets."""
    starts, ends, dts = [], [], [np.zeros(1, np.uint64)]
    ntok = 0
    for s, e, dt, base in parts:
        starts.append(np.asarray(s, np.uint64) + np.uint64(base))
        ends.append(np.asarray(e, np.uint64) + np.uint64(base))
        dts.append(np.asarray(dt[1:], np.uint64) + np.uint64(ntok))
        ntok += len(s)
    return np.concatenate(starts), np.concatenate(ends), np.concatenate(dts)
