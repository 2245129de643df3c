#!/usr/bin/env python3
"""Diagnostic: does cutting a shard as two half-shards on two streams (two
tokenizers, two captured graphs running at once) beat one pipeline over the
whole shard?  k_mark_walk is issue-bound and k_zh latency-bound, so one half's
k_zh could hide under the other half's k_mark_walk.  Prints ms per shard for
(a) one pipeline, (b) the halves back to back on one stream, (c) the halves on
two streams."""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _sub in ("oracle", "gen", os.path.join("jieba-go_amd", "python")):
    sys.path.insert(0, os.path.join(ROOT, _sub))

import torch  # noqa: E402

import jiebahip as J  # noqa: E402
import synth  # noqa: E402


def main():
    steps = int(os.environ.get("STEPS", "20"))
    nparts = int(os.environ.get("PARTS", "2"))
    s = synth.Synth(nwords=350_000)
    tmp = tempfile.mkdtemp()
    dp, ep = s.write_files(tmp)
    buf, off, _ = s.corpus(synth.KIND_DOCS, 0, target_bytes=128 << 20)
    nbytes, ndocs = int(off[-1]), len(off) - 1
    dev = torch.device("cuda", 0)

    def mk():
        return J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, kind=J.JB_DICT_PREFIX,
                                         size_override=J.JIEBA_SIZE, device=0))

    def upload(lo, hi):
        b0, b1 = int(off[lo]), int(off[hi])
        t = np.zeros(b1 - b0 + 64, np.uint8)
        t[: b1 - b0] = buf[b0:b1]
        o = (off[lo: hi + 1] - off[lo]).astype(np.int64)
        return torch.from_numpy(t).to(dev), torch.from_numpy(o).to(dev), b1 - b0, hi - lo

    full = upload(0, ndocs)
    cuts = [int(np.searchsorted(off, nbytes * k // nparts)) for k in range(nparts + 1)]
    cuts[0], cuts[-1] = 0, ndocs
    parts = [upload(cuts[k], cuts[k + 1]) for k in range(nparts)]
    tks = [mk() for _ in range(nparts)]
    streams = [torch.cuda.Stream(dev) for _ in range(nparts)]
    main_s = torch.cuda.current_stream(dev)

    def run_full():
        tks[0].cut_device(full[0].data_ptr(), full[2], full[1].data_ptr(), full[3], True, main_s.cuda_stream)

    def run_seq():
        for tk, p in zip(tks, parts):
            tk.cut_device(p[0].data_ptr(), p[2], p[1].data_ptr(), p[3], True, main_s.cuda_stream)

    def run_par():
        ev = torch.cuda.Event()
        ev.record(main_s)
        for tk, p, st in zip(tks, parts, streams):
            st.wait_event(ev)
            tk.cut_device(p[0].data_ptr(), p[2], p[1].data_ptr(), p[3], True, st.cuda_stream)
        for st in streams:
            main_s.wait_stream(st)

    def timeit(fn):
        for _ in range(4):
            fn()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / steps * 1e3

    # each tokenizer captures a graph per (buffers, sizes): keep the full run on its own tokenizer
    tk_full = mk()

    def run_full2():
        tk_full.cut_device(full[0].data_ptr(), full[2], full[1].data_ptr(), full[3], True, main_s.cuda_stream)

    for r in range(2):
        print(f"round {r}: full {timeit(run_full2):.4f} ms  seq{nparts} {timeit(run_seq):.4f} ms  "
              f"par{nparts} {timeit(run_par):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
