#!/usr/bin/env python3
"""bench.py — jieba-go Cut on MI355X: UTF-8 Chinese chars/s segmented.

Workload (BASELINE.json config 4, "1 GB synthetic Zipf corpus, doc-sharded
across 8 GPUs"): every rank segments its own shard of the synthetic C_syn
corpus — 1 GiB / 8 = 128 MiB of documents per GPU, HMM on (the reference's
big-text benchmark setting, tokenizer_test.go:510,521) — with the 350k-word
D_syn dictionary and E_syn emissions.  Per-GPU work is fixed,
so N GPUs process N x 128 MiB (weak scaling; N = 8 is config 4).  A step is
one full Cut pass (all kernels, spans out) over the shard, inputs resident in
HBM.  Documents shard with no data-path collective; ranks only meet at the
timing barriers.

Prints one JSON line (rank 0).  `roofline` is for the dominant kernel (by
average launch time; `roofline_kernels` has both big kernels),
`cpu_baseline` is the oracle (C restatement of tokenizer.go) on this host's
cores over a bounded sample of the same shard, checked token for token
against the GPU output of the same documents.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _sub in ("oracle", "gen", os.path.join("jieba-go_amd", "python")):
    sys.path.insert(0, os.path.join(ROOT, _sub))

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0   # float4 copy, same guide
DOC_STRIDE = 10_000_000     # rank r generates documents r*DOC_STRIDE, r*DOC_STRIDE+1, ...


def han_bytes(buf, n):
    """Bytes of `buf[:n]` that belong to \\p{Han} runes (3-byte BMP Han + 4-byte Han)."""
    b = buf[:n]
    lead3 = np.nonzero((b[:-2] >= 0xE0) & (b[:-2] < 0xF0))[0]
    cp = ((b[lead3].astype(np.uint32) & 0x0F) << 12) | ((b[lead3 + 1].astype(np.uint32) & 0x3F) << 6) | \
        (b[lead3 + 2].astype(np.uint32) & 0x3F)
    h3 = ((cp >= 0x3400) & (cp <= 0x4DBF)) | ((cp >= 0x4E00) & (cp <= 0x9FFC)) | \
        ((cp >= 0x2E80) & (cp <= 0x2FD5)) | ((cp >= 0xF900) & (cp <= 0xFAD9)) | (cp == 0x3005) | (cp == 0x3007) | \
        ((cp >= 0x3021) & (cp <= 0x3029)) | ((cp >= 0x3038) & (cp <= 0x303B))
    lead4 = int(np.count_nonzero((b >= 0xF0) & (b <= 0xF4)))  # synthetic corpora hold no 4-byte runes
    return int(h3.sum()) * 3 + lead4 * 4


def load_pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary (separate
    rocprofv3 --pmc passes, FETCH_SIZE x2 gfx950 correction), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
        for name, e in d["kernels"].items():  # e.g. "k_zh<true>" for kernel "k_zh"
            if name == kernel or name.startswith(kernel + "<"):
                return e["hbm_bytes_per_launch"]
        return None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mib", type=float, default=128.0, help="corpus MiB per GPU")
    ap.add_argument("--workload", choices=["docs", "s10k", "long-punct", "long-oov"], default="docs",
                    help="docs: C_syn document shard (config 4, the headline); s10k: 10,000 sentences (configs 2/3 "
                         "with --hmm 0/1); long-punct / long-oov: one 1,000,000-rune document (configs 5a / 5b)")
    ap.add_argument("--hmm", type=int, default=1)
    ap.add_argument("--nwords", type=int, default=350_000)
    ap.add_argument("--dict-kind", choices=["prefix", "txt"], default="prefix",
                    help="prefix: NewJiebaTokenizer semantics (prefix_dictionary.gob, size 60,101,967) as in the "
                         "reference's own benchmarks; txt: NewTokenizer(dict.txt)")
    ap.add_argument("--cpu-sample-mib", type=float, default=128.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu1-sample-mib", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import jiebahip as J
    import synth

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)

    # ---- data (synthetic, seeded) ---------------------------
    t0 = time.time()
    s = synth.Synth(nwords=args.nwords)
    tmp = tempfile.mkdtemp(prefix=f"jb_bench_r{rank}_")
    dpath, epath = s.write_files(tmp)
    if args.workload == "docs":
        buf, off, nrunes = s.corpus(synth.KIND_DOCS, rank * DOC_STRIDE, target_bytes=int(args.mib * (1 << 20)))
    elif args.workload == "s10k":
        buf, off, nrunes = s.corpus(synth.KIND_SENTENCES, rank * DOC_STRIDE, max_docs=10_000,
                                    target_bytes=64 << 20)
    else:
        buf, off, nrunes = s.corpus(synth.KIND_LONG_PUNCT if args.workload == "long-punct" else synth.KIND_LONG_OOV,
                                    rank, target_runes=1_000_000)
    nbytes = int(off[-1])
    ndocs = len(off) - 1
    hbytes = han_bytes(buf, nbytes)
    gen_s = time.time() - t0

    kind = J.JB_DICT_PREFIX if args.dict_kind == "prefix" else J.JB_DICT_TXT
    size_override = J.JIEBA_SIZE if args.dict_kind == "prefix" else 0
    tk = J.Tokenizer(J.make_config(dict_path=dpath, emit_path=epath, kind=kind, size_override=size_override,
                                   device=local))
    d_text = torch.from_numpy(buf).to(dev)                      # nbytes + 64 zero padding bytes
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        return tk.cut_device(d_text.data_ptr(), nbytes, d_off.data_ptr(), ndocs, bool(args.hmm), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # timed region: the pipeline replays as one captured HIP graph per step
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    ptrs = None
    for _ in range(args.steps):
        ptrs = step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    if dist:
        dist.barrier()

    # per-kernel durations: the same K steps again, launched kernel by kernel
    # with a HIP event pair around each launch on the launch stream
    prof = not args.no_profile
    kprof = {}
    prof_ms = None
    if prof:
        tk.profile(True)
        tk.profile_reset()
        torch.cuda.synchronize(dev)
        tp = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        prof_ms = (time.perf_counter() - tp) / args.steps * 1e3
        kprof = tk.profile_read()
        tk.profile(False)

    # whole-job aggregates: max time over ranks, sum of work
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        w = torch.tensor([nrunes, nbytes, hbytes], dtype=torch.float64, device=dev)
        dist.all_reduce(w, op=dist.ReduceOp.SUM)
        tot_runes, tot_bytes, tot_han = (float(x) for x in w.tolist())
    else:
        tot_runes, tot_bytes, tot_han = float(nrunes), float(nbytes), float(hbytes)

    ms_per_step = elapsed / args.steps * 1e3
    value = tot_runes * args.steps / elapsed

    # ---- roofline of the dominant kernel --------------------------------------
    # Algorithmic bytes: 1 B read per input byte + 2 output bits
    # per byte = 1.25 B per byte of the units a kernel processes: every input
    # byte for k_mark_walk (it classifies and walks the whole batch), the Han
    # bytes for k_zh (DP + Viterbi over zh blocks).
    roof = None
    rooflines = {}
    kernels = {}
    if kprof:
        for name, (ms, n) in kprof.items():
            if n:
                kernels[name] = {"avg_ms": ms / n, "launches": int(n)}
        dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
        units = {"k_mark_walk": float(nbytes), "k_zh": float(hbytes)}
        if args.workload == "long-oov":  # one unpunctuated block: its Han bytes all go through k_zh_long
            units["k_zh_long"] = float(hbytes)
        for kname, u in units.items():
            kk = kernels.get(kname)
            if not kk:
                continue
            alg = 1.25 * u
            achieved = alg / (kk["avg_ms"] * 1e-3) / 1e9
            rooflines[kname] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(achieved / HBM_PEAK_GBS, 5),
                                # the committed PMC summary is of the headline workload only
                                "traffic": load_pmc_traffic(kname) if args.workload == "docs" else None,
                                "kernel": kname, "alg_bytes_per_launch": alg, "avg_launch_ms": kk["avg_ms"],
                                "frac_of_measured_copy": round(achieved / HBM_MEASURED_GBS, 5)}
        if dom in rooflines:
            roof = dict(rooflines[dom], dominant_kernel=dom)
        elif rooflines:
            roof = dict(next(iter(rooflines.values())), dominant_kernel=dom)

    # ---- CPU baseline + parity sample (rank 0, N = 1) -----------------------
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle as O
        lim = int(args.cpu_sample_mib * (1 << 20))
        dend = int(np.searchsorted(off, min(lim, nbytes), side="right")) - 1
        dend = max(1, min(dend, ndocs))
        sbytes = int(off[dend])
        s_runes = int(np.count_nonzero((buf[:sbytes] & 0xC0) != 0x80))
        o = O.Oracle.from_files(dpath, epath, kind, size_override)
        backptr = args.workload.startswith("long")  # the literal path copy is O(m^2) on a 1M-rune run
        O.set_viterbi_backptr(backptr)
        threads = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
        tc = time.perf_counter()
        os_, oe, od = o.cut_batch(buf[: sbytes + 16], off[: dend + 1], bool(args.hmm), nthreads=threads)
        cpu_s = time.perf_counter() - tc
        cpu = {"value": round(s_runes / cpu_s, 1), "unit": "chars/s", "cores": threads, "kind": "port",
               "sample": f"first {dend} documents ({sbytes / 2**20:.1f} MiB, {s_runes} chars) of rank 0's shard, "
                         f"oracle/jieba_oracle.c (C restatement of tokenizer.go, "
                         f"{'O(n) back-pointer' if backptr else 'literal path-copy'} Viterbi), "
                         f"{threads} threads over documents, {cpu_s:.2f} s",
               "cpu_model": _cpu_model()}
        ps, pe, pd, pn = ptrs
        ntok = int(J.dev_to_host(pn, 8, np.uint64)[0])
        gd = J.dev_to_host(pd, 8 * (ndocs + 1), np.uint64)
        k1 = int(gd[dend])
        gs = J.dev_to_host(ps, 4 * k1, np.uint32)
        ge = J.dev_to_host(pe, 4 * k1, np.uint32)
        ok = bool(np.array_equal(gs, os_) and np.array_equal(ge, oe) and np.array_equal(gd[: dend + 1], od))
        parity = {"docs": dend, "tokens": int(len(os_)), "bit_exact": ok, "gpu_tokens_total": ntok}
        # one-thread oracle on a smaller sample (SURVEY.md §8d asks for 1 and n threads)
        d1 = max(1, min(ndocs, int(np.searchsorted(off, min(int(args.cpu1_sample_mib * (1 << 20)), nbytes),
                                                   side="right")) - 1))
        b1 = int(off[d1])
        r1 = int(np.count_nonzero((buf[:b1] & 0xC0) != 0x80))
        tc = time.perf_counter()
        o.cut_batch(buf[: b1 + 16], off[: d1 + 1], bool(args.hmm), nthreads=1)
        c1 = time.perf_counter() - tc
        cpu["value_1thread"] = round(r1 / c1, 1)
        cpu["sample_1thread"] = f"first {d1} documents ({b1 / 2**20:.1f} MiB, {r1} chars), 1 thread, {c1:.2f} s"
        del o

    # ---- end to end from host memory (PCIe in and out; rank 0, N = 1) -------
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        res = tk.cut_batch_into(buf, off, bool(args.hmm))  # warm the pinned staging and the output arrays
        te = time.perf_counter()
        for _ in range(3):
            res = tk.cut_batch_into(buf, off, bool(args.hmm), res[3])
        e2e_s = (time.perf_counter() - te) / 3
        e2e = {"value": round(nrunes / e2e_s, 1), "unit": "chars/s", "ms": round(e2e_s * 1e3, 2),
               "what": "jb_cut_batch_into from host memory: pinned staging, H2D text + offsets, all kernels, "
                       "D2H spans, u64 batch offsets into caller arrays"}

    if rank == 0:
        line = {
            "metric": "UTF-8 Chinese chars/sec segmented (whole node) + achieved HBM GB/s vs peak",
            "value": round(value, 1), "unit": "chars/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (seeded D_syn 350k-word dict, E_syn emissions, C_syn Zipf corpus)",
            "config": {"workload": (f"C_syn corpus shard {args.mib:g} MiB/GPU (1 GiB over 8 GPUs = config 4), "
                                    if args.workload == "docs" else
                                    "S10k: 10,000 synthetic sentences (configs 2/3), " if args.workload == "s10k" else
                                    f"L1M: one 1,000,000-rune document, "
                                    f"{'punctuated (5a)' if args.workload == 'long-punct' else 'unpunctuated, 30% OOV (5b)'}, ")
                                   + f"Cut hmm={'on' if args.hmm else 'off'}, "
                                   f"{'NewJiebaTokenizer (prefix dict, size 60,101,967)' if args.dict_kind == 'prefix' else 'NewTokenizer(dict.txt)'}",
                       "bytes_per_gpu": nbytes, "chars_per_gpu": nrunes, "han_bytes_per_gpu": hbytes,
                       "docs_per_gpu": ndocs, "dict_words": s.nwords, "parallelism": f"doc-shard x{world}, no collectives"},
            "roofline": roof,
            "roofline_kernels": rooflines,
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "end_to_end_host": e2e,
            "han_chars_per_s": round(tot_han / 3 * args.steps / elapsed, 1),
            "input_GBps": round(tot_bytes * args.steps / elapsed / 1e9, 3),
            "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
            "ms_per_step_kernel_by_kernel": round(prof_ms, 4) if prof_ms else None,
            "gen_s": round(gen_s, 2),
            "loaded": J.loaded_runtime(),
        }
        print(json.dumps(line), flush=True)
    tk.close()
    if dist:
        dist.destroy_process_group()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for l in f:
                if l.startswith("model name"):
                    return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
