#!/usr/bin/env python3
"""bench.py — jieba-go Cut on MI355X: UTF-8 Chinese chars/s segmented.

Headline workload (BASELINE.json configs[3], the config the metric is quoted
on): ONE fixed 1 GiB corpus of synthetic C_syn documents (seeded Zipf text,
SURVEY.md §8d), cut with HMM on (the reference's big-text benchmark setting,
tokenizer_test.go:608-609) against the 350k-word D_syn dictionary and E_syn
emissions.  `--gpus N` strong-scales that same corpus: rank r cuts the
byte-balanced document range shard.shard_bounds(...)[r] (jb_shard_bounds, the
rule jb_cut_batch uses across the devices of one context), so N = 1 cuts the
whole GiB on one GPU.  Documents are independent (tokenizer.go:158-160): no
data-path collective, ranks only meet at the timing barriers and for the
job-level sums, over gloo (CPU tensors; no RCCL).

Ranks: `python bench.py --gpus N` starts N child processes of itself, one per
GPU (RANK = LOCAL_RANK = r), before any GPU call, and exits non-zero when
fewer than N GPUs are visible or a rank fails; under torch.distributed.run
(WORLD_SIZE set) the ranks come from the environment and --gpus must match.
Rank 0 generates the fixed corpus once and the other ranks map it.

A step is one full Cut pass (every kernel, token spans out) over the rank's
shard, inputs already resident in HBM.  `value` = all ranks' runes x K / the
slowest rank's time for the K timed steps.

After timing, every rank downloads its spans and checks ALL of its shard
token for token against the oracle (oracle/jieba_oracle.c, the C restatement
of tokenizer.go) on the host's CPUs; at N = 1 that full-corpus oracle run is
also `cpu_baseline` (threads = the CPUs this process may use).  `roofline` is
the dominant kernel's, from HIP event pairs around each launch on the launch
stream (a second pass of the K steps, kernel by kernel).

Other BASELINE configs: --workload sentence (config 1: jb_cut latency on the
19-rune sentence of tokenizer_test.go:531), s10k (configs 2/3 with --hmm 0/1),
long-punct / long-oov (configs 5a / 5b).
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
    _p = os.path.join(ROOT, _sub)
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0   # float4 copy, same guide
METRIC = "UTF-8 Chinese chars/sec segmented (whole node) + achieved HBM GB/s vs peak"
SENTENCE = "我昨天去上海交通大學與老師討論量子力學"  # tokenizer_test.go:531
REF_SENTENCE_NS = 30726                         # tokenizer_test.go:610 (i5-9400)
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


# ---------------------------------------------------------------------------
# host helpers
# ---------------------------------------------------------------------------
def effective_cpus():
    """CPUs this process may use: its affinity set, capped by a cgroup CPU quota
    (cpu.max) when one is set.  On the GPU box `nproc` shows the whole machine
    while the job's share is enforced by the quota."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def han_bytes(buf, n, chunk=64 << 20):
    """Bytes of buf[:n] that belong to \\p{Han} runes (3-byte BMP Han + 4-byte forms)."""
    total = 0
    for a in range(0, n, chunk):
        b = np.asarray(buf[a:min(n, a + chunk) + 2])
        m = len(b) - 2 if a + chunk < n else min(len(b), n - a)
        lead3 = np.nonzero((b[:m] >= 0xE0) & (b[:m] < 0xF0))[0]
        lead3 = lead3[lead3 + 2 < len(b)]
        cp = ((b[lead3].astype(np.uint32) & 0x0F) << 12) | ((b[lead3 + 1].astype(np.uint32) & 0x3F) << 6) | \
            (b[lead3 + 2].astype(np.uint32) & 0x3F)
        h3 = ((cp >= 0x3400) & (cp <= 0x4DBF)) | ((cp >= 0x4E00) & (cp <= 0x9FFC)) | \
            ((cp >= 0x2E80) & (cp <= 0x2FD5)) | ((cp >= 0xF900) & (cp <= 0xFAD9)) | (cp == 0x3005) | \
            (cp == 0x3007) | ((cp >= 0x3021) & (cp <= 0x3029)) | ((cp >= 0x3038) & (cp <= 0x303B))
        total += int(h3.sum()) * 3 + int(np.count_nonzero((b[:m] >= 0xF0) & (b[:m] <= 0xF4))) * 4
    return total


def count_runes(buf, n, chunk=256 << 20):
    return sum(int(np.count_nonzero((np.asarray(buf[a:min(n, a + chunk)]) & 0xC0) != 0x80))
               for a in range(0, n, chunk))


def load_pmc_traffic(kernel, workload_key):
    """HBM bytes per launch of `kernel` from the committed PMC summary (separate
    rocprofv3 --pmc passes, corrected as MI355X_MICROARCH.md prescribes), when
    that summary was collected on this same workload; else None."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        if d.get("workload_key") != workload_key:
            return None
        for name, e in d["kernels"].items():  # e.g. "k_zh<true>" for kernel "k_zh"
            if name == kernel or name.startswith(kernel + "<"):
                return e["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    return None


# ---------------------------------------------------------------------------
# workload
# ---------------------------------------------------------------------------
def shared_corpus_dir():
    """Where rank 0 leaves the generated corpus for the other ranks of a job (one
    directory per rendezvous port, under the temp dir)."""
    return os.path.join(tempfile.gettempdir(), f"jb_bench_corpus_{os.environ.get('MASTER_PORT', 'local')}")


def make_workload(args, s, rank, world=1, dist=None):
    """(buf, doc_off, description) of the WHOLE job's input (every rank sees the
    same one and takes its shard) — or of this rank's own input for the
    single-document / per-GPU workloads.  With several ranks, rank 0 generates the
    fixed corpus on all the job's CPUs and writes it to a temp directory; the other
    ranks map it read-only after a barrier (one generation per job, not per rank)."""
    import synth
    if args.workload == "docs":
        mib = args.corpus_mib
        desc = f"C_syn corpus, {mib:g} MiB fixed ({'1 GiB = config 4' if mib == 1024 else 'reduced'})"
        if dist is None or world == 1:
            buf, off, _ = s.corpus_parallel(synth.KIND_DOCS, 0, target_bytes=int(mib * (1 << 20)),
                                            threads=max(1, min(16, effective_cpus()[0])))
            return buf, off, desc
        d = shared_corpus_dir()
        if rank == 0:
            buf, off, _ = s.corpus_parallel(synth.KIND_DOCS, 0, target_bytes=int(mib * (1 << 20)),
                                            threads=max(1, min(16, effective_cpus()[0])))
            os.makedirs(d, exist_ok=True)
            np.save(os.path.join(d, "buf.npy"), buf)
            np.save(os.path.join(d, "off.npy"), off)
        dist.barrier()
        if rank != 0:
            buf = np.load(os.path.join(d, "buf.npy"), mmap_mode="r")
            off = np.load(os.path.join(d, "off.npy"))
        return buf, off, desc
    if args.workload == "s10k":
        buf, off, _ = s.corpus(synth.KIND_SENTENCES, 0, max_docs=10_000, target_bytes=64 << 20)
        return buf, off, "S10k: 10,000 synthetic sentences (configs 2/3)"
    if args.workload in ("long-punct", "long-oov"):
        kind = synth.KIND_LONG_PUNCT if args.workload == "long-punct" else synth.KIND_LONG_OOV
        buf, off, _ = s.corpus(kind, rank, target_runes=1_000_000)
        return buf, off, ("L1M: one 1,000,000-rune document, " +
                          ("punctuated (5a)" if args.workload == "long-punct" else "unpunctuated, 30% OOV (5b)"))
    raise ValueError(args.workload)


def shard_for(buf, off, world, rank, sharded):
    """(shard buffer with 64 padding bytes, rebased offsets, first doc, base byte)."""
    import shard
    if not sharded or world == 1:
        return buf, np.asarray(off, np.uint64), 0, 0
    cut = shard.shard_bounds(off, world)
    d0, d1 = cut[rank], cut[rank + 1]
    base, end = int(off[d0]), int(off[d1])
    sub = np.zeros(end - base + 64, np.uint8)
    sub[: end - base] = buf[base:end]
    return sub, np.asarray(off[d0:d1 + 1], np.uint64) - np.uint64(base), d0, base


# ---------------------------------------------------------------------------
# the measured path
# ---------------------------------------------------------------------------
class GpuCutter:
    """jb_cut_device on HBM-resident input: one rank's shard, one GPU."""

    def __init__(self, tk, buf, off, hmm, local):
        import torch
        import jiebahip as J
        self.torch, self.J, self.tk = torch, J, tk
        self.dev = torch.device("cuda", local)
        self.nbytes = int(off[-1])
        self.ndocs = len(off) - 1
        self.hmm = bool(hmm)
        self.d_text = torch.from_numpy(np.asarray(buf[: self.nbytes + 64])).to(self.dev)
        self.d_off = torch.from_numpy(np.asarray(off, np.int64)).to(self.dev)
        self.stream = torch.cuda.current_stream(self.dev).cuda_stream
        self.ptrs = None

    def step(self):
        self.ptrs = self.tk.cut_device(self.d_text.data_ptr(), self.nbytes, self.d_off.data_ptr(), self.ndocs,
                                       self.hmm, self.stream)

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def profile(self, steps):
        """Per-kernel (total ms, launches) over `steps` more steps, launched kernel
        by kernel with HIP events on the launch stream; and their ms per step."""
        self.tk.profile(True)
        self.tk.profile_reset()
        self.sync()
        t = time.perf_counter()
        for _ in range(steps):
            self.step()
        self.sync()
        ms = (time.perf_counter() - t) / steps * 1e3
        k = self.tk.profile_read()
        self.tk.profile(False)
        return k, ms

    def results(self):
        """(starts u32, ends u32, doc_tok u64[ndocs+1]) of the last step; raises if that
        pipeline reported an error (jb_device_status)."""
        J = self.J
        ps, pe, pd, pn = self.ptrs
        self.sync()
        self.tk.device_status(self.stream)
        ntok = int(J.dev_to_host(pn, 8, np.uint64)[0])
        return (J.dev_to_host(ps, 4 * ntok, np.uint32), J.dev_to_host(pe, 4 * ntok, np.uint32),
                J.dev_to_host(pd, 8 * (self.ndocs + 1), np.uint64))

    def ties(self):
        return self.tk.last_ties()


def check_shard(results, o, buf, off, hmm, threads):
    """The rank's GPU spans against the oracle over its WHOLE shard (timed: at
    N = 1 this run is cpu_baseline).  Returns a dict."""
    gs, ge, gd = results
    t = time.perf_counter()
    os_, oe, od = o.cut_batch(buf, off, bool(hmm), nthreads=threads)
    cpu_s = time.perf_counter() - t
    ok = bool(np.array_equal(gs, os_) and np.array_equal(ge, oe) and np.array_equal(gd, od))
    mism = 0
    if not ok:
        n = min(len(gs), len(os_))
        mism = int(np.count_nonzero((gs[:n] != os_[:n]) | (ge[:n] != oe[:n]))) + abs(len(gs) - len(os_))
        mism = max(mism, 1)
    return {"ok": ok, "mismatches": mism, "tokens": int(len(os_)), "gpu_tokens": int(len(gs)), "cpu_s": cpu_s,
            "oracle_ties": int(o.ties)}


def job_sums(dist, agg_dev, vals, op="sum"):
    """Element-wise sum (or max) of a list of floats over ranks."""
    if dist is None:
        return [float(v) for v in vals]
    import torch
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=agg_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return [float(x) for x in t.tolist()]


# The timed step's output (jb_cut_device): u32 (start, end) spans, 8 B per token
# ("with (start,end) uint32 spans: 8 B x tokens").
OUTPUT_FORMAT = "u32 (start, end) token spans, 8 B per token"
SPAN_BYTES = 8


def alg_bytes_per_byte(step_bytes, step_tokens):
    """SURVEY.md §8d's algorithmic bytes per input byte of the timed step: 1 B read
    + the output written, here the spans (8 B per token) spread over the input bytes."""
    return 1.0 + SPAN_BYTES * step_tokens / step_bytes if step_bytes else 1.0


def roofline_of(kernels, units, traffic_of, per_byte):
    """Per kernel: algorithmic bytes per launch = `per_byte` (alg_bytes_per_byte of the
    step) x the unit bytes the launch processes, over its average launch time.  Units:
    every input byte for k_mark_walk (it classifies and walks the whole batch), the Han
    bytes for k_zh / k_long / k_long_dp (DP + Viterbi over zh blocks)."""
    out = {}
    for kname, u in units.items():
        kk = kernels.get(kname)
        if not kk or not u:
            continue
        alg = per_byte * u
        achieved = alg / (kk["avg_ms"] * 1e-3) / 1e9
        out[kname] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic_of(kname),
                      "kernel": kname, "output_format": OUTPUT_FORMAT, "alg_bytes_per_unit_byte": round(per_byte, 5),
                      "alg_bytes_per_launch": alg, "avg_launch_ms": kk["avg_ms"],
                      "frac_of_measured_copy": round(achieved / HBM_MEASURED_GBS, 5)}
    return out


def roofline_step(step_bytes, step_tokens, ms_per_step):
    """The whole timed step against HBM: its algorithmic bytes (input read + spans
    written) over ms_per_step."""
    alg = step_bytes + SPAN_BYTES * step_tokens
    achieved = alg / (ms_per_step * 1e-3) / 1e9 if ms_per_step else 0.0
    return {"bound": "hbm", "output_format": OUTPUT_FORMAT, "alg_bytes_per_step": int(alg),
            "input_bytes": int(step_bytes), "tokens": int(step_tokens), "ms_per_step": ms_per_step,
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5)}


def run(args, world, rank, dist, agg_dev, make_cutter, open_oracle, log=print):
    """Everything but process setup: workload, shard, timing, per-rank parity,
    job-level aggregation.  make_cutter(buf, off, hmm) gives the rank's measured
    path (GpuCutter on a GPU); open_oracle() the checker.  Returns rank 0's bench
    line (a dict), None on other ranks."""
    import synth
    t0 = time.time()
    s = synth.Synth(nwords=args.nwords)
    sharded = args.workload == "docs"
    buf, off, wdesc = make_workload(args, s, rank, world, dist)
    emul = sharded and world == 1 and args.shard_of > 1  # one GPU's shard of an N-GPU job, on one GPU
    if emul:
        if not 0 <= args.shard_rank < args.shard_of:
            raise ValueError(f"--shard-rank {args.shard_rank} outside 0..{args.shard_of - 1}")
        sbuf, soff, d0, base = shard_for(buf, off, args.shard_of, args.shard_rank, True)
        wdesc += f"; ONLY shard {args.shard_rank} of {args.shard_of} (one GPU's share at {args.shard_of} GPUs)"
        del buf
    else:
        sbuf, soff, d0, base = shard_for(buf, off, world, rank, sharded)
    if sharded and world > 1:
        del buf
        dist.barrier()  # every rank holds its own copy of its shard: the shared corpus file can go
        if rank == 0:
            import shutil
            shutil.rmtree(shared_corpus_dir(), ignore_errors=True)
    nbytes = int(soff[-1])
    nrunes = count_runes(sbuf, nbytes)
    hbytes = han_bytes(sbuf, nbytes)
    gen_s = time.time() - t0

    cutter = make_cutter(sbuf, soff, args.hmm)
    for _ in range(args.warmup):
        cutter.step()
    cutter.sync()
    if dist:
        dist.barrier()
    cutter.sync()
    t = time.perf_counter()
    for _ in range(args.steps):
        cutter.step()
    cutter.sync()
    elapsed = time.perf_counter() - t
    if dist:
        dist.barrier()
    results = cutter.results()
    ties = cutter.ties()
    ntok = int(len(results[0]))

    kprof, prof_ms = ({}, None) if args.no_profile else cutter.profile(args.steps)
    kernels = {k: {"avg_ms": ms / n, "launches": int(n)} for k, (ms, n) in kprof.items() if n}

    # ---- parity: this rank's whole shard against the oracle ----------------
    ncpu, nproc, quota = effective_cpus()
    par = None
    o = None
    if not args.no_parity:
        o = open_oracle()
        import oracle as O
        O.set_viterbi_backptr(args.workload.startswith("long"))  # path copy is O(m^2) on a 1M-rune run
        par = check_shard(results, o, sbuf, soff, args.hmm, max(1, ncpu // world))

    # ---- job-level aggregates ----------------------------------------------
    (elapsed_max,) = job_sums(dist, agg_dev, [elapsed], "max")
    sums = job_sums(dist, agg_dev, [nrunes, nbytes, hbytes, len(soff) - 1, ties,
                                    par["mismatches"] if par else 0, par["tokens"] if par else 0,
                                    0 if par is None else (0 if par["ok"] else 1),
                                    par["oracle_ties"] if par else 0, ntok])
    tot_runes, tot_bytes, tot_han, tot_docs, tot_ties, tot_mism, tot_tok, bad_ranks, tot_oties, tot_gtok = sums
    # every rank's own numbers (an N > 1 line shows a straggler)
    mine = {"rank": rank, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
            "shard_bytes": nbytes, "shard_docs": len(soff) - 1, "shard_chars": nrunes, "first_doc": d0,
            "tokens": ntok, "bit_exact": None if par is None else par["ok"]}
    if dist is not None and world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    else:
        per_rank = [mine]

    cpu = None
    if rank == 0 and world == 1 and par is not None:
        cpu = {"value": round(nrunes / par["cpu_s"], 1), "unit": "chars/s", "cores": max(1, ncpu // world),
               "kind": "port",
               "sample": (f"the whole workload ({nbytes / 2**20:.1f} MiB, {nrunes} chars, {len(soff) - 1} docs): "
                          f"oracle/jieba_oracle.c (C restatement of tokenizer.go, "
                          f"{'O(n) back-pointer' if args.workload.startswith('long') else 'literal path-copy'} "
                          f"Viterbi), threads over documents, {par['cpu_s']:.2f} s; the same run is the parity check"),
               "cpu_model": cpu_model(), "nproc": nproc, "cgroup_quota_cpus": quota}
        if args.cpu1_sample_mib > 0 and args.workload == "docs":
            lim = int(args.cpu1_sample_mib * (1 << 20))
            d1 = max(1, min(len(soff) - 1, int(np.searchsorted(soff, min(lim, nbytes), side="right")) - 1))
            b1 = int(soff[d1])
            r1 = count_runes(sbuf, b1)
            tc = time.perf_counter()
            o.cut_batch(sbuf[: b1 + 16], soff[: d1 + 1], bool(args.hmm), nthreads=1)
            c1 = time.perf_counter() - tc
            cpu["value_1thread"] = round(r1 / c1, 1)
            cpu["sample_1thread"] = f"first {d1} documents ({b1 / 2**20:.1f} MiB, {r1} chars), 1 thread, {c1:.2f} s"

    if rank != 0:
        return None
    units = {"k_mark_walk": float(nbytes), "k_zh": float(hbytes)}
    if args.workload == "long-oov":  # one unpunctuated block: its Han bytes all go through the long-block path
        units["k_long"] = float(hbytes)  # (its kernels as one launch, JB_LONG_FUSED=1)
        units["k_long_dp"] = float(hbytes)  # (separate launches)
    wkey = f"{args.workload}:{nbytes}:{'hmm' if args.hmm else 'nohmm'}:{args.dict_kind}"
    rooflines = roofline_of(kernels, units, lambda k: load_pmc_traffic(k, wkey), alg_bytes_per_byte(nbytes, ntok))
    roof = None
    if kernels:
        dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
        if dom in rooflines:
            roof = dict(rooflines[dom], dominant_kernel=dom)
        elif rooflines:
            roof = dict(max(rooflines.values(), key=lambda r: r["avg_launch_ms"]), dominant_kernel=dom)
    ms_per_step = elapsed_max / args.steps * 1e3
    value = tot_runes * args.steps / elapsed_max
    parity = None
    if par is not None:
        parity = {"scope": "every token of every rank's shard" if sharded else "every token of the workload",
                  "bytes": int(tot_bytes), "docs": int(tot_docs), "tokens": int(tot_tok),
                  "bit_exact": bad_ranks == 0 and tot_mism == 0, "mismatches": int(tot_mism),
                  "ranks_checked": world, "oracle_threads_per_rank": max(1, ncpu // world)}
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "chars/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded D_syn 350k-word dict, E_syn emissions, C_syn Zipf corpus)",
        "config": {"workload": f"{wdesc}, Cut hmm={'on' if args.hmm else 'off'}, "
                               f"{'NewJiebaTokenizer (prefix dict, size 60,101,967)' if args.dict_kind == 'prefix' else 'NewTokenizer(dict.txt)'}",
                   "corpus_bytes": int(tot_bytes), "corpus_chars": int(tot_runes), "corpus_han_bytes": int(tot_han),
                   "corpus_docs": int(tot_docs), "rank0_shard_bytes": nbytes, "dict_words": s.nwords,
                   "parallelism": f"doc-shard x{world} (byte-balanced contiguous ranges), no collectives",
                   "emulated_shard": {"of": args.shard_of, "rank": args.shard_rank} if emul else None,
                   "per_rank": per_rank},
        "roofline": roof,
        "roofline_kernels": rooflines,
        "roofline_step": roofline_step(tot_bytes, tot_gtok, ms_per_step),
        "cpu_baseline": cpu,
        "parity": parity,
        "viterbi_ties": {"gpu": int(tot_ties), "oracle": int(tot_oties) if par else None,
                         "what": "exact stateTransitionRoute ties a == b > minFloat (Q12, tokenizer.go:748-753), "
                                 "resolved in stateChange order; the reference resolves them in Go map order"},
        "han_chars_per_s": round(tot_han / 3 * args.steps / elapsed_max, 1),
        "input_GBps": round(tot_bytes * args.steps / elapsed_max / 1e9, 3),
        "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
        "ms_per_step_kernel_by_kernel": round(prof_ms, 4) if prof_ms else None,
        "gen_s": round(gen_s, 2),
        "workload_key": wkey,
    }
    return line, (sbuf, soff, cutter)


def end_to_end(tk, buf, off, hmm, nrunes, reps=3):
    """The host-memory paths a drop-in caller gets (never the line's `value`): the batch
    in host memory, text pieces copied up while earlier pieces are cut and their
    results come back (three streams).  `value`: jb_cut_batch_mask (2 bits per byte)
    from pageable memory; `spans`: jb_cut_batch_into (u64 spans into caller arrays);
    `masks_pinned`: masks with the text in jb_host_alloc memory (no staging copy).
    The masks are checked against the spans."""
    import jiebahip as J

    def timed(fn):
        r = fn(None)  # warm the pinned staging and the output arrays
        t = time.perf_counter()
        for _ in range(reps):
            r = fn(r)
        return r, (time.perf_counter() - t) / reps

    res, s_sp = timed(lambda r: tk.cut_batch_into(buf, off, bool(hmm), r[3] if r else None))
    r32, s_32 = timed(lambda r: tk.cut_batch_into32(buf, off, bool(hmm), r[3] if r else None))
    ok32 = bool(np.array_equal(r32[0].astype(np.uint64) + np.uint64(off[0]), res[0]) and
                np.array_equal(r32[1].astype(np.uint64) + np.uint64(off[0]), res[1]) and np.array_equal(r32[2], res[2]))
    del r32
    ms, me, _ = tk.cut_batch_mask(buf, off, bool(hmm))
    (ms, me, ntok), s_m = timed(lambda r: tk.cut_batch_mask(buf, off, bool(hmm), (r[0], r[1]) if r else None))
    nb = int(off[-1] - off[0])
    ms2, me2 = J.mask_to_spans(ms, me, nb, int(off[0]))
    ok_mask = bool(np.array_equal(ms2, res[0]) and np.array_equal(me2, res[1]))
    hb = J.HostBuffer(len(buf))
    try:
        hb.array[:] = buf
        (pms, pme, _), s_p = timed(lambda r: tk.cut_batch_mask(hb.array, off, bool(hmm), (r[0], r[1]) if r else None))
        ok_pin = bool(np.array_equal(pms, ms) and np.array_equal(pme, me))
    finally:
        hb.free()

    def rate(sec):
        return {"value": round(nrunes / sec, 1), "unit": "chars/s", "ms": round(sec * 1e3, 2)}
    out = rate(s_m)
    out["what"] = ("jb_cut_batch_mask from pageable host memory: pieces of 64 MiB staged into pinned memory and "
                   "copied up while earlier pieces are cut, token boundaries back as 2 bits per input byte "
                   "(SURVEY.md §8d's output format); checked against the spans below")
    out["tokens"] = int(ntok)
    out["same_tokens_as_spans"] = ok_mask
    out["spans"] = dict(rate(s_sp), what="jb_cut_batch_into from pageable host memory: the same pipeline with the "
                                         "spans packed on the GPU (k_span_pack: 2 B per token, gap | length, rare "
                                         "escapes in a side list), decoded on the host into u64 batch offsets in "
                                         "caller arrays (16 B written per token)",
                        span_pack=os.environ.get("JB_SPAN_PACK", "1") != "0")
    out["spans32"] = dict(rate(s_32), what="jb_cut_batch_into32, what the Go binding's Cut / CutBatch call: the same, "
                                           "decoded into u32 offsets from the batch's first byte in caller arrays "
                                           "(8 B written per token)", same_as_spans=ok32)
    out["masks_pinned"] = dict(rate(s_p), what="jb_cut_batch_mask with the text in jb_host_alloc (pinned) memory: "
                                               "no staging copy", same_as_pageable=ok_pin)
    return out


def sentence_latency(tk, o, n):
    """Config 1: Cut(sentence, hmm=true) through jb_cut (host string in, spans out,
    the same call a Go caller makes); the oracle on one core beside it."""
    import ctypes as C
    import jiebahip as J
    import oracle as O
    t = SENTENCE.encode("utf-8")
    sp = J.jb_spans()
    L = J.lib()
    assert tk.Cut(SENTENCE, True) == o.cut(SENTENCE, True)
    for _ in range(50):
        J._check(L.jb_cut(tk.h, t, len(t), 1, C.byref(sp)))
        L.jb_spans_free(C.byref(sp))
    lat = np.empty(n)
    for i in range(n):
        a = time.perf_counter_ns()
        J._check(L.jb_cut(tk.h, t, len(t), 1, C.byref(sp)))
        lat[i] = time.perf_counter_ns() - a
        L.jb_spans_free(C.byref(sp))
    ol = O.lib()
    s = np.zeros(64, np.uint32)
    e = np.zeros(64, np.uint32)
    olat = np.empty(n)
    for i in range(n):
        a = time.perf_counter_ns()
        ol.or_cut(o.h, t, len(t), 1, s.ctypes.data, e.ctypes.data, 64)
        olat[i] = time.perf_counter_ns() - a
    return lat, olat


STAMPS_LIB = os.path.join(ROOT, "jieba-go_amd", "lib_st", "libjiebahip.so")


def parse_zh_clocks(err):
    """The last "[jb] k_zh clocks/wave" line a STAMPS build printed: (DP cycles per
    wave, DP loop trips per wave, k_zh cycles per wave, DP lane use)."""
    import re
    last = None
    for ln in err.splitlines():
        m = re.search(r"k_zh clocks/wave: setup (\S+) dp (\S+) .* total (\S+); chunks/wave \S+; "
                      r"lane DP steps (\S+) vs 64\*max (\S+) \(DP lane use (\S+)\)", ln)
        if m:
            last = m
    if not last:
        return None
    dp, total, max64, use = float(last.group(2)), float(last.group(3)), float(last.group(5)), float(last.group(6))
    return dp, max64 / 64.0, total, use


def latency_probe(args):
    """Child process (JB_LIB = the STAMPS build, JB_STAMPS=1): k_zh's per-wave phase
    clocks on a loaded chip (the first 128 MiB of the headline corpus: every wave has
    ~11 groups) and on one wave alone (a 1 KiB batch: one group), printed by the
    library to stderr and parsed by the parent."""
    import torch
    import jiebahip as J
    import synth
    s = synth.Synth(nwords=args.nwords)
    tmp = tempfile.mkdtemp(prefix="jb_lat_")
    dpath, epath = s.write_files(tmp)
    tk = J.Tokenizer(J.make_config(dict_path=dpath, emit_path=epath, kind=J.JB_DICT_PREFIX,
                                   size_override=J.JIEBA_SIZE, device=0))
    buf, off, _ = s.corpus_parallel(synth.KIND_DOCS, 0, target_bytes=128 << 20,
                                    threads=max(1, min(16, effective_cpus()[0])))
    one = int(np.searchsorted(off, 1024, side="right")) - 1  # whole documents in the first KiB
    small = (np.concatenate([np.asarray(buf[: int(off[max(one, 1)])]), np.zeros(64, np.uint8)]),
             np.asarray(off[: max(one, 1) + 1], np.uint64))
    for tag, (b, o) in (("loaded", (buf, off)), ("one_wave", small)):
        c = GpuCutter(tk, b, o, True, 0)
        for _ in range(2):
            c.step()
            c.sync()
        print(f"[probe] {tag} done", file=sys.stderr, flush=True)
    tk.close()


def roofline_latency(timeout=240):
    """k_zh's DP against its latency floor: cycles per DP step
    per wave with every wave busy, beside the same for one wave alone on an idle
    chip (the step's own dependent chain: record and weight loads, ring reads,
    float64 adds and compares).  frac = floor / loaded: 1.0 would mean the 4 waves
    per SIMD only share the SIMD, none slows another.  From the STAMPS build in a
    child process; None when it is absent or fails."""
    import subprocess
    if not os.path.exists(STAMPS_LIB):
        return None
    # (JB_ZH_WIDE=1: the one-wave batch runs k_zh's wide form too, the form the headline batch gets)
    env = dict(os.environ, JB_LIB=STAMPS_LIB, JB_STAMPS="1", JB_GRAPH="0", JB_ZH_WIDE="1")
    try:
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--latency-probe"], env=env,
                           capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return None
    err = p.stderr
    parts = err.split("[probe] loaded done")
    if p.returncode != 0 or len(parts) != 2:
        return {"error": err[-400:]}
    loaded, alone = parse_zh_clocks(parts[0]), parse_zh_clocks(parts[1])
    if not loaded or not alone:
        return {"error": "no k_zh clocks in the probe's output"}
    cl, ca = loaded[0] / loaded[1], alone[0] / alone[1]
    lines = [ln.split("] ", 1)[1] for ln in parts[0].splitlines()
             if ln.startswith("[jb] k_zh clocks") or ln.startswith("[jb] k_mark_walk clocks")]
    return {"bound": "latency", "unit": "cycles per DP step per wave",
            "achieved": round(cl, 1), "floor": round(ca, 1), "frac": round(ca / cl, 4),
            "dp_share_of_k_zh": round(loaded[0] / loaded[2], 4), "dp_lane_use": loaded[3],
            "waves_per_simd": 4, "workgroup_waves": 16, "phase_clocks_loaded": lines[-2:],
            "what": "k_zh's backward DP (calcDagProba + maxIndexProba): s_memtime cycles per step of a wave's "
                    "DP loop, every wave busy (first 128 MiB of the corpus) vs one wave alone (a 1 KiB batch); "
                    "STAMPS build of the same source, per-wave clocks cost a few %"}


class GpuBackend:
    """The measured path: one jb context on the rank's GPU, GpuCutter over it."""
    name = "gpu"

    def device_count(self):
        import torch
        return torch.cuda.device_count()  # (counts devices without initialising one)

    def open(self, cfg_kw, local):
        import torch
        import jiebahip as J
        torch.cuda.set_device(local)
        self.tk = J.Tokenizer(J.make_config(device=local, **cfg_kw))
        return self.tk

    def make_cutter(self, buf, off, hmm, local):
        return GpuCutter(self.tk, buf, off, hmm, local)

    def close(self):
        self.tk.close()


def load_backend():
    """GpuBackend, or — for the CPU test of the N-rank launcher only — the class
    JB_BENCH_TEST_BACKEND names ("module:Class", e.g. an oracle stand-in).  A
    test backend's line says so in `data`; the driver never sets the variable."""
    spec = os.environ.get("JB_BENCH_TEST_BACKEND")
    if not spec:
        return GpuBackend()
    import importlib
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)()


def share_gpu():
    """JB_BENCH_SHARE_GPU=1 (testing only): every rank on GPU (LOCAL_RANK mod the GPUs
    visible), so the N-rank path runs end to end on a one-GPU box; the line's `data`
    and `config.ranks` say so, and it is never a scaling number."""
    return os.environ.get("JB_BENCH_SHARE_GPU") == "1"


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch(n, argv, backend):
    """`--gpus N` without an inherited WORLD_SIZE: start N fresh child processes of
    this script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on
    127.0.0.1), before this process makes any GPU call.  The children meet over
    gloo (barriers and job sums on CPU tensors; no RCCL); rank 0 prints the line on
    the inherited stdout.  If a child fails, the others are stopped (they would
    wait at a barrier forever) and the launcher exits non-zero."""
    import signal
    import subprocess
    have = backend.device_count()
    if have < n and not (share_gpu() and have >= 1):
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible; not running a smaller job in its place",
              file=sys.stderr)
        return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, JB_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      start_new_session=True))
    rc = 0
    alive = list(procs)
    while alive:
        time.sleep(0.2)
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr)
                for q in alive:
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
    return rc


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one process each). Without WORLD_SIZE in the environment bench.py starts the "
                         "N ranks itself; under torch.distributed.run it must equal WORLD_SIZE. Default 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["docs", "sentence", "s10k", "long-punct", "long-oov"], default="docs")
    ap.add_argument("--corpus-mib", type=float, default=1024.0,
                    help="docs: the fixed corpus (MiB), strong-scaled over the ranks; 1024 = config 4")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="docs, one process: cut only shard --shard-rank of the corpus split N ways (the shard one "
                         "GPU of an N-GPU job gets), to know the per-GPU rate at N GPUs on one GPU; the line's "
                         "value is then that one GPU's chars/s, not a job's")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--hmm", type=int, default=1)
    ap.add_argument("--nwords", type=int, default=350_000)
    ap.add_argument("--dict-kind", choices=["prefix", "txt"], default="prefix",
                    help="prefix: NewJiebaTokenizer semantics (prefix_dictionary.gob, size 60,101,967) as in the "
                         "reference's own benchmarks; txt: NewTokenizer(dict.txt)")
    ap.add_argument("--cpu1-sample-mib", type=float, default=96.0,
                    help="one-thread oracle sample (docs, N = 1); 0: skip")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check (and cpu_baseline)")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--sentence-iters", type=int, default=5000)
    ap.add_argument("--no-latency", action="store_true", help="skip the roofline_latency probe")
    ap.add_argument("--latency-probe", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.latency_probe:
        latency_probe(args)
        return 0

    backend = load_backend()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if (args.gpus or 1) > 1:
            return launch(args.gpus, argv, backend)
        world, rank, local = 1, 0, 0
    else:
        world = int(env_world)
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if args.gpus is not None and args.gpus != world:
            print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}", file=sys.stderr)
            return 2
    if share_gpu() and backend.device_count() >= 1:
        local %= backend.device_count()
    if local >= backend.device_count():
        print(f"bench.py: rank {rank} wants GPU {local}, only {backend.device_count()} visible", file=sys.stderr)
        return 2

    import torch
    import jiebahip as J
    import synth

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")  # barriers + scalar sums only: no RCCL
    agg_dev = torch.device("cpu")

    tmp = tempfile.mkdtemp(prefix=f"jb_bench_r{rank}_")
    dpath, epath = synth.Synth(nwords=args.nwords).write_files(tmp)
    kind = J.JB_DICT_PREFIX if args.dict_kind == "prefix" else J.JB_DICT_TXT
    size_override = J.JIEBA_SIZE if args.dict_kind == "prefix" else 0
    tk = backend.open(dict(dict_path=dpath, emit_path=epath, kind=kind, size_override=size_override), local)

    def open_oracle():
        import oracle as O
        return O.Oracle.from_files(dpath, epath, kind, size_override)

    if args.workload == "sentence":
        o = open_oracle()
        lat, olat = sentence_latency(tk, o, args.sentence_iters)
        med = float(np.median(lat))
        line = {"metric": METRIC, "value": round(19 / (med * 1e-9), 1), "unit": "chars/s", "n_gpus": 1,
                "steps": args.sentence_iters, "warmup": 50, "ms_per_step": round(med * 1e-6, 5),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                "data": "the reference's benchmark sentence", "config": {
                    "workload": f"config 1: Cut({SENTENCE!r}, hmm=true) through jb_cut, one call at a time "
                                "(host string in, one k_small launch with the text in its kernel arguments, "
                                "spans back in pinned host memory), 19 runes / 57 bytes",
                    "parallelism": "one call"},
                "vs_reference_ns_per_op": round(REF_SENTENCE_NS / med, 3),
                "latency_ns": {"median": med, "p10": float(np.percentile(lat, 10)),
                               "p99": float(np.percentile(lat, 99)), "mean": float(lat.mean())},
                "reference_ns_per_op": {"value": REF_SENTENCE_NS, "hardware": "i5-9400 (tokenizer_test.go:610)"},
                "cpu_baseline": {"value": round(19 / (float(np.median(olat)) * 1e-9), 1), "unit": "chars/s",
                                 "cores": 1, "kind": "port", "latency_ns_median": float(np.median(olat)),
                                 "sample": f"{args.sentence_iters} calls of or_cut (oracle/jieba_oracle.c) on the "
                                           "same sentence, ctypes call overhead included", "cpu_model": cpu_model()},
                "roofline": None}
        print(json.dumps(line), flush=True)
        backend.close()
        return 0

    out = run(args, world, rank, dist, agg_dev,
              lambda b, o_, h: backend.make_cutter(b, o_, h, local), open_oracle)
    if rank == 0:
        line, (sbuf, soff, _) = out
        launcher = os.environ.get("JB_BENCH_LAUNCHER") or ("torch.distributed.run" if world > 1 else "single process")
        line["config"]["ranks"] = {"launcher": launcher, "processes": world, "rank_to_gpu": "rank r -> GPU r",
                                   "host_group": "gloo (timing barriers + job sums; no RCCL)" if world > 1 else None,
                                   "per_rank": line["config"].pop("per_rank")}
        if share_gpu():
            line["config"]["ranks"]["rank_to_gpu"] = "TEST (JB_BENCH_SHARE_GPU): rank r -> GPU r mod the GPUs visible"
            line["data"] = "TEST (JB_BENCH_SHARE_GPU, ranks share a GPU): not a scaling measurement; " + line["data"]
        if backend.name != "gpu":
            line["data"] = f"TEST BACKEND {backend.name}: not a measurement"
        if world == 1 and not args.no_e2e:
            line["end_to_end_host"] = end_to_end(tk, sbuf, soff, args.hmm, line["config"]["corpus_chars"])
        if world == 1 and args.workload == "docs" and not args.no_latency:
            line["roofline_latency"] = roofline_latency()
        line["loaded"] = J.loaded_runtime() if backend.name == "gpu" else None
        print(json.dumps(line), flush=True)
    backend.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
