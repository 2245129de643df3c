"""CPU, world_size 2 over gloo: the multi-GPU path's sharding and job-level
aggregation (bench.py's max-over-ranks time, summed work), with the oracle
standing in for each rank's device."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import shard
from bench_backend import OracleCutter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, dict_path, emit_path, corpus_mib, corrupt_rank, out_dir):
    import json
    import types
    import bench
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = types.SimpleNamespace(workload="docs", corpus_mib=corpus_mib, nwords=20_000, hmm=1, steps=3, warmup=1,
                                 no_profile=True, no_parity=False, cpu1_sample_mib=0, dict_kind="txt")
    seen = {}

    def make_cutter(buf, off, hmm):
        c = OracleCutter(O.Oracle.from_files(dict_path, emit_path, 0), buf, off, hmm, corrupt=rank == corrupt_rank)
        seen["c"] = c
        return c

    out = bench.run(args, world, rank, dist, "cpu", make_cutter, lambda: O.Oracle.from_files(dict_path, emit_path, 0))
    c = seen["c"]
    s, e, d = c.o.cut_batch(c.buf, c.off, True, nthreads=2)
    parts = [None] * world
    dist.all_gather_object(parts, (s, e, d, len(c.off) - 1, c.steps))
    if rank == 0:
        line = out[0]
        with open(os.path.join(out_dir, "line.json"), "w") as f:
            json.dump(line, f)
        np.savez(os.path.join(out_dir, "parts.npz"),
                 **{f"s{r}": p[0] for r, p in enumerate(parts)}, **{f"e{r}": p[1] for r, p in enumerate(parts)},
                 **{f"d{r}": p[2] for r, p in enumerate(parts)},
                 nd=np.array([p[3] for p in parts]), steps=np.array([p[4] for p in parts]))
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover_and_balance():
    rng = np.random.default_rng(0)
    sizes = rng.integers(0, 5000, size=1001)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    for world in (1, 2, 3, 4, 8):
        cut = shard.shard_bounds(off, world)
        assert cut[0] == 0 and cut[-1] == 1001 and all(a <= b for a, b in zip(cut, cut[1:]))
        per = [int(off[cut[r + 1]] - off[cut[r]]) for r in range(world)]
        assert sum(per) == int(off[-1])
        assert max(per) - min(per) <= 2 * 5000


def test_library_shard_bounds_equal_python():
    """jb_shard_bounds (the partition jb_cut_batch gives each device of a ctx)
    and shard.shard_bounds (bench.py's per-rank partition) are the same rule."""
    import jiebahip as J
    rng = np.random.default_rng(5)
    cases = [np.zeros(1, np.uint64), np.array([0, 10], np.uint64), np.array([7, 7, 7, 20], np.uint64)]
    for n in (1, 2, 3, 17, 1000):
        sizes = rng.integers(0, 3000, size=n)
        sizes[rng.random(n) < 0.2] = 0  # empty documents
        cases.append((np.concatenate([[0], np.cumsum(sizes)]) + rng.integers(0, 50)).astype(np.uint64))
    big = np.cumsum(np.full(9, 1 << 40, np.uint64))  # offsets past 2^32
    cases.append(np.concatenate([[0], big]).astype(np.uint64))
    for off in cases:
        for parts in (1, 2, 3, 4, 8, 13):
            assert J.shard_bounds(off, parts) == shard.shard_bounds(off, parts), (len(off), parts)
    with pytest.raises(J.JbError):
        J.shard_bounds(np.array([0, 5, 3], np.uint64), 2)  # not monotonic


@pytest.mark.parametrize("corrupt_rank", [-1, 1])
def test_bench_two_ranks_gloo(syn_small, corrupt_rank):
    """bench.run's N > 1 path on CPU over gloo, world size 2: each rank takes its
    jb_shard_bounds range of the fixed corpus, times its steps, checks its whole
    shard against the oracle; rank 0's line carries the max-over-ranks time and
    the job-level sums.  The per-rank outputs merged in rank order equal one
    process cutting the whole corpus, and one corrupted token on rank 1 makes
    the job's parity fail."""
    import json
    import oracle as O
    import synth
    dp, ep, s = syn_small
    mib = 0.75
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(2, _free_port(), dp, ep, mib, corrupt_rank, out), nprocs=2, join=True,
                           start_method="spawn")
        with open(os.path.join(out, "line.json")) as f:
            line = json.load(f)
        parts = np.load(os.path.join(out, "parts.npz"))
    buf, off, nr = s.corpus_parallel(synth.KIND_DOCS, 0, target_bytes=int(mib * (1 << 20)), threads=2)
    cut = shard.shard_bounds(off, 2)
    assert list(parts["nd"]) == [cut[1] - cut[0], cut[2] - cut[1]] and list(parts["steps"]) == [4, 4]
    merged = shard.merge([(parts[f"s{r}"], parts[f"e{r}"], parts[f"d{r}"], int(off[cut[r]])) for r in range(2)])
    o = O.Oracle.from_files(dp, ep, 0)
    s1, e1, d1 = o.cut_batch(buf, off, True, nthreads=4)
    assert np.array_equal(merged[0], s1) and np.array_equal(merged[1], e1) and np.array_equal(merged[2], d1)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["corpus_bytes"] == int(off[-1]) and line["config"]["corpus_docs"] == len(off) - 1
    assert line["config"]["corpus_chars"] == nr
    assert line["parity"]["bytes"] == int(off[-1]) and line["parity"]["tokens"] == len(s1)
    assert line["parity"]["bit_exact"] == (corrupt_rank < 0)
    assert line["parity"]["mismatches"] == (0 if corrupt_rank < 0 else 1)
    assert line["cpu_baseline"] is None  # (rank 0 at N = 1 only)
    assert abs(line["value"] - nr * 3 / (line["ms_per_step"] * 3e-3)) / line["value"] < 0.05  # (ms rounded)
    # every rank's own step time, kernel times and shard (a straggler shows in the line)
    pr = line["config"]["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1]
    assert [r["shard_docs"] for r in pr] == [cut[1] - cut[0], cut[2] - cut[1]]
    assert [r["shard_bytes"] for r in pr] == [int(off[cut[1]] - off[cut[0]]), int(off[cut[2]] - off[cut[1]])]
    assert [r["first_doc"] for r in pr] == [0, cut[1]]
    assert sum(r["shard_chars"] for r in pr) == nr
    assert max(r["ms_per_step"] for r in pr) == pytest.approx(line["ms_per_step"], rel=1e-3, abs=1e-3)
    assert [r["bit_exact"] for r in pr] == [True, corrupt_rank != 1]
    assert all(isinstance(r["kernels_ms"], dict) for r in pr)
    st = line["roofline_step"]
    assert st["tokens"] == sum(r["tokens"] for r in pr) and st["input_bytes"] == int(off[-1])
    assert st["alg_bytes_per_step"] == int(off[-1]) + 8 * st["tokens"]


def _bench_cmd(*extra):
    return [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "docs", "--corpus-mib", "0.75",
            "--nwords", "20000", "--steps", "3", "--warmup", "1", "--no-profile", "--no-e2e", "--no-latency",
            "--cpu1-sample-mib", "0", "--dict-kind", "txt", *extra]


def _bench_env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    tests = os.path.dirname(os.path.abspath(__file__))
    env.update(JB_BENCH_TEST_BACKEND="bench_backend:OracleBackend",
               PYTHONPATH=os.pathsep.join([tests, ROOT] + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else [])),
               **kw)
    return env


@pytest.mark.parametrize("corrupt_rank", [-1, 1])
def test_bench_launcher_two_ranks(corrupt_rank):
    """`python bench.py --gpus 2` with no WORLD_SIZE: bench.py starts the two ranks
    itself (child processes, gloo), each cuts its shard of the fixed corpus and
    checks it; one JSON line comes out, from rank 0, with n_gpus 2 and both
    ranks' parity in it.  The measured path is the oracle stand-in
    (tests/bench_backend.py), so this checks the launcher, not a GPU."""
    import json
    p = subprocess.run(_bench_cmd("--gpus", "2"), env=_bench_env(JB_TEST_CORRUPT_RANK=str(corrupt_rank)),
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["parity"]["ranks_checked"] == 2
    assert line["config"]["ranks"]["launcher"] == "bench.py" and line["config"]["ranks"]["processes"] == 2
    assert line["parity"]["bit_exact"] == (corrupt_rank < 0)
    assert line["parity"]["mismatches"] == (0 if corrupt_rank < 0 else 1)
    assert line["data"].startswith("TEST BACKEND")
    assert line["value"] > 0 and line["cpu_baseline"] is None
    pr = line["config"]["ranks"]["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1] and sum(r["shard_bytes"] for r in pr) == line["config"]["corpus_bytes"]
    assert [r["bit_exact"] for r in pr] == [True, corrupt_rank != 1]


def test_roofline_charges_the_output_format():
    """bench.roofline_of charges SURVEY.md §8d's bytes for the format the timed step
    writes: 1 B read per input byte + 8 B per u32 (start, end) span."""
    import bench
    nbytes, ntok, han = 1_000_000, 123_457, 700_002
    per = bench.alg_bytes_per_byte(nbytes, ntok)
    assert per == pytest.approx(1.0 + 8.0 * ntok / nbytes)
    kern = {"k_mark_walk": {"avg_ms": 2.0}, "k_zh": {"avg_ms": 1.0}}
    r = bench.roofline_of(kern, {"k_mark_walk": float(nbytes), "k_zh": float(han)}, lambda k: None, per)
    assert r["k_mark_walk"]["alg_bytes_per_launch"] == pytest.approx(nbytes + 8 * ntok)
    assert r["k_zh"]["alg_bytes_per_launch"] == pytest.approx(han * per)
    assert r["k_mark_walk"]["achieved"] == pytest.approx((nbytes + 8 * ntok) / 2e-3 / 1e9, abs=0.01)
    assert "spans" in r["k_mark_walk"]["output_format"]
    st = bench.roofline_step(nbytes, ntok, 0.5)
    assert st["alg_bytes_per_step"] == nbytes + 8 * ntok
    assert st["achieved"] == pytest.approx((nbytes + 8 * ntok) / 0.5e-3 / 1e9, abs=0.01)
    assert st["frac"] == pytest.approx(st["achieved"] / bench.HBM_PEAK_GBS, abs=1e-5)


def test_bench_launcher_refuses_missing_devices():
    """`--gpus 2` on a box with one GPU fails loudly instead of printing a 1-GPU line."""
    p = subprocess.run(_bench_cmd("--gpus", "2"), env=_bench_env(JB_TEST_DEVICES="1"),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode != 0 and "only 1 GPU" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_gpus_must_match_world_size():
    """Under torch.distributed.run (WORLD_SIZE set), a different --gpus is an error."""
    p = subprocess.run(_bench_cmd("--gpus", "4"),
                       env=_bench_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                      MASTER_PORT=str(_free_port())),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode != 0 and "disagrees with WORLD_SIZE=2" in p.stderr
