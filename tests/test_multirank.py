"""CPU, world_size 2 over gloo: the multi-GPU path's sharding and job-level
aggregation (bench.py's max-over-ranks time, summed work), with the oracle
standing in for each rank's device."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, dict_path, emit_path, buf, off, out_dir):
    import torch
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sub, soff, d0, base = shard.shard_of(buf, off, world, rank)
    o = O.Oracle.from_files(dict_path, emit_path, 0)
    s, e, dt = o.cut_batch(sub, soff, True)
    parts = [None] * world
    dist.all_gather_object(parts, (s, e, dt, base))
    # job-level aggregates as bench.py computes them
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    w = torch.tensor([float(len(sub) - 16)], dtype=torch.float64)
    dist.all_reduce(w, op=dist.ReduceOp.SUM)
    if rank == 0:
        S, E, DT = shard.merge(parts)
        np.savez(os.path.join(out_dir, "merged.npz"), s=S, e=E, dt=DT, tmax=t.item(), wsum=w.item())
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


def test_two_ranks_gloo_equals_single_process(syn_small):
    import oracle as O
    import synth
    dp, ep, s = syn_small
    buf, off, nr = s.corpus(synth.KIND_DOCS, 40, target_bytes=300_000)
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(2, _free_port(), dp, ep, buf, off, out), nprocs=2, join=True,
                           start_method="spawn")
        m = np.load(os.path.join(out, "merged.npz"))
        o = O.Oracle.from_files(dp, ep, 0)
        s1, e1, d1 = o.cut_batch(buf, off, True)
        assert np.array_equal(m["s"], s1) and np.array_equal(m["e"], e1) and np.array_equal(m["dt"], d1)
        assert m["tmax"] == 2.0 and m["wsum"] == float(off[-1])
