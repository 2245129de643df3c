"""GPU: BASELINE config 4 at its full size, the multi-device host path and
concurrent device-resident callers — each against the oracle, bit-exact, through
the C ABI.  Every test here needs the GPU."""
import os
import threading

import numpy as np
import pytest

import jiebahip as J
import oracle as O
import synth

pytestmark = pytest.mark.gpu


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _cmp(gs, ge, gd, os_, oe, od, label):
    if not (len(gs) == len(os_) and np.array_equal(gs, os_) and np.array_equal(ge, oe)):
        n = min(len(gs), len(os_))
        bad = int(np.argmax((gs[:n] != os_[:n]) | (ge[:n] != oe[:n]))) if n else 0
        raise AssertionError(f"{label}: {len(gs)} vs {len(os_)} tokens, first difference at token {bad}")
    assert np.array_equal(gd, od), label


def _device_cut(tk, buf, off, hmm):
    """The bench's measured path (bench.GpuCutter): input resident in HBM,
    jb_cut_device on the current stream, results copied back afterwards."""
    import torch
    nbytes, nd = int(off[-1]), len(off) - 1
    d_text = torch.from_numpy(np.ascontiguousarray(buf[: nbytes + 64])).cuda()
    d_off = torch.from_numpy(np.asarray(off, np.int64)).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    ps, pe, pd, pn = tk.cut_device(d_text.data_ptr(), nbytes, d_off.data_ptr(), nd, hmm, stream)
    torch.cuda.synchronize()
    n = int(J.dev_to_host(pn, 8, np.uint64)[0])
    out = (J.dev_to_host(ps, 4 * n, np.uint32).astype(np.uint64), J.dev_to_host(pe, 4 * n, np.uint32).astype(np.uint64),
           J.dev_to_host(pd, 8 * (nd + 1), np.uint64))
    del d_text, d_off
    return out


def test_config4_full_corpus(syn_full):
    """BASELINE config 4 at the size its metric is quoted on: the 1 GiB C_syn corpus
    (the bench's workload, 73k documents), cut on the device as bench.py times it,
    every token against the oracle (tokenizer_test.go:16-26 cut big texts the same
    way).  A 1M-rune unpunctuated document with 30 % OOV runes (config 5b) rides at
    the end of the batch, so the long-block kernels run in the same pipeline."""
    dp, ep, s = syn_full
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus_parallel(synth.KIND_DOCS, 0, target_bytes=1 << 30, threads=_threads())
    lbuf, loff, _ = s.corpus(synth.KIND_LONG_OOV, 5, target_runes=1_000_000)
    n0, nl = int(off[-1]), int(loff[-1])
    big = np.zeros(n0 + nl + 64, np.uint8)
    big[:n0] = buf[:n0]
    big[n0:n0 + nl] = lbuf[:nl]
    del buf
    boff = np.concatenate([np.asarray(off, np.uint64), np.asarray(loff[1:], np.uint64) + np.uint64(n0)])
    assert n0 >= (1 << 30) - (1 << 20) and len(boff) - 1 > 70_000
    O.set_viterbi_backptr(True)  # same decisions as path copying (test_oracle_kats), O(m) on the long run
    try:
        for hmm in (True, False):
            gs, ge, gd = _device_cut(tk, big, boff, hmm)
            st = tk.last_stats()
            if hmm:
                assert st["long_blocks"] >= 1, st  # the 1M-rune document's Han runs
            os_, oe, od = o.cut_batch(big, boff, hmm, nthreads=_threads())
            _cmp(gs, ge, gd, os_, oe, od, f"config 4 (1 GiB) + 5b, hmm={hmm}")
            assert st["tokens"] == len(os_)
            del gs, ge, gd, os_, oe, od
    finally:
        O.set_viterbi_backptr(False)
    tk.close()


@pytest.mark.parametrize("ndev", [2, 3])
def test_multi_device_host_path(syn_small, ndev, monkeypatch):
    """jb_cut_batch over several devices: byte-balanced document ranges, one host
    thread, stream and workspace per device, spans concatenated in document order
    (SURVEY.md §8e).  JB_DEVICE_WRAP maps the devices onto the one GPU here."""
    dp, ep, s = syn_small
    monkeypatch.setenv("JB_DEVICE_WRAP", "1")
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, ndevices=ndev))
    monkeypatch.delenv("JB_DEVICE_WRAP")
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus(synth.KIND_DOCS, 40 + ndev, target_bytes=6 << 20)
    for hmm in (False, True):
        gs, ge, gd = tk.cut_batch(buf, off, hmm)
        os_, oe, od = o.cut_batch(buf, off, hmm, nthreads=8)
        _cmp(gs, ge, gd, os_, oe, od, f"{ndev} devices hmm={hmm}")
        assert tk.last_stats()["tokens"] == len(os_)  # summed over the devices
        s2, e2, d2, _ = tk.cut_batch_into(buf, off, hmm)
        _cmp(s2, e2, d2, os_, oe, od, f"{ndev} devices into caller arrays hmm={hmm}")
    # a batch smaller than the device count, and one tiny batch (k_small on one device)
    few = off[:2]
    gs, ge, gd = tk.cut_batch(buf, few, True)
    os_, oe, od = o.cut_batch(buf, few, True)
    _cmp(gs, ge, gd, os_, oe, od, "one document over several devices")
    t = "我昨天去上海交通大學與老師討論量子力學"
    assert tk.Cut(t, True) == o.cut(t, True)
    st = tk.last_stats()
    assert st["tokens"] == len(o.cut(t, True))  # no stale counts from the devices that got nothing
    tk.close()


def test_cut_device_into_concurrent_threads(syn_small):
    """jb_cut_device_into from two threads on two streams at once, each with its
    own output arrays: the shared workspace is ordered on the device, and neither
    thread sees the other's tokens."""
    import torch
    dp, ep, s = syn_small
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
    o = O.Oracle.from_files(dp, ep, 0)
    batches = [s.corpus(synth.KIND_DOCS, 60 + k, target_bytes=(3 + k) << 20)[:2] for k in range(2)]
    want = [o.cut_batch(b, f, True, nthreads=8) for b, f in batches]
    errs = []

    def run(k):
        try:
            buf, off = batches[k]
            nbytes, nd = int(off[-1]), len(off) - 1
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                d_text = torch.from_numpy(np.ascontiguousarray(buf[: nbytes + 64])).cuda()
                d_off = torch.from_numpy(np.asarray(off, np.int64)).cuda()
                o_s = torch.empty(nbytes + 1, dtype=torch.int32, device="cuda")
                o_e = torch.empty(nbytes + 1, dtype=torch.int32, device="cuda")
                o_d = torch.empty(nd + 1, dtype=torch.int64, device="cuda")
                o_n = torch.zeros(1, dtype=torch.int64, device="cuda")
                for rep in range(6):
                    o_s.fill_(-1)
                    tk.cut_device_into(d_text.data_ptr(), nbytes, d_off.data_ptr(), nd, True, o_s.data_ptr(),
                                       o_e.data_ptr(), nbytes + 1, o_d.data_ptr(), o_n.data_ptr(), st.cuda_stream)
                    st.synchronize()
                    n = int(o_n.item())
                    got = (o_s[:n].cpu().numpy().view(np.uint32).astype(np.uint64),
                           o_e[:n].cpu().numpy().view(np.uint32).astype(np.uint64), o_d.cpu().numpy().view(np.uint64))
                    _cmp(*got, *want[k], f"thread {k} rep {rep}")
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    with pytest.raises(J.JbError) as e:  # outputs must hold a token per byte
        tk.cut_device_into(0, 100, 0, 1, True, 1, 1, 99, 1, 1)
    assert e.value.code == J.JB_EINVAL
    tk.close()


def _mask_spans(tk, buf, off, hmm):
    ms, me, n = tk.cut_batch_mask(buf, off, hmm)
    base = int(off[0])
    s, e = J.mask_to_spans(ms, me, int(off[-1]) - base, base)
    assert len(s) == len(e) == n
    return s, e


@pytest.mark.parametrize("piece_kib", [256, 65536])
def test_host_pipeline_pieces_and_masks(syn_small, piece_kib, monkeypatch):
    """Host batches cut in pieces of whole documents, pipelined over three streams
    (JB_PIECE_KIB; 256 KiB makes dozens of pieces here, and the 1M-rune document one
    piece of its own): spans, caller arrays, boundary masks (jb_cut_batch_mask),
    pinned input (jb_host_alloc) and the summed counters all equal the oracle's."""
    dp, ep, s = syn_small
    monkeypatch.setenv("JB_PIECE_KIB", str(piece_kib))
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
    monkeypatch.delenv("JB_PIECE_KIB")
    ref = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus(synth.KIND_DOCS, 70, target_bytes=5 << 20)
    lbuf, loff, _ = s.corpus(synth.KIND_LONG_PUNCT, 71, target_runes=1_000_000)
    n0, nl = int(off[-1]), int(loff[-1])
    big = np.zeros(n0 + nl + 64, np.uint8)
    big[:n0], big[n0:n0 + nl] = buf[:n0], lbuf[:nl]
    boff = np.concatenate([np.asarray(off, np.uint64), np.asarray(loff[1:], np.uint64) + np.uint64(n0)])
    for hmm in (False, True):
        os_, oe, od = o.cut_batch(big, boff, hmm, nthreads=8)
        gs, ge, gd = tk.cut_batch(big, boff, hmm)
        _cmp(gs, ge, gd, os_, oe, od, f"pieces of {piece_kib} KiB, hmm={hmm}")
        st = tk.last_stats()
        ref.cut_batch(big, boff, hmm)
        rst = ref.last_stats()
        assert st["tokens"] == len(os_) and st["blocks"] == rst["blocks"] and st["zh_blocks"] == rst["zh_blocks"], \
            (st, rst)
        s2, e2, d2, _ = tk.cut_batch_into(big, boff, hmm)
        _cmp(s2, e2, d2, os_, oe, od, f"into, pieces of {piece_kib} KiB")
        ms, me = _mask_spans(tk, big, boff, hmm)
        _cmp(ms, me, od, os_, oe, od, f"masks, pieces of {piece_kib} KiB, hmm={hmm}")
        assert tk.last_stats()["tokens"] == len(os_)
    # a batch that starts inside the buffer (mask bit 0 = byte doc_off[0]), and documents
    # of it from pinned memory
    sub = boff[5:400]
    os_, oe, od = o.cut_batch(big, sub, True)
    ms, me = _mask_spans(tk, big, sub, True)
    _cmp(ms, me, od, os_, oe, od, "masks of a batch at an offset")
    hb = J.HostBuffer(len(big))
    try:
        hb.array[:] = big
        gs, ge, gd = tk.cut_batch(hb.array, boff, True)
        os_, oe, od = o.cut_batch(big, boff, True, nthreads=8)
        _cmp(gs, ge, gd, os_, oe, od, "pinned input")
        ms, me = _mask_spans(tk, hb.array, boff, True)
        _cmp(ms, me, od, os_, oe, od, "masks from pinned input")
    finally:
        hb.free()
    # tiny batches (k_small) and empty ones
    for t in ("", "中文", "我昨天去上海交通大學與老師討論量子力學", "abc 中文 x"):
        b = np.frombuffer(t.encode() + b"\0" * 16, np.uint8)
        f = np.array([0, len(t.encode())], np.uint64)
        ms, me = _mask_spans(tk, b, f, True)
        os_, oe = o.cut_spans(t.encode(), True)
        assert ms.tolist() == os_.tolist() and me.tolist() == oe.tolist(), t
    rc = J.lib().jb_cut_batch_mask(tk.h, big.ctypes.data, boff.ctypes.data, len(boff) - 1, 1, None, None, 3,
                                   J.C.byref(J.C.c_uint64()))
    assert rc == J.JB_EINVAL  # 3 words cannot hold the batch
    # caller arrays longer than the batch (reused after a larger one): every word is
    # written, the tail past the batch as zeros, so a popcount counts the batch's tokens
    nw = (int(boff[-1]) + 63) // 64
    ws = np.full(nw, ~np.uint64(0), np.uint64)
    we = np.full(nw, ~np.uint64(0), np.uint64)
    small_off = boff[:40]
    os_, oe, od = o.cut_batch(big, small_off, True)
    n = J.C.c_uint64()
    J._check(J.lib().jb_cut_batch_mask(tk.h, big.ctypes.data, small_off.ctypes.data, len(small_off) - 1, 1,
                                       ws.ctypes.data, we.ctypes.data, nw, J.C.byref(n)))
    need = (int(small_off[-1]) + 63) // 64
    assert n.value == len(os_) and not ws[need:].any() and not we[need:].any()
    pop = lambda a: int(np.unpackbits(a.view(np.uint8)).sum())  # noqa: E731
    assert pop(ws) == pop(we) == len(os_)
    ms, me, nt = tk.cut_batch_mask(big, small_off, True, (ws, we))
    assert len(ms) == need and nt == len(os_)
    tk.close()
    ref.close()


@pytest.mark.parametrize("ndev", [2, 3])
def test_multi_device_masks(syn_small, ndev, monkeypatch):
    """Boundary masks over several devices: the words two device ranges share are
    ORed together, the others written once."""
    dp, ep, s = syn_small
    monkeypatch.setenv("JB_DEVICE_WRAP", "1")
    monkeypatch.setenv("JB_PIECE_KIB", "512")
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, ndevices=ndev))
    monkeypatch.delenv("JB_DEVICE_WRAP")
    monkeypatch.delenv("JB_PIECE_KIB")
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus(synth.KIND_DOCS, 80 + ndev, target_bytes=4 << 20)
    for hmm in (False, True):
        os_, oe, od = o.cut_batch(buf, off, hmm, nthreads=8)
        ms, me = _mask_spans(tk, buf, off, hmm)
        _cmp(ms, me, od, os_, oe, od, f"masks over {ndev} devices, hmm={hmm}")
    tk.close()


@pytest.mark.parametrize("ndev,piece_kib", [(1, 1024), (2, 65536), (4, 512)])
def test_one_large_document_split(syn_small, ndev, piece_kib, monkeypatch):
    """One 1M-rune document (config 5a, ~3 MB) cut as several units at Han-run starts
    (jb_split_points): over devices (JB_DEVICE_WRAP) and over pipeline pieces within a
    device (JB_PIECE_KIB smaller than the document).  Spans, doc_tok, masks and the
    counters equal the oracle's on the whole document."""
    dp, ep, s = syn_small
    monkeypatch.setenv("JB_DEVICE_WRAP", "1")
    monkeypatch.setenv("JB_PIECE_KIB", str(piece_kib))
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, ndevices=ndev))
    monkeypatch.delenv("JB_DEVICE_WRAP")
    monkeypatch.delenv("JB_PIECE_KIB")
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off, _ = s.corpus(synth.KIND_LONG_PUNCT, 90 + ndev, target_runes=1_000_000)
    # the document alone, and between two short ones
    pre = "短句。".encode()
    b2 = np.frombuffer(pre + bytes(buf[: int(off[-1])]) + pre + b"\0" * 64, np.uint8)
    off2 = np.array([0, len(pre), len(pre) + int(off[-1]), 2 * len(pre) + int(off[-1])], np.uint64)
    for bb, ff in ((buf, off), (b2, off2)):
        for hmm in (False, True):
            os_, oe, od = o.cut_batch(bb, ff, hmm)
            gs, ge, gd = tk.cut_batch(bb, ff, hmm)
            _cmp(gs, ge, gd, os_, oe, od, f"1M runes over {ndev} devices / {piece_kib} KiB pieces, hmm={hmm}")
            assert tk.last_stats()["tokens"] == len(os_)
            s2, e2, d2, _ = tk.cut_batch_into(bb, ff, hmm)
            _cmp(s2, e2, d2, os_, oe, od, "into")
            ms, me = _mask_spans(tk, bb, ff, hmm)
            _cmp(ms, me, od, os_, oe, od, "masks")
    tk.close()


def test_cut_device_into_unaligned_outputs(syn_small):
    """Caller span arrays that are not 16-byte aligned: k_tok's write pass then stores
    one span per lane instead of four (its 16-byte stores need aligned outputs)."""
    import torch
    dp, ep, s = syn_small
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
    o = O.Oracle.from_files(dp, ep, 0)
    buf, off = s.corpus(synth.KIND_DOCS, 65, target_bytes=2 << 20)[:2]
    want = o.cut_batch(buf, off, True, nthreads=8)
    nbytes, nd = int(off[-1]), len(off) - 1
    d_text = torch.from_numpy(np.ascontiguousarray(buf[: nbytes + 64])).cuda()
    d_off = torch.from_numpy(np.asarray(off, np.int64)).cuda()
    o_s = torch.full((nbytes + 8,), -1, dtype=torch.int32, device="cuda")
    o_e = torch.full((nbytes + 8,), -1, dtype=torch.int32, device="cuda")
    o_d = torch.empty(nd + 1, dtype=torch.int64, device="cuda")
    o_n = torch.zeros(1, dtype=torch.int64, device="cuda")
    for sh in (1, 2, 3):  # 4, 8, 12 bytes past a 16-byte boundary
        o_s.fill_(-1)
        o_e.fill_(-1)
        tk.cut_device_into(d_text.data_ptr(), nbytes, d_off.data_ptr(), nd, True, o_s.data_ptr() + 4 * sh,
                           o_e.data_ptr() + 4 * sh, nbytes + 1, o_d.data_ptr(), o_n.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        n = int(o_n.item())
        got = (o_s[sh:sh + n].cpu().numpy().view(np.uint32).astype(np.uint64),
               o_e[sh:sh + n].cpu().numpy().view(np.uint32).astype(np.uint64), o_d.cpu().numpy().view(np.uint64))
        _cmp(*got, *want, f"outputs {4 * sh} bytes past alignment")
        assert int(o_s[sh - 1].item()) == -1 and int(o_s[sh + n].item()) == -1  # nothing written outside
    tk.close()


def test_bench_two_ranks_on_the_gpu(tmp_path):
    """`bench.py --gpus 2` end to end on the GPU: the launcher starts two ranks
    (JB_BENCH_SHARE_GPU puts both on GPU 0 of a one-GPU box, testing only), each cuts
    its byte-balanced shard of the corpus through the C ABI and checks every token
    against the oracle, and rank 0 prints one line with the job's aggregate
    (the driver's N-GPU scaling run takes the same path with one GPU per rank)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, JB_BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--corpus-mib", "32",
                        "--steps", "2", "--warmup", "1", "--no-e2e", "--no-latency", "--no-profile",
                        "--cpu1-sample-mib", "0"], capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["ranks"]["processes"] == 2
    assert line["parity"]["bit_exact"] and line["parity"]["ranks_checked"] == 2, line["parity"]
    assert "JB_BENCH_SHARE_GPU" in line["data"]
    assert line["value"] > 0
