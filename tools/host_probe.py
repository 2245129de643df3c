"""Where the host-memory path's time goes (diagnostic, GPU box): PCIe copy rates
from pinned memory both ways (alone and at once), then jb_cut_batch_into on the
1 GiB C_syn corpus with the library's JB_DEBUG phase clocks.
usage: python tools/host_probe.py [--mib 1024]"""
import argparse
import os
import sys
import tempfile
import time

os.environ.setdefault("JB_DEBUG", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "gen", os.path.join("jieba-go_amd", "python")):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402


def pcie(torch, nbytes, reps=5):
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out[name] = nbytes * reps / (time.perf_counter() - t) / 1e9
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    out["both_each_way"] = nbytes * reps / (time.perf_counter() - t) / 1e9
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=1024)
    args = ap.parse_args()
    import torch
    import jiebahip as J
    import synth
    print("pcie GB/s (256 MiB pinned):", pcie(torch, 256 << 20), flush=True)
    tmp = tempfile.mkdtemp()
    s = synth.Synth(nwords=350_000)
    dp, ep = s.write_files(tmp)
    tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep, kind=J.JB_DICT_PREFIX, size_override=J.JIEBA_SIZE))
    buf, off, _ = s.corpus_parallel(synth.KIND_DOCS, 0, target_bytes=int(args.mib * (1 << 20)), threads=16)
    nchars = int(np.count_nonzero((np.asarray(buf[: int(off[-1])]) & 0xC0) != 0x80))
    res = tk.cut_batch_into(buf, off, True)
    for r in range(4):
        t = time.perf_counter()
        res = tk.cut_batch_into(buf, off, True, res[3])
        dt = time.perf_counter() - t
        print(f"cut_batch_into rep {r}: {dt * 1e3:.2f} ms, {nchars / dt / 1e9:.2f} G chars/s", flush=True)
    r32 = tk.cut_batch_into32(buf, off, True)
    for r in range(4):
        t = time.perf_counter()
        r32 = tk.cut_batch_into32(buf, off, True, r32[3])
        dt = time.perf_counter() - t
        print(f"cut_batch_into32 rep {r}: {dt * 1e3:.2f} ms, {nchars / dt / 1e9:.2f} G chars/s", flush=True)
    del r32
    if hasattr(tk, "cut_batch_mask"):
        m = tk.cut_batch_mask(buf, off, True)
        for r in range(4):
            t = time.perf_counter()
            m = tk.cut_batch_mask(buf, off, True, m)
            dt = time.perf_counter() - t
            print(f"cut_batch_mask rep {r}: {dt * 1e3:.2f} ms, {nchars / dt / 1e9:.2f} G chars/s", flush=True)
        hb = J.HostBuffer(len(buf))
        hb.array[:] = buf
        m = tk.cut_batch_mask(hb.array, off, True, m)
        for r in range(3):
            t = time.perf_counter()
            m = tk.cut_batch_mask(hb.array, off, True, m)
            dt = time.perf_counter() - t
            print(f"cut_batch_mask pinned rep {r}: {dt * 1e3:.2f} ms, {nchars / dt / 1e9:.2f} G chars/s", flush=True)
        hb.free()
    # per-kernel times: the host path (one call, masks) against the device-resident path on the same batch
    import torch
    nb = int(off[-1])
    tk.profile(True)
    tk.profile_reset()
    tk.cut_batch_mask(buf, off, True, m)
    host_k = tk.profile_read()
    tk.profile_reset()
    d_text = torch.from_numpy(np.asarray(buf[: nb + 64])).cuda()
    d_off = torch.from_numpy(np.asarray(off, np.int64)).cuda()
    for _ in range(2):
        tk.cut_device(d_text.data_ptr(), nb, d_off.data_ptr(), len(off) - 1, True, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    dev_k = tk.profile_read()
    for k in host_k:
        if host_k[k][1] or dev_k[k][1]:
            print(f"  {k:14s} host path {host_k[k][0]:8.3f} ms / {host_k[k][1]} launches   device path "
                  f"{dev_k[k][0] / max(1, dev_k[k][1]) * (host_k[k][1] and 1):8.3f} ms per launch", flush=True)
    tk.close()


if __name__ == "__main__":
    main()
