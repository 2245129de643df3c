"""conc_trace.py — summarise a JB_SMALL_TRACE file (one line per k_small batch: slot,
calls, and the host clocks in us of staging start, launch return, completion word, split
end) over the last SECONDS of the run: per-slot busy share, gaps between a slot's
batches, batch sizes, and how many batches were on the GPU at once.
Diagnostic tool, not part of the product.  usage: conc_trace.py TRACE [SECONDS]"""
import sys

import numpy as np

a = np.loadtxt(sys.argv[1], ndmin=2)
win = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 0.07e6
sel = a[a[:, 2] > a[:, 5].max() - win]
span = sel[:, 5].max() - sel[:, 2].min()
st, sy, sp = sel[:, 3] - sel[:, 2], sel[:, 4] - sel[:, 3], sel[:, 5] - sel[:, 4]
print(f"{sys.argv[1]}: {len(sel)} batches, {int(sel[:, 1].sum())} calls in {span:.0f} us "
      f"({sel[:, 1].sum() / span * 1e6:.0f} calls/s), mean batch {sel[:, 1].mean():.2f}")
for nm, x in (("stage+launch", st), ("sync", sy), ("split", sp)):
    print(f"  {nm:13s} med {np.median(x):6.1f} mean {x.mean():6.1f} p90 {np.percentile(x, 90):6.1f} us")
for k in range(int(a[:, 0].max()) + 1):
    s = sel[sel[:, 0] == k]
    if len(s) < 2:
        continue
    s = s[np.argsort(s[:, 2])]
    g = s[1:, 2] - s[:-1, 5]
    print(f"  slot {k}: {len(s)} batches, busy {(s[:, 5] - s[:, 2]).sum() / span:.2f}, "
          f"mean batch {s[:, 1].mean():.2f}, gap med {np.median(g):.1f} mean {g.mean():.1f} us")
ev = sorted([(x, 1) for x in sel[:, 3]] + [(x, -1) for x in sel[:, 4]])
c, last, hist = 0, ev[0][0], {}
for x, dlt in ev:
    hist[c] = hist.get(c, 0.0) + x - last
    c += dlt
    last = x
print("  batches on the GPU at once (share of time):", {k: round(v / span, 2) for k, v in sorted(hist.items())})
