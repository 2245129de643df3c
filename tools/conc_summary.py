"""Summarise JB_DEBUG's k_small batch lines: batch sizes, host stage+launch and sync times."""
import re
import sys

import numpy as np

for path in sys.argv[1:]:
    rows = []
    for ln in open(path):
        m = re.match(r"\[jb\] k_small (\d+) bytes, (\d+) calls: stage\+launch ([\d.]+) us, sync ([\d.]+) us; phases \(us\): ([\d. ]+);", ln)
        if m and len(m.group(5).split()) == 15:
            ph = [float(x.rstrip(";")) for x in m.group(5).split()]
            rows.append([int(m.group(1)), int(m.group(2)), float(m.group(3)), float(m.group(4)), ph[10]])  # clk[11]: kernel end
    if not rows:
        print(path, "no batch lines")
        continue
    a = np.array(rows)
    big = a[a[:, 1] > 1]
    print(f"{path}: {len(a)} batches; calls/batch mean {a[:,1].mean():.2f} max {a[:,1].max():.0f}; "
          f"bytes mean {a[:,0].mean():.0f}; stage+launch us mean {a[:,2].mean():.1f}; sync us mean {a[:,3].mean():.1f} "
          f"p90 {np.percentile(a[:,3],90):.1f}; kernel us (first to last clock) mean {a[:,4].mean():.1f}")
    for n in (1, 2, 4, 8, 16):
        s = a[(a[:, 1] >= n) & (a[:, 1] < 2 * n)]
        if len(s):
            print(f"   calls {n}-{2*n-1}: {len(s)} batches, bytes {s[:,0].mean():.0f}, sync {s[:,3].mean():.1f} us, "
                  f"kernel {s[:,4].mean():.1f} us")
