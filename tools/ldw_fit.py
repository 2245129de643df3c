"""k_long_dp per-window chain clocks (STAMPS build, JB_LDW_OUT): a least-squares
fit of a window's cycles on its register-form groups (four runes with items of
lengths 1..m each), its class-1 runes (other fast forms, read from the ring in a
general group) and class-3 runes (item lists); the rest of the window's 64 groups
are general groups.  Diagnostic tool."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4).astype(np.float64)
a = a[a[:, 0] > 0]
cyc, nf, n1, n3 = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
ng = 64.0 - nf
X = np.stack([nf, ng, n1, n3], 1)
coef, *_ = np.linalg.lstsq(X, cyc, rcond=None)
pred = X @ coef
print(f"windows {len(a)}: cycles/window mean {cyc.mean():.0f} (per rune {cyc.mean() / 256:.1f}); register-form "
      f"groups {nf.mean():.1f}/64, class-1 runes {n1.mean():.2f}, class-3 runes {n3.mean():.2f} per window")
print(f"fit: per register-form group {coef[0]:.0f} cycles, per general group {coef[1]:.0f}, per class-1 rune "
      f"{coef[2]:.0f}, per class-3 rune {coef[3]:.0f}; residual rms {np.sqrt(np.mean((cyc - pred) ** 2)):.0f}")
