"""Per-walker cost model of the fix-up sweeps from a MM_FIX_TRACE_DUMP file:
least squares of a walker's time (10 ns ticks) on its walked tiles, jumped tiles
and visited super-tiles, per sweep.  Usage: python tools/fix_fit.py <dump>"""
import sys

import numpy as np

tr = np.fromfile(sys.argv[1], dtype=np.uint32)
gs = tr.size // (16 * 3 * 4)
tr = tr.reshape(16, 3, gs, 4)
for k in range(16):
    r = tr[k].reshape(-1, 4).astype(np.float64)
    live = (r[:, 0] > 0) | (r[:, 3] > 0)
    if not live.any():
        continue
    r = r[live]
    t_us = r[:, 0] / 100.0
    X = np.column_stack([r[:, 1], r[:, 2], r[:, 3], np.ones(len(r))])
    coef, *_ = np.linalg.lstsq(X, t_us, rcond=None)
    print(f"sweep {k}: {len(r)} walkers, max {t_us.max():.1f} us, walked {int(r[:, 1].sum())} jumped {int(r[:, 2].sum())} "
          f"visited {int(r[:, 3].sum())}; fit us = {coef[0]:.3f}*walked + {coef[1]:.3f}*jumped + {coef[2]:.3f}*visited + "
          f"{coef[3]:.2f}")
    top = np.argsort(-t_us)[:6]
    print("   longest walkers (us, walked, jumped, visited):",
          "; ".join(f"{t_us[i]:.1f} {int(r[i, 1])} {int(r[i, 2])} {int(r[i, 3])}" for i in top))
    one = (r[:, 3] == 1) & (r[:, 1] == 0) & (r[:, 2] == 0)
    if one.any():
        print(f"   walkers that stop at once (coalesced on entry): {int(one.sum())}, median {np.median(t_us[one]):.1f} us, "
              f"max {t_us[one].max():.1f} us")
