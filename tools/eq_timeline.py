"""Per-block timeline of one eq launch from an MM_EQ_STAMPS build
(MM_EQ_STAMPS_DUMP=<file>): u64 per block {entry, ticket, pass 1 done, carry
done, end, HW_ID, -, -} in 100 MHz ticks.  Prints the spread of each phase, the
look-back wait and the last blocks to finish.
Usage: python tools/eq_timeline.py <dump>"""
import sys

import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8)
d = d[d[:, 0] > 0]
t0 = d[:, 0].min()
us = lambda x: (x.astype(np.float64) - float(t0)) / 100.0  # noqa: E731
entry, ticket, p1, carry, end = (us(d[:, k]) for k in range(5))
print(f"{len(d)} blocks; kernel span {end.max():.1f} us (first entry 0)")
for name, v in [("entry", entry), ("pass 1 end", p1), ("carry end", carry), ("end", end)]:
    print(f"  {name:11s} min {v.min():7.1f}  median {np.median(v):7.1f}  max {v.max():7.1f}")
w = carry - p1
print(f"  pass 1 {np.median(p1 - ticket):.1f} us median ({(p1 - ticket).min():.1f}-{(p1 - ticket).max():.1f}); "
      f"look-back wait {np.median(w):.1f} median ({w.min():.1f}-{w.max():.1f}); "
      f"pass 2 {np.median(end - carry):.1f} median ({(end - carry).min():.1f}-{(end - carry).max():.1f})")
order = np.argsort(-end)[:5]
print("  last blocks (ticket, entry, pass1 end, carry end, end):")
for i in order:
    print(f"    {i:4d} {entry[i]:7.1f} {p1[i]:7.1f} {carry[i]:7.1f} {end[i]:7.1f}")
