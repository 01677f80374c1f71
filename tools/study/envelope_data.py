"""Raw per-(chunk, band) compacted M sequences for tools/study/envelope_model.c:
python tools/study/coalesce_data.py full 300 && python tools/study/envelope_data.py full
-> /tmp/study/<which>.idx (path band frames attack release per line) + .bin files."""
import os
import sys

import numpy as np

which = sys.argv[1] if len(sys.argv) > 1 else "full"
d = np.load(f"/tmp/coalesce_{which}.npz")
os.makedirs("/tmp/study", exist_ok=True)
with open(f"/tmp/study/{which}.idx", "w") as f:
    for k in sorted(d.files):
        if k.startswith("c"):
            b = int(k.split("_b")[1])
            d[k].astype(np.float64).tofile(f"/tmp/study/{which}_{k}.bin")
            f.write(f"/tmp/study/{which}_{k}.bin {b} {len(d[k])} {float(d[f'A_b{b}'])!r} {float(d[f'R_b{b}'])!r}\n")
