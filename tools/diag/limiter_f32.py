"""Diagnostic: where the f32 soft limiter differs from numpy (prints a few cases)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd")]
from mastering_amd import ops  # noqa: E402

d = np.load(os.path.join(ROOT, "tests", "golden", "primitives.npz"))
x = d["prim_lim_in"].astype(np.float32)
ref = d["prim_lim_out_f32"]
y = ops.soft_limiter(x.copy())
bad = np.flatnonzero(y != ref)
print("mismatches", bad.size, "of", x.size)
for i in bad[:10]:
    a = np.abs(x[i]); dd = a - np.float32(0.98); t = dd / np.float32(0.02)
    den = np.sqrt(np.float32(1) + t * t)
    print(i, repr(x[i]), "gpu", repr(y[i]), "ref", repr(ref[i]), "d", repr(dd), "t", repr(t), "den", repr(den),
          "q", repr(dd / den))
