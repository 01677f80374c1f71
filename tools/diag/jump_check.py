"""GPU diagnostic: one track per parameter set through master_pcm against the CPU
oracle; prints the identical-sample fraction and the envelope solve's statistics.
python tools/diag/jump_check.py [seconds]   (MM_COMP_NOJUMP=1: release jumps off)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd")]
import bench  # noqa: E402
from mastering_amd import master_pcm  # noqa: E402
from mastering_amd.synth import pink_noise_pcm16  # noqa: E402
from oracle import mastering_oracle as mo  # noqa: E402

secs = int(sys.argv[1]) if len(sys.argv) > 1 else 60
rate = 44100
pcm = pink_noise_pcm16(secs * rate, rate, 2, track=0)
for name, params in (("full", bench.P_FULL), ("hot", bench.P_HOT)):
    t0 = time.time()
    ref = mo.master(pcm, rate, params)
    out, info = master_pcm(pcm, rate, params)
    same = out == ref
    bad = np.flatnonzero(~same.all(axis=1)) if out.ndim == 2 else np.flatnonzero(~same)
    print(f"{name}: exact={same.mean():.7f} first_bad={bad[:5].tolist()} n_bad_frames={bad.size} "
          f"iters={info['comp_iters']} walked={info['comp_walked']} jumped={info['comp_jumped']} "
          f"active={info['comp_active']} ({time.time() - t0:.1f}s)", flush=True)
