"""GPU diagnostic: a device-resident batch (mm_master_batch) of pink-noise tracks
against the oracle, per track: identical-sample fraction, RMS, solve statistics.
python tools/diag/batch_check.py [n_tracks] [seconds]   (MM_COMP_NOJUMP=1: jumps off)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mastering_amd import Job, master_batch, native  # noqa: E402
from mastering_amd.synth import pink_noise_pcm16  # noqa: E402
from oracle import mastering_oracle as mo  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
secs = int(sys.argv[2]) if len(sys.argv) > 2 else 180
rate = 44100
P = bench.P_FULL
pcms = [pink_noise_pcm16(secs * rate, rate, 2, 400 + t) for t in range(n)]
xs = [torch.from_numpy(p.astype(np.float32) / 32768).cuda() for p in pcms]
jobs = [Job(secs * rate, rate, 2, P) for _ in range(n)]
outs = [torch.empty((j.frames_proc, 2), dtype=torch.int16, device="cuda") for j in jobs]
res = master_batch(native.context(0), jobs, [x.data_ptr() for x in xs], [o.data_ptr() for o in outs])
for t in range(n):
    got = outs[t].cpu().numpy()
    ref = mo.master(pcms[t], rate, P)
    bad = np.flatnonzero((got != ref).any(axis=1))
    r = float(np.sqrt(np.mean(((got.astype(np.float64) - ref) / 32768) ** 2)))
    print(f"track {t}: exact={np.mean(got == ref):.7f} rms={r:.2e} n_bad={bad.size} first={bad[:4].tolist()} "
          f"iters={res[t].comp_iters} walked={res[t].comp_walked} jumped={res[t].comp_jumped}", flush=True)
