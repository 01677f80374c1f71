"""Dump the compacted per-(chunk, band) M sequences of a bench track (for
tools/study/coalesce.c).  python tools/study/coalesce_data.py [full|hot] [seconds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "python-audio-mastering_amd"))
import bench  # noqa: E402
from mastering_amd import design  # noqa: E402
from mastering_amd.synth import pink_noise_pcm16  # noqa: E402
from oracle import mastering_oracle as mo  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "full"
secs = int(sys.argv[2]) if len(sys.argv) > 2 else 120
st = bench.P_HOT if which == "hot" else bench.P_FULL
rate = 44100
pcm = pink_noise_pcm16(secs * rate, rate, 2, track=0)
thr, rat = mo.multiband_params(st)
out = {}
for ci, (s, e) in enumerate(mo.chunk_ranges(pcm.shape[0], rate)):
    c = pcm[s:min(e, pcm.shape[0])]
    x = mo.pcm_to_float(c)
    x = mo.saturation(x, st.get("saturation", 0))
    x = mo.equalize(x, rate, st)
    x = mo.stereo_width(x, st["width"])
    q = mo.quantize(x)
    for b, (band, t, r, (at, rel)) in enumerate(zip(mo.band_split(q, rate), thr, rat, mo.BAND_TIMES)):
        bc = design.band_constants(rate, t, r, at, rel)
        look = bc["look"]
        e2 = (band.astype(np.int64) ** 2).sum(axis=1)
        cs = np.concatenate([[0], np.cumsum(e2)])
        i = np.arange(band.shape[0])
        lo = np.maximum(i - look, 0)
        S = cs[i] - cs[lo]
        n = (i - lo) * 2
        rms = np.zeros(band.shape[0], np.int64)
        nz = n > 0
        rms[nz] = np.floor(np.sqrt(S[nz] / n[nz])).astype(np.int64)
        M = bc["table"][np.minimum(rms, 32768)]
        M = M[M != 0]
        out[f"c{ci}_b{b}"] = M
        out[f"A_b{b}"] = np.float64(bc["attack_frames"])
        out[f"R_b{b}"] = np.float64(bc["release_frames"])
np.savez(f"/tmp/coalesce_{which}.npz", **out)
print({k: v.shape for k, v in out.items() if k.startswith("c")})
