"""Dev helper: compare loudness / mix of one golden case between GPU and oracle."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd")]
from mastering_amd import Job, master_pcm, native  # noqa: E402
from oracle import mastering_oracle as mo  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "chunks_hot_31s"
d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
st = json.loads(str(d["settings"]))
rate = int(d["rate"])
out, info = master_pcm(d["pcm"], rate, st)
print("L gpu", info["loudness"], "L ref", float(d["loudness"]), "gain", info["gain_linear"], "iters", info["comp_iters"])
ref = d["out"]
print("exact", np.mean(out == ref), "maxdiff", np.abs(out.astype(int) - ref).max())
job = Job(d["pcm"].shape[0], rate, d["pcm"].shape[1] if d["pcm"].ndim == 2 else 1, st)
ctx = native.context(0)
import torch  # noqa: E402
x = torch.from_numpy(np.ascontiguousarray(d["pcm"].astype(np.float32) / 32768)).cuda()
ctx.check(ctx.lib.mm_stage_chunks(ctx.ptr, ctypes.byref(job.job), ctypes.c_void_p(x.data_ptr())), "stage")
mix = np.empty((job.frames_proc, 2), np.int16)
ctx.check(ctx.lib.mm_read_mix(ctx.ptr, mix.ctypes.data_as(ctypes.POINTER(ctypes.c_int16))), "read_mix")
thr, rat = mo.multiband_params(st)
refmix = []
pcm = d["pcm"]
for s, e in mo.chunk_ranges(pcm.shape[0], rate):
    c = pcm[s:min(e, pcm.shape[0])]
    y = mo.saturation(mo.pcm_to_float(c), st.get("saturation", 0))
    y = mo.equalize(y, rate, st)
    if st.get("width", 1.0) != 1.0:
        y = mo.stereo_width(y, st["width"])
    q = mo.quantize(y)
    if st.get("multiband"):
        q = mo.multiband(q, rate, thr, rat)
    refmix.append(q)
refmix = np.concatenate(refmix)
print("mix exact", np.mean(mix == refmix), "first diff frame", np.argmax(np.any(mix != refmix, axis=1)))
