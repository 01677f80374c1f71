"""Where do the remaining output differences come from?  For a few configurations:
the pre-gain mix against the oracle's, the loudness against the oracle's, and the
final output (diagnostic, GPU)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd")]

from mastering_amd import Job, master_batch, master_pcm, native  # noqa: E402
from mastering_amd.synth import pink_noise_pcm16  # noqa: E402
from oracle import mastering_oracle as mo  # noqa: E402

mo.build()
P_FULL = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
          "saturation": 30, "width": 1.3, "multiband": True, "lufs": -14.0}
P_HOT = dict(P_FULL, low_thresh=-16.0, mid_thresh=-21.0, high_thresh=-27.0)


def staged_mix(pcm, rate, params):
    import torch
    job = Job(pcm.shape[0], rate, 2, params)
    ctx = native.context(0)
    d_in = torch.from_numpy(np.ascontiguousarray(pcm.astype(np.float32) / 32768)).cuda()
    ctx.check(ctx.lib.mm_stage_chunks(ctx.ptr, ctypes.byref(job.job), ctypes.c_void_p(d_in.data_ptr())), "stage")
    mix = np.empty((job.frames_proc, 2), np.int16)
    ctx.check(ctx.lib.mm_read_mix(ctx.ptr, mix.ctypes.data_as(ctypes.POINTER(ctypes.c_int16))), "read_mix")
    return mix


def oracle_mix(pcm, rate, params):
    thr, rat = mo.multiband_params(params)
    ref = []
    for s, e in mo.chunk_ranges(pcm.shape[0], rate):
        x = mo.saturation(mo.pcm_to_float(pcm[s:e]), params.get("saturation", 0))
        y = mo.quantize(mo.stereo_width(mo.equalize(x, rate, params), params.get("width", 1.0)))
        ref.append(mo.multiband(y, rate, thr, rat) if params.get("multiband") else y)
    return np.concatenate(ref)


def one(name, pcm, rate, params):
    mix, rmix = staged_mix(pcm, rate, params), oracle_mix(pcm, rate, params)
    nm = min(len(mix), len(rmix))
    mix, rmix = mix[:nm], rmix[:nm]
    out, info = master_pcm(pcm, rate, params)
    ref, L = mo.master(pcm, rate, params, return_loudness=True)
    print(f"{name}: mix exact {np.mean(mix == rmix):.7f}  dL {info['loudness'] - L:+.3e} (L {L:.12f})  "
          f"out exact {np.mean(out == ref):.7f}", flush=True)


one("44056 hot 40s", pink_noise_pcm16(40 * 44056, 44056, 2, 21), 44056, P_HOT)
one("44100 full 4.1s", pink_noise_pcm16(int(4.1 * 44100), 44100, 2, 700), 44100, P_FULL)
one("44100 hot 3.3s", pink_noise_pcm16(int(3.3 * 44100), 44100, 2, 703), 44100, P_HOT)
one("44100 full 1.5s", pink_noise_pcm16(int(1.5 * 44100), 44100, 2, 705), 44100, P_FULL)
