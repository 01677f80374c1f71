"""TEST INFRASTRUCTURE ONLY — CPU oracle of the reference's legacy engine
(root main.py:46-192), the checker of mastering_amd/legacy.py.

Restates main.py's chunked chain with numpy/scipy (the same dtype flow: f32
samples, f64 out of every sosfilt, numpy's weak-scalar rules) and the pydub
compressor loop in C (oracle/compressor_oracle.c via mastering_oracle).  Pinned
bit for bit to tests/golden/legacy_*.npz, which tests/golden/make_golden_legacy.py
produced by running main.py itself (tests/test_legacy.py).  Never imported by
the product package.
"""
from __future__ import annotations

import numpy as np
import scipy.signal

from . import mastering_oracle as mo


def saturation(x, amount):  # main.py:94-97
    if amount == 0:
        return x
    gain = 1.0 + (amount / 100.0) * 4.0
    return np.tanh(x * gain) / gain


def shelf(x, rate, cutoff, gain_db, kind, order=5):  # main.py:133-143
    if gain_db == 0:
        return x
    sos = scipy.signal.butter(order, cutoff / (0.5 * rate), btype=kind, analog=False, output="sos")
    f = scipy.signal.sosfilt(sos, x)
    g = 10 ** (gain_db / 20.0)
    return x + (f * (g - 1)) if gain_db > 0 else x * g + (f * (1 - g))


def peak(x, rate, center, gain_db, q=1.0):  # main.py:145-154
    if gain_db == 0:
        return x
    c = center / (0.5 * rate)
    e1, e2 = c / np.sqrt(q), c * np.sqrt(q)
    lo, hi = min(e1, e2), max(e1, e2)
    if lo >= hi:
        hi = lo + 1e-9
    if hi >= 1.0:
        hi = 0.999999
    sos = scipy.signal.butter(2, [lo, hi], btype="bandpass", output="sos")
    return x + (scipy.signal.sosfilt(sos, x) * (10 ** (gain_db / 20.0) - 1))


def equalize(x, rate, st):  # main.py:116-131 (mono passes through)
    if not (x.ndim > 1 and x.shape[1] == 2):
        return x
    l, r = x[:, 0], x[:, 1]
    for fn, hz, g, extra in ((shelf, 250, float(st.get("bass_boost", 0.0)), ("low",)),
                             (peak, 1000, -float(st.get("mid_cut", 0.0)), ()),
                             (peak, 4000, float(st.get("presence_boost", 0.0)), ()),
                             (shelf, 8000, float(st.get("treble_boost", 0.0)), ("high",))):
        l, r = fn(l, rate, hz, g, *extra), fn(r, rate, hz, g, *extra)
    return np.array([l, r]).T


def multiband(q, rate, st):  # main.py:156-177
    x = mo.pcm_to_float(q)
    b = scipy.signal.butter
    lo = scipy.signal.sosfilt(b(4, 250, btype="lowpass", fs=rate, output="sos"), x, axis=0)
    mid = scipy.signal.sosfilt(b(4, 250, btype="highpass", fs=rate, output="sos"), x, axis=0)
    mid = scipy.signal.sosfilt(b(4, 4000, btype="lowpass", fs=rate, output="sos"), mid, axis=0)
    hi = scipy.signal.sosfilt(b(4, 4000, btype="highpass", fs=rate, output="sos"), x, axis=0)
    thr = (float(st.get("low_band_threshold", -25.0)), float(st.get("mid_band_threshold", -20.0)),
           float(st.get("high_band_threshold", -15.0)))
    rat = (float(st.get("low_band_ratio", 6.0)), float(st.get("mid_band_ratio", 3.0)),
           float(st.get("high_band_ratio", 4.0)))
    outs = [mo.compress_band(mo.quantize(band), rate, t, r, at, rel)
            for band, t, r, (at, rel) in zip((lo, mid, hi), thr, rat, mo.BAND_TIMES)]
    out = mo.overlay_add(mo.overlay_add(outs[0], outs[1]), outs[2])
    n1 = mo.overlay_length(q.shape[0], rate)
    if n1 != q.shape[0]:
        pad = np.zeros((n1,) + q.shape[1:], np.int16)
        pad[:min(n1, q.shape[0])] = out[:min(n1, q.shape[0])]
        out = pad
    return out


def soft_limiter(x, thr=0.98):  # main.py:189-192
    x = x.copy()
    k = np.abs(x) > thr
    x[k] = np.tanh(x[k]) * thr
    return x


def master(pcm, rate, st):  # main.py:48-72
    n = pcm.shape[0]
    chunks = []
    for s, e in mo.chunk_ranges(n, rate):
        c = pcm[s:min(e, n)]
        if e > n:
            c = np.concatenate([c, np.zeros((e - n,) + pcm.shape[1:], np.int16)])
        x = mo.pcm_to_float(c)
        if float(st.get("saturation", 0.0)) > 0:
            x = saturation(x, float(st.get("saturation")))
        y = equalize(x, rate, st)
        if float(st.get("width", 1.0)) != 1.0:
            y = mo.stereo_width(y, float(st.get("width")))
        q = mo.quantize(y)
        if st.get("use_multiband"):
            q = multiband(q, rate, st)
        chunks.append(q)
    out = np.concatenate(chunks) if chunks else np.zeros((0,) + pcm.shape[1:], np.int16)
    y = mo.pcm_to_float(out)
    if st.get("lufs") is not None:
        y, _ = mo.normalize_to_lufs(y, rate, float(st.get("lufs")))
    with np.errstate(invalid="ignore"):
        return mo.quantize(soft_limiter(y))
