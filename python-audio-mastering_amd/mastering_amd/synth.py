"""Synthetic pink-noise programme material (SURVEY.md §8d "Synthetic input").

Per channel: white N(0,1) from ``numpy.random.default_rng(1000 + track)``,
coloured by the Kellet/Smith pink IIR (streamed per 30 s with carried state),
right = 0.6 * P_L + 0.8 * P_R' (correlated stereo), each channel scaled to
-18 dBFS RMS, then quantised to the int16 grid so that the PCM16 and f32 forms
of a track are the same numbers (the reference only handles 16-bit PCM
correctly, SURVEY.md §7 hard part 6).
"""
from __future__ import annotations

import numpy as np
import scipy.signal

_PINK_B = np.array([0.049922035, -0.095993537, 0.050612699, -0.004408786])
_PINK_A = np.array([1.0, -2.494956002, 2.017265875, -0.522189400])


def pink_noise_pcm16(frames: int, rate: int = 44100, channels: int = 2, track: int = 0,
                     level_dbfs: float = -18.0) -> np.ndarray:
    """int16 [frames, channels] (or [frames] for mono) pink noise at `level_dbfs` RMS."""
    rng = np.random.default_rng(1000 + track)
    step = 30 * rate
    raw = np.empty((frames, 2), np.float32)
    zi = [np.zeros(3), np.zeros(3)]
    for s in range(0, frames, step):
        n = min(step, frames - s)
        w = rng.standard_normal((n, 2))
        for c in range(2):
            raw[s:s + n, c], zi[c] = scipy.signal.lfilter(_PINK_B, _PINK_A, w[:, c], zi=zi[c])
    left = raw[:, 0].astype(np.float64)
    right = 0.6 * left + 0.8 * raw[:, 1]
    target = 10.0 ** (level_dbfs / 20.0)
    out = np.empty((frames, channels), np.int16)
    for c, x in enumerate([left, right][:channels]):
        rms = np.sqrt(np.mean(x * x)) if frames else 1.0
        y = x * (target / rms if rms > 0 else 0.0)
        out[:, c] = np.clip(np.round(y * 32768.0), -32768, 32767).astype(np.int16)
    return out[:, 0] if channels == 1 else out


def pink_noise_chunks(c0: int, c1: int, rate: int = 44100, channels: int = 2, track: int = 0,
                      level_dbfs: float = -18.0, chunk_s: int = 30) -> np.ndarray:
    """Frames of 30 s chunks [c0, c1) of a long synthetic track, each chunk its own
    pink-noise block (seeded by track and chunk index, scaled to `level_dbfs`), so a
    time-sharded rank (BASELINE C4: 2 h = 240 chunks) generates only its own range."""
    n = chunk_s * rate
    out = np.empty(((c1 - c0) * n, channels) if channels > 1 else ((c1 - c0) * n,), np.int16)
    for k, c in enumerate(range(c0, c1)):
        out[k * n:(k + 1) * n] = pink_noise_pcm16(n, rate, channels, track=100003 * (track + 1) + c,
                                                  level_dbfs=level_dbfs)
    return out
