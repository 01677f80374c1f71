"""TEST INFRASTRUCTURE ONLY — the faithful-cost CPU baseline.

Only `bench.py`'s `cpu_baseline` leg uses this module; it is never part of the
product path.  It times the reference's hot path with the reference's own cost
structure, because the reference itself cannot run on the GPU box (pydub,
pyloudnorm and ffmpeg are absent there and here):

* per 30 s chunk (AME:54-76): int16 -> f32, exciter, 4-biquad EQ (sosfilt per
  stage), width and int16 in numpy/scipy (mastering_oracle), then the multiband
  stage (AME:196-210) through pydub 0.25.1's per-frame Python loop
  (thirdparty_restated.compress_dynamic_range over AudioSegment byte slices,
  audioop rms/mul) and pydub's overlay — ~97 % of the reference's CPU time;
* the whole-track tail (AME:80-89): concat, f32, pyloudnorm-restated loudness,
  gain, soft limiter, int16.

Chunks are independent and cost-linear, so a sample of whole chunks is timed and
extrapolated to the track (stated as such in the bench line); the N-core figure
runs one chunk per worker process at once (multiprocessing over chunks, as a
chunked CPU deployment would).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time

import numpy as np

from . import mastering_oracle as mo
from . import thirdparty_restated as tp


def master_chunk(pcm: np.ndarray, rate: int, settings: dict) -> np.ndarray:
    """AME:55-76 on one int16 chunk with the pydub-structured compressor loop."""
    ch = 1 if pcm.ndim == 1 else pcm.shape[1]
    x = mo.pcm_to_float(pcm)
    x = mo.saturation(x, settings.get("saturation", 0))
    x = mo.equalize(x, rate, settings)
    if settings.get("width", 1.0) != 1.0:
        x = mo.stereo_width(x, settings.get("width"))
    q = mo.quantize(x)
    if not settings.get("multiband"):
        return q
    thr, rat = mo.multiband_params(settings)
    bands = mo.band_split(q, rate)
    segs = []
    for b, t, r, (at, rel) in zip(bands, thr, rat, mo.BAND_TIMES):
        seg = tp.AudioSegment(np.ascontiguousarray(b).tobytes(), 2, rate, ch)
        segs.append(tp.compress_dynamic_range(seg, threshold=t, ratio=r, attack=at, release=rel))
    out = segs[0].overlay(segs[1]).overlay(segs[2])
    o = np.frombuffer(out._data, np.int16)
    return o.reshape(-1, ch) if ch > 1 else o


def master_tail(mix: np.ndarray, rate: int, settings: dict) -> np.ndarray:
    """AME:80-89 on the concatenated mix."""
    y = mo.pcm_to_float(mix)
    if settings.get("lufs") is not None:
        y, _ = mo.normalize_to_lufs(y, rate, settings.get("lufs"))
    with np.errstate(invalid="ignore"):
        return mo.quantize(mo.soft_limiter(y))


def _time_chunk(args):
    pcm, rate, settings = args
    os.environ["OMP_NUM_THREADS"] = "1"
    t0 = time.perf_counter()
    master_chunk(pcm, rate, settings)
    return time.perf_counter() - t0


def time_track(pcm: np.ndarray, rate: int, settings: dict, chunks_1core: int = 2, procs: int | None = None) -> dict:
    """Seconds to master `pcm` with the reference's cost structure: `chunks_1core`
    whole chunks timed back to back on one core, then one chunk per process on
    `procs` cores at once, each extrapolated to every chunk of the track; the
    tail is timed on the whole track."""
    bounds = mo.chunk_ranges(pcm.shape[0], rate)
    full = [(s, e) for s, e in bounds if e - s == bounds[0][1] - bounds[0][0]]
    sample = [pcm[s:e] for s, e in full[:max(1, chunks_1core)]]
    t0 = time.perf_counter()
    for c in sample:
        master_chunk(c, rate, settings)
    per_chunk_1 = (time.perf_counter() - t0) / len(sample)
    t0 = time.perf_counter()
    master_tail(pcm[: len(pcm)], rate, settings)
    tail = time.perf_counter() - t0
    n_chunks = len(bounds)
    out = {"chunks": n_chunks, "chunk_frames": full[0][1] - full[0][0], "sampled_chunks_1core": len(sample),
           "per_chunk_s_1core": per_chunk_1, "tail_s": tail, "track_s_1core": per_chunk_1 * n_chunks + tail}
    procs = procs or 1
    if procs > 1:
        work = [(pcm[full[k % len(full)][0]:full[k % len(full)][1]], rate, settings) for k in range(procs)]
        ctx = mp.get_context("fork")
        with ctx.Pool(procs) as pool:
            t0 = time.perf_counter()
            pool.map(_time_chunk, work, chunksize=1)
            wall = time.perf_counter() - t0
        # `procs` chunks per `wall` seconds; the tail (one whole-track pass) stays serial
        out.update({"procs": procs, "wall_s_per_round": wall,
                    "track_s_ncore": wall * (-(-n_chunks // procs)) + tail})
    return out
