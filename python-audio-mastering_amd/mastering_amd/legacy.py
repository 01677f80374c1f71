"""The reference's legacy engine (root main.py) as an
alternate DSP profile on the GPU.

`main.py` is the older monolithic Cloud Function the worker engine replaced.  Its
chunked chain (main.py:48-72) differs from AME's:

  exciter      tanh(x * g) / g, g = 1 + 4 * amount / 100, only if amount > 0  (main.py:94-97)
  EQ           stereo only (mono passes through); each stage is a PARALLEL mix of
               a butter() filter: shelves y = x + (g-1) * butter5(x) (boost) or
               g * x + (1-g) * butter5(x) (cut), peaks y = x + (g-1) * bandpass2(x)
               (main.py:116-154)
  width        as AME (main.py:107-113)
  multiband    key `use_multiband`; bands LP4(250), LP4(4000)(HP4(250)(x)) and
               HP4(4000); thresholds/ratios from `low_band_threshold` ...
               (main.py:156-177); pydub compressor + overlay as AME
  loudness     as AME, without the print (main.py:179-187)
  limiter      |x| > 0.98 -> tanh(x) * 0.98 (main.py:189-192)

The functions below keep main.py's names and signatures; every per-sample step
is one HIP operator of the library (include/mastering.h: mm_op_saturation_legacy,
mm_op_sosfilt_mix, mm_op_sosfilt, mm_op_quantize, mm_op_compress_bands,
mm_op_loudness/mm_op_gain, mm_op_soft_limiter_legacy).  Filter design (scipy
butter, host f64) is the reference's own expression.  No CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.signal

from . import design, native, ops, wavio
from .engine import Job

__all__ = ["apply_saturation", "apply_eq_to_samples", "apply_shelf_filter", "apply_peak_filter",
           "apply_stereo_width", "apply_multiband_compressor", "normalize_to_lufs", "soft_limiter",
           "master_pcm", "process"]

CHUNK_MS = 30 * 1000  # main.py:50


def _sections(sos):
    out = []
    for row in np.asarray(sos, np.float64):
        if row[3] != 1.0:
            raise ValueError("unnormalised SOS section")
        out.append((row[0], row[1], row[2], row[4], row[5]))
    return out


def _iir(sections, ch):
    f = native.MMIir()
    Job._fill_iir(f, sections, [len(sections)], design.OPS_TILE, design.LB_THREADS // ch)
    return f


def _sosfilt_mix(samples, sos, a, c, device=0):
    """a * samples + c * scipy.signal.sosfilt(sos, samples) on one channel, f64 out."""
    x, dt = ops._float_input(samples, "sosfilt")
    out = np.empty(x.shape, np.float64)
    ctx = native.context(device)
    ctx.check(ctx.lib.mm_op_sosfilt_mix(ctx.ptr, dt, ops._ptr(x), x.shape[0], 1, ctypes.byref(_iir(_sections(sos), 1)),
                                        float(a), float(c), ops._ptr(out)), "mm_op_sosfilt_mix")
    return out


def _sosfilt(samples, sos, device=0):
    """scipy.signal.sosfilt(sos, samples, axis=0) on [N] or [N, 2], f64 out."""
    x, dt = ops._float_input(samples, "sosfilt")
    return ops._sosfilt(x, dt, 1 if x.ndim == 1 else x.shape[1], _sections(sos), device=device)


# ------------------------------------------------------------------ main.py:94-192
def apply_saturation(samples, amount, device: int = 0):
    if amount == 0:
        return samples
    x, dt = ops._float_input(samples, "apply_saturation")
    out = np.empty_like(x)
    ctx = native.context(device)
    ctx.check(ctx.lib.mm_op_saturation_legacy(ctx.ptr, dt, ops._ptr(x), x.size, float(amount), ops._ptr(out)),
              "mm_op_saturation_legacy")
    return out


apply_stereo_width = ops.apply_stereo_width  # main.py:107-113 == AME:136-144


def apply_shelf_filter(samples, sample_rate, cutoff_hz, gain_db, filter_type, order=5, device: int = 0):
    if gain_db == 0:
        return samples
    nyquist = 0.5 * sample_rate
    normal_cutoff = cutoff_hz / nyquist
    sos = scipy.signal.butter(order, normal_cutoff, btype=filter_type, analog=False, output="sos")
    gain_factor = 10 ** (gain_db / 20.0)
    if gain_db > 0:
        return _sosfilt_mix(samples, sos, 1.0, gain_factor - 1, device)
    return _sosfilt_mix(samples, sos, gain_factor, 1 - gain_factor, device)


def apply_peak_filter(samples, sample_rate, center_hz, gain_db, q=1.0, device: int = 0):
    if gain_db == 0:
        return samples
    nyquist = 0.5 * sample_rate
    normal_center = center_hz / nyquist
    edge1, edge2 = normal_center / np.sqrt(q), normal_center * np.sqrt(q)
    low_freq, high_freq = min(edge1, edge2), max(edge1, edge2)
    if low_freq >= high_freq:
        high_freq = low_freq + 1e-9
    if high_freq >= 1.0:
        high_freq = 0.999999
    sos = scipy.signal.butter(2, [low_freq, high_freq], btype="bandpass", output="sos")
    gain_factor = 10 ** (gain_db / 20.0)
    return _sosfilt_mix(samples, sos, 1.0, gain_factor - 1, device)


def apply_eq_to_samples(samples, sample_rate, settings, device: int = 0):
    if not (samples.ndim > 1 and samples.shape[1] == 2):
        return samples  # main.py:131-132: the legacy EQ leaves mono untouched
    left, right = samples[:, 0], samples[:, 1]
    stages = [(apply_shelf_filter, 250, float(settings.get("bass_boost", 0.0)), ("low",)),
              (apply_peak_filter, 1000, -float(settings.get("mid_cut", 0.0)), ()),
              (apply_peak_filter, 4000, float(settings.get("presence_boost", 0.0)), ()),
              (apply_shelf_filter, 8000, float(settings.get("treble_boost", 0.0)), ("high",))]
    for fn, hz, gain, extra in stages:
        left = fn(left, sample_rate, hz, gain, *extra, device=device)
        right = fn(right, sample_rate, hz, gain, *extra, device=device)
    return np.array([left, right]).T


def _band_settings(settings):
    return (float(settings.get("low_band_threshold", -25.0)), float(settings.get("low_band_ratio", 6.0)),
            float(settings.get("mid_band_threshold", -20.0)), float(settings.get("mid_band_ratio", 3.0)),
            float(settings.get("high_band_threshold", -15.0)), float(settings.get("high_band_ratio", 4.0)))


def apply_multiband_compressor(chunk, settings, frame_rate=None, device: int = 0):
    """main.py:156-177 on a 16-bit segment (or int16 ndarray with frame_rate)."""
    pcm, ch, rate = ops._pcm16(chunk)
    rate = int(frame_rate if frame_rate is not None else rate)
    lt, lr, mt, mr, ht, hr = _band_settings(settings)
    lo_x, hi_x = 250, 4000
    samples = ops.audio_segment_to_float_array(pcm, device=device)
    low = _sosfilt(samples, scipy.signal.butter(4, lo_x, btype="lowpass", fs=rate, output="sos"), device)
    mid_sos = np.concatenate([scipy.signal.butter(4, lo_x, btype="highpass", fs=rate, output="sos"),
                              scipy.signal.butter(4, hi_x, btype="lowpass", fs=rate, output="sos")])
    mid = _sosfilt(samples, mid_sos, device)  # two sosfilt calls in f64 == one 4-section cascade
    high = _sosfilt(samples, scipy.signal.butter(4, hi_x, btype="highpass", fs=rate, output="sos"), device)
    bands = [ops._quantize(b, device) for b in (low, mid, high)]
    n = pcm.shape[0]
    params = {"multiband": True, "low_thresh": lt, "low_ratio": lr, "mid_thresh": mt, "mid_ratio": mr,
              "high_thresh": ht, "high_ratio": hr}
    job = Job(n, rate, ch, params, single_chunk=True)
    mix = np.empty_like(pcm)
    if n:
        ctx = native.context(device)
        ctx.check(ctx.lib.mm_op_compress_bands(ctx.ptr, ctypes.byref(job.job), ops._ptr(bands[0]), ops._ptr(bands[1]),
                                               ops._ptr(bands[2]), ops._ptr(mix)), "mm_op_compress_bands")
    n1 = design.pydub_frame(design.pydub_len_ms(n, rate), rate)  # pydub overlay's ms re-slicing
    n2 = design.pydub_frame(design.pydub_len_ms(n1, rate), rate)  # the second overlay re-slices again
    if n2 != n1:
        raise NotImplementedError(f"pydub overlay re-slicing is not stable at {rate} Hz")
    if n1 != n:
        out = np.zeros((n1,) + pcm.shape[1:], np.int16)
        out[:min(n, n1)] = mix[:min(n, n1)]
        mix = out
    spawn = getattr(chunk, "_spawn", None)
    return spawn(mix.tobytes()) if spawn is not None and not isinstance(chunk, np.ndarray) else mix


def normalize_to_lufs(samples, sample_rate, target_lufs=-14.0, device: int = 0):
    x, dt, loudness = ops._loudness(samples, sample_rate, target_lufs, device)
    gain_db = target_lufs - loudness
    gain_linear = 10.0 ** (gain_db / 20.0)
    out = np.empty(x.shape, np.float64)
    ctx = native.context(device)
    ctx.check(ctx.lib.mm_op_gain(ctx.ptr, dt, ops._ptr(x), x.size, float(gain_linear), ops._ptr(out)), "mm_op_gain")
    return out


def soft_limiter(samples, threshold=0.98, device: int = 0):
    x, dt = ops._float_input(samples, "soft_limiter")
    ctx = native.context(device)
    ctx.check(ctx.lib.mm_op_soft_limiter_legacy(ctx.ptr, dt, ops._ptr(x), x.size, float(threshold)),
              "mm_op_soft_limiter_legacy")
    if x is not samples:
        samples[...] = x
    return samples


# ------------------------------------------------------------------ main.py:48-72
def master_pcm(pcm: np.ndarray, rate: int, settings: dict, device: int = 0) -> np.ndarray:
    """The legacy chain on int16 PCM [N] or [N, 2] -> int16 PCM (main.py:48-72)."""
    settings = dict(settings or {})
    n = pcm.shape[0]
    chunks = []
    bounds = design.chunk_bounds(n, rate)
    if settings.get("use_multiband"):  # the overlay's ms re-slicing must keep every chunk's length
        design.check_chunk_geometry(bounds, design.pydub_frame(design.CHUNK_MS, rate), rate, True)
    for a, b in bounds:
        c = pcm[a:min(b, n)]
        if b > n:  # pydub pads <= 2 ms of silence
            c = np.concatenate([c, np.zeros((b - n,) + pcm.shape[1:], np.int16)])
        x = ops.audio_segment_to_float_array(c, device=device)
        if float(settings.get("saturation", 0.0)) > 0:
            x = apply_saturation(x, float(settings.get("saturation")), device=device)
        y = apply_eq_to_samples(x, rate, settings, device=device)
        if float(settings.get("width", 1.0)) != 1.0:
            y = apply_stereo_width(y, float(settings.get("width")), device=device)
        q = ops._quantize(y, device)
        if settings.get("use_multiband"):
            q = apply_multiband_compressor(q, settings, frame_rate=rate, device=device)
        chunks.append(q)
    out = np.concatenate(chunks) if chunks else np.zeros((0,) + pcm.shape[1:], np.int16)
    y = ops.audio_segment_to_float_array(out, device=device)
    if settings.get("lufs") is not None:
        y = normalize_to_lufs(y, rate, float(settings.get("lufs")), device=device)
    y = soft_limiter(y, device=device)
    return ops._quantize(y, device)


def process(input_path: str, output_path: str, settings: dict, device: int = 0) -> dict:
    """main.py:46-72 with local files: decode a 16-bit WAV, master, export WAV."""
    pcm, rate = wavio.read_wav(input_path)
    if pcm.dtype != np.int16:
        raise ValueError("the legacy profile takes 16-bit PCM WAV (what pydub decodes it to)")
    out = master_pcm(pcm, rate, settings, device=device)
    wavio.write_wav(output_path, out, rate)
    return {"frames": int(out.shape[0]), "rate": rate, "output_path": output_path}
