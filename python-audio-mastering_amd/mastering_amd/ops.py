"""The reference's per-stage DSP surface on the GPU.

Same names, arguments and return conventions as the helpers in
worker/audio_mastering_engine.py ("AME"), so a caller can swap in ONE stage:

  audio_segment_to_float_array   AME:117-121
  float_array_to_audio_segment   AME:123-126
  apply_saturation               AME:128-134
  apply_stereo_width             AME:136-144
  apply_eq_to_samples            AME:146-163
  apply_shelf_filter             AME:165-183
  apply_peak_filter              AME:185-194
  apply_multiband_compressor     AME:196-210
  normalize_to_lufs              AME:212-222
  soft_limiter                   AME:224-227
  integrated_loudness            pyloudnorm Meter(rate).integrated_loudness (AME:218)

numpy in, numpy out; every per-sample computation runs in the HIP library
(include/mastering.h, "per-stage operators").  Results follow numpy's dtype rules
for the reference's expressions: float32 stays float32 through the pointwise
stages, scipy's sosfilt returns float64, and the LUFS gain is an np.float64 so
normalize_to_lufs returns float64.  "Segments" are pydub-AudioSegment-like objects
(`get_array_of_samples`, `channels`, `sample_width`, `frame_rate`, `_spawn`); a
plain int16 ndarray is accepted too (with `frame_rate=` where a rate is needed).
Only 16-bit samples are supported (sample_width 2: what AME's int16 conversions
produce); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import design, native
from .engine import Job

__all__ = ["audio_segment_to_float_array", "float_array_to_audio_segment", "apply_saturation",
           "apply_stereo_width", "apply_eq_to_samples", "apply_shelf_filter", "apply_peak_filter",
           "apply_multiband_compressor", "normalize_to_lufs", "soft_limiter", "integrated_loudness"]

_vp = ctypes.c_void_p


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_vp)


def _float_input(samples, what: str):
    x = np.asarray(samples)
    if x.dtype == np.float32:
        return np.ascontiguousarray(x), native.MM_F32
    if x.dtype == np.float64:
        return np.ascontiguousarray(x), native.MM_F64
    raise TypeError(f"{what}: float32 or float64 samples expected, got {x.dtype}")


def _ctx(device: int):
    return native.context(device)


def _pcm16(segment):
    """(int16 samples [N] or [N, ch], channels, frame_rate) of a segment or ndarray."""
    if isinstance(segment, np.ndarray):
        if segment.dtype != np.int16:
            raise TypeError("int16 PCM expected")
        ch = 1 if segment.ndim == 1 else segment.shape[1]
        return np.ascontiguousarray(segment), ch, None
    if getattr(segment, "sample_width", 2) != 2:
        raise ValueError("only 16-bit segments are supported (sample_width 2)")
    ch = int(segment.channels)
    s = np.array(segment.get_array_of_samples()).astype(np.int16)
    if ch == 2:
        s = s.reshape((-1, 2))
    return np.ascontiguousarray(s), ch, getattr(segment, "frame_rate", None)


# ------------------------------------------------------------------ AME:117-126
def audio_segment_to_float_array(audio_segment, device: int = 0) -> np.ndarray:
    """int16 samples / 32768 as float32, reshaped (-1, 2) for stereo (AME:117-121)."""
    pcm, ch, _ = _pcm16(audio_segment)
    out = np.empty(pcm.shape, np.float32)
    ctx = _ctx(device)
    ctx.check(ctx.lib.mm_op_pcm_to_float(ctx.ptr, _ptr(pcm), pcm.size, _ptr(out)), "mm_op_pcm_to_float")
    return out


def _quantize(float_array, device: int) -> np.ndarray:
    x, dt = _float_input(float_array, "float_array_to_audio_segment")
    out = np.empty(x.shape, np.int16)
    ctx = _ctx(device)
    ctx.check(ctx.lib.mm_op_quantize(ctx.ptr, dt, _ptr(x), x.size, _ptr(out)), "mm_op_quantize")
    return out


def float_array_to_audio_segment(float_array, audio_segment_template, device: int = 0):
    """clip to [-1, 1], * 32768, astype(int16) (AME:123-126); returns
    `template._spawn(bytes)`, or the int16 array when the template has no _spawn."""
    if getattr(audio_segment_template, "sample_width", 2) != 2:
        raise ValueError("only 16-bit templates are supported (sample_width 2)")
    q = _quantize(float_array, device)
    spawn = getattr(audio_segment_template, "_spawn", None)
    return spawn(q.tobytes()) if spawn is not None else q


# ------------------------------------------------------------------ pointwise
def apply_saturation(samples, saturation_percent, device: int = 0):
    """(1 - mix) x + mix tanh(x (1 + 4 mix)), mix = (s / 100)^2 (AME:128-134).
    float32 samples on the int16 grid (what audio_segment_to_float_array makes)
    take the values of design.saturation_table (numpy's own float32 tanh); others
    the device tanhf."""
    if saturation_percent == 0:
        return samples
    x, dt = _float_input(samples, "apply_saturation")
    out = np.empty_like(x)
    ctx = _ctx(device)
    tab = None
    if dt == native.MM_F32:
        tab = design.saturation_table(saturation_percent)[0].ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    ctx.check(ctx.lib.mm_op_saturation_table(ctx.ptr, dt, _ptr(x), x.size, float(saturation_percent), tab,
                                             _ptr(out)), "mm_op_saturation_table")
    return out


def apply_stereo_width(samples, width_factor, device: int = 0):
    """Mid/side scaling of a [N, 2] array; anything else passes through (AME:136-144)."""
    if samples.ndim == 1 or samples.shape[1] != 2:
        return samples
    x, dt = _float_input(samples, "apply_stereo_width")
    out = np.empty_like(x)
    ctx = _ctx(device)
    ctx.check(ctx.lib.mm_op_stereo_width(ctx.ptr, dt, _ptr(x), x.shape[0], float(width_factor), _ptr(out)),
              "mm_op_stereo_width")
    return out


def soft_limiter(samples, threshold=0.98, device: int = 0):
    """Knee above `threshold` with asymptote 1.0, IN PLACE, returns `samples` (AME:224-227)."""
    x, dt = _float_input(samples, "soft_limiter")
    ctx = _ctx(device)
    ctx.check(ctx.lib.mm_op_soft_limiter(ctx.ptr, dt, _ptr(x), x.size, float(threshold)), "mm_op_soft_limiter")
    if x is not samples:  # non-contiguous input: write the result back into it
        samples[...] = x
    return samples


# ------------------------------------------------------------------ EQ (sosfilt)
def _sosfilt(x: np.ndarray, dt: int, ch: int, sections, round_f32: bool = False, device: int = 0) -> np.ndarray:
    iir = native.MMIir()
    Job._fill_iir(iir, sections, [len(sections)], design.OPS_TILE, design.LB_THREADS // ch)
    frames = x.shape[0]
    out = np.empty((frames, ch) if ch == 2 else (frames,), np.float64)
    ctx = _ctx(device)
    ctx.check(ctx.lib.mm_op_sosfilt(ctx.ptr, dt, _ptr(x), frames, ch, ctypes.byref(iir), int(round_f32), _ptr(out)),
              "mm_op_sosfilt")
    return out


def _filter_1d(samples, section, device):
    x, dt = _float_input(samples, "sosfilt")
    if x.ndim != 1:
        raise NotImplementedError("shelf/peak filters take one channel (AME calls them per channel)")
    return _sosfilt(x, dt, 1, [section], device=device)


def apply_shelf_filter(samples, sample_rate, cutoff_hz, gain_db, filter_type, q=0.707, device: int = 0):
    """One RBJ-style shelf biquad as AME:165-183 writes it (w0 = 4 pi f / fs,
    gain = 10^(dB/20)); f64 out; 0 dB returns `samples` unchanged."""
    if gain_db == 0:
        return samples
    return _filter_1d(samples, design.shelf_section(sample_rate, cutoff_hz, gain_db,
                                                    "low" if filter_type == "low" else "high", q), device)


def apply_peak_filter(samples, sample_rate, center_hz, gain_db, q=1.0, device: int = 0):
    """One peaking biquad as AME:185-194 writes it; f64 out; 0 dB is the identity."""
    if gain_db == 0:
        return samples
    return _filter_1d(samples, design.peak_section(sample_rate, center_hz, gain_db, q), device)


def apply_eq_to_samples(samples, sample_rate, settings, device: int = 0):
    """Low shelf 250 Hz, peak 1 kHz (-mid_cut), peak 4 kHz, high shelf 8 kHz, per
    channel, each skipped at 0 dB (AME:146-163), as ONE cascade launch."""
    sections = design.eq_sections(sample_rate, settings)
    stereo = samples.ndim > 1 and samples.shape[1] == 2
    if not sections:  # every stage returned its input (AME:171, 186)
        return np.array([samples[:, 0], samples[:, 1]]).T if stereo else samples
    x, dt = _float_input(samples, "apply_eq_to_samples")
    if not stereo and x.ndim != 1:
        raise NotImplementedError("mono EQ takes a 1-D array")
    return _sosfilt(x, dt, 2 if stereo else 1, sections, device=device)


# ------------------------------------------------------------------ multiband
def apply_multiband_compressor(chunk, low_thresh, low_ratio, mid_thresh, mid_ratio, high_thresh, high_ratio,
                               low_crossover=250, high_crossover=4000, frame_rate=None, device: int = 0):
    """butter(4) crossover at (low_crossover, high_crossover), mid = x - lo - hi,
    pydub compress_dynamic_range per band with attack/release 10/200, 5/150 and
    1/50 ms, overlay lo + mid + hi (AME:196-210), on the GPU.  Returns
    `chunk._spawn(bytes)` for a segment, an int16 array for an ndarray input."""
    pcm, ch, rate = _pcm16(chunk)
    rate = int(frame_rate if frame_rate is not None else rate)
    if not rate:
        raise ValueError("frame_rate is required for an ndarray chunk")
    n = pcm.shape[0]
    params = {"multiband": True, "low_thresh": low_thresh, "low_ratio": low_ratio, "mid_thresh": mid_thresh,
              "mid_ratio": mid_ratio, "high_thresh": high_thresh, "high_ratio": high_ratio}
    job = Job(n, rate, ch, params, single_chunk=True, crossover=(low_crossover, high_crossover))
    job.job.in_kind = native.MM_IN_I16
    mix = np.empty_like(pcm)
    ctx = _ctx(device)
    if n:
        ctx.check(ctx.lib.mm_op_multiband(ctx.ptr, ctypes.byref(job.job), _ptr(pcm), _ptr(mix)), "mm_op_multiband")
    # pydub overlay re-slices its first operand by ms: seg[0:len(seg)] has
    # int(round(1000 n / rate) * rate / 1000) frames (padded with silence or cut)
    n1 = design.pydub_frame(design.pydub_len_ms(n, rate), rate)
    n2 = design.pydub_frame(design.pydub_len_ms(n1, rate), rate)
    if n2 != n1:
        raise NotImplementedError(f"pydub overlay re-slicing is not stable at {rate} Hz")
    if n1 != n:
        out = np.zeros((n1,) + pcm.shape[1:], np.int16)
        k = min(n, n1)
        out[:k] = mix[:k]
        mix = out
    spawn = getattr(chunk, "_spawn", None)
    return spawn(mix.tobytes()) if spawn is not None and not isinstance(chunk, np.ndarray) else mix


# ------------------------------------------------------------------ loudness
def _loudness(samples, sample_rate, target, device):
    x, dt = _float_input(samples, "integrated_loudness")
    ch = 2 if x.ndim == 2 else 1
    if x.ndim == 2 and x.shape[1] != 2:
        raise NotImplementedError("mono or stereo samples only")
    job = Job(x.shape[0], sample_rate, ch, {"lufs": float(target)}, single_chunk=True)  # raises if < 0.4 s
    out = np.zeros(2)
    ctx = _ctx(device)
    ctx.check(ctx.lib.mm_op_loudness(ctx.ptr, ctypes.byref(job.job), dt, _ptr(x), out.ctypes.data_as(native.c_double_p)),
              "mm_op_loudness")
    return x, dt, np.float64(out[0])


def integrated_loudness(data, rate, device: int = 0) -> np.float64:
    """pyloudnorm 0.1.1 Meter(rate).integrated_loudness of a mono signal (or of
    the mean of a stereo one), in LUFS."""
    return _loudness(data, rate, 0.0, device)[2]


def normalize_to_lufs(samples, sample_rate, target_lufs=-14.0, device: int = 0):
    """Measure the mono mean's loudness and scale to `target_lufs` (AME:212-222)."""
    x, dt, loudness = _loudness(samples, sample_rate, target_lufs, device)
    gain_db = target_lufs - loudness
    gain_linear = 10.0 ** (gain_db / 20.0)
    print(f"Current loudness: {loudness:.2f} LUFS. Applying {gain_db:.2f} dB gain...")
    out = np.empty(x.shape, np.float64)
    ctx = _ctx(device)
    ctx.check(ctx.lib.mm_op_gain(ctx.ptr, dt, _ptr(x), x.size, float(gain_linear), _ptr(out)), "mm_op_gain")
    return out
