"""TEST INFRASTRUCTURE ONLY — restatement of the third-party pieces the reference
hot path calls but does not vendor.  Never imported by the product package.

The reference (`worker/audio_mastering_engine.py`, "AME" below) imports
`pydub` (requirements.txt:2, unpinned; latest at the 2025-08-29 snapshot: 0.25.1)
and `pyloudnorm` (requirements.txt:5, unpinned; latest: 0.1.1).  Neither is
installed here and there is no network, so their published algorithms are
restated below, written for this repo, covering exactly the surface AME uses:

* pydub.AudioSegment: decode (AME:43), ms slicing (AME:54), `_spawn`
  (AME:126), `get_array_of_samples` (AME:118), `overlay` (AME:210),
  `sum()` concatenation (AME:80), WAV `export` (AME:98);
* pydub.effects.compress_dynamic_range (AME:207-209) — the per-frame loop,
  kept in pydub's own loop structure (this is also the "faithful-cost" CPU
  baseline: it is as slow as the reference);
* pyloudnorm.Meter(rate).integrated_loudness (AME:213,218) — BS.1770-4 K-weighted
  gated loudness.

int16 arithmetic goes through stdlib `audioop` (present in Python 3.10) exactly
as pydub does.  Parity at this boundary is "parity unpinned": the reference's own
tests hold no fixture for it (it has no tests).
"""
from __future__ import annotations

import array
import audioop
import io
import math
import wave

import numpy as np
import scipy.signal


# --------------------------------------------------------------------------
# WAV decode (stands in for ffmpeg's pcm_s16le decode of a PCM16 WAV; AME:43)
# --------------------------------------------------------------------------
def _read_wav_pcm16(buf: bytes):
    with wave.open(io.BytesIO(buf), "rb") as w:
        ch, sw, rate, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        data = w.readframes(n)
    if sw != 2:
        raise ValueError("restated decoder handles 16-bit PCM only")
    return data, sw, rate, ch


class AudioSegment:
    """Subset of pydub 0.25.1 `AudioSegment` used by AME."""

    def __init__(self, data=b"", sample_width=2, frame_rate=44100, channels=1):
        self._data = bytes(data)
        self.sample_width = sample_width
        self.frame_rate = frame_rate
        self.channels = channels
        self.frame_width = channels * sample_width

    # -- construction -------------------------------------------------------
    @classmethod
    def from_file(cls, file, format=None, **kw):
        if hasattr(file, "read"):
            buf = file.read()
        else:
            with open(file, "rb") as f:
                buf = f.read()
        data, sw, rate, ch = _read_wav_pcm16(buf)
        return cls(data, sw, rate, ch)

    def _spawn(self, data, overrides=None):
        if isinstance(data, list):
            data = b"".join(data)
        if isinstance(data, array.array):
            data = data.tobytes()
        if hasattr(data, "read"):
            if hasattr(data, "seek"):
                data.seek(0)
            data = data.read()
        o = overrides or {}
        return AudioSegment(data, o.get("sample_width", self.sample_width),
                            o.get("frame_rate", self.frame_rate),
                            o.get("channels", self.channels))

    # -- geometry -----------------------------------------------------------
    def frame_count(self, ms=None):
        if ms is not None:
            return ms * (self.frame_rate / 1000.0)
        return float(len(self._data) // self.frame_width)

    def __len__(self):
        return round(1000 * (self.frame_count() / self.frame_rate))

    @property
    def max_possible_amplitude(self):
        bits = self.sample_width * 8
        return float(1 << bits) / 2

    @property
    def rms(self):
        return audioop.rms(self._data, self.sample_width)

    def _parse_position(self, val):
        if val < 0:
            val = len(self) - abs(val)
        val = self.frame_count(ms=len(self)) if val == float("inf") else self.frame_count(ms=val)
        return int(val)

    def __getitem__(self, millisecond):
        if isinstance(millisecond, slice):
            start = millisecond.start if millisecond.start is not None else 0
            end = millisecond.stop if millisecond.stop is not None else len(self)
            start = min(start, len(self))
            end = min(end, len(self))
        else:
            start, end = millisecond, millisecond + 1
        start = self._parse_position(start) * self.frame_width
        end = self._parse_position(end) * self.frame_width
        data = self._data[start:end]
        missing = (end - start - len(data)) // self.frame_width
        if missing:
            if missing > self.frame_count(ms=2):
                raise ValueError("TooManyMissingFrames: %s" % missing)
            silence = audioop.mul(data[: self.frame_width], self.sample_width, 0)
            data += silence * missing
        return self._spawn(data)

    def get_sample_slice(self, start_sample=None, end_sample=None):
        max_val = int(self.frame_count())

        def bounded(val, default):
            if val is None:
                return default
            if val < 0:
                return 0
            if val > max_val:
                return max_val
            return val

        s = bounded(start_sample, 0) * self.frame_width
        e = bounded(end_sample, max_val) * self.frame_width
        return self._spawn(self._data[s:e])

    def get_frame(self, index):
        s = index * self.frame_width
        return self._data[s:s + self.frame_width]

    def get_array_of_samples(self):
        return array.array({1: "b", 2: "h", 4: "i"}[self.sample_width], self._data)

    # -- combination --------------------------------------------------------
    def append(self, seg, crossfade=100):
        if crossfade != 0:
            raise NotImplementedError("only crossfade=0 is reached from AME:80")
        return self._spawn(self._data + seg._data)

    def __add__(self, arg):
        if isinstance(arg, AudioSegment):
            return self.append(arg, crossfade=0)
        raise NotImplementedError

    def __radd__(self, rarg):
        if rarg == 0:
            return self
        raise TypeError

    def overlay(self, seg, position=0, loop=False, times=None, gain_during_overlay=None):
        if loop:
            times = -1
        elif times is None:
            times = 1
        out = io.BytesIO()
        seg1, seg2 = self, seg  # AME always overlays same-format segments (_sync is a no-op)
        sw = seg1.sample_width
        out.write(seg1[:position]._data)
        s1 = seg1[position:]._data
        s2 = seg2._data
        pos, n1, n2 = 0, len(s1), len(s2)
        while times:
            remaining = max(0, n1 - pos)
            if n2 >= remaining:
                s2 = s2[:remaining]
                n2 = remaining
                times = 1
            out.write(audioop.add(s1[pos:pos + n2], s2, sw))
            pos += n2
            times -= 1
        out.write(s1[pos:])
        return seg1._spawn(out)

    def export(self, out_f, format="wav", **kw):
        if format != "wav":
            raise NotImplementedError
        with wave.open(out_f, "wb") as w:
            w.setnchannels(self.channels)
            w.setsampwidth(self.sample_width)
            w.setframerate(self.frame_rate)
            w.setnframes(int(self.frame_count()))
            w.writeframesraw(self._data)
        return out_f


def db_to_float(db, using_amplitude=True):
    db = float(db)
    return 10 ** (db / 20) if using_amplitude else 10 ** (db / 10)


def ratio_to_db(ratio, val2=None, using_amplitude=True):
    ratio = float(ratio)
    if val2 is not None:
        ratio = ratio / val2
    if ratio == 0:
        return -float("inf")
    return 20 * math.log(ratio, 10) if using_amplitude else 10 * math.log(ratio, 10)


def compress_dynamic_range(seg, threshold=-20.0, ratio=4.0, attack=5.0, release=50.0):
    """pydub.effects.compress_dynamic_range, in pydub's per-frame loop form."""
    thresh_rms = seg.max_possible_amplitude * db_to_float(threshold)
    look_frames = int(seg.frame_count(ms=attack))

    def rms_at(i):
        return seg.get_sample_slice(i - look_frames, i).rms

    def db_over_threshold(rms):
        if rms == 0:
            return 0.0
        return max(ratio_to_db(rms / thresh_rms), 0)

    output = []
    attenuation = 0.0
    attack_frames = seg.frame_count(ms=attack)
    release_frames = seg.frame_count(ms=release)
    for i in range(int(seg.frame_count())):
        rms_now = rms_at(i)
        max_att = (1 - (1.0 / ratio)) * db_over_threshold(rms_now)
        inc = max_att / attack_frames
        dec = max_att / release_frames
        if rms_now > thresh_rms and attenuation <= max_att:
            attenuation += inc
            attenuation = min(attenuation, max_att)
        else:
            attenuation -= dec
            attenuation = max(attenuation, 0)
        frame = seg.get_frame(i)
        if attenuation != 0.0:
            frame = audioop.mul(frame, seg.sample_width, db_to_float(-attenuation))
        output.append(frame)
    return seg._spawn(data=b"".join(output))


# --------------------------------------------------------------------------
# pyloudnorm 0.1.1 (Meter with the default "K-weighting", block_size 0.4 s)
# --------------------------------------------------------------------------
class IIRfilter:
    def __init__(self, G, Q, fc, rate, filter_type, passband_gain=1.0):
        self.G, self.Q, self.fc, self.rate = G, Q, fc, rate
        self.filter_type = filter_type
        self.passband_gain = passband_gain
        self.b, self.a = self._coefficients()

    def _coefficients(self):
        A = 10 ** (self.G / 40.0)
        w0 = 2.0 * np.pi * (self.fc / self.rate)
        alpha = np.sin(w0) / (2.0 * self.Q)
        if self.filter_type == "high_shelf":
            b0 = A * ((A + 1) + (A - 1) * np.cos(w0) + 2 * np.sqrt(A) * alpha)
            b1 = -2 * A * ((A - 1) + (A + 1) * np.cos(w0))
            b2 = A * ((A + 1) + (A - 1) * np.cos(w0) - 2 * np.sqrt(A) * alpha)
            a0 = (A + 1) - (A - 1) * np.cos(w0) + 2 * np.sqrt(A) * alpha
            a1 = 2 * ((A - 1) - (A + 1) * np.cos(w0))
            a2 = (A + 1) - (A - 1) * np.cos(w0) - 2 * np.sqrt(A) * alpha
        elif self.filter_type == "high_pass":
            b0 = (1 + np.cos(w0)) / 2
            b1 = -(1 + np.cos(w0))
            b2 = (1 + np.cos(w0)) / 2
            a0 = 1 + alpha
            a1 = -2 * np.cos(w0)
            a2 = 1 - alpha
        else:
            raise NotImplementedError(self.filter_type)
        return np.array([b0, b1, b2]) / a0, np.array([a0, a1, a2]) / a0

    def apply_filter(self, data):
        return self.passband_gain * scipy.signal.lfilter(self.b, self.a, data)


class Meter:
    def __init__(self, rate, filter_class="K-weighting", block_size=0.400):
        if filter_class != "K-weighting":
            raise NotImplementedError
        self.rate = rate
        self.block_size = block_size
        self._filters = {
            "high_shelf": IIRfilter(4.0, 1 / np.sqrt(2), 1500.0, rate, "high_shelf"),
            "high_pass": IIRfilter(0.0, 0.5, 38.0, rate, "high_pass"),
        }

    def integrated_loudness(self, data):
        x = data.copy()
        if not isinstance(x, np.ndarray):
            raise ValueError("Data must be of type numpy.ndarray.")
        if not np.issubdtype(x.dtype, np.floating):
            raise ValueError("Data must be floating point.")
        if x.ndim == 2 and x.shape[1] > 5:
            raise ValueError("Audio must have five channels or less.")
        if x.shape[0] < self.block_size * self.rate:
            raise ValueError("Audio must have length greater than the block size.")
        if x.ndim == 1:
            x = np.reshape(x, (x.shape[0], 1))
        nch, ns = x.shape[1], x.shape[0]
        for f in self._filters.values():
            for c in range(nch):
                x[:, c] = f.apply_filter(x[:, c])
        G = [1.0, 1.0, 1.0, 1.41, 1.41]
        T_g, gamma_a, step = self.block_size, -70.0, 1.0 - 0.75
        T = ns / self.rate
        nblocks = int(np.round(((T - T_g) / (T_g * step)))) + 1
        jr = np.arange(0, nblocks)
        z = np.zeros(shape=(nch, nblocks))
        for c in range(nch):
            for j in jr:
                lo = int(T_g * (j * step) * self.rate)
                hi = int(T_g * (j * step + 1) * self.rate)
                z[c, j] = (1.0 / (T_g * self.rate)) * np.sum(np.square(x[lo:hi, c]))
        with np.errstate(divide="ignore", invalid="ignore"):
            lj = [-0.691 + 10.0 * np.log10(np.sum([G[c] * z[c, j] for c in range(nch)])) for j in jr]
            J = [j for j, v in enumerate(lj) if v >= gamma_a]
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", category=RuntimeWarning)
                zavg = [np.mean([z[c, j] for j in J]) for c in range(nch)]
                gamma_r = -0.691 + 10.0 * np.log10(np.sum([G[c] * zavg[c] for c in range(nch)])) - 10.0
                J = [j for j, v in enumerate(lj) if (v > gamma_r and v > gamma_a)]
                zavg = np.nan_to_num(np.array([np.mean([z[c, j] for j in J]) for c in range(nch)]))
            return -0.691 + 10.0 * np.log10(np.sum([G[c] * zavg[c] for c in range(nch)]))
