"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own code.

Run here only (the reference tree is not on the GPU box):

    python tests/golden/make_golden.py

`worker/audio_mastering_engine.py` ("AME") imports pydub, pyloudnorm and
google.cloud.storage, none of which are installed.  We register stand-in modules
whose contents are the restatements in oracle/thirdparty_restated.py (pydub
0.25.1 AudioSegment subset + compress_dynamic_range, pyloudnorm 0.1.1 Meter) and a
local in-memory fake of the GCS client, then call the reference's own
`process_audio_from_gcs` end to end and its own per-stage helpers.  Everything
AME itself does (chunking, dtype flow, EQ/crossover design, quantisation,
concat, limiter) is therefore the reference's code; the third-party boundary is
restated ("parity unpinned" there — the reference has no tests).

Each fixture is an .npz of data only: inputs, settings (JSON), expected outputs
and the loudness the reference measured.
"""
from __future__ import annotations

import importlib.util
import io
import json
import os
import sys
import types
import wave

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "python-audio-mastering_amd"))

from oracle import thirdparty_restated as tp  # noqa: E402
from mastering_amd.synth import pink_noise_pcm16  # noqa: E402

AME_PATH = "/root/reference/worker/audio_mastering_engine.py"

# --------------------------------------------------------------------------
# stand-in third-party modules
# --------------------------------------------------------------------------
_BUCKETS: dict[str, dict[str, bytes]] = {}
_LOUDNESS: list[float] = []


class _Blob:
    def __init__(self, bucket, name):
        self.b, self.name = bucket, name

    def download_to_file(self, f):
        f.write(_BUCKETS[self.b][self.name])

    def upload_from_file(self, f, content_type=None):
        _BUCKETS[self.b][self.name] = f.read()

    def upload_from_string(self, s):
        _BUCKETS[self.b][self.name] = s.encode() if isinstance(s, str) else s


class _Bucket:
    def __init__(self, name):
        self.name = name
        _BUCKETS.setdefault(name, {})

    def blob(self, name):
        return _Blob(self.name, name)


class _Client:
    def bucket(self, name):
        return _Bucket(name)


class _RecordingMeter(tp.Meter):
    def integrated_loudness(self, data):
        L = super().integrated_loudness(data)
        _LOUDNESS.append(float(L))
        return L


def load_reference():
    mods = {n: types.ModuleType(n) for n in
            ["pydub", "pydub.effects", "pyloudnorm", "google", "google.cloud", "google.cloud.storage"]}
    mods["pydub"].AudioSegment = tp.AudioSegment
    mods["pydub.effects"].compress_dynamic_range = tp.compress_dynamic_range
    mods["pyloudnorm"].Meter = _RecordingMeter
    mods["google.cloud.storage"].Client = _Client
    mods["google.cloud"].storage = mods["google.cloud.storage"]
    mods["google"].cloud = mods["google.cloud"]
    sys.modules.update(mods)
    spec = importlib.util.spec_from_file_location("reference_ame", AME_PATH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def wav_bytes(pcm: np.ndarray, rate: int) -> bytes:
    ch = 1 if pcm.ndim == 1 else pcm.shape[1]
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(np.ascontiguousarray(pcm, dtype="<i2").tobytes())
    return buf.getvalue()


def read_wav(b: bytes):
    with wave.open(io.BytesIO(b), "rb") as w:
        ch, n = w.getnchannels(), w.getnframes()
        d = np.frombuffer(w.readframes(n), dtype="<i2")
    return d.reshape(-1, ch) if ch > 1 else d


def run_reference(ame, pcm, rate, settings):
    _BUCKETS.clear()
    _LOUDNESS.clear()
    _BUCKETS["bkt"] = {"in/track.wav": wav_bytes(pcm, rate)}
    ame.process_audio_from_gcs("gs://bkt/in/track.wav", dict(settings))
    out = read_wav(_BUCKETS["bkt"]["processed/mastered_track.wav"])
    assert "processed/mastered_track.wav.complete" in _BUCKETS["bkt"]
    return out, (_LOUDNESS[-1] if _LOUDNESS else None)


P_EQLUFS = {"bass_boost": 2.0, "mid_cut": 0.0, "presence_boost": 3.5, "treble_boost": 2.5,
            "saturation": 0, "width": 1.0, "multiband": False, "lufs": -14.0}
P_FULL = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
          "saturation": 30, "width": 1.3, "multiband": True, "lufs": -14.0}
# thresholds near each band's median level so attack, hold and release all fire
P_HOT = dict(P_FULL, low_thresh=-16.0, mid_thresh=-21.0, high_thresh=-27.0)


def cases():
    sr = 44100
    yield "eqlufs_3s", pink_noise_pcm16(3 * sr, sr, 2, 1), sr, P_EQLUFS
    yield "full_4s", pink_noise_pcm16(4 * sr, sr, 2, 2), sr, P_FULL
    yield "hot_4s", pink_noise_pcm16(4 * sr, sr, 2, 3), sr, P_HOT
    yield "nolufs_dubstep_3s", pink_noise_pcm16(3 * sr, sr, 2, 4), sr, dict(
        P_HOT, bass_boost=5.0, mid_cut=4.0, presence_boost=2.0, treble_boost=3.5, width=0.5, lufs=None)
    yield "mono_hot_2s", pink_noise_pcm16(2 * sr, sr, 1, 5), sr, P_HOT
    yield "ragged_hot", pink_noise_pcm16(2 * sr + 22050 + 13, sr, 2, 6), sr, dict(P_HOT, lufs=-16.0)
    yield "loud_sat100", pink_noise_pcm16(2 * sr, sr, 2, 7, level_dbfs=-4.0), sr, dict(
        P_HOT, saturation=100, bass_boost=6.0, lufs=-6.0, mid_thresh=-12.0, low_thresh=-10.0)
    yield "noeq_width_2s", pink_noise_pcm16(2 * sr, sr, 2, 8), sr, {
        "saturation": 20, "width": 1.6, "multiband": True, "lufs": -12.0}
    yield "rock_nomb_2s", pink_noise_pcm16(2 * sr, sr, 2, 9), sr, {
        "bass_boost": 1.5, "mid_cut": -2.0, "presence_boost": 2.5, "treble_boost": 1.0,
        "saturation": 10, "width": 1.2, "multiband": False, "lufs": -14.0}
    yield "hot_96k_1s", pink_noise_pcm16(96000, 96000, 2, 10), 96000, P_HOT
    yield "silence_1s", np.zeros((sr, 2), np.int16), sr, P_FULL
    yield "chunks_hot_31s", pink_noise_pcm16(31 * sr, sr, 2, 11), sr, P_HOT


def primitives(ame):
    """Per-stage vectors from the reference's own helpers (AME:117-227)."""
    rng = np.random.default_rng(7)
    sr = 44100
    q = pink_noise_pcm16(8192, sr, 2, 20)
    x = q.astype(np.float32) / 32768
    d = {"prim_q": q}
    d["prim_sat30"] = ame.apply_saturation(x, 30)
    d["prim_sat100"] = ame.apply_saturation(x * np.float32(3.0), 100)
    for name, st in [("techno", ame.EQ_PRESETS["techno"]), ("rock", ame.EQ_PRESETS["rock"])]:
        d[f"prim_eq_{name}"] = ame.apply_eq_to_samples(x, sr, st)
    d["prim_eq_96k_dubstep"] = ame.apply_eq_to_samples(x, 96000, ame.EQ_PRESETS["dubstep"])
    d["prim_width13_f64"] = ame.apply_stereo_width(x.astype(np.float64), 1.3)
    d["prim_width07_f32"] = ame.apply_stereo_width(x, 0.7)
    lim = rng.standard_normal(4096) * 1.2
    d["prim_lim_in"] = lim
    d["prim_lim_out_f64"] = ame.soft_limiter(lim.copy())
    d["prim_lim_out_f32"] = ame.soft_limiter(lim.astype(np.float32))

    class _Seg:
        sample_width, channels = 2, 2

        def _spawn(self, data):
            return data

    edge = np.array([1.0, 32767.9 / 32768, -1.0, -0.7 / 32768, np.nan, 1.5, -2.0, 0.49999], np.float64)
    d["prim_quant_in"] = edge
    d["prim_quant_out"] = np.frombuffer(ame.float_array_to_audio_segment(edge, _Seg()), np.int16)
    # apply_multiband_compressor (AME:196-210) on pydub segments: 2.5 s stereo with
    # thresholds where every branch fires, a ragged 8192-frame chunk (overlay pads it
    # to 186 ms = 8202 frames) and mono at 48 kHz with custom crossovers
    mb = [("prim_mb_hot", pink_noise_pcm16(110250, sr, 2, 21), sr, (-16.0, 6.0, -21.0, 3.0, -27.0, 4.0), {}),
          ("prim_mb_ragged", q, sr, (-25.0, 6.0, -20.0, 3.0, -15.0, 4.0), {}),
          ("prim_mb_mono48k", pink_noise_pcm16(72000, 48000, 1, 22), 48000, (-18.0, 4.0, -24.0, 2.0, -30.0, 8.0),
           {"low_crossover": 300, "high_crossover": 5000})]
    for name, pcm, rate, args, kw in mb:
        ch = 1 if pcm.ndim == 1 else 2
        seg = tp.AudioSegment(np.ascontiguousarray(pcm, dtype="<i2").tobytes(), 2, rate, ch)
        out = ame.apply_multiband_compressor(seg, *args, **kw)
        o = np.frombuffer(out._data, np.int16)
        d[f"{name}_in"] = pcm
        d[f"{name}_out"] = o.reshape(-1, 2) if ch == 2 else o
        d[f"{name}_args"] = np.array(list(args) + [kw.get("low_crossover", 250), kw.get("high_crossover", 4000), rate],
                                     np.float64)
    # normalize_to_lufs (AME:212-222): f32 stereo (f64 out) and f64 mono
    for name, x, rate, target in [("prim_norm_f32", pink_noise_pcm16(3 * sr, sr, 2, 23).astype(np.float32) / 32768,
                                   sr, -14.0),
                                  ("prim_norm_f64_mono", rng.standard_normal(2 * 48000) * 0.05, 48000, -16.0)]:
        _LOUDNESS.clear()
        d[f"{name}_in"] = x
        d[f"{name}_out"] = ame.normalize_to_lufs(x.copy(), rate, target)
        d[f"{name}_meta"] = np.array([rate, target, _LOUDNESS[-1]], np.float64)
    return d


def main():
    ame = load_reference()
    meta = {}
    only = set(sys.argv[1:])
    if only == {"primitives"}:  # per-stage vectors only
        np.savez_compressed(os.path.join(HERE, "primitives.npz"), **primitives(ame))
        return
    for name, pcm, rate, st in cases():
        if only and name not in only:
            continue
        out, L = run_reference(ame, pcm, rate, st)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), pcm=pcm, rate=rate, out=out,
                            settings=json.dumps(st), loudness=np.nan if L is None else L)
        meta[name] = {"frames_in": int(pcm.shape[0]), "frames_out": int(out.shape[0]), "rate": rate,
                      "loudness": L}
        print(name, meta[name], flush=True)
    if not only:
        np.savez_compressed(os.path.join(HERE, "primitives.npz"), **primitives(ame))
        # short audio with a loudness target must raise (pyloudnorm valid_audio)
        try:
            run_reference(ame, pink_noise_pcm16(10000, 44100, 2, 30), 44100, P_EQLUFS)
            meta["short_raises"] = False
        except ValueError as e:
            meta["short_raises"] = str(e)
        with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
