"""The WAV file path of the C-ABI (mm_wav_probe / mm_master_wav):
RIFF parsing against mastering_amd.wavio on the CPU (no GPU needed: a NULL context),
and on the GPU every reference golden pushed through process() as a WAV file and
compared with the reference's own exported output (AME:43-98 end to end)."""
import ctypes
import glob
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN


def _probe(path):
    from mastering_amd import native
    lib = native.load()
    info = native.MMWavInfo()
    rc = lib.mm_wav_probe(None, os.fsencode(str(path)), ctypes.byref(info))
    return rc, info


def _extensible_wav(path, x, rate, subformat):
    """WAVE_FORMAT_EXTENSIBLE header + a LIST chunk with odd size before the data."""
    ch = x.shape[1] if x.ndim > 1 else 1
    bits = x.dtype.itemsize * 8
    ba = ch * bits // 8
    payload = x.tobytes()
    fmt = struct.pack("<HHIIHH", 0xFFFE, ch, rate, rate * ba, ba, bits) + struct.pack("<HHI", 22, bits, 3)
    fmt += struct.pack("<H", subformat) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
    lst = b"LIST" + struct.pack("<I", 3) + b"abc\x00"
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + lst + b"data" + struct.pack("<I", len(payload))
    body += payload
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_probe_matches_wavio(tmp_path):
    from mastering_amd import wavio
    rng = np.random.default_rng(3)
    cases = {
        "s16.wav": rng.integers(-32768, 32767, (1001, 2), dtype=np.int16),
        "m16.wav": rng.integers(-32768, 32767, 777, dtype=np.int16),
        "f32.wav": rng.uniform(-1, 1, (500, 2)).astype(np.float32),
    }
    for name, x in cases.items():
        p = tmp_path / name
        wavio.write_wav(str(p), x, 48000)
        rc, info = _probe(p)
        assert rc == 0, name
        y, rate = wavio.read_wav(str(p))
        ch = 1 if y.ndim == 1 else y.shape[1]
        assert (info.frames, info.rate, info.channels) == (y.shape[0], rate, ch)
        assert (info.format, info.bits) == ((1, 16) if y.dtype == np.int16 else (3, 32))
        assert info.data_offset == 44
    p = tmp_path / "ext.wav"
    _extensible_wav(str(p), cases["f32.wav"], 44100, 3)
    rc, info = _probe(p)
    assert rc == 0 and info.format == 3 and info.frames == 500 and info.data_offset == 44 + 24 + 12
    y, _ = wavio.read_wav(str(p))
    assert y.shape == (500, 2)


def test_probe_rejects_bad_files(tmp_path):
    from mastering_amd import wavio
    p = tmp_path / "junk.wav"
    p.write_bytes(b"not a wav file at all")
    assert _probe(p)[0] < 0
    assert _probe(tmp_path / "missing.wav")[0] < 0
    x = np.zeros((10, 2), np.int16)
    q = tmp_path / "s24.wav"
    wavio.write_wav(str(q), x, 44100)
    data = bytearray(q.read_bytes())
    data[34:36] = struct.pack("<H", 24)  # claim 24-bit
    q.write_bytes(bytes(data))
    assert _probe(q)[0] < 0
    # a data chunk that claims more than the file holds is truncated to whole frames
    t = tmp_path / "trunc.wav"
    wavio.write_wav(str(t), np.ones((100, 2), np.int16), 44100)
    t.write_bytes(t.read_bytes()[:-5])
    rc, info = _probe(t)
    assert rc == 0 and info.frames == 98


GOLDEN_CASES = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz")) if not p.endswith("primitives.npz") and not os.path.basename(p).startswith("legacy"))


def _golden(path):
    d = np.load(path)
    return d["pcm"], int(d["rate"]), json.loads(str(d["settings"])), d["out"], float(d["loudness"])


def check_against_golden(got, info, ref, L):
    """north_star tolerances: PCM RMS <= 1e-5 (decoded /32768), |dL| <= 0.1 LU; internal
    loudness bar 4e-4 LU."""
    assert got.shape == ref.shape and got.dtype == np.int16
    rms = float(np.sqrt(np.mean(((got.astype(np.float64) - ref) / 32768.0) ** 2))) if ref.size else 0.0
    assert rms <= 1e-5, rms
    if np.isfinite(L):
        assert abs(info["loudness"] - L) <= 4e-4
    return rms


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN_CASES, ids=[os.path.basename(p)[:-4] for p in GOLDEN_CASES])
def test_process_wav_matches_reference_golden(tmp_path, path):
    """AME:43 decode -> chain -> AME:98 export, end to end through files: the golden
    input written as the PCM16 WAV the reference decoded, process() -> the output
    WAV against the reference's own exported samples and measured loudness."""
    from mastering_amd import process, wavio
    pcm, rate, settings, ref, L = _golden(path)
    src, dst = tmp_path / "in.wav", tmp_path / "out.wav"
    wavio.write_wav(str(src), pcm, rate)
    info = process(str(src), str(dst), settings)
    got, r2 = wavio.read_wav(str(dst))
    assert r2 == rate
    check_against_golden(got, info, ref, L)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["full_4s", "mono_hot_2s", "ragged_hot"])
def test_process_float_wav_and_float_output(tmp_path, name):
    """A 32-bit float WAV holding the same samples (PCM16 / 32768) masters to the same
    result, and output_format='f32' writes that result / 32768.  (The reference would
    decode a float WAV through ffmpeg as pcm_s32le with sample_width 4, which AME:121,
    125 mis-scale: DESIGN.md §2 documents this deliberate deviation.)"""
    from mastering_amd import process, wavio
    pcm, rate, settings, ref, L = _golden(os.path.join(GOLDEN, name + ".npz"))
    src, dst = tmp_path / "in.wav", tmp_path / "out.wav"
    wavio.write_wav(str(src), pcm.astype(np.float32) / 32768, rate)
    info = process(str(src), str(dst), dict(settings, output_format="f32"))
    got, _ = wavio.read_wav(str(dst))
    assert got.dtype == np.float32
    assert np.array_equal(got * 32768, np.round(got * 32768))  # on the int16 grid
    check_against_golden((got * 32768).astype(np.int16), info, ref, L)


@pytest.mark.gpu
def test_master_wav_streams_large_files(tmp_path, oracle):
    """70 s stereo PCM16 = 12 MB: crosses the 8 MB staging buffers in both directions;
    the file result against the oracle on the same samples."""
    from mastering_amd import process, wavio
    from mastering_amd.synth import pink_noise_pcm16
    P = {"saturation": 10, "multiband": True, "lufs": -16.0}
    pcm = pink_noise_pcm16(70 * 44100, 44100, 2, 8)
    src, dst = tmp_path / "in.wav", tmp_path / "out.wav"
    wavio.write_wav(str(src), pcm, 44100)
    info = process(str(src), str(dst), P)
    got, _ = wavio.read_wav(str(dst))
    ref, L = oracle.master(pcm, 44100, P, return_loudness=True)
    check_against_golden(got, info, ref, L)


@pytest.mark.gpu
def test_process_raises_value_error_on_bad_input(tmp_path):
    from mastering_amd import process
    p = tmp_path / "junk.wav"
    p.write_bytes(b"RIFF\x04\x00\x00\x00WAVE")
    with pytest.raises(ValueError):
        process(str(p), str(tmp_path / "o.wav"), {})
