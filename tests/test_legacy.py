"""The legacy engine profile (reference root main.py).

CPU: the legacy oracle (oracle/legacy_oracle.py) against the vectors that the
reference's main.py itself produced (tests/golden/make_golden_legacy.py), bit for
bit.  GPU: mastering_amd.legacy (HIP operators) against the same vectors:
end-to-end PCM RMS <= 1e-5 (north_star tolerance), per-stage f64 filters 1e-12,
f32 tanh stages 2 ulp, int16 stages >= 99.99 % identical."""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

CASES = sorted(glob.glob(os.path.join(GOLDEN, "legacy_*_*s.npz")))


@pytest.fixture(scope="module")
def lo():
    from oracle import legacy_oracle
    from oracle import mastering_oracle as mo
    mo.build()
    return legacy_oracle


@pytest.fixture(scope="module")
def prim():
    return np.load(os.path.join(GOLDEN, "legacy_primitives.npz"))


def test_cases_present():
    assert len(CASES) == 4


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_legacy_oracle_matches_reference(lo, path):
    d = np.load(path)
    got = lo.master(d["pcm"], int(d["rate"]), json.loads(str(d["settings"])))
    assert got.shape == d["out"].shape and np.array_equal(got, d["out"])


def test_legacy_oracle_primitives(lo, prim):
    x = prim["lp_q"].astype(np.float32) / 32768
    sr = 44100
    assert np.array_equal(lo.saturation(x, 40.0), prim["lp_sat40"])
    assert np.array_equal(lo.shelf(x[:, 0], sr, 250, 4.0, "low"), prim["lp_shelf_low_boost"])
    assert np.array_equal(lo.shelf(x[:, 1], sr, 8000, -3.0, "high"), prim["lp_shelf_high_cut"])
    assert np.array_equal(lo.peak(x[:, 0], sr, 1000, -2.0), prim["lp_peak_cut"])
    from test_legacy_settings import LEGACY_FULL
    assert np.array_equal(lo.equalize(x, sr, LEGACY_FULL), prim["lp_eq_full"])
    assert np.array_equal(lo.soft_limiter(prim["lp_lim_in"]), prim["lp_lim_out"])
    assert np.array_equal(lo.multiband(prim["lp_q"], sr, LEGACY_FULL), prim["lp_mb_out"])


def _ulp_close(a, b, n):
    return np.all(np.abs(a - b) <= n * np.spacing(np.abs(b).astype(b.dtype)))


@pytest.mark.gpu
def test_legacy_primitives_on_gpu(prim):
    from mastering_amd import legacy
    from test_legacy_settings import LEGACY_FULL
    x = prim["lp_q"].astype(np.float32) / 32768
    sr = 44100
    y = legacy.apply_saturation(x, 40.0)
    assert y.dtype == np.float32 and _ulp_close(y, prim["lp_sat40"], 2)
    for got, key in [(legacy.apply_shelf_filter(x[:, 0], sr, 250, 4.0, "low"), "lp_shelf_low_boost"),
                     (legacy.apply_shelf_filter(x[:, 1], sr, 8000, -3.0, "high"), "lp_shelf_high_cut"),
                     (legacy.apply_peak_filter(x[:, 0], sr, 1000, -2.0), "lp_peak_cut"),
                     (legacy.apply_eq_to_samples(x, sr, LEGACY_FULL), "lp_eq_full")]:
        assert got.dtype == np.float64 and got.shape == prim[key].shape
        assert np.max(np.abs(got - prim[key])) <= 1e-12, key
    lim = prim["lp_lim_in"].copy()
    assert legacy.soft_limiter(lim) is lim
    assert np.max(np.abs(lim - prim["lp_lim_out"])) <= 2 * np.spacing(1.0)  # f64 tanh: 2 ulp
    mb = legacy.apply_multiband_compressor(prim["lp_q"], LEGACY_FULL, frame_rate=sr)
    assert mb.shape == prim["lp_mb_out"].shape and np.mean(mb == prim["lp_mb_out"]) >= 0.9999


@pytest.mark.gpu
@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_legacy_end_to_end_on_gpu(tmp_path, path):
    """main.py's whole job through files: PCM16 WAV in, legacy.process, WAV out."""
    from mastering_amd import legacy, wavio
    d = np.load(path)
    src, dst = tmp_path / "in.wav", tmp_path / "out.wav"
    wavio.write_wav(str(src), d["pcm"], int(d["rate"]))
    legacy.process(str(src), str(dst), json.loads(str(d["settings"])))
    got, rate = wavio.read_wav(str(dst))
    ref = d["out"]
    assert rate == int(d["rate"]) and got.shape == ref.shape
    rms = float(np.sqrt(np.mean(((got.astype(np.float64) - ref) / 32768.0) ** 2)))
    assert rms <= 1e-5, rms
