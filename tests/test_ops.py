"""The per-stage operator surface (mastering_amd.ops, the reference's AME:117-227
helpers one at a time).  CPU: the identity / pass-through paths that never reach
the library, and argument checks.  GPU (through the C-ABI's mm_op_* entry
points): every vector of tests/golden/primitives.npz, which the reference's OWN
helpers produced (tests/golden/make_golden.py), within the tolerance written on
each check.

Tolerances: integer outputs (quantise, multiband int16) bit-exact except where a
floating-point stage before a truncation can land on the other side of an
integer (stated per test); f64 IIR outputs 1e-12 absolute (the look-back composes
tile carries in a different order than scipy's sequential loop); f32 tanh 2 ulp
(numpy's f32 tanh is not correctly rounded); everything else bit-exact."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, record_exact


@pytest.fixture(scope="module")
def prim():
    return np.load(os.path.join(GOLDEN, "primitives.npz"))


# ----------------------------------------------------------------- CPU
def test_identity_paths_do_not_copy():
    from mastering_amd import ops
    x = np.zeros((16, 2), np.float32)
    assert ops.apply_saturation(x, 0) is x  # AME:129
    m = np.zeros(16, np.float32)
    assert ops.apply_stereo_width(m, 1.5) is m  # AME:137
    assert ops.apply_eq_to_samples(m, 44100, {}) is m
    assert ops.apply_shelf_filter(m, 44100, 250, 0, "low") is m  # AME:171
    assert ops.apply_peak_filter(m, 44100, 1000, 0) is m  # AME:186
    y = ops.apply_eq_to_samples(x, 44100, {"bass_boost": 0.0})
    assert y is not x and y.dtype == np.float32 and np.array_equal(y, x)


def test_argument_checks():
    from mastering_amd import ops
    with pytest.raises(TypeError):
        ops.apply_saturation(np.zeros(4, np.int16), 30)
    with pytest.raises(ValueError):  # pyloudnorm valid_audio: shorter than one 0.4 s block
        ops.normalize_to_lufs(np.zeros((1000, 2), np.float32), 44100)

    class Seg24:
        sample_width, channels, frame_rate = 3, 2, 44100
    with pytest.raises(ValueError):
        ops.audio_segment_to_float_array(Seg24())


@pytest.mark.parametrize("pct", [30, 100, 1, 55.5])
def test_saturation_table_is_numpys_own(pct, oracle):
    """design.saturation_table (the exciter's int16-grid table the device gathers) is
    the reference expression evaluated by numpy: equal, bit for bit, to the oracle's
    apply_saturation on decoded PCM16 in the reference's [N, 2] layout, in random
    order and through a strided view (numpy's float32 tanh depends on the value only),
    and to the primitives fixture the reference's own helper produced."""
    from mastering_amd import design
    tab, key = design.saturation_table(pct)
    assert tab.dtype == np.float32 and tab.shape == (65536,) and key != 0
    rng = np.random.default_rng(7)
    pcm = rng.integers(-32768, 32768, size=(200_003, 2)).astype(np.int16)
    x = oracle.pcm_to_float(pcm)
    ref = oracle.saturation(x, pct)
    assert np.array_equal(tab[pcm.astype(np.int32) + 32768], ref)
    assert np.array_equal(tab[pcm[:, 1].astype(np.int32) + 32768], oracle.saturation(x[:, 1], pct))
    if pct == 30:
        prim = np.load(os.path.join(GOLDEN, "primitives.npz"))
        q = prim["prim_q"].astype(np.int32)
        assert np.array_equal(tab[q + 32768], prim["prim_sat30"])


# ----------------------------------------------------------------- GPU
class _Seg:
    """pydub-AudioSegment-like (the attributes AME's helpers touch)."""

    def __init__(self, data, channels, rate):
        self._data, self.channels, self.frame_rate, self.sample_width = data, channels, rate, 2

    def get_array_of_samples(self):
        import array
        return array.array("h", self._data)

    def _spawn(self, data):
        return _Seg(bytes(data), self.channels, self.frame_rate)


@pytest.mark.gpu
def test_pcm_conversions(prim):
    from mastering_amd import ops
    q = prim["prim_q"]
    x = ops.audio_segment_to_float_array(_Seg(q.tobytes(), 2, 44100))
    assert x.dtype == np.float32 and x.shape == q.shape and np.array_equal(x, q.astype(np.float32) / 32768)
    with np.errstate(invalid="ignore"):
        out = ops.float_array_to_audio_segment(prim["prim_quant_in"], _Seg(b"", 1, 44100))
    assert np.array_equal(np.frombuffer(out._data, np.int16), prim["prim_quant_out"])  # bit-exact


@pytest.mark.gpu
def test_saturation(prim):
    from mastering_amd import ops
    x = prim["prim_q"].astype(np.float32) / 32768
    for got_in, pct, key in [(x, 30, "prim_sat30"), (x * np.float32(3.0), 100, "prim_sat100")]:
        y = ops.apply_saturation(got_in, pct)
        ref = prim[key]
        assert y.dtype == ref.dtype == np.float32
        # on the int16 grid (|k| < 32768 after the x3): the table, numpy's own bits
        grid = (got_in * 32768 == np.trunc(got_in * 32768)) & (got_in >= -1) & (got_in < 1)
        assert grid.mean() > 0.3
        assert np.array_equal(y[grid], ref[grid]), np.mean(y[grid] == ref[grid])
        record_exact(np.mean(y == ref), "f32")
        ulp = np.spacing(np.abs(ref).astype(np.float32))
        assert np.all(np.abs(y - ref) <= 2 * ulp), np.max(np.abs(y - ref) / ulp)  # off the grid: tanhf, 2 ulp


@pytest.mark.gpu
@pytest.mark.parametrize("name,preset,rate", [("techno", "techno", 44100), ("rock", "rock", 44100),
                                              ("96k_dubstep", "dubstep", 96000)])
def test_eq(prim, name, preset, rate):
    from mastering_amd import EQ_PRESETS, ops
    x = prim["prim_q"].astype(np.float32) / 32768
    y = ops.apply_eq_to_samples(x, rate, EQ_PRESETS[preset])
    ref = prim[f"prim_eq_{name}"]
    assert y.dtype == ref.dtype == np.float64 and y.shape == ref.shape
    record_exact(np.mean(y == ref), "f64")
    assert np.max(np.abs(y - ref)) <= 1e-12


@pytest.mark.gpu
def test_shelf_and_peak_match_scipy(prim):
    """apply_shelf_filter / apply_peak_filter per channel == the reference's per-stage
    sosfilt chain (prim_eq_techno is their composition on each channel)."""
    from mastering_amd import EQ_PRESETS, ops
    st = EQ_PRESETS["techno"]
    x = prim["prim_q"].astype(np.float32) / 32768
    for c in range(2):
        y = ops.apply_shelf_filter(x[:, c], 44100, 250, st["bass_boost"], "low")
        y = ops.apply_peak_filter(y, 44100, 1000, -st["mid_cut"])
        y = ops.apply_peak_filter(y, 44100, 4000, st["presence_boost"])
        y = ops.apply_shelf_filter(y, 44100, 8000, st["treble_boost"], "high")
        assert y.dtype == np.float64 and np.max(np.abs(y - prim["prim_eq_techno"][:, c])) <= 1e-12


@pytest.mark.gpu
def test_width(prim):
    from mastering_amd import ops
    x = prim["prim_q"].astype(np.float32) / 32768
    y64 = ops.apply_stereo_width(x.astype(np.float64), 1.3)
    y32 = ops.apply_stereo_width(x, 0.7)
    assert y64.dtype == np.float64 and np.array_equal(y64, prim["prim_width13_f64"])  # bit-exact
    assert y32.dtype == np.float32 and np.array_equal(y32, prim["prim_width07_f32"])


@pytest.mark.gpu
def test_soft_limiter(prim):
    from mastering_amd import ops
    x64 = prim["prim_lim_in"].copy()
    x32 = prim["prim_lim_in"].astype(np.float32)
    assert ops.soft_limiter(x64) is x64 and np.array_equal(x64, prim["prim_lim_out_f64"])  # in place, bit-exact
    assert ops.soft_limiter(x32) is x32 and np.array_equal(x32, prim["prim_lim_out_f32"])
    strided = np.repeat(prim["prim_lim_in"][:, None], 2, axis=1)[:, 0]  # non-contiguous view
    ops.soft_limiter(strided)
    assert np.array_equal(strided, prim["prim_lim_out_f64"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["prim_mb_hot", "prim_mb_ragged", "prim_mb_mono48k"])
def test_multiband(prim, name):
    """int16 out of the crossover + pydub compressor + overlay: identical to the
    reference's vectors (the quantised crossover pass runs scipy's operation order; a
    look-back carry differing in its last bit next to an int16 boundary is the only
    way a sample could move), with the overlay's padded length exact."""
    from mastering_amd import ops
    a = prim[f"{name}_args"]
    pcm, ref = prim[f"{name}_in"], prim[f"{name}_out"]
    ch = 1 if pcm.ndim == 1 else 2
    seg = ops.apply_multiband_compressor(_Seg(pcm.tobytes(), ch, int(a[8])), a[0], a[1], a[2], a[3], a[4], a[5],
                                         low_crossover=a[6], high_crossover=a[7])
    got = np.frombuffer(seg._data, np.int16)
    got = got.reshape(-1, 2) if ch == 2 else got
    arr = ops.apply_multiband_compressor(pcm, *a[:6], low_crossover=a[6], high_crossover=a[7], frame_rate=int(a[8]))
    assert np.array_equal(arr, got)
    assert got.shape == ref.shape
    record_exact(np.mean(got == ref), "i16")
    assert np.array_equal(got, ref), np.mean(got == ref)  # measured: identical (scipy-order passes)
    assert np.sqrt(np.mean(((got.astype(np.float64) - ref) / 32768) ** 2)) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["prim_norm_f32", "prim_norm_f64_mono"])
def test_normalize_to_lufs(prim, name):
    """Loudness within the north star's 0.1 LU and the internal 4e-4 LU; the output
    (f64, = samples * np.float64 gain) then differs only by that gain ratio."""
    from mastering_amd import ops
    rate, target, L = prim[f"{name}_meta"]
    x = prim[f"{name}_in"]
    Lg = ops.integrated_loudness(x if x.ndim == 1 else x.mean(axis=1), int(rate))
    assert abs(Lg - L) <= 4e-4
    y = ops.normalize_to_lufs(x, int(rate), target)
    ref = prim[f"{name}_out"]
    assert y.dtype == ref.dtype == np.float64 and y.shape == ref.shape
    assert np.max(np.abs(y - ref)) <= 1e-4 * np.max(np.abs(ref))
