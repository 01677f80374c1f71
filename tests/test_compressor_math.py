"""The compressor's two hand-made elementary functions, evaluated on the device
through mm_check_compressor_math:

* exp10_tab (csrc/compressor.hip), the gain 10^y of comp_apply for y = -att/20 in
  [-3, 0]: within 2 ulp of numpy's 10.0 ** y (libm pow) on a dense grid and on
  random points, and exactly 1.0 at y = 0 and y = -0 (the identity gain pydub
  skips, AME:207-209);
* rms_exact1, comp_rms's audioop.rms: isqrt(floor(S / n)) exactly, at the edges
  S = n k^2 - 1, n k^2, n k^2 + 1 for every k <= 32768 and the window sample
  counts n the product uses (look * channels, and the shorter windows at a chunk
  start).  The f32 estimate's error budget (2^-22 against a 2^-19 bias) is what
  makes one upward correction enough; these edges are where it would fail."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from mastering_amd import native
    c = native.Context()
    yield c
    c.close()


def _run(ctx, what, a, b=None):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b if b is not None else np.zeros(1), np.float64)
    out = np.empty_like(a)
    P = ctypes.POINTER(ctypes.c_double)
    ctx.check(ctx.lib.mm_check_compressor_math(ctx.ptr, what, a.ctypes.data_as(P), b.ctypes.data_as(P), a.size,
                                               out.ctypes.data_as(P)), "mm_check_compressor_math")
    return out


def _ulps(x, y):
    """ulp distance of positive doubles (their bit patterns are ordered)."""
    return np.abs(x.view(np.int64) - y.view(np.int64))


def test_exp10_tab_within_two_ulp(ctx):
    rng = np.random.default_rng(7)
    y = np.concatenate([np.linspace(-3.0, 0.0, 2_000_001), -3.0 * rng.random(1_000_000),
                        -np.logspace(-300, 0, 20_001) * 3.0])
    got = _run(ctx, 0, y)
    ref = np.power(10.0, y)
    d = _ulps(got, ref)
    assert d.max() <= 2, (d.max(), y[np.argmax(d)], got[np.argmax(d)], ref[np.argmax(d)])


def test_exp10_tab_exact_at_zero(ctx):
    got = _run(ctx, 0, np.array([0.0, -0.0]))
    assert got[0] == 1.0 and got[1] == 1.0, got


def _isqrt(q):
    r = np.floor(np.sqrt(q.astype(np.float64))).astype(np.int64)
    for _ in range(2):
        r = np.where((r + 1) * (r + 1) <= q, r + 1, r)
        r = np.where(r * r > q, r - 1, r)
    return r


@pytest.mark.parametrize("n", [1, 2, 3, 5, 64, 220, 441, 882, 1323, 2205, 4410, 8820, 19200])
def test_rms_exact1_edges(ctx, n):
    k = np.arange(0, 32769, dtype=np.int64)
    S = np.concatenate([n * k * k - 1, n * k * k, n * k * k + 1])
    S = S[(S >= 0) & (S <= n * 32768 * 32768)]
    got = _run(ctx, 1, S.astype(np.float64), np.full(S.size, float(n)))
    ref = _isqrt(S // n)
    bad = np.flatnonzero(got.astype(np.int64) != ref)
    assert bad.size == 0, (n, S[bad[:5]], got[bad[:5]], ref[bad[:5]])
