"""pyloudnorm's block energies in numpy's own reduction order (CPU, no GPU).

pyloudnorm computes z_j = (1/(0.4 rate)) * np.sum(np.square(x[lo:hi])) on the
float32 K-weighted line (AME:218): an f32 sum whose bits depend on numpy's order
(8192-element buffer chunks summed in order, each chunk a pairwise tree with
eight-accumulator leaves of <= 128 elements).  The device's kw_blocks_kernel runs a
program the library builds per block length; mm_np_sum_f32 evaluates that same
program on the host, so these tests pin the device's summation order to np.sum
bit for bit."""
import ctypes

import numpy as np
import pytest

LENGTHS = [0, 1, 5, 7, 8, 9, 100, 127, 128, 129, 136, 200, 1000, 4410, 8191, 8192, 8193, 8200, 9000,
           16384, 16385, 17640, 17641, 19200, 38400, 76800, 8820, 6615, 14112]


def np_sum_lib(x):
    from mastering_amd import native
    lib = native.load()
    out = ctypes.c_float()
    x = np.ascontiguousarray(x, dtype=np.float32)
    assert lib.mm_np_sum_f32(x.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), x.size, ctypes.byref(out)) == 0
    return np.float32(out.value)


@pytest.mark.parametrize("n", LENGTHS)
def test_program_equals_np_sum(n):
    rng = np.random.default_rng(n)
    for scale in (1e-3, 0.3, 1.0):
        x = np.square((rng.standard_normal(n) * scale).astype(np.float32))
        assert np_sum_lib(x) == np.sum(x), (n, scale)


def test_pyloudnorm_block_slices():
    """The reference's own expression on column slices of an (N, 1) float32 line at
    the blocks design.loudness_blocks produces (44.1 and 96 kHz, clamped last blocks)."""
    from mastering_amd import design
    rng = np.random.default_rng(3)
    for rate, seconds in ((44100, 3.7), (96000, 2.05), (48000, 1.0)):
        frames = int(seconds * rate)
        x = (rng.standard_normal((frames, 1)) * 0.05).astype(np.float32)
        nb, lo, hi, _, scale = design.loudness_blocks(frames, rate)
        for j in range(nb):
            ref = (1.0 / (0.4 * rate)) * np.sum(np.square(x[lo[j]:hi[j], 0]))  # pyloudnorm, NEP 50: f32
            got = np.float32(scale) * np_sum_lib(np.square(x[lo[j]:hi[j], 0]))
            assert ref.dtype == np.float32 and got == ref, (rate, j)
