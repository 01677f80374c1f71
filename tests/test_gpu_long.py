"""Track length on one GPU: a track above round 3's single-plane envelope-solve
limit (~511 M frames: ~3.2 h at 44.1 kHz, ~89 min at 96 kHz) runs through the
device-resident entry point (mm_master_device) — the compressor's M plane is now
one plane per 30 s chunk (chunks are independent, AME:48-77), so no length below
2^31 frames is refused (tests/test_abi.py checks the planning arithmetic there).

Checked, as the whole-track oracle would take minutes at this size:
  * the gated loudness against the oracle's pyloudnorm restatement of the
    device's own pre-gain mix (the K-weighting line runs across all 200 chunks);
  * three sampled chunks' pre-gain mixes against the oracle chain (exciter, EQ,
    width, int16, crossover, pydub compressor, overlay: AME:55-80), with the
    identical-sample floor of test_gpu_parity.py;
  * those chunks' output against the oracle's gain + soft limiter + int16
    (AME:84-89) applied to the device mix."""
import ctypes

import numpy as np
import pytest

from conftest import record_exact
from test_gpu_parity import MIN_EXACT, P_FULL, rms_diff

pytestmark = pytest.mark.gpu


def _oracle_chunk_mix(oracle, pcm, rate, params):
    thr, rat = oracle.multiband_params(params)
    x = oracle.saturation(oracle.pcm_to_float(pcm), params.get("saturation", 0))
    y = oracle.quantize(oracle.stereo_width(oracle.equalize(x, rate, params), params.get("width", 1.0)))
    return oracle.multiband(y, rate, thr, rat)


@pytest.mark.timeout(900)
def test_100_min_96k_track_on_one_gpu(oracle):
    import torch

    from mastering_amd import Job, engine, native
    from mastering_amd.synth import pink_noise_chunks
    rate, nch = 96000, 200
    CF = 30 * rate
    pcm = pink_noise_chunks(0, nch, rate, 2, track=11)
    N = pcm.shape[0]
    assert N == 576_000_000  # > 511 M frames
    job = Job(N, rate, 2, P_FULL)
    ctx = native.context(0)
    x = torch.from_numpy(pcm).cuda().to(torch.float32).div_(32768)
    out = torch.empty((job.frames_proc, 2), dtype=torch.int16, device="cuda")
    res = native.MMResult()
    engine.master_device(ctx, job, x.data_ptr(), out.data_ptr(), res)
    ctx.sync()
    del x
    print(f"100 min @ 96 kHz: L={res.loudness:.6f} comp_iters={res.comp_iters}", flush=True)
    mix = np.empty((job.frames_proc, 2), np.int16)
    ctx.check(ctx.lib.mm_read_mix(ctx.ptr, mix.ctypes.data_as(ctypes.POINTER(ctypes.c_int16))), "read_mix")
    got = out.cpu().numpy()
    del out
    # loudness of the device's mix, pyloudnorm restated (as normalize_to_lufs)
    L = oracle.integrated_loudness(oracle.pcm_to_float(mix).mean(axis=1), rate)
    print(f"oracle L of the device mix: {L:.6f} (|dL| {abs(L - res.loudness):.2e})", flush=True)
    assert abs(res.loudness - L) <= 4e-4
    gain = 10.0 ** ((P_FULL["lufs"] - res.loudness) / 20.0)
    assert res.gain_linear == pytest.approx(gain, rel=1e-12)
    for c in (0, nch // 2 + 1, nch - 1):
        s, e = c * CF, (c + 1) * CF
        ref = _oracle_chunk_mix(oracle, pcm[s:e], rate, P_FULL)
        exact = float(np.mean(mix[s:e] == ref))
        record_exact(exact, "mix")
        print(f"chunk {c}: mix identical {exact:.7f}", flush=True)
        assert exact >= MIN_EXACT and rms_diff(mix[s:e], ref) <= 1e-5
        with np.errstate(invalid="ignore"):  # (the reference's gain is an np.float64: f64 from here, AME:86)
            fin = oracle.quantize(oracle.soft_limiter(oracle.pcm_to_float(mix[s:e]) * np.float64(res.gain_linear)))
        assert np.array_equal(got[s:e], fin)
