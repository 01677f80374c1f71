"""Parity at BASELINE.json's full single-GPU size (C2: one 5-min 44.1 kHz stereo
track, full chain) and its C4 orchestration, plus size-independent properties.
The oracle masters the whole track on the CPU in seconds, so the comparison is
direct.  Tolerances as in test_gpu_parity.py (north_star)."""
import threading

import numpy as np
import pytest

from test_gpu_parity import P_FULL, _check, _ThreadCollectives, rms_diff

pytestmark = pytest.mark.gpu

RATE = 44100
C2_SECONDS = 300


@pytest.fixture(scope="module")
def c2_track():
    from mastering_amd.synth import pink_noise_pcm16
    return pink_noise_pcm16(C2_SECONDS * RATE, RATE, 2, 0)  # bench.py's rank-0 track


@pytest.fixture(scope="module")
def c2_reference(oracle, c2_track):
    return oracle.master(c2_track, RATE, P_FULL, return_loudness=True)


# C2's identical-sample floor: bit-identical since round 6 (exciter codes, numpy-order
# loudness block energies); a K-weighting carry flip could move a few samples
# (test_gpu_parity.MIN_EXACT's note), so the floor leaves room for that alone
C2_MIN_EXACT = 0.9999


def test_c2_full_track_vs_oracle(c2_track, c2_reference):
    from mastering_amd import master_pcm
    out, info = master_pcm(c2_track, RATE, P_FULL)
    ref, L = c2_reference
    _, exact = _check(out, info, ref, L, min_exact=C2_MIN_EXACT)
    print(f"C2 full track: identical int16 samples {exact:.7f} (floor {C2_MIN_EXACT}), "
          f"comp_iters {info['comp_iters']}")


def test_c2_deterministic(c2_track):
    """Same input, same bits: the look-back carries, the Jacobi sweeps and the loudness
    reductions run in fixed orders regardless of block scheduling."""
    from mastering_amd import master_pcm
    a, ia = master_pcm(c2_track, RATE, P_FULL)
    b, ib = master_pcm(c2_track, RATE, P_FULL)
    assert np.array_equal(a, b)
    assert ia["loudness"] == ib["loudness"] and ia["comp_iters"] == ib["comp_iters"]


def test_c4_time_sharded_full_track(c2_track, c2_reference):
    """The 300 s track split over two ranks (threads with their own contexts on one
    GPU): stitched output matches the oracle; every rank gates the same loudness."""
    import torch

    from mastering_amd import distributed as D
    from mastering_amd import native
    world = 2
    coll = _ThreadCollectives(world)
    outs, infos, errs = [None] * world, [None] * world, []

    def rank_main(r):
        try:
            plan = D.plan_time_shards(c2_track.shape[0], RATE, 2, world, r)
            be = D.GpuBackend(native.Context(0))
            x = torch.from_numpy(c2_track[plan.in_lo:plan.in_hi].astype(np.float32) / 32768).cuda()
            out = torch.empty((plan.frames, 2), dtype=torch.int16, device="cuda")
            infos[r] = D.master_time_sharded(be, plan, P_FULL, x.data_ptr(), out.data_ptr(), coll.bind(r))
            be.ctx.sync()
            outs[r] = out.cpu().numpy()
            be.ctx.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            coll.bar.abort()

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errs, errs
    assert infos[0]["loudness"] == infos[1]["loudness"]
    ref, L = c2_reference
    _check(np.concatenate(outs), infos[0], ref, L)


def test_c2_chunk_independence(oracle, c2_track):
    """AME:48-77 processes every 30 s chunk on its own: the staged pre-gain mix of a
    chunk inside the full track equals the oracle's mix of that chunk alone (exciter
    off, so the only differences are last-bit IIR carries)."""
    from test_gpu_parity import _oracle_mix, _staged_mix
    params = dict(P_FULL, saturation=0)
    mix = _staged_mix(c2_track, params)
    bounds = oracle.chunk_ranges(c2_track.shape[0], RATE)
    for ci in (0, len(bounds) // 2, len(bounds) - 1):
        s, e = bounds[ci]
        ref = _oracle_mix(oracle, c2_track[s:e], params)
        assert np.mean(mix[s:e] == ref) >= 0.999999, (ci, np.mean(mix[s:e] == ref))
        assert rms_diff(mix[s:e], ref) <= 1e-6
