"""Multi-rank paths on CPU (gloo): the time-sharded orchestration of
mastering_amd/distributed.py (BASELINE C4) driven by an oracle-backed rank backend,
and the file sharding of C3/C5.  The GPU backend (C-ABI) of the same orchestration
is covered by tests/test_gpu_parity.py::test_time_sharded_on_one_gpu."""
import os
import socket

import numpy as np
import pytest
import scipy.signal

from conftest import ROOT  # noqa: F401  (sys.path setup)

P_FULL = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
          "saturation": 30, "width": 1.3, "multiband": True, "lufs": -14.0}
RATE = 44100


class OracleBackend:
    """Test-only rank backend: the CPU oracle computes the rank's chunk chain and
    its K-weighted segment energies with an explicit filter state carry."""

    def __init__(self, pcm_full):
        self.pcm = pcm_full

    def make_job(self, plan, params, out_kind):
        self.plan, self.params = plan, params
        return None

    def stage(self, job, d_in):
        from oracle import mastering_oracle as mo
        p, P = self.plan, self.params
        x = d_in  # the rank's slice of the decoded track (int16)
        thr, rat = mo.multiband_params(P)
        chunks = []
        for s, e in mo.chunk_ranges(x.shape[0], RATE):
            c = x[s:min(e, x.shape[0])]
            if e > x.shape[0]:
                c = np.concatenate([c, np.zeros((e - x.shape[0],) + x.shape[1:], np.int16)])
            y = mo.saturation(mo.pcm_to_float(c), P.get("saturation", 0))
            y = mo.equalize(y, RATE, P)
            if P.get("width", 1.0) != 1.0:
                y = mo.stereo_width(y, P["width"])
            q = mo.quantize(y)
            if P.get("multiband"):
                q = mo.multiband(q, RATE, thr, rat)
            chunks.append(q)
        self.mix = np.concatenate(chunks)
        assert self.mix.shape[0] == p.frames

    def _kweight(self, carry):
        from mastering_amd import design
        mono = (self.mix.astype(np.float32) / 32768).mean(axis=1)  # AME:215
        (b0, b1, b2, a1, a2), (c0, c1, c2, d1, d2) = design.kweight_sections(RATE)
        y1, z1 = scipy.signal.lfilter([b0, b1, b2], [1, a1, a2], mono.astype(np.float64), zi=carry[:2])
        y1 = y1.astype(np.float32)
        y2, z2 = scipy.signal.lfilter([c0, c1, c2], [1, d1, d2], y1.astype(np.float64), zi=carry[2:])
        return y2.astype(np.float32), np.concatenate([z1, z2])

    def kweight_range_end(self):
        return self._kweight(np.zeros(4))[1]

    def hop_energies(self, carry):
        y, _ = self._kweight(np.asarray(carry, np.float64))
        b = self.plan.local_bounds
        e = y.astype(np.float64) ** 2
        cs = np.concatenate([[0.0], np.cumsum(e)])
        return cs[b[1:]] - cs[b[:-1]]

    def finalize(self, gain, use_gain, d_out):
        from oracle import mastering_oracle as mo
        y = mo.pcm_to_float(self.mix)
        if use_gain:
            y = y * gain
        with np.errstate(invalid="ignore"):
            d_out[:] = mo.quantize(mo.soft_limiter(y))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, seconds, outdir):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd")]
    import torch.distributed as dist

    from mastering_amd import distributed as D
    from mastering_amd.synth import pink_noise_pcm16
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    pcm = pink_noise_pcm16(int(seconds * RATE), RATE, 2, 7)
    plan = D.plan_time_shards(pcm.shape[0], RATE, 2, world, rank)
    be = OracleBackend(pcm)
    out = np.empty((plan.frames, 2), np.int16)
    info = D.master_time_sharded(be, plan, P_FULL, pcm[plan.in_lo:plan.in_hi], out, D.TorchCollectives())
    np.save(os.path.join(outdir, f"out{rank}.npy"), out)
    np.save(os.path.join(outdir, f"L{rank}.npy"), np.array([info["loudness"], plan.f0, plan.f1]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_chunks_balanced():
    from mastering_amd.distributed import shard_chunks, shard_files
    assert shard_chunks(240, 8) == [(30 * r, 30 * r + 30) for r in range(8)]  # C4: 2 h / 8 GPUs
    r = shard_chunks(7, 3)
    assert r == [(0, 3), (3, 5), (5, 7)]
    assert sorted(sum((shard_files(64, 8, k) for k in range(8)), [])) == list(range(64))  # C3


def test_plan_segments_cover_track():
    from mastering_amd.distributed import plan_time_shards
    frames = 95 * RATE + 1234
    plans = [plan_time_shards(frames, RATE, 2, 3, r) for r in range(3)]
    assert plans[0].f0 == 0 and plans[-1].f1 == plans[-1].frames_proc_total
    for a, b in zip(plans, plans[1:]):
        assert a.f1 == b.f0
    for p in plans:  # every local segment lies inside one global segment
        g = p.local_to_global
        lo = p.local_bounds[:-1] + p.f0
        hi = p.local_bounds[1:] + p.f0
        assert np.all(p.seg_bounds[g] <= lo) and np.all(hi <= p.seg_bounds[g + 1])


def test_gate_matches_meter(oracle):
    """Host gating on segment energies == the pyloudnorm restatement."""
    from mastering_amd import distributed as D
    from mastering_amd.synth import pink_noise_pcm16
    pcm = pink_noise_pcm16(7 * RATE + 1323, RATE, 2, 4)  # whole ms: no pydub padding
    pcm[RATE:2 * RATE] //= 300  # a quiet second exercises both gates
    plan = D.plan_time_shards(pcm.shape[0], RATE, 2, 1, 0)
    be = OracleBackend(pcm)
    be.plan = plan
    be.mix = pcm[: plan.frames]
    L = D.gate_loudness(be.hop_energies(np.zeros(4)), plan)
    ref = oracle.integrated_loudness((pcm[: plan.frames].astype(np.float32) / 32768).mean(axis=1), RATE)
    assert L == pytest.approx(ref, abs=1e-5)


def test_compose_carry_exact():
    """Carry composition over ranges == one K-weighting run over the whole mix."""
    from mastering_amd import design
    from mastering_amd.distributed import compose_carry
    rng = np.random.default_rng(0)
    x = rng.standard_normal(50000) * 0.1
    (b0, b1, b2, a1, a2), (c0, c1, c2, d1, d2) = design.kweight_sections(RATE)

    def run(seg, zi):
        y1, z1 = scipy.signal.lfilter([b0, b1, b2], [1, a1, a2], seg, zi=zi[:2])
        _, z2 = scipy.signal.lfilter([c0, c1, c2], [1, d1, d2], y1, zi=zi[2:])
        return np.concatenate([z1, z2])

    cuts = [0, 12000, 31000, 50000]
    z = np.stack([run(x[a:b], np.zeros(4)) for a, b in zip(cuts, cuts[1:])])
    lens = np.diff(cuts)
    for r in range(3):
        want = run(x[: cuts[r]], np.zeros(4)) if r else np.zeros(4)
        np.testing.assert_allclose(compose_carry(z, lens, RATE, r), want, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("world", [2])
def test_time_sharded_gloo(tmp_path, oracle, world):
    """world_size 2 over gloo: the stitched ranks == the single-process oracle."""
    import torch.multiprocessing as mp
    seconds = 65.0  # chunks 30 + 30 + 5 s -> ranks own [0, 60 s) and [60, 65 s)
    port = _free_port()
    mp.start_processes(_rank_main, args=(world, port, seconds, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    from mastering_amd.synth import pink_noise_pcm16
    pcm = pink_noise_pcm16(int(seconds * RATE), RATE, 2, 7)
    ref, Lref = oracle.master(pcm, RATE, P_FULL, return_loudness=True)
    outs = [np.load(tmp_path / f"out{r}.npy") for r in range(world)]
    Ls = [np.load(tmp_path / f"L{r}.npy") for r in range(world)]
    assert all(L[0] == Ls[0][0] for L in Ls)  # every rank gates the same vector
    out = np.concatenate(outs)
    assert out.shape == ref.shape
    assert abs(Ls[0][0] - Lref) <= 4e-4
    rms = np.sqrt(np.mean(((out.astype(np.float64) - ref) / 32768) ** 2))
    assert rms <= 1e-5


def _small_rank(seconds=3.0):
    from mastering_amd import distributed as D
    from mastering_amd.synth import pink_noise_pcm16
    pcm = pink_noise_pcm16(int(seconds * RATE), RATE, 2, 3)
    plan = D.plan_time_shards(pcm.shape[0], RATE, 2, 1, 0)
    return D, pcm, plan, OracleBackend(pcm)


def test_time_sharded_refuses_non_consecutive_segments():
    """a plan whose local segments are not consecutive global ones raises
    (it used to fall back to the host path silently)."""
    D, pcm, plan, be = _small_rank()
    plan.local_to_global = plan.local_to_global.copy()
    plan.local_to_global[1:] += 1  # a gap after the first segment
    out = np.empty((plan.frames, 2), np.int16)
    with pytest.raises(ValueError, match="consecutive"):
        D.master_time_sharded(be, plan, P_FULL, pcm, out, D.LocalCollectives())


@pytest.mark.parametrize("mismatch", ["context", "world"])
def test_time_sharded_refuses_foreign_library_collectives(mismatch):
    """LibraryCollectives must wrap the backend's own context over the
    plan's world; anything else raises instead of taking the host path."""
    D, pcm, plan, be = _small_rank()
    be.ctx = object()
    # no communicator needed: the check comes before any work or collective
    coll = D.LibraryCollectives(object() if mismatch == "context" else be.ctx,
                                plan.world + (1 if mismatch == "world" else 0))
    out = np.empty((plan.frames, 2), np.int16)
    with pytest.raises(ValueError, match="LibraryCollectives"):
        D.master_time_sharded(be, plan, P_FULL, pcm, out, coll)
