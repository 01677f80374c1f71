"""The library's own RCCL path (mm_comm_unique_id / mm_comm_init /
mm_allreduce_sum_f64 / mm_allgather_f64 and their device-pointer variants) and the
device loudness steps (mm_shard_energies_device / mm_gate_finalize_device /
mm_shard_loudness_device) on the one-GPU box: a world-size-1
communicator runs ncclCommInitRank, the HBM staging and the real collectives,
then the C4 orchestration (distributed.master_time_sharded) uses it and is checked
against the oracle.  RCCL forbids two ranks of one
communicator on the same GPU, so N > 1 is covered by the gloo tests
(test_distributed.py) and the driver's multi-GPU bench."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def coll():
    from mastering_amd import distributed as D
    from mastering_amd import native
    ctx = native.Context(0)
    c = D.LibraryCollectives.create(ctx, 0, 1, D.rccl_unique_id())
    yield c
    c.close()
    ctx.close()


def test_rccl_collectives_world1(coll):
    n = 72_000  # loudness segments of a 2-h track (0.1 s each)
    v = np.random.default_rng(0).standard_normal(n)
    assert np.array_equal(coll.all_reduce_sum(v), v)
    g = coll.all_gather(v[:20])
    assert g.shape == (1, 20) and np.array_equal(g[0], v[:20])


def test_time_sharded_with_library_rccl(coll, oracle):
    import torch

    from mastering_amd import distributed as D
    from mastering_amd.synth import pink_noise_pcm16
    from test_gpu_parity import P_FULL, _check
    rate = 44100
    pcm = pink_noise_pcm16(65 * rate, rate, 2, 12)
    plan = D.plan_time_shards(pcm.shape[0], rate, 2, 1, 0)
    be = D.GpuBackend(coll.ctx)
    x = torch.from_numpy(pcm.astype(np.float32) / 32768).cuda()
    out = torch.empty((plan.frames, 2), dtype=torch.int16, device="cuda")
    info = D.master_time_sharded(be, plan, P_FULL, x.data_ptr(), out.data_ptr(), coll)
    coll.ctx.sync()
    ref, L = oracle.master(pcm, rate, P_FULL, return_loudness=True)
    _check(out.cpu().numpy(), info, ref, L)
    assert info.get("device_gate"), "the library-RCCL path keeps the energies, gating and gain on the device"


def test_device_gate_matches_host_gate(coll, oracle):
    """mm_shard_loudness_device (energies -> whole-track vector -> gate_kernel -> device
    gain -> finalize) against the host orchestration of the same staged range (host
    energies, numpy gating, host gain): same loudness to 1e-6 LU, the same output but for one-ulp gain differences."""
    import torch

    from mastering_amd import distributed as D
    from mastering_amd.synth import pink_noise_pcm16
    from test_gpu_parity import P_FULL
    rate = 44100
    pcm = pink_noise_pcm16(95 * rate, rate, 2, 13)
    plan = D.plan_time_shards(pcm.shape[0], rate, 2, 1, 0)
    be = D.GpuBackend(coll.ctx)
    x = torch.from_numpy(pcm.astype(np.float32) / 32768).cuda()
    outs, infos = [], []
    for c in (coll, D.TorchLikeHost()):
        out = torch.empty((plan.frames, 2), dtype=torch.int16, device="cuda")
        infos.append(D.master_time_sharded(be, plan, P_FULL, x.data_ptr(), out.data_ptr(), c))
        coll.ctx.sync()
        outs.append(out.cpu().numpy())
    assert infos[0].get("device_gate") and not infos[1].get("device_gate")
    assert abs(infos[0]["loudness"] - infos[1]["loudness"]) <= 1e-6
    assert np.mean(outs[0] == outs[1]) >= 0.9999


def test_device_gate_returns_the_applied_gain(coll, oracle):
    """The gain master_time_sharded reports is the one finalize applied (read back from
    the device, gate.hip's pow), within 4 ulp of the reference's float64 expression
    10 ** ((target - L) / 20) on the same L (AME:219-222)."""
    import torch

    from mastering_amd import distributed as D
    from mastering_amd.synth import pink_noise_pcm16
    from test_gpu_parity import P_FULL
    rate = 44100
    pcm = pink_noise_pcm16(40 * rate, rate, 2, 14)
    plan = D.plan_time_shards(pcm.shape[0], rate, 2, 1, 0)
    be = D.GpuBackend(coll.ctx)
    x = torch.from_numpy(pcm.astype(np.float32) / 32768).cuda()
    out = torch.empty((plan.frames, 2), dtype=torch.int16, device="cuda")
    info = D.master_time_sharded(be, plan, P_FULL, x.data_ptr(), out.data_ptr(), coll)
    host = 10.0 ** ((float(P_FULL["lufs"]) - info["loudness"]) / 20.0)
    assert info["device_gate"]
    assert abs(info["gain_linear"] - host) <= 4 * np.spacing(host), (info["gain_linear"], host)


def _staged_rank(ctx, pcm, rate, world, rank):
    import torch

    from mastering_amd import distributed as D
    from mastering_amd import native
    from test_gpu_parity import P_FULL
    plan = D.plan_time_shards(pcm.shape[0], rate, 2, world, rank)
    be = D.GpuBackend(ctx)
    x = torch.from_numpy(pcm[plan.in_lo:plan.in_hi].astype(np.float32) / 32768).cuda()
    be.stage(be.make_job(plan, P_FULL, native.MM_OUT_I16), x.data_ptr())
    return plan, be, x


def test_rank_of_multi_rank_plan_device_energies_and_gate(coll):
    """Rank 1 of a 3-rank plan on one GPU: its energies land at its
    global offset (> 0) of a whole-track device vector that is zero elsewhere and
    equal the host path's mm_hop_energies; the device gate of a full vector equals
    the numpy restatement of pyloudnorm's gating (distributed.gate_loudness)."""
    import torch

    from mastering_amd import distributed as D
    from mastering_amd.synth import pink_noise_pcm16
    rate = 44100
    pcm = pink_noise_pcm16(95 * rate, rate, 2, 15)
    plan, be, x = _staged_rank(coll.ctx, pcm, rate, 3, 1)
    n_glob = len(plan.seg_bounds) - 1
    assert plan.local_to_global[0] > 0 and len(plan.local_to_global) < n_glob
    carry = np.array([1e-3, -2e-3, 5e-4, 1e-4])  # any carry-in state: both paths take the same
    full = torch.full((n_glob,), 7.0, dtype=torch.float64, device="cuda")
    torch.cuda.current_stream().synchronize()  # the fill is on torch's stream, the library uses its own
    be.shard_energies_device(carry, plan, full.data_ptr())
    got = full.cpu().numpy()
    host = be.hop_energies(carry)
    o = int(plan.local_to_global[0])
    assert np.all(got[:o] == 0) and np.all(got[o + len(host):] == 0)
    np.testing.assert_allclose(got[o:o + len(host)], host, rtol=1e-12, atol=0)
    # gate a whole-track vector (every rank's segments present) on the device
    vec = np.random.default_rng(3).uniform(1e-6, 1e-2, n_glob)
    vec[::97] = 1e-12  # some blocks below the absolute gate
    dv = torch.from_numpy(vec).cuda()
    out = torch.empty((plan.frames, 2), dtype=torch.int16, device="cuda")
    L, gain = be.gate_finalize_device(dv.data_ptr(), plan, -14.0, out.data_ptr())
    Lh = D.gate_loudness(vec, plan)
    assert abs(L - Lh) <= 1e-6, (L, Lh)
    assert abs(gain - 10.0 ** ((-14.0 - L) / 20.0)) <= 4 * np.spacing(gain)


def test_multi_rank_plan_needs_the_communicator(coll):
    """A world-2 plan on a context whose communicator spans one rank is refused
    (MM_ERR_STATE), not gated on a half-empty vector."""
    import torch

    from mastering_amd.synth import pink_noise_pcm16
    rate = 44100
    pcm = pink_noise_pcm16(65 * rate, rate, 2, 16)
    plan, be, x = _staged_rank(coll.ctx, pcm, rate, 2, 0)
    out = torch.empty((plan.frames, 2), dtype=torch.int16, device="cuda")
    with pytest.raises(RuntimeError, match="communicator"):
        be.shard_loudness_device(np.zeros(4), plan, -14.0, out.data_ptr())


def test_device_collectives_world1(coll):
    """mm_allreduce_sum_f64_device / mm_allgather_f64_device on device buffers."""
    import torch
    v = torch.from_numpy(np.random.default_rng(1).standard_normal(4096)).cuda()
    ref = v.cpu().numpy().copy()
    coll.all_reduce_sum_device(v.data_ptr(), v.numel())
    assert np.array_equal(v.cpu().numpy(), ref)
    o = torch.empty_like(v)
    coll.all_gather_device(v.data_ptr(), o.data_ptr(), v.numel())
    assert np.array_equal(o.cpu().numpy(), ref)


def test_time_sharded_with_torch_nccl(oracle):
    """The torch.distributed path (backend "nccl" = RCCL) at world 1: the library's
    energy vector is a torch tensor all-reduced in place in HBM (no host copies),
    then gated on the device; same loudness as the library-RCCL path."""
    import os

    import torch
    import torch.distributed as dist

    from mastering_amd import distributed as D
    from mastering_amd import native
    from mastering_amd.synth import pink_noise_pcm16
    from test_gpu_parity import P_FULL, _check
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rate = 44100
        pcm = pink_noise_pcm16(65 * rate, rate, 2, 12)
        plan = D.plan_time_shards(pcm.shape[0], rate, 2, 1, 0)
        ctx = native.Context(0)
        be = D.GpuBackend(ctx)
        x = torch.from_numpy(pcm.astype(np.float32) / 32768).cuda()
        out = torch.empty((plan.frames, 2), dtype=torch.int16, device="cuda")
        info = D.master_time_sharded(be, plan, P_FULL, x.data_ptr(), out.data_ptr(), D.TorchCollectives())
        ctx.sync()
        assert info["device_gate"]
        ref, L = oracle.master(pcm, rate, P_FULL, return_loudness=True)
        _check(out.cpu().numpy(), info, ref, L)
        ctx.close()
    finally:
        dist.destroy_process_group()
