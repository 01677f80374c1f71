"""The library's own RCCL path (mm_comm_unique_id / mm_comm_init /
mm_allreduce_sum_f64 / mm_allgather_f64) on the one-GPU box: a world-size-1
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
