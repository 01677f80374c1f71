"""Multi-GPU sharding of the mastering hot path.

Two ways to spread work over the GPUs of a node, one process per GPU:

* by file (BASELINE C3/C5): every rank masters its own tracks end to end; there
  is no data-path collective (`shard_files`).
* by time (BASELINE C4, one long track): the reference's per-chunk chain
  (AME:48-77) is independent between 30 s chunks, so every rank runs a
  contiguous range of whole chunks.  The only whole-track couplings are the
  K-weighting IIR and the gated loudness (AME:84-86, pyloudnorm):
    1. each rank stages its chunks and computes the zero-start end state z_r of
       the K-weighting recurrence over its range;
    2. all-gather of (z_r, range length): every rank composes its exact carry-in
       s_r = A^{L_{r-1}} s_{r-1} + z_{r-1} (A = the K-weighting state transition);
    3. every rank computes the K-weighted energy of each 0.1 s loudness segment
       of its range from that carry-in, scattered into a zeroed whole-track vector;
    4. ONE sum all-reduce of that f64 vector (RCCL over xGMI when the process
       group is "nccl"; gloo in the CPU tests);
    5. every rank gates the same vector (pyloudnorm's block gating) and applies
       the same gain + soft limiter + int16 quantisation to its own range.

The per-rank compute is behind a small backend protocol so that the
orchestration is testable on CPU (tests/test_distributed.py drives it with an
oracle-backed backend over gloo); `GpuBackend` is the product implementation
over the C-ABI (include/mastering.h: mm_stage_chunks, mm_kweight_range_end,
mm_hop_energies, mm_finalize).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import design, native
from .engine import Job


# ----------------------------------------------------------------------------
# partitioning
# ----------------------------------------------------------------------------
def shard_files(n_files: int, world: int, rank: int):
    """Round-robin file indices of `rank` (C3: 64 tracks / 8 GPUs; C5: 128 / 8)."""
    return list(range(rank, n_files, world))


def shard_chunks(n_chunks: int, world: int):
    """Contiguous, balanced ranges of whole 30 s chunks: [(c0, c1)] per rank."""
    base, extra = divmod(n_chunks, world)
    out, c = [], 0
    for r in range(world):
        n = base + (1 if r < extra else 0)
        out.append((c, c + n))
        c += n
    return out


@dataclass
class RankPlan:
    """Geometry of one rank's share of a time-sharded track."""
    rank: int
    world: int
    rate: int
    channels: int
    frames_total: int        # decoded frames of the whole track
    frames_proc_total: int   # processed frames of the whole track (pydub slicing)
    f0: int                  # first processed frame of this rank
    f1: int                  # one past the last processed frame of this rank
    in_lo: int               # input slice [in_lo, in_hi) this rank reads
    in_hi: int
    ranges: list             # [(f0, f1)] of every rank
    # whole-track loudness geometry (pyloudnorm blocks) and this rank's segments
    n_blocks: int
    block_lo: np.ndarray
    block_hi: np.ndarray
    seg_bounds: np.ndarray   # whole-track distinct block bounds
    local_bounds: np.ndarray  # this rank's segment bounds, relative to f0
    local_to_global: np.ndarray  # global segment index of every local segment
    block_scale: float

    @property
    def frames(self):
        return self.f1 - self.f0


def plan_time_shards(frames_total: int, rate: int, channels: int, world: int, rank: int) -> RankPlan:
    bounds = design.chunk_bounds(frames_total, rate)
    if not bounds:
        raise ValueError("empty track")
    if len(bounds) < world:
        raise ValueError(f"{len(bounds)} chunks cannot be time-sharded over {world} ranks")
    if frames_total < 0.4 * rate:
        raise ValueError("Audio must have length greater than the block size.")
    cr = shard_chunks(len(bounds), world)
    ranges = [(bounds[c0][0], bounds[c1 - 1][1]) for c0, c1 in cr]
    f0, f1 = ranges[rank]
    frames_proc_total = bounds[-1][1]
    nb, lo, hi, segb, scale = design.loudness_blocks(frames_proc_total, rate)
    inner = segb[(segb > f0) & (segb < f1)]
    local = np.concatenate([[f0], inner, [f1]]).astype(np.int64)
    # global segment s covers [segb[s], segb[s+1]); a local segment starting at x
    # lies inside the global segment with the largest bound <= x
    l2g = np.searchsorted(segb, local[:-1], side="right") - 1
    l2g = np.clip(l2g, 0, len(segb) - 2)
    return RankPlan(rank, world, rate, channels, frames_total, frames_proc_total, f0, f1,
                    min(f0, frames_total), min(f1, frames_total), ranges, nb, lo, hi, segb,
                    (local - f0).astype(np.int64), l2g.astype(np.int64), scale)


def kweight_transition(rate: int, frames: int) -> np.ndarray:
    """A^frames of the K-weighting state recurrence (4x4, f64)."""
    A = design.transition_matrix(design.kweight_sections(rate), [2])[:4, :4]
    return np.linalg.matrix_power(A, int(frames))


def compose_carry(z_all: np.ndarray, len_all, rate: int, rank: int) -> np.ndarray:
    """Carry-in state of `rank` from every rank's zero-start end state."""
    s = np.zeros(4)
    for q in range(rank):
        s = kweight_transition(rate, len_all[q]) @ s + z_all[q]
    return s


def block_segments(plan: RankPlan):
    """Every loudness block's whole-track segment range [s0, s1) (int32), as
    gate_loudness derives it."""
    n = len(plan.seg_bounds) - 1
    s0 = np.minimum(np.searchsorted(plan.seg_bounds, plan.block_lo), n).astype(np.int32)
    s1 = np.minimum(np.searchsorted(plan.seg_bounds, plan.block_hi), n).astype(np.int32)
    return s0, s1


def gate_loudness(seg_energy: np.ndarray, plan: RankPlan) -> float:
    """pyloudnorm 0.1.1 integrated_loudness gating on whole-track segment energies
    (same restatement as mm_gate_loudness in csrc/mastering.hip)."""
    cs = np.concatenate([[0.0], np.cumsum(seg_energy)])
    s0 = np.searchsorted(plan.seg_bounds, plan.block_lo)
    s1 = np.searchsorted(plan.seg_bounds, plan.block_hi)
    z = plan.block_scale * (cs[np.minimum(s1, len(seg_energy))] - cs[np.minimum(s0, len(seg_energy))])
    with np.errstate(divide="ignore"):
        lb = -0.691 + 10.0 * np.log10(z)
    gated = z[lb >= -70.0]
    with np.errstate(invalid="ignore", divide="ignore"):
        gamma_r = -0.691 + 10.0 * np.log10(np.mean(gated) if gated.size else np.nan) - 10.0
        sel = z[(lb > gamma_r) & (lb > -70.0)]
        zavg = np.nan_to_num(np.mean(sel)) if sel.size else 0.0
        return float(-0.691 + 10.0 * np.log10(zavg))


# ----------------------------------------------------------------------------
# collectives (torch.distributed: backend "nccl" is RCCL over xGMI on ROCm)
# ----------------------------------------------------------------------------
class TorchCollectives:
    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"

    def all_gather(self, vec: np.ndarray) -> np.ndarray:
        import torch
        t = torch.from_numpy(np.ascontiguousarray(vec, dtype=np.float64)).to(self.device)
        out = [torch.empty_like(t) for _ in range(self.dist.get_world_size(self.group))]
        self.dist.all_gather(out, t, group=self.group)
        return np.stack([o.cpu().numpy() for o in out])

    def all_reduce_sum(self, vec: np.ndarray) -> np.ndarray:
        import torch
        t = torch.from_numpy(np.ascontiguousarray(vec, dtype=np.float64)).to(self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy()

    def all_reduce_sum_device(self, t):
        """In-place sum all-reduce of a device tensor (RCCL over xGMI with "nccl"), no
        host copies; complete on return (the library reads the buffer next)."""
        import torch
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        torch.cuda.current_stream(t.device).synchronize()
        return t


def rccl_unique_id() -> bytes:
    """A fresh RCCL unique id (128 bytes) for mm_comm_init; rank 0 makes it and
    hands it to the other ranks out of band (bench.py: a gloo broadcast)."""
    lib = native.load()
    buf = ctypes.create_string_buffer(128)
    rc = lib.mm_comm_unique_id(buf)
    if rc != 0:
        raise RuntimeError(f"mm_comm_unique_id failed ({rc})")
    return buf.raw


class LibraryCollectives:
    """The same two collectives through the library's own RCCL communicator
    (mm_comm_init / mm_allgather_f64 / mm_allreduce_sum_f64): one rank per GPU,
    RCCL over xGMI between them."""

    def __init__(self, ctx: native.Context, world: int):
        self.ctx, self.world = ctx, world

    @classmethod
    def create(cls, ctx: native.Context, rank: int, world: int, unique_id: bytes) -> "LibraryCollectives":
        if len(unique_id) != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        ctx.check(ctx.lib.mm_comm_init(ctx.ptr, int(rank), int(world), unique_id), "mm_comm_init")
        return cls(ctx, world)

    def close(self):
        self.ctx.check(self.ctx.lib.mm_comm_destroy(self.ctx.ptr), "mm_comm_destroy")

    def all_gather(self, vec: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(vec, dtype=np.float64)
        out = np.empty(v.size * self.world)
        self.ctx.check(self.ctx.lib.mm_allgather_f64(self.ctx.ptr, v.ctypes.data_as(native.c_double_p),
                                                     out.ctypes.data_as(native.c_double_p), v.size),
                       "mm_allgather_f64")
        return out.reshape(self.world, v.size)

    def all_reduce_sum(self, vec: np.ndarray) -> np.ndarray:
        v = np.array(vec, dtype=np.float64)
        self.ctx.check(self.ctx.lib.mm_allreduce_sum_f64(self.ctx.ptr, v.ctypes.data_as(native.c_double_p),
                                                         v.size), "mm_allreduce_sum_f64")
        return v

    def all_reduce_sum_device(self, d_buf: int, n: int):
        """In-place sum all-reduce of n doubles at device address d_buf (this context's
        device), no host staging (mm_allreduce_sum_f64_device)."""
        self.ctx.check(self.ctx.lib.mm_allreduce_sum_f64_device(self.ctx.ptr, ctypes.c_void_p(d_buf), int(n)),
                       "mm_allreduce_sum_f64_device")

    def all_gather_device(self, d_in: int, d_out: int, n: int):
        """All-gather of n doubles per rank between device buffers (d_out: world * n)."""
        self.ctx.check(self.ctx.lib.mm_allgather_f64_device(self.ctx.ptr, ctypes.c_void_p(d_in),
                                                            ctypes.c_void_p(d_out), int(n)),
                       "mm_allgather_f64_device")


class TorchLikeHost:
    """world == 1 through the host orchestration (energies to the host, numpy gating):
    the reference for the device-resident path in the tests."""

    def all_gather(self, vec):
        return np.asarray(vec, dtype=np.float64)[None, :]

    def all_reduce_sum(self, vec):
        return np.asarray(vec, dtype=np.float64)


class LocalCollectives:
    """world == 1 (no communication)."""

    def all_gather(self, vec):
        return np.asarray(vec, dtype=np.float64)[None, :]

    def all_reduce_sum(self, vec):
        return np.asarray(vec, dtype=np.float64)


# ----------------------------------------------------------------------------
# per-rank compute backend over the C-ABI
# ----------------------------------------------------------------------------
class GpuBackend:
    """Stages one rank's chunks on its GPU and exposes the four steps the
    orchestration needs.  `d_in` / `d_out` are device pointers (e.g. torch)."""

    def __init__(self, ctx: native.Context):
        self.ctx = ctx
        self.job = None

    def make_job(self, plan: RankPlan, params: dict, out_kind: int) -> Job:
        return Job(plan.in_hi - plan.in_lo, plan.rate, plan.channels, params, out_kind,
                   seg_bounds=plan.local_bounds, check_length=False)

    def stage(self, job: Job, d_in: int):
        self.job = job
        self.ctx.check(self.ctx.lib.mm_stage_chunks(self.ctx.ptr, ctypes.byref(job.job), ctypes.c_void_p(d_in)),
                       "mm_stage_chunks")

    def kweight_range_end(self) -> np.ndarray:
        z = np.zeros(4)
        self.ctx.check(self.ctx.lib.mm_kweight_range_end(self.ctx.ptr, z.ctypes.data_as(native.c_double_p)),
                       "mm_kweight_range_end")
        return z

    def hop_energies(self, carry: np.ndarray) -> np.ndarray:
        c = np.ascontiguousarray(carry, dtype=np.float64)
        e = np.zeros(int(self.job.job.n_segs))
        self.ctx.check(self.ctx.lib.mm_hop_energies(self.ctx.ptr, c.ctypes.data_as(native.c_double_p),
                                                    e.ctypes.data_as(native.c_double_p)), "mm_hop_energies")
        return e

    def shard_loudness_device(self, carry: np.ndarray, plan: "RankPlan", target: float, d_out: int):
        """Steps 3-5 with the energy vector kept in HBM (mm_shard_loudness_device): this
        rank's segment energies into the whole-track vector, the RCCL sum all-reduce
        in place (the context's communicator, which must span plan.world ranks), device
        gating and the device gain into mm_finalize.  Returns (L, the gain applied)."""
        c = np.ascontiguousarray(carry, dtype=np.float64)
        n_glob = len(plan.seg_bounds) - 1
        s0, s1 = block_segments(plan)
        lg = np.zeros(2)
        self.ctx.check(self.ctx.lib.mm_shard_loudness_device(
            self.ctx.ptr, c.ctypes.data_as(native.c_double_p), n_glob, int(plan.local_to_global[0]), len(s0),
            s0.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), s1.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            float(plan.block_scale), float(target), int(plan.world), ctypes.c_void_p(d_out),
            lg.ctypes.data_as(native.c_double_p)), "mm_shard_loudness_device")
        return float(lg[0]), float(lg[1])

    def shard_energies_device(self, carry: np.ndarray, plan: "RankPlan", d_full: int):
        """Step 3 into a caller's device vector of the whole track's segments."""
        c = np.ascontiguousarray(carry, dtype=np.float64)
        self.ctx.check(self.ctx.lib.mm_shard_energies_device(
            self.ctx.ptr, c.ctypes.data_as(native.c_double_p), len(plan.seg_bounds) - 1,
            int(plan.local_to_global[0]), ctypes.c_void_p(d_full)), "mm_shard_energies_device")

    def gate_finalize_device(self, d_full: int, plan: "RankPlan", target: float, d_out: int):
        """Step 5 from the summed device vector: (L, the gain applied)."""
        s0, s1 = block_segments(plan)
        lg = np.zeros(2)
        self.ctx.check(self.ctx.lib.mm_gate_finalize_device(
            self.ctx.ptr, ctypes.c_void_p(d_full), len(plan.seg_bounds) - 1, len(s0),
            s0.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), s1.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            float(plan.block_scale), float(target), ctypes.c_void_p(d_out), lg.ctypes.data_as(native.c_double_p)),
            "mm_gate_finalize_device")
        return float(lg[0]), float(lg[1])

    def shard_loudness_torch(self, carry: np.ndarray, plan: "RankPlan", target: float, d_out: int, coll):
        """Steps 3-5 with torch.distributed ("nccl" = RCCL) summing the library's energy
        vector in place in HBM: the vector is a torch tensor on this context's device."""
        import torch
        dev = torch.device("cuda", self.ctx.device)
        # empty, not zeros: mm_shard_energies_device zeroes the vector on the library's
        # own (non-blocking) stream; a torch fill would be queued on torch's stream,
        # unordered with it.  Drain torch's stream first so no earlier
        # torch work on a recycled block can land after the library's writes.
        full = torch.empty(len(plan.seg_bounds) - 1, dtype=torch.float64, device=dev)
        torch.cuda.current_stream(dev).synchronize()
        self.shard_energies_device(carry, plan, full.data_ptr())
        coll.all_reduce_sum_device(full)
        return self.gate_finalize_device(full.data_ptr(), plan, target, d_out)

    def finalize(self, gain: float, use_gain: bool, d_out: int):
        self.ctx.check(self.ctx.lib.mm_finalize(self.ctx.ptr, float(gain), int(use_gain), ctypes.c_void_p(d_out)),
                       "mm_finalize")


def master_time_sharded(backend, plan: RankPlan, params: dict, d_in, d_out, coll,
                        out_kind: int = native.MM_OUT_I16) -> dict:
    """Run this rank's share of a time-sharded track (steps 1-5 above).
    `d_in` holds the rank's input slice [plan.in_lo, plan.in_hi) (decoded f32);
    `d_out` receives its processed frames [plan.f0, plan.f1)."""
    # checked before any work or collective: the path depends only on the collective's
    # kind and the plan, the same on every rank (raises since round 5)
    if isinstance(coll, LibraryCollectives) and (coll.ctx is not getattr(backend, "ctx", None)
                                                 or coll.world != plan.world):
        raise ValueError("LibraryCollectives must wrap the backend's own context (its RCCL communicator) "
                         "over the plan's world")
    l2g = plan.local_to_global
    if params.get("lufs") is not None and not (len(l2g) and np.all(np.diff(l2g) == 1)):
        raise ValueError("a rank's loudness segments must be consecutive global segments")
    job = backend.make_job(plan, params, out_kind)
    backend.stage(job, d_in)
    lufs = params.get("lufs")
    L, gain = None, 1.0
    if lufs is not None:
        z = backend.kweight_range_end()
        zl = coll.all_gather(np.concatenate([z, [float(plan.frames)]]))
        carry = compose_carry(zl[:, :4], zl[:, 4].astype(np.int64), plan.rate, plan.rank)
        mode = None
        if hasattr(backend, "shard_loudness_device"):
            if isinstance(coll, LibraryCollectives) or (isinstance(coll, LocalCollectives) and plan.world == 1):
                mode = "library"
            elif isinstance(coll, TorchCollectives) and coll.device == "cuda":
                mode = "torch"
        if mode is not None:
            # energies, all-reduce, gating and gain stay on the device; the gain returned
            # is the one finalize applied (gate.hip), not a host recomputation
            if mode == "library":
                L, gain = backend.shard_loudness_device(carry, plan, float(lufs), d_out)
            else:
                L, gain = backend.shard_loudness_torch(carry, plan, float(lufs), d_out, coll)
            return {"loudness": L, "gain_linear": gain, "frames": plan.frames, "f0": plan.f0, "f1": plan.f1,
                    "device_gate": True}
        local = backend.hop_energies(carry)
        full = np.zeros(len(plan.seg_bounds) - 1)
        np.add.at(full, plan.local_to_global, local)
        full = coll.all_reduce_sum(full)
        L = gate_loudness(full, plan)
        gain = 10.0 ** ((float(lufs) - L) / 20.0)
    backend.finalize(gain, lufs is not None, d_out)
    return {"loudness": L, "gain_linear": gain, "frames": plan.frames, "f0": plan.f0, "f1": plan.f1}
