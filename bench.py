"""Benchmark: stereo frames/s through the full mastering chain (BASELINE.json metric).

Workloads (`--workload`, BASELINE.json configs; a "step" masters every track of
the rank's share once, inputs and outputs resident in HBM):
  C2  one 5-min 44.1 kHz stereo f32 track per GPU (default; BASELINE's 1-GPU
      config).  With N > 1 every rank masters its own track: file sharding, no
      data-path collective, "scaling": "weak".
  C3  8 x 3-min 44.1 kHz tracks per GPU (64 tracks over 8 GPUs), file-sharded,
      run as one mm_master_batch: same-settings tracks fused into timelines
      (two units here, every stage launched once per unit), units in flight on
      their own streams.
  C4  one 2-h 44.1 kHz track time-sharded over the N ranks: each rank stages its
      contiguous 30 s chunks, then the K-weighting carry all-gather and ONE sum
      all-reduce of the 0.1 s loudness energies run through the library's own RCCL
      communicator (mm_comm_init; RCCL over xGMI), "scaling": "strong".
  C5  16 x 3-min 96 kHz f32 tracks per GPU (128 over 8 GPUs), f32 out, batched.
  C1  one 30 s 44.1 kHz track, EQ + LUFS only (pop preset; no exciter, no
      multiband, width 1.0): BASELINE's CPU-path config, timed here on the GPU with
      the reference's CPU path (faithful-cost leg) beside it.
Full chain settings P_FULL (exciter 30 %, techno EQ, width 1.3, 3-band compressor
with the worker's default thresholds, LUFS -14); `--params hot` switches to the
P_HOT thresholds (every compressor branch fires: the envelope solve's worst case
measured here).

Timing: W warm-up steps, then K steps timed with no instrumentation, bracketed
by a barrier + device sync on both sides (max over ranks).  A separate pass with
HIP events around every launch on the library's streams gives per-kernel device
times.  roofline: the chain's algorithmic bytes (16 B per stereo frame: f32 L,R
in + f32 L,R out) over ms_per_step is the headline; the dominant
kernel's own algorithmic bytes per launch over its event-timed average launch sit
beside it.  `traffic` = PMC bytes per step from profiles/<tag>_pmc_summary.json,
used only when that profile was measured on these exact kernel sources (its
source_sha matches).  `limiter` comes from the SQ issue/wait shares recorded next
to it.  cpu_baseline: the faithful-cost CPU path (oracle/faithful_cost.py: the
reference's numpy/scipy stages + pydub's per-frame Python compressor loop) on
whole chunks, extrapolated, on 1 core and on the box's cores; it runs before
anything touches the GPU (its worker processes are forked).

Run:  python bench.py [--workload C2|C3|C4|C5] [--gpus N] [--steps K] [--warmup W]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ... (each rank
reads RANK / LOCAL_RANK / WORLD_SIZE; --gpus must equal WORLD_SIZE), or `python bench.py
--gpus N` alone: that process becomes the launcher (launch_ranks) and starts the N ranks itself.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")  # CPU baseline leg: one core per process
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("MKL_NUM_THREADS", "1")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "python-audio-mastering_amd"))

import numpy as np  # noqa: E402

METRIC = "stereo frames/sec through full mastering chain, 44.1 kHz f32; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
CHAIN_BYTES_PER_FRAME = 16  # f32 L,R in + f32 L,R out
PROFILE_ROUND = "r06"  # profiles/<round>_<workload>_pmc_summary.json carry the PMC traffic
P_FULL = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
          "saturation": 30, "width": 1.3, "multiband": True, "lufs": -14.0}
P_HOT = dict(P_FULL, low_thresh=-16.0, mid_thresh=-21.0, high_thresh=-27.0)
P_EQLUFS = {"bass_boost": 2.0, "mid_cut": 0.0, "presence_boost": 3.5, "treble_boost": 2.5,  # pop (AME:15-20)
            "saturation": 0, "width": 1.0, "multiband": False, "lufs": -14.0}
PARAMS = {"full": P_FULL, "hot": P_HOT, "eqlufs": P_EQLUFS}
PARAMS_DESC = {"full": "full chain (sat 30, techno EQ, width 1.3, multiband defaults, LUFS -14)",
               "hot": "full chain P_HOT thresholds", "eqlufs": "EQ + LUFS only (pop preset, LUFS -14)"}
VALU_PEAK_G = 256 * 4 * 2.4e9 / 4 / 1e9  # G wave64 VALU instr/s: 1024 SIMDs x 2.4 GHz / 4 cycles (f64 FMA rate)
WORKLOADS = {
    "C1": {"rate": 44100, "seconds": 30, "tracks": 1, "params": "eqlufs",
           "desc": "C1: one 30 s 44.1 kHz stereo f32 track"},
    "C2": {"rate": 44100, "seconds": 300, "tracks": 1, "desc": "C2: 5-min 44.1 kHz stereo f32 track per GPU"},
    "C3": {"rate": 44100, "seconds": 180, "tracks": 8, "desc": "C3: 8 x 3-min 44.1 kHz stereo f32 tracks per GPU "
                                                             "(64 over 8 GPUs), file-sharded, batched"},
    "C4": {"rate": 44100, "seconds": 7200, "tracks": 1, "desc": "C4: one 2-h 44.1 kHz stereo f32 track time-sharded "
                                                              "over the ranks, RCCL carry all-gather + energy "
                                                              "all-reduce"},
    "C5": {"rate": 96000, "seconds": 180, "tracks": 16, "desc": "C5: 16 x 3-min 96 kHz stereo f32 tracks per GPU "
                                                              "(128 over 8 GPUs), f32 hi-res out, batched"},
}


def source_sha() -> str:
    """Hash of everything that shapes the kernels' work (HIP sources, header, host
    geometry): a profile under profiles/ is used only for the exact same code."""
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "python-audio-mastering_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")))
    files += [os.path.join(ROOT, "include", "mastering.h"),
              os.path.join(ROOT, "python-audio-mastering_amd", "mastering_amd", "engine.py"),
              os.path.join(ROOT, "python-audio-mastering_amd", "mastering_amd", "design.py")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def intermediate_bytes(kernel, n, g, active, walked_per_launch):
    """HBM bytes one launch moves for its own inputs/outputs in this design (stereo,
    n frames, g tiles, `active` compressor frames over the 3 bands), intermediates
    included: the kernel's own data-flow floor, NOT SURVEY §8(d)'s algorithmic
    bytes (16 B per stereo frame for the whole chain, which the headline and the
    dominant kernel's `frac` use)."""
    table = {
        "eq": 8 * n + 4 * n,                  # f32 L,R in; int16 pair q1 out
        "pre_pointwise": 8 * n + 4 * n,
        "xover": 4 * n + 12 * n,              # q1 in; three int16-pair bands out
        "comp_rms": 12 * n + 24 * n,          # bands in; f64 M of every band-frame out (the M plane)
        "comp_describe": 8 * active,          # M of every active band-frame (links + release-jump records: 128 B per active tile)
        "comp_pass0": 8 * active,             # M of every active band-frame
        "comp_fix": 8 * walked_per_launch,    # M of the re-walked frames
        "comp_apply": 8 * active + 12 * n + 4 * n,  # M of the active frames, bands in; mix out
        "kweight": 4 * n + 4 * n,             # mix in; f32 squares out (exact block energies)
        "kw_blocks": 16 * n,                  # the squares, once per overlapping 0.4 s block (4x)
        "seg_reduce": g * 24,
        "gate": 0,
        "finalize": 4 * n + 8 * n,            # mix in; f32 L,R out
    }
    return table.get(kernel)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU). Under torch.distributed.run it must equal WORLD_SIZE; without it, "
                         "N > 1 makes this process a launcher that starts and times N rank processes itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher test: every rank prints its rank / local rank / world as JSON and exits "
                         "before anything touches the GPU")
    ap.add_argument("--cpu-baseline-from", default=None, help=argparse.SUPPRESS)  # launcher -> rank 0
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="C2")
    ap.add_argument("--params", choices=sorted(PARAMS), default=None,
                    help="settings (default: the workload's own: eqlufs for C1, else full)")
    ap.add_argument("--profile-steps", type=int, default=5, help="steps of the per-kernel event-timed pass")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-chunks", type=int, default=2, help="whole chunks timed on one core (faithful-cost leg)")
    ap.add_argument("--cpu-procs", type=int, default=0, help="worker processes of the N-core leg (0: the CPU "
                                                              "share the job was given: MAX_JOBS when set, else "
                                                              "every CPU of the process's affinity)")
    ap.add_argument("--profile-tag", default=None, help="profiles/<tag>_pmc_summary.json for traffic/limiter")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=INT",
                    help="tuning experiments only: set engine.NAME (COMP_WARMUP, COMP_SUPER_FRAMES) or "
                         "design.DEFAULT_TILE before the jobs are planned")
    args = ap.parse_args(argv)
    if args.params is None:
        args.params = WORKLOADS[args.workload].get("params", "full")
    for kv in args.tune:
        name, val = kv.split("=")
        from mastering_amd import design, engine
        mod = design if name == "DEFAULT_TILE" else engine
        if not hasattr(mod, name):
            raise SystemExit(f"--tune: unknown knob {name}")
        setattr(mod, name, int(val))
    return args


# ----------------------------------------------------------------- CPU baseline
def cpu_baseline(args, wl, params):
    """Faithful-cost CPU path (oracle/faithful_cost.py), 1 core and N cores."""
    from mastering_amd.synth import pink_noise_pcm16
    from oracle import faithful_cost
    from oracle import mastering_oracle as mo
    rate = wl["rate"]
    frames = int(wl["seconds"] * rate)
    pcm = pink_noise_pcm16(frames if wl["seconds"] <= 300 else 300 * rate, rate, 2, track=0)
    affinity = len(os.sched_getaffinity(0))
    share = os.environ.get("MAX_JOBS")
    procs = args.cpu_procs or (int(share) if share and share.isdigit() and int(share) > 0 else affinity)
    n_chunks = len(mo.chunk_ranges(pcm.shape[0], rate))
    if n_chunks == 1:
        procs = 1  # one chunk: nothing to spread over cores
    r = faithful_cost.time_track(pcm, rate, params, chunks_1core=args.cpu_chunks, procs=procs)
    reps = 1
    while r["track_s_1core"] * reps < 2.0 and reps < 50:  # short tracks (C1): best of repeats, >= 2 s of CPU work
        r2 = faithful_cost.time_track(pcm, rate, params, chunks_1core=args.cpu_chunks, procs=1)
        for k in ("per_chunk_s_1core", "tail_s"):
            r[k] = min(r[k], r2[k])
        reps += 1
    scale = frames / pcm.shape[0]  # C4: a 5-min sample track, chunk cost extrapolated to the 2-h track
    t1 = (r["per_chunk_s_1core"] * r["chunks"] + r["tail_s"]) * scale
    tn = r.get("track_s_ncore", t1) * scale
    best = min(t1, tn)
    stages = ("numpy/scipy stages + pydub's per-frame Python compressor loop, pyloudnorm restated"
              if params.get("multiband") else "numpy/scipy stages, pyloudnorm restated; no multiband stage")
    ncore = (f" and {r['procs']} chunks on {r['procs']} cores at once ({r['wall_s_per_round']:.2f} s)"
             if r.get("procs", 1) > 1 else "")
    return {"value": frames / best, "unit": "stereo frames/s", "cores": r.get("procs", 1) if tn <= t1 else 1,
            "kind": "port",
            "sample": (f"faithful-cost reference path ({stages}): {r['sampled_chunks_1core']} whole 30 s chunk(s) "
                       f"on 1 core ({r['per_chunk_s_1core']:.3f} s each, best of {reps}){ncore}, the whole-track "
                       f"tail ({r['tail_s']:.3f} s), extrapolated to the {wl['desc'].split(':')[0]} track "
                       f"({frames} frames, {r['chunks'] * scale:.0f} chunks); value = the faster of the 1-core and "
                       f"N-core legs"),
            "single_core": {"value": frames / t1, "cores": 1, "track_s": t1},
            "multi_core": ({"value": frames / tn, "cores": r["procs"], "track_s": tn} if r.get("procs", 1) > 1
                           else None),
            "extrapolated": r["chunks"] * scale > r["sampled_chunks_1core"],
            "host_cpus": {"os_cpu_count": os.cpu_count(), "affinity": affinity, "max_jobs_env": share,
                          "leg_processes": r.get("procs", 1),
                          "policy": ("one chunk: 1 process" if n_chunks == 1 else "--cpu-procs" if args.cpu_procs
                                     else "MAX_JOBS (the CPU share the GPU box gives one GPU's job)"
                                     if procs != affinity else "every CPU of the affinity mask")}}


class stdout_to_stderr:
    """Redirect file descriptor 1 to 2 (native libraries print on it) for a block."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


# ----------------------------------------------------------------- workloads
class Runner:
    """One rank's share of a workload; step() masters it once."""

    def __init__(self, args, wl, params, rank, world, local, dist):
        import torch

        from mastering_amd import Job, native
        from mastering_amd.synth import pink_noise_chunks, pink_noise_pcm16
        self.args, self.wl, self.params, self.rank, self.world = args, wl, params, rank, world
        self.torch = torch
        self.dev = f"cuda:{local}"
        self.ctx = native.context(local)
        rate = wl["rate"]
        frames = int(wl["seconds"] * rate)
        self.kind = args.workload
        out_kind = native.MM_OUT_F32
        if self.kind == "C4":
            from mastering_amd import distributed as D
            self.D = D
            self.plan = D.plan_time_shards(frames, rate, 2, world, rank)
            c0 = self.plan.f0 // (30 * rate)
            c1 = -(-self.plan.f1 // (30 * rate))
            pcm = pink_noise_chunks(c0, c1, rate, 2, track=0)
            self.x = torch.from_numpy(pcm.astype(np.float32) / 32768).to(self.dev)
            self.out = torch.empty((self.plan.frames, 2), dtype=torch.float32, device=self.dev)
            uid = D.rccl_unique_id() if rank == 0 else None
            if world > 1:
                obj = [uid]
                dist.broadcast_object_list(obj, src=0)
                uid = obj[0]
            with stdout_to_stderr():  # RCCL prints its version banner on stdout: keep stdout the JSON line
                self.coll = D.LibraryCollectives.create(self.ctx, rank, world, uid)
            self.backend = D.GpuBackend(self.ctx)
            self.frames_step = self.plan.frames
            self.total_frames_step = frames  # the whole track per step (strong scaling)
            self.jobs = [self.backend.make_job(self.plan, params, out_kind)]
        else:
            tracks = wl["tracks"]
            self.jobs, self.xs, self.outs = [], [], []
            # the batch's tracks back to back in one device buffer (per-track views): a
            # fused unit of whole-chunk tracks then reads them in place (mm_master_batch)
            self.x_all = torch.empty((tracks * frames, 2), dtype=torch.float32, device=self.dev)
            for t in range(tracks):
                pcm = pink_noise_pcm16(frames, rate, 2, track=rank * tracks + t)
                self.x_all[t * frames:(t + 1) * frames].copy_(torch.from_numpy(pcm.astype(np.float32) / 32768))
                self.xs.append(self.x_all[t * frames:(t + 1) * frames])
                job = Job(frames, rate, 2, params, out_kind=out_kind)
                self.jobs.append(job)
                self.outs.append(torch.empty((job.frames_proc, 2), dtype=torch.float32, device=self.dev))
            self.frames_step = frames * tracks
            self.total_frames_step = frames * tracks * world
        self.results = None

    def step(self, want_results=False):
        from mastering_amd import engine, native
        if self.kind == "C4":
            info = self.D.master_time_sharded(self.backend, self.plan, self.params, self.x.data_ptr(),
                                              self.out.data_ptr(), self.coll, out_kind=native.MM_OUT_F32)
            self.ctx.sync()
            if want_results:
                self.results = [info]
        elif len(self.jobs) == 1:
            res = native.MMResult() if want_results else None
            engine.master_device(self.ctx, self.jobs[0], self.xs[0].data_ptr(), self.outs[0].data_ptr(), res)
            if want_results:
                self.results = [res]
        else:
            r = engine.master_batch(self.ctx, self.jobs, [x.data_ptr() for x in self.xs],
                                    [o.data_ptr() for o in self.outs], with_results=want_results)
            if want_results:
                self.results = r


def valu_ceiling(prof, dom):
    """The f64-VALU ceiling beside the HBM one, from the profile's SQ pass:
    SQ_INSTS_VALU (wave64 VALU instructions per launch, chip total) over the
    kernel's average duration, against 1024 SIMDs issuing one wave64 f64 FMA
    every 4 cycles at 2.4 GHz (MI355X_MICROARCH.md: 78.6 TF f64 vector)."""
    ks = prof.get("kernels", {})

    def one(k):
        q = ks.get(k, {})
        n, ns = (q.get("sq") or {}).get("SQ_INSTS_VALU"), q.get("avg_ns")
        if not n or not ns:
            return None
        g = n / (ns * 1e-9) / 1e9
        return {"achieved": g, "frac": g / VALU_PEAK_G, "instrs_per_launch": n, "avg_launch_ms": ns / 1e6}

    per = {k: one(k) for k in ks}
    per = {k: v for k, v in per.items() if v}
    tot_ns = sum(ks[k]["avg_ns"] * ks[k].get("launches_per_step", 1) for k in per)
    chain = (sum(v["frac"] * ks[k]["avg_ns"] * ks[k].get("launches_per_step", 1) for k, v in per.items()) / tot_ns
             if tot_ns else None)
    return {"unit": "G wave64 VALU instr/s", "peak": VALU_PEAK_G, "dominant_kernel": per.get(dom),
            "chain_time_weighted_frac": chain,
            "per_kernel_frac": {k: round(v["frac"], 4) for k, v in per.items()}}


LANE_OPS_PEAK = 1024 * 16 * 2.4e9  # VALU lane-instructions/s: 1024 SIMDs x 16 lanes x 2.4 GHz (39.3 T)


def valu_floor(prof, n_frames, ms_step):
    """The chain's VALU floor: lane-instructions per stereo frame
    (SQ_INSTS_VALU x 64 lanes x launches per step over the step's frames, per kernel
    and summed) and the time the chip needs to issue them at one wave64 instruction
    per SIMD every 4 cycles (39.3 T lane-instr/s), against ms_per_step."""
    ks = prof.get("kernels", {})
    per = {}
    for k, q in ks.items():
        n = (q.get("sq") or {}).get("SQ_INSTS_VALU")
        if n:
            per[k] = n * 64.0 * q.get("launches_per_step", 1.0) / n_frames
    if not per:
        return None
    tot = sum(per.values())
    floor_ms = tot * n_frames / LANE_OPS_PEAK * 1e3
    return {"lane_instr_per_frame": tot, "floor_ms": floor_ms, "frac": floor_ms / ms_step,
            "peak_lane_instr_per_s": LANE_OPS_PEAK,
            "per_kernel_lane_instr_per_frame": {k: round(v, 1) for k, v in sorted(per.items(), key=lambda kv: -kv[1])},
            "scope": "SQ_INSTS_VALU x 64 x launches per step / frames per step, summed over the chain's kernels"}


# Arithmetic the exact recurrences themselves need, per stereo frame (DESIGN.md §4's
# column): fixed per frame, or per active / re-walked band-frame.
NEEDED_OPS_PER_FRAME = {"eq": 120, "xover": 122, "comp_rms": 39, "comp_apply": 45, "kweight": 22, "finalize": 10,
                        "kw_blocks": 4}  # (kw_blocks: numpy's f32 adds, 4 overlapping 0.4 s blocks per frame)
NEEDED_OPS_PER_ACTIVE = {"comp_describe": 16, "comp_pass0": 8}  # per active band-frame
NEEDED_OPS_PER_REWALKED = {"comp_fix": 8}  # per re-walked band-frame


def needed_floor(per_kernel_ms, n_frames, active, walked, ms_step):
    """The time the chip needs for the arithmetic the exact algorithm needs (not the
    instructions issued: no addressing, conversions, divergence or two-pass IIR
    overhead) at 39.3 T lane-ops/s, and the HBM fraction the 16 B/frame roofline
    would reach at that floor: the ceiling of an exact f64 implementation."""
    per = {k: float(v) for k, v in NEEDED_OPS_PER_FRAME.items() if k in per_kernel_ms}
    for k, v in NEEDED_OPS_PER_ACTIVE.items():
        if k in per_kernel_ms:
            per[k] = v * active / n_frames
    for k, v in NEEDED_OPS_PER_REWALKED.items():
        if k in per_kernel_ms:
            per[k] = v * walked / n_frames
    tot = sum(per.values())
    floor_ms = tot * n_frames / LANE_OPS_PEAK * 1e3
    return {"ops_per_frame": tot, "needed_floor_ms": floor_ms, "frac": floor_ms / ms_step,
            "hbm_frac_at_needed_floor": CHAIN_BYTES_PER_FRAME * n_frames / (floor_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
            "per_kernel_ops_per_frame": {k: round(v, 2) for k, v in per.items()},
            "scope": "f64/f32 operations the exact recurrences need per stereo frame (active and re-walked "
                     "band-frames from the run), at 1024 SIMDs x 16 lanes x 2.4 GHz"}


def profile_summary(tag):
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.json")
    try:
        with open(path) as f:
            return json.load(f), path
    except (OSError, ValueError):
        return None, path


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """`--gpus N` (N > 1) outside torch.distributed.run: this process becomes the
    launcher.  It runs the CPU baseline (rank 0's leg, before any GPU work), then
    starts N child processes of this script with RANK = LOCAL_RANK = 0..N-1,
    WORLD_SIZE = N and a 127.0.0.1 rendezvous, exactly the environment
    torch.distributed.run would give them; the ranks time themselves (barrier,
    max over ranks) and rank 0's JSON line is printed here.  The launcher never
    touches the GPU and never re-execs: the ranks are ordinary child processes,
    and a failing rank stops the others (by PID) and fails the launch."""
    import subprocess
    import tempfile
    wl, params = WORKLOADS[args.workload], PARAMS[args.params]
    child_argv = list(argv)
    tmp = tempfile.mkdtemp(prefix="mm_bench_")
    if not args.no_cpu_baseline and not args.dry_run:
        cpu = cpu_baseline(args, wl, params)
        path = os.path.join(tmp, "cpu_baseline.json")
        with open(path, "w") as f:
            json.dump(cpu, f)
        child_argv += ["--cpu-baseline-from", path]
    env = dict(os.environ, WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    procs, outs = [], []
    for r in range(args.gpus):
        out = open(os.path.join(tmp, f"rank{r}.out"), "w+")
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + child_argv,
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=out))
    rc = 0
    pending = set(range(args.gpus))
    while pending:
        for r in list(pending):
            code = procs[r].poll()
            if code is None:
                continue
            pending.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench launcher: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in pending:
                    procs[q].terminate()
        time.sleep(0.05)
    for r, out in enumerate(outs):
        out.seek(0)
        text = out.read()
        out.close()
        if args.dry_run or r == 0:
            sys.stdout.write(text)
        elif text:
            sys.stderr.write(text)
    sys.stdout.flush()
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        raise SystemExit(launch_ranks(args, argv))
    rank = int(os.environ.get("RANK", "0"))
    world = int(env_world or "1")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch N ranks with "
                         f"torch.distributed.run --nproc-per-node N, or run bench.py --gpus N alone")
    if args.dry_run:  # the control plane the timed run uses (gloo rendezvous, max over ranks), no GPU
        ranks_seen = 1
        if world > 1:
            import torch
            import torch.distributed as dist
            with stdout_to_stderr():  # gloo prints its connection banner on stdout
                dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            ranks_seen = int(t.item())
            dist.destroy_process_group()
        print(json.dumps({"rank": rank, "local_rank": local, "world": world, "ranks_in_group": ranks_seen,
                          "workload": args.workload,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        return
    wl = WORKLOADS[args.workload]
    params = PARAMS[args.params]

    # the CPU baseline first: its worker processes fork before anything initialises the GPU
    cpu = None
    if rank == 0 and args.cpu_baseline_from:
        with open(args.cpu_baseline_from) as f:
            cpu = json.load(f)  # measured by the launcher before it started the ranks
    elif rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, wl, params)

    import torch
    import torch.distributed as dist
    if world > 1:
        with stdout_to_stderr():  # gloo prints its connection banner on stdout: keep stdout the JSON line
            dist.init_process_group("gloo")  # control plane only (barrier, max of timings, RCCL id broadcast)
    torch.cuda.set_device(local)
    run = Runner(args, wl, params, rank, world, local, dist if world > 1 else None)

    for _ in range(args.warmup):
        run.step()
    run.ctx.sync()
    torch.cuda.synchronize()

    # ---- timed region: no instrumentation
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run.step()
    run.ctx.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = t1 - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # ---- profiling pass: HIP events around every launch
    run.ctx.timing(True)
    P = max(1, args.profile_steps)
    for i in range(P):
        run.step(want_results=(i == P - 1))
    stats = run.ctx.kernel_stats()
    run.ctx.timing(False)
    if world > 1 and args.workload == "C4":
        # every rank gated the same all-reduced vector: the same loudness and gain on
        # every rank, checked before rank 0 reports
        lg = [None] * world
        dist.all_gather_object(lg, (run.results[0]["loudness"], run.results[0]["gain_linear"]))
        if any(v != lg[0] for v in lg):
            raise SystemExit(f"C4: ranks disagree on loudness / gain: {lg}")

    if rank == 0:
        from mastering_amd import native
        ms_step = dt / args.steps * 1e3
        value = run.total_frames_step * args.steps / dt
        per = {k: (ms / P, n / P) for k, (ms, n) in stats.items()}  # per step: ms, launches
        dom = max(per, key=lambda k: per[k][0])
        dom_ms, launches = per[dom]
        avg_s = dom_ms / 1e3 / max(launches, 1)
        res = run.results
        active = sum(int(getattr(r, "comp_active", 0) or 0) for r in res) if res and not isinstance(res[0], dict) \
            else 0
        walked = sum(int(getattr(r, "comp_walked", 0) or 0) for r in res) if res and not isinstance(res[0], dict) \
            else 0
        jumped = sum(int(getattr(r, "comp_jumped", 0) or 0) for r in res) if res and not isinstance(res[0], dict) \
            else 0
        iters = [int(r.comp_iters) for r in res] if res and not isinstance(res[0], dict) else None
        job0 = run.jobs[0]
        n_frames = run.frames_step
        g_tiles = sum(j.G for j in run.jobs)
        walked_per_launch = walked / max(launches, 1) if dom == "comp_fix" else 0
        ibl = intermediate_bytes(dom, n_frames, g_tiles, active, walked_per_launch)
        # 16 B per stereo frame; a launch processes the step's frames over
        # its launches per step (a kernel launched once per step: every frame)
        bpl = CHAIN_BYTES_PER_FRAME * n_frames / max(launches, 1)
        k_achieved = bpl / avg_s / 1e9
        chain_gbs = CHAIN_BYTES_PER_FRAME * n_frames / (ms_step / 1e3) / 1e9
        # PMC traffic and SQ shares, only from a profile of these exact sources
        sha = source_sha()
        default_params = WORKLOADS[args.workload].get("params", "full")
        tag = args.profile_tag or f"{PROFILE_ROUND}_{args.workload}" + ("" if args.params == default_params else args.params)
        prof, prof_path = profile_summary(tag)
        traffic = limiter = dom_traffic = None
        valu = vfloor = None
        prof_note = f"no profile at {os.path.relpath(prof_path, ROOT)}"
        if prof is not None:
            if prof.get("source_sha") != sha:
                prof_note = (f"{os.path.relpath(prof_path, ROOT)} was measured on sources {prof.get('source_sha')}, "
                             f"these are {sha}: traffic not reported")
            else:
                prof_note = os.path.relpath(prof_path, ROOT)
                traffic = prof.get("chain", {}).get("bytes_per_step")
                limiter = prof.get("chain", {}).get("limiter")
                k = prof.get("kernels", {}).get(dom, {})
                dom_traffic = k.get("bytes_per_launch")
                valu = valu_ceiling(prof, dom)
                vfloor = valu_floor(prof, n_frames, ms_step)
        if vfloor is None:
            vfloor = {}
        vfloor["needed"] = needed_floor({k: v[0] for k, v in per.items()}, n_frames, active, walked, ms_step)
        vfloor["needed_floor_ms"] = vfloor["needed"]["needed_floor_ms"]
        line = {
            "metric": METRIC, "value": value, "unit": "stereo frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
            "scaling": "strong" if args.workload == "C4" else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": wl["desc"] + ", " + PARAMS_DESC[args.params],
                       "frames_per_track": int(wl["seconds"] * wl["rate"]), "tracks_per_gpu": wl["tracks"],
                       "rate": wl["rate"], "frames_per_rank_step": n_frames,
                       "parallelism": (f"time-sharded x{world} (library RCCL)" if args.workload == "C4"
                                       else f"file-sharded x{world}"),
                       "in": "f32 interleaved (decoded PCM16)", "out": "f32 interleaved"},
            "roofline": {"bound": "hbm", "limiter": limiter, "achieved": chain_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": chain_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_step": CHAIN_BYTES_PER_FRAME * n_frames,
                         "scope": "whole chain: 16 B per stereo frame over ms_per_step",
                         "profile": prof_note, "source_sha": sha,
                         "dominant_kernel": {"name": dom, "achieved": k_achieved,
                                             "frac": k_achieved / HBM_PEAK_GBS,
                                             "algorithmic_bytes_per_launch": bpl,
                                             "scope": "16 B per stereo frame (SURVEY §8(d)) x frames per launch "
                                                      "(the step's frames / launches per step), over the "
                                                      "kernel's event-timed average launch",
                                             "intermediate_bytes_per_launch": ibl,
                                             "intermediate_frac": (ibl / avg_s / 1e9 / HBM_PEAK_GBS
                                                                   if ibl is not None else None),
                                             "avg_launch_ms": avg_s * 1e3,
                                             "launches_per_step": launches, "traffic": dom_traffic},
                         "valu_ceiling": valu, "valu": vfloor},
            "chain": {"device_ms_per_step": sum(v[0] for v in per.values()),
                      "comp_iters": iters, "comp_active_frames": active, "comp_rewalked_frames": walked, "comp_jumped_frames": jumped,
                      "kernels_ms_per_step": {k: round(v[0], 4) for k, v in per.items()},
                      # launches per step (library kernels; comp_fix counts every queued sweep,
                      # quiet ones included; runtime copies / fills are not library launches)
                      "launches_per_step": round(sum(v[1] for v in per.values()), 2),
                      "kernel_launches_per_step": {k: round(v[1], 2) for k, v in per.items()}},
        }
        if args.workload == "C4":
            line["chain"]["loudness"] = res[0]["loudness"] if res else None
        if cpu is not None:
            line["cpu_baseline"] = cpu
        del native
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
