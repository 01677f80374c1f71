"""Benchmark: stereo frames/s through the full mastering chain (BASELINE.json metric).

Workload at N=1 is BASELINE config C2: one 5-min 44.1 kHz stereo f32 track, full
chain (exciter 30 %, techno EQ, width 1.3, 3-band compressor with the worker's
default thresholds, LUFS -14) on one MI355X.  For N>1 every rank masters its own
5-min track (file sharding as in C3: no data-path collective) -> "scaling": "weak".
A "step" = one complete mastering of the track with input and output resident
in HBM (mm_master_device: every kernel of the chain plus its single host sync).

Timing: W warm-up steps, then K steps timed with no instrumentation, bracketed
by a barrier + device sync on both sides (max over ranks).  A separate profiling
pass (HIP events around every launch on the library's stream) gives per-kernel
device times; the dominant kernel's roofline uses its ALGORITHMIC bytes per
launch over its average launch duration.  `traffic` comes from the
committed rocprofv3 PMC summary of the same command (tools/pmc.sh ->
profiles/<round>_pmc_summary.json) when present.

Run:  python bench.py [--gpus N] [--steps K] [--warmup W]
Multi-GPU (driver): python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")  # CPU baseline leg: one core
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("MKL_NUM_THREADS", "1")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "python-audio-mastering_amd"))

import numpy as np  # noqa: E402

METRIC = "stereo frames/sec through full mastering chain, 44.1 kHz f32; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_pmc_summary.json")
P_FULL = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
          "saturation": 30, "width": 1.3, "multiband": True, "lufs": -14.0}


ENVELOPE_NOTE = ("the compressor envelope is a sequential non-linear recurrence solved exactly by speculative "
                 "super-tile walks (one lane each, ~0.4 waves per SIMD): VALU-issue and dependent-latency bound, "
                 "not HBM bound; the warm-up re-reads each M from the memory fabric ~7x (PMC traffic) "
                 "(DESIGN.md §4)")


def algorithmic_bytes(kernel, n, g, active, walked_per_launch):
    """Minimum HBM bytes one launch must move for its own inputs/outputs (stereo,
    n frames, g tiles, `active` compressor frames over the 3 bands)."""
    table = {
        "eq": 8 * n + 4 * n,                  # f32 L,R in; int16 pair q1 out
        "pre_pointwise": 8 * n + 4 * n,
        "xover": 4 * n + 12 * n,              # q1 in; three int16-pair bands out
        "comp_rms": 12 * n + 6 * n,           # bands in; uint16 rms x3 out
        "comp_offsets": 3 * g * 8,            # counts in, offsets out
        "comp_compact": 6 * n + 8 * active,   # rms in; M of active frames out
        "comp_pass0": 8 * active,             # M of every active frame
        "comp_fix": 8 * walked_per_launch,    # M of the re-walked frames
        "comp_record": 16 * active,           # M in, att out
        "comp_tstart": 3 * g * 12,
        "comp_apply": 6 * n + 12 * n + 4 * n,  # rms, bands in; mix out
        "kweight": 4 * n,                     # mix in
        "seg_reduce": g * 24,
        "gate": 0,
        "finalize": 4 * n + 8 * n,            # mix in; f32 L,R out
    }
    return table.get(kernel)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--profile-steps", type=int, default=5, help="steps of the per-kernel event-timed pass")
    ap.add_argument("--seconds", type=float, default=300.0, help="track length (C2: 300 s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=300.0,
                    help="CPU baseline sample (default: the whole C2 track)")
    return ap.parse_args()


def cpu_baseline(pcm, rate, seconds):
    """The oracle (CPU restatement of the reference chain, 'port'): numpy/scipy
    stages + the pydub compressor loop in C, one thread, on a prefix of the track."""
    from oracle import mastering_oracle as mo
    n = min(int(seconds * rate), pcm.shape[0])
    sample = np.ascontiguousarray(pcm[:n])
    mo.master(sample[: rate * 2], rate, P_FULL)  # build / warm caches
    t0 = time.perf_counter()
    mo.master(sample, rate, P_FULL)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "stereo frames/s", "cores": 1, "kind": "port",
            "sample": f"first {n / rate:.0f} s ({n} frames) of the rank-0 C2 track, full chain (oracle/: "
                      f"numpy/scipy stages + pydub compressor loop in C + pyloudnorm restatement), 1 thread, "
                      f"{dt:.2f} s"}


def pmc_traffic(kernel):
    try:
        with open(PMC_SUMMARY) as f:
            k = json.load(f)["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    return None if k is None else k.get("bytes_per_launch")


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")  # control plane only (barrier, max of timings)
    torch.cuda.set_device(local)

    from mastering_amd import Job, engine, native
    from mastering_amd.synth import pink_noise_pcm16

    rate = 44100
    frames = int(args.seconds * rate)
    pcm = pink_noise_pcm16(frames, rate, 2, track=rank)
    x = torch.from_numpy(np.ascontiguousarray(pcm.astype(np.float32) / 32768)).to(f"cuda:{local}")
    job = Job(frames, rate, 2, P_FULL, out_kind=native.MM_OUT_F32)
    out = torch.empty((job.frames_proc, 2), dtype=torch.float32, device=f"cuda:{local}")
    ctx = native.context(local)

    def step(res=None):
        return engine.master_device(ctx, job, x.data_ptr(), out.data_ptr(), res)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    torch.cuda.synchronize()

    # ---- timed region: no instrumentation
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
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
    res = native.MMResult()
    ctx.timing(True)
    for i in range(args.profile_steps):
        step(res if i == args.profile_steps - 1 else None)
    stats = ctx.kernel_stats()
    ctx.timing(False)

    if rank == 0:
        P = args.profile_steps
        total_frames = frames * world * args.steps
        value = total_frames / dt
        per = {k: (ms / P, n / P) for k, (ms, n) in stats.items()}  # per step: ms, launches
        dom = max(per, key=lambda k: per[k][0])
        ms_step, launches = per[dom]
        avg_s = ms_step / 1e3 / max(launches, 1)
        walked_per_launch = res.comp_walked / max(launches, 1) if dom == "comp_fix" else 0
        bpl = algorithmic_bytes(dom, job.frames_proc, job.G, res.comp_active, walked_per_launch)
        achieved = bpl / avg_s / 1e9 if bpl is not None else None
        traffic = pmc_traffic(dom)
        dev_ms = sum(v[0] for v in per.values())
        line = {
            "metric": METRIC, "value": value, "unit": "stereo frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "C2: 5-min 44.1 kHz stereo f32 pink-noise track per GPU, full chain "
                                   "(sat 30, techno EQ, width 1.3, multiband defaults, LUFS -14)",
                       "frames_per_track": frames, "tracks_per_gpu": 1, "rate": rate,
                       "parallelism": f"file-sharded x{world}", "out": "f32 interleaved (decoded PCM16)"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved is not None else None,
                         "traffic": traffic, "algorithmic_bytes_per_launch": bpl,
                         "avg_launch_ms": avg_s * 1e3, "launches_per_step": launches,
                         "note": ENVELOPE_NOTE if dom in ("comp_pass0", "comp_fix", "comp_record") else None},
            "chain": {"algorithmic_bytes_per_frame": 16, "device_ms_per_step": dev_ms,
                      "achieved_GBps": 16 * job.frames_proc / (dt / args.steps) / 1e9,
                      "frac_of_peak": 16 * job.frames_proc / (dt / args.steps) / 1e9 / HBM_PEAK_GBS,
                      "comp_iters": res.comp_iters, "comp_active_frames": res.comp_active,
                      "comp_rewalked_frames": res.comp_walked,
                      "kernels_ms_per_step": {k: round(v[0], 4) for k, v in per.items()}},
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(pcm, rate, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
