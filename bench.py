"""Benchmark: stereo frames/s through the full mastering chain (BASELINE.json metric).

Workload at N=1 is BASELINE config C2: one 5-min 44.1 kHz stereo f32 track, full
chain (exciter 30 %, techno EQ, width 1.3, 3-band compressor with the worker's
default thresholds, LUFS -14) on one MI355X.  For N>1 every rank masters its own
5-min track (file sharding as in C3: no data-path collective) -> "scaling": "weak".
A "step" = one complete mastering of the track with input and output resident
in HBM (mm_master_device), including the host-side loudness gating.

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
P_FULL = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
          "saturation": 30, "width": 1.3, "multiband": True, "lufs": -14.0}

# Algorithmic HBM bytes per frame of each kernel ("Kernels"): the
# bytes the kernel must move at minimum for its own inputs/outputs (stereo).
KERNEL_BYTES_PER_FRAME = {
    "eq_pass1": 8, "eq_pass2": 8 + 4, "pre_pointwise": 8 + 4,
    "xover_pass1": 4, "xover_pass2": 4 + 12,
    "comp_rms": 12 + 24, "comp_pass0": 24, "comp_apply": 24 + 12 + 4,
    "kw_pass1": 4, "kw_pass2": 4, "finalize": 4 + 8,
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=300.0, help="track length (C2: 300 s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=60.0, help="CPU baseline sample length")
    return ap.parse_args()


def cpu_baseline(pcm, rate, seconds):
    """Oracle (CPU restatement, 'port') on a bounded sample of the same workload."""
    from oracle import mastering_oracle as mo
    n = int(seconds * rate)
    sample = np.ascontiguousarray(pcm[:n])
    mo.master(sample[: rate * 2], rate, P_FULL)  # warm caches / build
    t0 = time.perf_counter()
    mo.master(sample, rate, P_FULL)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "stereo frames/s", "cores": 1, "kind": "port",
            "sample": f"first {seconds:.0f} s ({n} frames) of the rank-0 C2 track, full chain incl. "
                      f"compressor loop in C and pyloudnorm-restated LUFS, 1 thread, {dt:.2f} s"}


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

    def step():
        return engine.master_device(ctx, job, x.data_ptr(), out.data_ptr())

    for _ in range(args.warmup):
        step()
    ctx.sync()
    torch.cuda.synchronize()

    ctx.timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
    ctx.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = t1 - t0
    stats = ctx.kernel_stats()
    ctx.timing(False)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    if rank == 0:
        total_frames = frames * world * args.steps
        value = total_frames / dt
        # dominant kernel by total device time
        per = {k: (ms, n) for k, (ms, n) in stats.items()}
        dom = max(per, key=lambda k: per[k][0])
        ms, n = per[dom]
        avg_s = ms / 1e3 / max(n, 1)
        bpf = KERNEL_BYTES_PER_FRAME.get(dom)
        if bpf is None:  # fix sweeps re-read M for re-run tiles only; price per frame of M (24 B)
            bpf = 24
        achieved = bpf * frames / avg_s / 1e9
        kern_ms = sum(v[0] for v in per.values()) / args.steps
        line = {
            "metric": METRIC, "value": value, "unit": "stereo frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "C2: 5-min 44.1 kHz stereo f32 pink-noise track per GPU, full chain "
                                   "(sat 30, techno EQ, width 1.3, multiband defaults, LUFS -14)",
                       "frames_per_track": frames, "tracks_per_gpu": 1, "rate": rate,
                       "parallelism": f"file-sharded x{world}", "out": "f32 interleaved (decoded PCM16)"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "bytes_per_frame": bpf, "avg_launch_ms": avg_s * 1e3, "launches_per_step": n / args.steps},
            "chain": {"algorithmic_bytes_per_frame": 16, "device_ms_per_step": kern_ms,
                      "achieved_GBps": 16 * frames / (dt / args.steps) / 1e9,
                      "frac_of_peak": 16 * frames / (dt / args.steps) / 1e9 / HBM_PEAK_GBS,
                      "comp_iters": res.comp_iters if res is not None else None,
                      "kernels_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in per.items()}},
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(pcm, rate, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
