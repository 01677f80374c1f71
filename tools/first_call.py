"""First-call cost: master_pcm on a FRESH context queues
COMP_SWEEPS = 8 fix-up sweeps (mastering.hip comp_queue: later solves on the same
context queue the last solve's need + 1).  Times, in this fresh process, the first
three master_pcm calls of the C2 track (host PCM16 in -> host PCM16 out, PCIe
included) and the device-resident chain (mm_master_device) on a fresh context and
on a warm one, with the queued-sweep launch counts from the per-kernel stats.
Usage (GPU box): python tools/first_call.py [seconds]   -> one JSON line"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-audio-mastering_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import bench
    from mastering_amd import Job, engine, master_pcm, native
    from mastering_amd.synth import pink_noise_pcm16
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
    rate = 44100
    pcm = pink_noise_pcm16(int(secs * rate), rate, 2, track=0)
    out = {"frames": int(pcm.shape[0]), "params": "P_FULL"}
    walls = []
    for _ in range(3):  # the process's one context (native.context) is fresh before the first
        t0 = time.perf_counter()
        master_pcm(pcm, rate, bench.P_FULL)
        walls.append((time.perf_counter() - t0) * 1e3)
    out["master_pcm_ms"] = walls
    # device-resident: a fresh context each for "first", then the same context again
    x = torch.from_numpy(pcm.astype(np.float32) / 32768).cuda()
    job = Job(pcm.shape[0], rate, 2, bench.P_FULL, out_kind=native.MM_OUT_F32)
    y = torch.empty((job.frames_proc, 2), dtype=torch.float32, device="cuda")
    ctx = native.Context(0)
    dev = []
    for i in range(4):
        ctx.timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = native.MMResult()
        engine.master_device(ctx, job, x.data_ptr(), y.data_ptr(), res)
        ctx.sync()
        dt = (time.perf_counter() - t0) * 1e3
        st = ctx.kernel_stats()
        ctx.timing(False)
        dev.append({"wall_ms": dt, "comp_fix_launches": st.get("comp_fix", (0, 0))[1],
                    "comp_fix_ms": st.get("comp_fix", (0, 0))[0], "kernel_ms": sum(v[0] for v in st.values()),
                    "sweeps_needed": int(res.comp_iters)})
    ctx.close()
    out["master_device_fresh_then_warm"] = dev
    print(json.dumps(out))


if __name__ == "__main__":
    main()
