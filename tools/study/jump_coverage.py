"""CPU study: how often could the envelope solve's release jumps apply on the TRUE
trajectory, and how long does a walk from the pass-0 guess (the M of its first
frame) take to coalesce with it?  Informs SEG / JB / e0 choice and the warm-up.
python tools/study/jump_coverage.py [seconds] [full|hot]"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd"), os.path.join(ROOT, "tests")]
import bench  # noqa: E402
import test_envelope_jumps as tj  # noqa: E402

secs = int(sys.argv[1]) if len(sys.argv) > 1 else 20
which = sys.argv[2] if len(sys.argv) > 2 else "full"
bench.P_HOT = bench.P_FULL if which == "full" else bench.P_HOT
SEG = tj.SEG


def describe(M, R, e0, jb):
    MANT = tj.MANT
    r0 = [tj._from(((e0 + k // 2 + 1023) << 52) | (MANT - 63 + k % 2)) for k in range(2 * jb)]
    r = list(r0)
    for m in M:
        dec = m / R
        r = [x - dec for x in r]
    q = []
    for k in range(2 * jb):
        rb = tj._bits(r[k])
        ok = (rb >> 52) == e0 + k // 2 + 1023 and (rb & MANT) != 0
        q.append(r0[k] - r[k] if ok else math.nan)
    return max(M), e0, q


def jump(desc, att, jb):
    mx, e0, q = desc
    if not att > 0.0:
        return None
    ab = tj._bits(att)
    k = (ab >> 52) - 1023 - e0
    if k < 0 or k >= jb:
        return None
    x = att - q[2 * k + (ab & 1)]
    if math.isnan(x):
        return None
    xb = tj._bits(x)
    if not x > mx or (xb >> 52) != (ab >> 52) or (xb & tj.MANT) == 0:
        return None
    return x


for bi, (M, A, R) in enumerate(tj._band_M(secs)):
    M = [float(v) for v in M]
    traj = [0.0]
    for m in M:
        traj.append(tj._step(traj[-1], m, A, R))
    nseg = len(M) // SEG
    cnt = {}
    above = 0
    for s in range(nseg):
        seg = M[s * SEG:(s + 1) * SEG]
        att = traj[s * SEG]
        if att > max(seg):
            above += 1
        for name, e0 in (("e0=M0", (tj._bits(seg[0]) >> 52) - 1023), ("e0=max", (tj._bits(max(seg)) >> 52) - 1023)):
            for jb in (4, 8):
                d = describe(seg, R, e0, jb)
                cnt[(name, jb)] = cnt.get((name, jb), 0) + (jump(d, att, jb) is not None)
    print(f"band {bi}: frames {len(M)} A={A:.1f} R={R:.1f} segs {nseg} state>max(M) {above / nseg:.3f} "
          + " ".join(f"{k[0]},JB{k[1]}:{v / nseg:.3f}" for k, v in cnt.items()))
    # coalescence from the guess M[p] at tile starts p (every 1000 frames)
    dist = []
    for p in range(1000, len(M) - 20000, 1000):
        a = M[p]
        n = 0
        while a != traj[p + n] and n < 20000:
            a = tj._step(a, M[p + n], A, R)
            n += 1
        dist.append(n)
    d = np.array(dist or [0])
    print(f"   coalescence from guess: median {np.median(d):.0f} p90 {np.percentile(d, 90):.0f} "
          f"p99 {np.percentile(d, 99):.0f} max {d.max()} >6000: {(d > 6000).mean():.3f} n={d.size}")
