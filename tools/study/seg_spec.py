"""CPU study: a segment-level speculative warm-up for pass 0.  Per SEG-frame
segment, precomputed in parallel: the release-jump descriptor and the exits of a
few reference entries (exact walks).  A lane then crosses a segment in O(1): an
exact jump when its state is a release entry, else the exit of the reference
entries when they all merged (the segment forgets its entry), else the exit of
the nearest reference (a guess).  Measures how often the state reached at a tile
start equals the true one, by warm-up length in segments.
python tools/study/seg_spec.py [seconds] [full|hot]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "python-audio-mastering_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools", "study")]
import bench  # noqa: E402
import test_envelope_jumps as tj  # noqa: E402

secs = int(sys.argv[1]) if len(sys.argv) > 1 else 20
which = sys.argv[2] if len(sys.argv) > 2 else "full"
if which == "full":
    bench.P_HOT = bench.P_FULL
SEG, U = tj.SEG, 1000


def walk(a, seg, A, R):
    for m in seg:
        a = tj._step(a, m, A, R)
    return a


for bi, (M, A, R) in enumerate(tj._band_M(secs)):
    M = [float(v) for v in M]
    nseg = len(M) // SEG
    if nseg < 300:
        print(f"band {bi}: {len(M)} active frames, skipped")
        continue
    traj = [0.0]
    for m in M:
        traj.append(tj._step(traj[-1], m, A, R))
    desc, refs = [], []
    cls = {"jump": 0, "merged": 0, "merged_wrong": 0, "other": 0}
    for s in range(nseg):
        seg = M[s * SEG:(s + 1) * SEG]
        d = tj._describe(seg, R)
        mx = d[0]
        ent = (0.0, seg[0], mx)
        ex = tuple(walk(e, seg, A, R) for e in ent)
        desc.append(d)
        refs.append((ent, ex))
        t_in, t_out = traj[s * SEG], traj[(s + 1) * SEG]
        if tj._jump(d, t_in) is not None:
            cls["jump"] += 1
        elif ex[0] == ex[1] == ex[2]:
            cls["merged" if ex[0] == t_out else "merged_wrong"] += 1
        else:
            cls["other"] += 1

    def cross(a, s):
        x = tj._jump(desc[s], a)
        if x is not None:
            return x
        ent, ex = refs[s]
        if ex[0] == ex[1] == ex[2]:
            return ex[0]
        k = int(np.argmin([abs(a - e) for e in ent]))
        return ex[k]

    print(f"band {bi}: segs {nseg} " + " ".join(f"{k}={v / nseg:.4f}" for k, v in cls.items()))
    for ws in (10, 30, 60, 100, 200):
        ok = tot = 0
        for t0 in range(ws, nseg - 1, U // SEG):
            a = M[(t0 - ws) * SEG]
            for s in range(t0 - ws, t0):
                a = cross(a, s)
            ok += a == traj[t0 * SEG]
            tot += 1
        print(f"   warm-up {ws:3d} segments: tile start exact {ok / tot:.4f} ({tot} tiles)")
