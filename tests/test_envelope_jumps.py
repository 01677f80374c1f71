"""The envelope solve's release jumps (csrc/compressor.hip Describer /
release_jump) restated in Python and checked on the CPU: every jump
the device would take lands bit for bit on the state pydub's step-by-step loop
reaches (AME:207-209).

The per-frame M sequences (inactive frames M = 0 included: the solve runs in
frame space, one descriptor per 125-frame tile) come from the oracle's own band
split of a pink-noise track at P_HOT thresholds (every envelope branch fires), so
the check covers long release stretches, parity ties and binade crossings of real
trajectories."""
import math
import struct

import numpy as np
import pytest

from mastering_amd import design

SEG, JB = 125, 8  # tile length, binades per descriptor (== csrc/compressor.hip)
MANT = (1 << 52) - 1
NAN = float("nan")


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _from(b):
    return struct.unpack("<d", struct.pack("<Q", b))[0]


def _step(a, m, A, R):
    """pydub's update (Appendix A); M/A, M/R correctly rounded like the device's."""
    inc, dec = m / A, m / R
    if a <= m:
        return min(a + inc, m)
    return max(a - dec, 0.0)


def _describe(M, R):
    """The Describer for one active tile: (max M, e0, q[2 JB]), e0 = binade of max M."""
    e0 = (_bits(max(M)) >> 52) - 1023
    r0 = [_from(((e0 + k // 2 + 1023) << 52) | (MANT - 63 + k % 2)) for k in range(2 * JB)]
    r = list(r0)
    for m in M:
        dec = m / R
        r = [x - dec for x in r]
    q = []
    for k in range(2 * JB):
        rb = _bits(r[k])
        ok = (rb >> 52) == e0 + k // 2 + 1023 and (rb & MANT) != 0
        q.append(r0[k] - r[k] if ok else NAN)
    return max(M), e0, q


def _jump(desc, att):
    """release_jump: the state after the segment, or None."""
    mx, e0, q = desc
    if not att > 0.0:
        return None
    ab = _bits(att)
    k = (ab >> 52) - 1023 - e0
    if k < 0 or k >= JB:
        return None
    x = att - q[2 * k + (ab & 1)]
    if math.isnan(x):
        return None
    xb = _bits(x)
    if not x > mx or (xb >> 52) != (ab >> 52) or (xb & MANT) == 0:
        return None
    return x


def _band_M(seconds=20):
    import bench
    from mastering_amd.synth import pink_noise_pcm16
    from oracle import mastering_oracle as mo
    rate, st = 44100, bench.P_HOT
    pcm = pink_noise_pcm16(seconds * rate, rate, 2, track=7)
    x = mo.stereo_width(mo.equalize(mo.saturation(mo.pcm_to_float(pcm), st["saturation"]), rate, st), st["width"])
    thr, rat = mo.multiband_params(st)
    out = []
    for band, t, r, (at, rel) in zip(mo.band_split(mo.quantize(x), rate), thr, rat, mo.BAND_TIMES):
        bc = design.band_constants(rate, t, r, at, rel)
        e2 = (band.astype(np.int64) ** 2).sum(axis=1)
        cs = np.concatenate([[0], np.cumsum(e2)])
        i = np.arange(band.shape[0])
        lo = np.maximum(i - bc["look"], 0)
        n = (i - lo) * 2
        S = cs[i] - cs[lo]
        rms = np.zeros(band.shape[0], np.int64)
        nz = n > 0
        rms[nz] = np.floor(np.sqrt(S[nz] / n[nz])).astype(np.int64)  # == audioop.rms (test_oracle.py)
        M = bc["table"][np.minimum(rms, 32768)]
        out.append((M, bc["attack_frames"], bc["release_frames"]))
    return out


@pytest.mark.timeout(300)
def test_release_jumps_are_exact():
    jumps = checked = 0
    for M, A, R in _band_M():
        traj = [0.0]
        for m in M:
            traj.append(_step(traj[-1], m, A, R))
        for s0 in range(0, len(M) - SEG + 1, SEG):
            seg = [float(v) for v in M[s0:s0 + SEG]]
            if max(seg) == 0.0:
                continue  # inactive tile: held, never jumped
            desc = _describe(seg, R)
            true = traj[s0]
            # the true state, its neighbours (other parity / rounding), and states in
            # the descriptor's other binades
            for att in (true, math.nextafter(true, math.inf), math.nextafter(true, -math.inf), true * 1.5,
                        desc[0] * 1.0001, desc[0] * 2.01, desc[0] * 4.3):
                checked += 1
                x = _jump(desc, att)
                if x is None:
                    continue
                jumps += 1
                y = att
                for m in seg:
                    y = _step(y, m, A, R)
                assert x == y, (s0, att, x, y)
    assert jumps > 0.3 * checked, (jumps, checked)  # the jump conditions are not vacuous


SJ_TPS = 4  # tiles per super-tile with a composed record (== csrc/compressor.hip SJ_TPS)


def _binade(x):
    return (_bits(x) >> 52) - 1023


def _next_up(x):
    return math.nextafter(x, math.inf) if x > 0.0 else x


def _compose_super(descs):
    """compose_super: (e0s, entries[2 JB] of (L, [Q1..Q_TPS])) from SJ_TPS tile descriptors."""
    e0s = _binade(max(d[0] for d in descs))
    ents = []
    for k in range(2 * JB):
        e, par, Q, L, ok, qs = e0s + k // 2, k & 1, 0.0, 0.0, True, []
        for mx, e0t, q in descs:
            kt = e - e0t
            qv = q[2 * min(max(kt, 0), JB - 1) + par]
            ok = ok and 0 <= kt < JB and qv == qv
            Q += qv if ok else 0.0
            ok = ok and Q < math.ldexp(1.0, e)
            if ok:
                par ^= int(math.ldexp(qv, 52 - e)) & 1
            L = max(L, _next_up(mx + Q))
            qs.append(Q)
        ents.append((L if ok else NAN, qs))
    return e0s, ents


def _super_jump(rec, att):
    """The fix walker's super jump: the tiles' entry states and the exit state, or None."""
    e0s, ents = rec
    if not att > 0.0:
        return None
    ab = _bits(att)
    kb = (ab >> 52) - 1023 - e0s
    if kb < 0 or kb >= JB:
        return None
    L, qs = ents[2 * kb + (ab & 1)]
    x = att - qs[-1]
    xb = _bits(x)
    if not att > L or (xb >> 52) != (ab >> 52) or (xb & MANT) == 0:
        return None
    return [att] + [att - q for q in qs[:-1]], x


@pytest.mark.timeout(300)
def test_super_tile_jumps_are_exact():
    """Records composed from SJ_TPS consecutive active tiles' descriptors: a super
    jump lands on the state the step-by-step loop reaches, and every tile's entry
    state it writes equals the loop's."""
    jumps = checked = 0
    for M, A, R in _band_M():
        Ma = [float(v) for v in M if v != 0.0]  # the solve's compact (active) frames
        traj = [0.0]
        for m in Ma:
            traj.append(_step(traj[-1], m, A, R))
        span = SEG * SJ_TPS
        for s0 in range(0, len(Ma) - span + 1, span):
            segs = [Ma[s0 + t * SEG:s0 + (t + 1) * SEG] for t in range(SJ_TPS)]
            rec = _compose_super([_describe(sg, R) for sg in segs])
            true = traj[s0]
            for att in (true, math.nextafter(true, math.inf), math.nextafter(true, -math.inf), true * 1.5,
                        max(max(sg) for sg in segs) * 1.7):
                checked += 1
                r = _super_jump(rec, att)
                if r is None:
                    continue
                jumps += 1
                entries, x = r
                y = att
                for t, sg in enumerate(segs):
                    assert entries[t] == y, (s0, t, att)
                    for m in sg:
                        y = _step(y, m, A, R)
                assert x == y, (s0, att, x, y)
    assert jumps > 0.2 * checked, (jumps, checked)


def _e_walk(E, M, R):
    """The (max,+) release envelope the pass-0 guesses follow: every attack an
    instant clamp, E <- max(M, E - M/R) per frame (M/R correctly rounded)."""
    for m in M:
        E = max(m, E - m / R)
    return E


def _e_tile(E, ct, desc):
    """compressor.hip e_fold_tile: the tile's E exit from its entry E, exactly as the
    per-frame walk, from the tile's E walk from 0 (ct) and its release-jump record:
    E - q when the pure release from E stays in its binade (the release offsets do not
    depend on M), max'ed with ct (a trajectory that clamps ends on ct's: monotone
    steps); None when no record covers E (the device then takes E - D: inexact)."""
    if E == 0.0:
        return ct
    mx, e0, q = desc
    eb = _binade(E)
    if eb < e0:  # below the tile's largest M: it clamps there
        return ct
    if eb - e0 >= JB:
        return None
    x = E - q[2 * (eb - e0) + (_bits(E) & 1)]
    if math.isnan(x):
        return None
    xb = _bits(x)
    if (xb >> 52) != (_bits(E) >> 52) or (xb & MANT) == 0:
        return None
    return max(ct, x)


@pytest.mark.timeout(300)
def test_e_fold_by_tiles_is_exact():
    """The pass-0 guess folded tile by tile equals the per-frame (max,+) walk bit for
    bit whenever the tile records cover the state (so a guess coincides with a
    speculative walk's release values, as tools/study/envelope_model.c assumes)."""
    total = covered = 0
    for M, A, R in _band_M():
        Ma = [float(v) for v in M if v != 0.0]
        segs = [Ma[s0:s0 + SEG] for s0 in range(0, len(Ma) - SEG + 1, SEG)]
        E_frame = E_tile = 0.0
        for sg in segs:
            ct = _e_walk(0.0, sg, R)
            nxt = _e_tile(E_tile, ct, _describe(sg, R))
            E_frame = _e_walk(E_frame, sg, R)
            total += 1
            if nxt is None:  # not covered: restart the comparison from the exact value
                E_tile = E_frame
                continue
            covered += 1
            assert nxt == E_frame
            E_tile = nxt
    print(f"e fold: {covered} of {total} tiles covered by their records")
    assert covered > 0.9 * total
