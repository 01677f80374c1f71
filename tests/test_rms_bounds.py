"""CPU model of comp_rms_t_kernel's global addresses (csrc/compressor.hip): every
band-plane load (phase A: the frame entering the window and the one leaving it,
including the prefetch past the tile and the loads of lanes past the chunk's tiles
or the track, which load as lane 0 does) and every M-plane store (phase C: T rows
plus the padding to whole walk blocks) stays inside its buffer.  Round 5 found a
negative drop index for such invalid lanes this way (a GPU fault on a 40 s track);
the model restates the kernel's index arithmetic at the geometries the product
uses (design.choose_tile, 4-tile super-tiles, 64-column blocks)."""
import pytest

from mastering_amd import design


def _check(frames, rate, look, prefetch=24):
    chunk = 30 * rate
    T = design.choose_tile(chunk)
    K = chunk // T
    N = frames
    G = (N + T - 1) // T
    TPS = 4
    SPC = ((K + TPS - 1) // TPS + 63) // 64 * 64
    NS = ((G + K - 1) // K) * SPC
    WB = design.WALK_BLOCK
    TP = (T + WB - 1) // WB * WB
    RP = TPS * TP + 2 * WB
    chunk_elems = RP * SPC
    band_len = T * G
    bad = []
    for cbk in range(NS // 64):
        cc = (cbk * 64) // SPC
        jt0 = (cbk * 64 - cc * SPC) * 4
        chunk0 = cc * K * T
        for w in range(4):
            lanes = [(jt0 + w * 64 + l, cc * K + jt0 + w * 64 + l) for l in range(64)]
            valid = [jt < K and g < G for jt, g in lanes]
            if not any(valid):
                continue  # the wave loads nothing
            assert valid[0], "a wave's invalid lanes must be its last ones"
            info = []
            for (jt, g), v in zip(lanes, valid):
                g32 = g if v else lanes[0][1]
                f0 = g32 * T
                ln = min(T, N - f0) if v else 0
                d_first = max(f0 - look, chunk0)
                skip = d_first - (f0 - look) if v else 0
                gd = d_first // T
                info.append((v, g32, ln, skip, gd, d_first - gd * T))
            steady = all((not v) or (sk == 0 and ln == T) for v, _, ln, sk, _, _ in info) and look > 0
            dgo, nd_u = info[0][4] - info[0][1], info[0][5]
            for v, g32, ln, skip, gd, nd in info:
                for i in range(T + prefetch):
                    if steady:
                        ii = min(i, T - 1)
                        k = nd_u + ii
                        wrap = int(k >= T)
                        idx = (ii * G + g32, (k - wrap * T) * G + dgo + wrap + g32)
                    else:
                        ii = max(min(i, ln - 1), 0)
                        k = nd + max(ii - skip, 0)
                        wrap = int(k >= T)
                        idx = (ii * G + g32, (k - wrap * T) * G + gd + wrap)
                    bad += [("load", cbk, w, i, x) for x in idx if not 0 <= x < band_len]
        for w in range(4):
            for lane in range(64):
                jt = jt0 + lane * 4 + w
                if jt >= K or cc * K + jt >= G:
                    continue
                sl = (cc * SPC + jt // 4) % SPC
                e = (sl >> 6) * RP * 64 + (sl & 63) + w * TP * 64
                if not (e >= 0 and e + (TP - 1) * 64 < chunk_elems):
                    bad.append(("store", cbk, w, lane, e))
    return bad


@pytest.mark.parametrize("seconds,rate,look", [(40, 44100, 882), (95, 44100, 2205), (31, 44100, 882),
                                               (29, 44100, 882), (65, 44100, 20), (180, 96000, 1920),
                                               (61.3, 48000, 480)])
def test_comp_rms_t_addresses_in_bounds(seconds, rate, look):
    bad = _check(int(seconds * rate), rate, look)
    assert not bad, bad[:5]
