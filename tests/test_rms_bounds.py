"""CPU model of comp_rms_t_kernel's global addresses (csrc/compressor.hip): every
band-plane load (phase A: the frame entering the window and the one leaving it,
including the prefetch past the tile and the loads of lanes past the chunk's tiles
or the track, which load as lane 0 does) and every M-plane store (phase C: T rows
plus the padding to whole walk blocks) stays inside its buffer.  Round 5 found a
negative drop index for such invalid lanes this way (a GPU fault on a 40 s track);
the model restates the kernel's index arithmetic at the geometries the product
uses.  The geometry (tile, tiles per super-tile, columns per chunk and per
workgroup, rows per tile and per column) comes from the library's own planning
function mm_solve_geometry for a planned Job, not restated here, so the model
follows the kernel when its geometry moves."""
import ctypes

import pytest

from mastering_amd import engine, native


def _geometry(frames, rate):
    job = engine.Job(frames, rate, 2, {"multiband": True})
    g = native.MMSolveGeom()
    assert native.load().mm_solve_geometry(ctypes.byref(job.job), ctypes.byref(g)) == 0
    return job, g


def _check(frames, rate, look, prefetch=24):
    job, geo = _geometry(frames, rate)
    T, K, N = job.tile, job.tiles_per_chunk, job.frames_proc
    G = (N + T - 1) // T
    TPS, CB = geo.tps, geo.col_block
    assert geo.rms_group_tiles == TPS * CB == 256  # comp_rms_t: 256 threads, lane = tile in phase A
    SPC = geo.cols_per_chunk
    NS = geo.chunks * SPC
    TP, RP = geo.tile_rows, geo.rows
    chunk_elems = geo.chunk_plane_bytes // 8
    assert chunk_elems == RP * SPC
    band_len = T * G
    bad = []
    for cbk in range(NS // CB):
        cc = (cbk * CB) // SPC
        jt0 = (cbk * CB - cc * SPC) * TPS
        chunk0 = cc * K * T
        for w in range(TPS):
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
        for w in range(TPS):
            for lane in range(CB):
                jt = jt0 + lane * TPS + w
                if jt >= K or cc * K + jt >= G:
                    continue
                sl = (cc * SPC + jt // TPS) % SPC
                e = (sl // CB) * RP * CB + (sl % CB) + w * TP * CB
                if not (e >= 0 and e + (TP - 1) * CB < chunk_elems):
                    bad.append(("store", cbk, w, lane, e))
    return bad


@pytest.mark.parametrize("seconds,rate,look", [(40, 44100, 882), (95, 44100, 2205), (31, 44100, 882),
                                               (29, 44100, 882), (65, 44100, 20), (180, 96000, 1920),
                                               (61.3, 48000, 480)])
def test_comp_rms_t_addresses_in_bounds(seconds, rate, look):
    bad = _check(int(seconds * rate), rate, look)
    assert not bad, bad[:5]
