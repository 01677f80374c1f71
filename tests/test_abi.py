"""The C-ABI boundary on CPU: the HIP library loads, exports every entry point
include/mastering.h declares, and the ctypes struct layouts in
mastering_amd/native.py agree with the C compiler's (no compute calls: no GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mastering.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(mm_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ("mm_create", "mm_destroy", "mm_last_error", "mm_master", "mm_master_device", "mm_stage_chunks",
                 "mm_kweight_range_end", "mm_hop_energies", "mm_finalize", "mm_comm_init",
                 "mm_allreduce_sum_f64"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    from mastering_amd import native
    if not os.path.exists(native.LIB_PATH):
        pytest.fail(f"HIP library not built: {native.LIB_PATH} (run __graft_entry__.build())")
    lib = native.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert sorted(native.EXPORTS) == declared_functions()
    assert lib.mm_version() == native.ABI_VERSION


def test_library_was_built_from_these_sources():
    """The library carries the hash of the sources it was compiled from
    (Makefile -DMM_SOURCE_SHA): a stale build is caught here and in smoke()."""
    from mastering_amd import native, srcsha
    assert native.library_sha() == srcsha.library_sha()


def test_struct_layouts_match_c(tmp_path):
    from mastering_amd import native
    prog = tmp_path / "layout.c"
    fields = {
        "mm_job": [f[0] for f in native.MMJob._fields_],
        "mm_iir": [f[0] for f in native.MMIir._fields_],
        "mm_band": [f[0] for f in native.MMBand._fields_],
        "mm_result": [f[0] for f in native.MMResult._fields_],
        "mm_wav_info": [f[0] for f in native.MMWavInfo._fields_],
        "mm_solve_geom": [f[0] for f in native.MMSolveGeom._fields_],
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mastering.h"', "int main(void){"]
    for st, fl in fields.items():
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fl:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)])
    got = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)]).decode().splitlines())
    classes = {"mm_job": native.MMJob, "mm_iir": native.MMIir, "mm_band": native.MMBand,
               "mm_result": native.MMResult, "mm_wav_info": native.MMWavInfo, "mm_solve_geom": native.MMSolveGeom}
    for st, cls in classes.items():
        assert int(got[st]) == ctypes.sizeof(cls), st
        for f in fields[st]:
            assert int(got[f"{st}.{f}"]) == getattr(cls, f).offset, f"{st}.{f}"


def test_product_path_fails_loudly_without_gpu():
    """No CPU fallback: without a usable device the context cannot be created."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from mastering_amd import native
    with pytest.raises(RuntimeError):
        native.Context(0)


@pytest.mark.parametrize("rate", [44100, 44056, 96000, 192000])
def test_solve_geometry_up_to_2_31_frames(rate):
    """The envelope solve's planning arithmetic (mm_solve_geometry, the function
    stage C itself plans with) accepts every track length below 2^31 frames: each
    chunk's M plane, walked through 32-bit buffer offsets, stays below 2^31 bytes
    whatever the length (round 3 refused tracks above ~511 M frames)."""
    from mastering_amd import design, engine, native
    lib = native.load()
    chunk = 30 * rate
    tile = design.choose_tile(chunk)
    prev = None
    for frames in (1, chunk, 511_000_000, 576_000_000, 1_000_000_000, 2**31 - 1):
        j = native.MMJob()
        j.frames_in = j.frames_proc = frames
        j.channels, j.rate, j.tile, j.tiles_per_chunk = 2, rate, tile, chunk // tile
        j.comp_super = engine.comp_super_frames(rate, tile)
        g = native.MMSolveGeom()
        assert lib.mm_solve_geometry(ctypes.byref(j), ctypes.byref(g)) == 0, frames
        assert g.chunks == -(-frames // chunk)
        assert g.cols_per_chunk % 64 == 0 and g.cols_per_chunk * g.tps >= chunk // tile
        assert g.walk_block == design.WALK_BLOCK  # choose_tile's padding model is the library's
        assert g.tile_rows >= tile and g.tile_rows % g.walk_block == 0
        assert 0 < g.chunk_plane_bytes < 2**31
        assert g.plane_bytes == 3 * g.chunks * g.chunk_plane_bytes
        if prev is not None:  # per-chunk geometry does not depend on the length
            assert (g.tps, g.rows, g.cols_per_chunk, g.chunk_plane_bytes) == prev
        prev = (g.tps, g.rows, g.cols_per_chunk, g.chunk_plane_bytes)


@pytest.mark.parametrize("rate", [11025, 16000, 22050, 32000, 44056, 44100, 48000, 88200, 96000, 192000])
def test_tile_geometry_every_rate(rate):
    """Tiles divide the 30 s chunk at every supported rate (225 frames where it divides,
    else the nearest divisor counting the 25-row walk-block padding; 125 without the
    compressor), and a super-tile is 4 tiles: the count the super-tile release records
    assume (SJ_TPS in csrc/compressor.hip), so super jumps run at every rate."""
    from mastering_amd import design, engine
    chunk = design.pydub_frame(design.CHUNK_MS, rate)
    t = design.choose_tile(chunk)
    assert chunk % t == 0 and 64 <= t <= 512
    if chunk % design.DEFAULT_TILE == 0:
        assert t == design.DEFAULT_TILE
    else:  # the fallback stays near the preferred length and wastes < 10 % of the walk rows
        assert abs(t - design.DEFAULT_TILE) <= 40 and ((t + 24) // 25 * 25 - t) / t < 0.1
    assert engine.comp_super_frames(rate, t) == 4 * t
    tn = design.choose_tile(chunk, design.NOCOMP_TILE)
    assert chunk % tn == 0
    job_mb = engine.Job(chunk, rate, 2, {"multiband": True})
    job_eq = engine.Job(chunk, rate, 2, {"multiband": False, "lufs": -14.0})
    assert job_mb.tile == t and job_eq.tile == tn
