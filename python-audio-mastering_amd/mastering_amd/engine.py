"""MI355X mastering engine — the drop-in for the reference's hot path.

Reference boundary: `process_audio_from_gcs(gcs_uri, settings)`
(worker/audio_mastering_engine.py:24, "AME"), whose DSP is AME:43-98.  Here the
same chain runs behind `process(input_path, output_path, params)` with local WAV
IO instead of GCS; `params` uses the worker's settings keys and defaults
(AME:58-86).  All per-sample work runs in hand-written HIP kernels
(libmastering_amd.so, include/mastering.h) — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import functools
import os

import numpy as np

from . import design, native

# AME:15-20, verbatim values and descriptions.
EQ_PRESETS = {
    "techno": {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
               "description": "Boosted sub-bass and highs, scooped mids for a powerful club sound."},
    "dubstep": {"bass_boost": 5.0, "mid_cut": 4.0, "presence_boost": 2.0, "treble_boost": 3.5,
                "description": "Aggressive low-end and crisp highs, with a significant mid-cut."},
    "pop": {"bass_boost": 2.0, "mid_cut": 0.0, "presence_boost": 3.5, "treble_boost": 2.5,
            "description": "Focused on vocal clarity with a solid low-end and bright highs."},
    "rock": {"bass_boost": 1.5, "mid_cut": -2.0, "presence_boost": 2.5, "treble_boost": 1.0,
             "description": "Warm low-mids for guitars and punchy presence for snare/vocals."},
}

COMP_WARMUP = 0  # super-tiles of speculative warm-up walk before each one (none: the sweeps' jumps repair starts)
COMP_MAX_ITERS = 100000
# envelope solve unit: super-tiles of 4 tiles (900 frames at the default tile) at
# EVERY rate, the tile count the super-tile release records assume (SJ_TPS in
# csrc/compressor.hip).  Not scaled with the rate (comp_rms maps a wave to one tile
# position of 64 super-tiles, so its M stores are 512-byte runs at any length).
COMP_SUPER_FRAMES = 900


def comp_super_frames(rate: int, tile: int = design.DEFAULT_TILE) -> int:
    """Super-tile length in frames: COMP_SUPER_FRAMES / DEFAULT_TILE (4) whole tiles of
    the track's tile at every rate."""
    del rate  # (see COMP_SUPER_FRAMES)
    return max(1, int(round(COMP_SUPER_FRAMES / design.DEFAULT_TILE))) * tile


class Job:
    """A planned mastering job: the mm_job POD plus the host arrays it points to."""

    def __init__(self, frames_in: int, rate: int, channels: int, params: dict, out_kind: int = native.MM_OUT_I16,
                 seg_bounds=None, check_length: bool = True, single_chunk: bool = False,
                 crossover=(design.LOW_CROSSOVER, design.HIGH_CROSSOVER)):
        """`seg_bounds` (time-sharded ranks, distributed.py): this range's loudness
        segment bounds relative to its first frame; the whole-track gating then
        happens on the host after the all-reduce.  `check_length=False` skips
        pyloudnorm's minimum-length check (it applies to the whole track).
        `single_chunk`: the whole input is ONE line (the per-stage operators of
        ops.py, which the reference calls on one chunk) instead of AME:48's 30 s
        chunks; `crossover`: apply_multiband_compressor's (low, high) Hz."""
        if channels not in (1, 2):
            raise ValueError("only mono and stereo are supported (AME:119,137,152)")
        params = dict(params or {})
        self.params = params
        self.rate, self.channels, self.frames_in = int(rate), int(channels), int(frames_in)
        multiband = bool(params.get("multiband"))
        if single_chunk:
            bounds = [(0, self.frames_in)] if self.frames_in else []
            self.tile = design.OPS_TILE
            self.tiles_per_chunk = max(1, -(-self.frames_in // self.tile))
        else:
            bounds = design.chunk_bounds(self.frames_in, self.rate)
            nominal = design.pydub_frame(design.CHUNK_MS, self.rate)
            design.check_chunk_geometry(bounds, nominal, self.rate, multiband)
            # without the compressor the chain is the IIR stages alone, which want the
            # lanes of shorter tiles on a short track (C1: 0.139 ms at 125 against 0.188 at 225)
            self.tile = design.choose_tile(nominal, None if multiband else design.NOCOMP_TILE)
            self.tiles_per_chunk = nominal // self.tile
        self.chunks = bounds
        self.frames_proc = bounds[-1][1] if bounds else 0
        lufs = params.get("lufs")
        if check_length and lufs is not None and self.frames_proc < 0.4 * self.rate:
            # pyloudnorm util.valid_audio (AME:218)
            raise ValueError("Audio must have length greater than the block size.")

        j = native.MMJob()
        j.frames_in, j.frames_proc = self.frames_in, self.frames_proc
        j.channels, j.rate, j.tile, j.tiles_per_chunk = self.channels, self.rate, self.tile, self.tiles_per_chunk
        on, keep, mix, drive = design.saturation_consts(params.get("saturation", 0))
        j.sat_on, j.sat_keep, j.sat_mix, j.sat_drive = on, keep, mix, drive
        if on:  # the exciter on the int16 grid: numpy's own float32 values (design.saturation_table)
            self._sat_tab, j.sat_key = design.saturation_table(params.get("saturation", 0))
            j.sat_table = self._sat_tab.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        w = params.get("width", 1.0)
        j.width_on = int(w != 1.0 and self.channels == 2)
        j.width = float(w) if w is not None else 1.0
        j.multiband_on = int(multiband)
        j.lufs_on = int(lufs is not None)
        j.lufs_target = float(lufs) if lufs is not None else 0.0
        j.out_kind = out_kind
        G = -(-self.frames_proc // self.tile) if self.frames_proc else 0
        self.G = G
        tpb = design.LB_THREADS // self.channels  # stereo stages run lane pairs
        # --- EQ (1 branch)
        eq = design.eq_sections(self.rate, params)
        self._fill_iir(j.eq, eq, [len(eq)], self.tile, tpb)
        # --- crossover (2 branches of 2)
        if multiband:
            self._fill_iir(j.xover, design.crossover_sections(self.rate, *crossover), [2, 2], self.tile, tpb)
            self._tables = []
            for b in range(3):
                tk, td, rk, rd = design.BAND_DEFAULTS[b]
                at, rel = design.BAND_TIMES[b]
                bc = design.band_constants(self.rate, params.get(tk, td), params.get(rk, rd), at, rel)
                tab = np.ascontiguousarray(bc["lut"])
                self._tables.append(tab)
                jb = j.band[b]
                jb.thresh_rms, jb.attack_frames, jb.release_frames = bc["thresh_rms"], bc["attack_frames"], \
                    bc["release_frames"]
                jb.look = bc["look"]
                nz = np.flatnonzero(tab[:, 0])
                jb.r0 = int(nz[0]) if nz.size else 32769
                jb.lut = tab.ctypes.data_as(native.c_double_p)
                jb.lut_key = bc["lut_key"]
        j.comp_warmup = COMP_WARMUP
        j.comp_max_iters = COMP_MAX_ITERS
        j.comp_super = comp_super_frames(self.rate, self.tile)
        # --- loudness
        if lufs is not None:
            self._fill_iir(j.kweight, design.kweight_sections(self.rate), [2],
                           self.tile // design.kweight_sub(self.tile), design.LB_THREADS)
            if seg_bounds is None:
                nb, lo, hi, segb, scale = design.loudness_blocks(self.frames_proc, self.rate)
            else:  # rank-local segments; blocks are gated over the whole track elsewhere
                segb = np.asarray(seg_bounds, dtype=np.int64)
                nb, lo, hi, scale = 1, np.zeros(1, np.int64), segb[-1:].copy(), 1.0 / (0.4 * self.rate)
            self._lo, self._hi, self._segb = (np.ascontiguousarray(lo), np.ascontiguousarray(hi),
                                              np.ascontiguousarray(segb))
            j.n_blocks = nb
            j.block_lo = self._lo.ctypes.data_as(native.c_int64_p)
            j.block_hi = self._hi.ctypes.data_as(native.c_int64_p)
            j.n_segs = len(segb) - 1
            j.seg_bounds = self._segb.ctypes.data_as(native.c_int64_p)
            j.block_scale = scale
        self.job = j

    @staticmethod
    @functools.lru_cache(maxsize=32)
    def _tables(sections, branches, tile, tpb):
        A = design.transition_matrix(list(sections), list(branches))
        t = design.lookback_tables(A, tile, tpb)
        return (np.ascontiguousarray(t["tile_pow"].reshape(design.TILE_POW, -1)),
                np.ascontiguousarray(t["blk_pow"].reshape(design.BLK_POW, -1)))

    @classmethod
    def _fill_iir(cls, dst, sections, branches, tile, tpb):
        dst.nsec = len(sections)
        dst.nsec_branch0 = branches[0]
        dst.dim = 2 * len(sections)
        dst.tpb = tpb
        dst.tile = int(tile)
        for s, sec in enumerate(sections):
            for k in range(5):
                dst.sos[s][k] = float(sec[k])
        if not sections:
            return
        key = tuple(tuple(float(v) for v in sec) for sec in sections)
        tp, bp = cls._tables(key, tuple(branches), int(tile), int(tpb))
        ctypes.memmove(dst.phi_tile_pow, tp.ctypes.data, tp.nbytes)
        ctypes.memmove(dst.phi_blk_pow, bp.ctypes.data, bp.nbytes)


def _device_input(pcm: np.ndarray):
    """PCM as the library takes it: int16 stays int16 (decoded /32768 on the GPU,
    AME:117-121; half the PCIe bytes), float32 is taken as decoded PCM."""
    if pcm.dtype == np.int16:
        return np.ascontiguousarray(pcm), native.MM_IN_I16
    if pcm.dtype == np.float32:
        return np.ascontiguousarray(pcm), native.MM_IN_F32
    raise TypeError("PCM must be int16 or float32")


def _info(job: "Job", res: native.MMResult) -> dict:
    return {"loudness": res.loudness if job.job.lufs_on else None,
            "gain_db": (float(job.job.lufs_target) - res.loudness) if job.job.lufs_on else None,
            "gain_linear": res.gain_linear, "frames": job.frames_proc, "comp_iters": res.comp_iters,
            "comp_walked": res.comp_walked, "comp_jumped": res.comp_jumped, "comp_active": res.comp_active,
            "chunks": len(job.chunks), "tile": job.tile}


def master_pcm(pcm: np.ndarray, rate: int, params: dict, out_kind: int = native.MM_OUT_I16, device: int = 0):
    """Run the whole chain (AME:48-89) on a PCM array [N] or [N, ch] on the GPU.
    Returns (out_pcm, info) with out_pcm int16 (or f32 = int16/32768)."""
    ch = 1 if pcm.ndim == 1 else pcm.shape[1]
    job = Job(pcm.shape[0], rate, ch, params, out_kind)
    x, job.job.in_kind = _device_input(pcm)
    shape = (job.frames_proc,) if ch == 1 else (job.frames_proc, ch)
    out = np.empty(shape, np.int16 if out_kind == native.MM_OUT_I16 else np.float32)
    ctx = native.context(device)
    res = native.MMResult()
    ctx.check(ctx.lib.mm_master(ctx.ptr, ctypes.byref(job.job), x.ctypes.data_as(ctypes.c_void_p),
                                out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(res)), "mm_master")
    return out, _info(job, res)


def wav_info(path: str, device: int = 0) -> native.MMWavInfo:
    """RIFF/WAVE header of `path` (PCM16 or float32), parsed by the library."""
    ctx = native.context(device)
    info = native.MMWavInfo()
    ctx.check(ctx.lib.mm_wav_probe(ctx.ptr, os.fsencode(path), ctypes.byref(info)), "mm_wav_probe")
    return info


def master_device(ctx: native.Context, job: Job, d_in: int, d_out: int, res: native.MMResult | None = None):
    """Device-resident variant (pointers from e.g. torch tensors).  With `res`
    the loudness, gain and compressor statistics are returned in it."""
    ctx.check(ctx.lib.mm_master_device(ctx.ptr, ctypes.byref(job.job), ctypes.c_void_p(d_in),
                                       ctypes.c_void_p(d_out), ctypes.byref(res) if res is not None else None),
              "mm_master_device")
    return res


def master_batch(ctx: native.Context, jobs, d_ins, d_outs, with_results: bool = True):
    """A batch of independent tracks with device-resident inputs/outputs
    (mm_master_batch).  Tracks with the same settings run as ONE timeline (each on
    whole chunks, every stage launched once for the batch); otherwise up to
    native.BATCH_STREAMS of them are in flight at once, each on its own stream.
    Returns one MMResult per job (or None)."""
    n = len(jobs)
    arr = (native.MMJob * n)(*[j.job for j in jobs])
    ins = (ctypes.c_void_p * n)(*[ctypes.c_void_p(int(p)) for p in d_ins])
    outs = (ctypes.c_void_p * n)(*[ctypes.c_void_p(int(p)) for p in d_outs])
    res = (native.MMResult * n)() if with_results else None
    ctx.check(ctx.lib.mm_master_batch(ctx.ptr, n, arr, ins, outs, res), "mm_master_batch")
    return list(res) if with_results else None


def process(input_path: str, output_path: str, params: dict, device: int = 0, verbose: bool = False) -> dict:
    """Master `input_path` (16-bit PCM or 32-bit float WAV) into `output_path`
    (16-bit PCM WAV, as AME:98 exports; params['output_format']='f32' writes float).
    The file streams through pinned staging into HBM and back (mm_master_wav).
    Raises ValueError for unreadable/unsupported input and RuntimeError for device
    failures, like the reference (AME:110-113)."""
    params = dict(params or {})
    fmt = params.pop("output_format", "pcm16")
    kind = native.MM_OUT_F32 if fmt == "f32" else native.MM_OUT_I16
    wi = wav_info(input_path, device)
    if verbose:
        print(f"Loaded {input_path}: {wi.frames} frames @ {wi.rate} Hz")
    job = Job(wi.frames, wi.rate, wi.channels, params, kind)
    ctx = native.context(device)
    res = native.MMResult()
    ctx.check(ctx.lib.mm_master_wav(ctx.ptr, ctypes.byref(job.job), os.fsencode(input_path), os.fsencode(output_path),
                                    ctypes.byref(res)), "mm_master_wav")
    info = _info(job, res)
    if verbose and info["loudness"] is not None:
        print(f"Current loudness: {info['loudness']:.2f} LUFS. Applying {info['gain_db']:.2f} dB gain...")
    info["output_path"] = os.path.abspath(output_path)
    return info
