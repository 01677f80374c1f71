"""ctypes binding of libmastering_amd.so (C-ABI declared in include/mastering.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is
visible, every compute entry point raises.  Struct layouts mirror mastering.h
field for field (natural C alignment on x86-64).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# MM_LIB: an alternative build of the same library (tools/ablation experiments only)
LIB_PATH = os.environ.get("MM_LIB") or os.path.join(_HERE, "libmastering_amd.so")

MM_OUT_I16, MM_OUT_F32 = 0, 1
MM_IN_F32, MM_IN_I16 = 0, 1
MM_F32, MM_F64 = 0, 1  # per-stage operator sample dtypes
MM_ERR_ARG = -1
BATCH_STREAMS = 8  # MM_BATCH_STREAMS
MAX_DIM, TILE_POW, BLK_POW = 8, 8, 65

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int64_p = ctypes.POINTER(ctypes.c_int64)


class MMIir(ctypes.Structure):
    _fields_ = [("nsec", ctypes.c_int32), ("nsec_branch0", ctypes.c_int32), ("dim", ctypes.c_int32),
                ("tpb", ctypes.c_int32), ("tile", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("sos", (ctypes.c_double * 5) * 4),
                ("phi_tile_pow", (ctypes.c_double * (MAX_DIM * MAX_DIM)) * TILE_POW),
                ("phi_blk_pow", (ctypes.c_double * (MAX_DIM * MAX_DIM)) * BLK_POW)]


class MMBand(ctypes.Structure):
    _fields_ = [("thresh_rms", ctypes.c_double), ("attack_frames", ctypes.c_double),
                ("release_frames", ctypes.c_double), ("look", ctypes.c_int32), ("r0", ctypes.c_int32),
                ("lut", c_double_p), ("lut_key", ctypes.c_uint64)]


class MMJob(ctypes.Structure):
    _fields_ = [("frames_in", ctypes.c_int64), ("frames_proc", ctypes.c_int64),
                ("channels", ctypes.c_int32), ("rate", ctypes.c_int32), ("tile", ctypes.c_int32),
                ("tiles_per_chunk", ctypes.c_int32),
                ("sat_keep", ctypes.c_float), ("sat_mix", ctypes.c_float), ("sat_drive", ctypes.c_float),
                ("sat_on", ctypes.c_int32), ("width", ctypes.c_double), ("width_on", ctypes.c_int32),
                ("multiband_on", ctypes.c_int32), ("lufs_on", ctypes.c_int32), ("out_kind", ctypes.c_int32),
                ("lufs_target", ctypes.c_double), ("eq", MMIir), ("xover", MMIir), ("kweight", MMIir),
                ("band", MMBand * 3), ("comp_warmup", ctypes.c_int32), ("comp_max_iters", ctypes.c_int32),
                ("comp_super", ctypes.c_int32), ("in_kind", ctypes.c_int32),
                ("n_blocks", ctypes.c_int64), ("block_lo", c_int64_p), ("block_hi", c_int64_p),
                ("n_segs", ctypes.c_int64), ("seg_bounds", c_int64_p), ("block_scale", ctypes.c_double),
                ("sat_table", ctypes.POINTER(ctypes.c_float)), ("sat_key", ctypes.c_uint64)]


class MMResult(ctypes.Structure):
    _fields_ = [("loudness", ctypes.c_double), ("gain_linear", ctypes.c_double), ("frames_out", ctypes.c_int64),
                ("comp_iters", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("comp_active", ctypes.c_int64), ("comp_walked", ctypes.c_int64),
                ("comp_jumped", ctypes.c_int64)]


class MMSolveGeom(ctypes.Structure):
    _fields_ = [("tps", ctypes.c_int32), ("tile_rows", ctypes.c_int32), ("rows", ctypes.c_int32),
                ("walk_block", ctypes.c_int32), ("cols_per_chunk", ctypes.c_int64), ("chunks", ctypes.c_int64),
                ("chunk_plane_bytes", ctypes.c_int64), ("plane_bytes", ctypes.c_int64),
                ("col_block", ctypes.c_int32), ("rms_group_tiles", ctypes.c_int32)]


ABI_VERSION = 4  # MM_ABI_VERSION of include/mastering.h


class MMWavInfo(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_int64), ("data_offset", ctypes.c_int64), ("rate", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("format", ctypes.c_int32), ("bits", ctypes.c_int32)]


# every symbol include/mastering.h declares (checked by tests/test_abi.py)
EXPORTS = ("mm_create", "mm_destroy", "mm_last_error", "mm_sync", "mm_version", "mm_source_sha", "mm_master",
           "mm_master_device",
           "mm_stage_chunks", "mm_kweight_range_end", "mm_hop_energies", "mm_shard_loudness_device",
           "mm_shard_energies_device", "mm_gate_finalize_device", "mm_allreduce_sum_f64_device",
           "mm_allgather_f64_device",
           "mm_gate_loudness", "mm_finalize",
           "mm_read_mix", "mm_timing", "mm_kernel_stats", "mm_comm_unique_id", "mm_comm_init", "mm_comm_destroy",
           "mm_allreduce_sum_f64", "mm_allgather_f64", "mm_wav_probe", "mm_master_wav",
           "mm_op_pcm_to_float", "mm_op_saturation", "mm_op_saturation_table", "mm_op_stereo_width", "mm_op_quantize", "mm_op_soft_limiter",
           "mm_op_gain", "mm_op_sosfilt", "mm_op_loudness", "mm_op_multiband", "mm_master_batch",
           "mm_op_saturation_legacy", "mm_op_soft_limiter_legacy", "mm_op_sosfilt_mix", "mm_op_compress_bands",
           "mm_solve_geometry", "mm_np_sum_f32", "mm_check_compressor_math")

_lib = None
_lock = threading.Lock()


def load():
    """Load the HIP library; raise loudly if it was not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        try:  # share ONE HIP runtime with PyTorch when it is present (same soname)
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP extension not built: {LIB_PATH} missing (run __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        P = ctypes.POINTER
        sig = {
            "mm_create": ([ctypes.c_int, P(vp)], ctypes.c_int),
            "mm_destroy": ([vp], ctypes.c_int),
            "mm_last_error": ([vp], ctypes.c_char_p),
            "mm_sync": ([vp], ctypes.c_int),
            "mm_version": ([], ctypes.c_int),
            "mm_source_sha": ([], ctypes.c_char_p),
            "mm_master": ([vp, P(MMJob), vp, vp, P(MMResult)], ctypes.c_int),
            "mm_master_device": ([vp, P(MMJob), vp, vp, P(MMResult)], ctypes.c_int),
            "mm_master_batch": ([vp, ctypes.c_int, P(MMJob), P(vp), P(vp), P(MMResult)], ctypes.c_int),
            "mm_stage_chunks": ([vp, P(MMJob), vp], ctypes.c_int),
            "mm_wav_probe": ([vp, ctypes.c_char_p, P(MMWavInfo)], ctypes.c_int),
            "mm_master_wav": ([vp, P(MMJob), ctypes.c_char_p, ctypes.c_char_p, P(MMResult)], ctypes.c_int),
            "mm_kweight_range_end": ([vp, c_double_p], ctypes.c_int),
            "mm_hop_energies": ([vp, c_double_p, c_double_p], ctypes.c_int),
            "mm_shard_energies_device": ([vp, c_double_p, ctypes.c_int64, ctypes.c_int64, vp], ctypes.c_int),
            "mm_gate_finalize_device": ([vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                                         ctypes.POINTER(ctypes.c_int32), ctypes.c_double, ctypes.c_double, vp,
                                         c_double_p], ctypes.c_int),
            "mm_shard_loudness_device": ([vp, c_double_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                          ctypes.c_double, ctypes.c_double, ctypes.c_int32, vp, c_double_p],
                                         ctypes.c_int),
            "mm_gate_loudness": ([P(MMJob), c_double_p, c_double_p], ctypes.c_int),
            "mm_finalize": ([vp, ctypes.c_double, ctypes.c_int, vp], ctypes.c_int),
            "mm_read_mix": ([vp, P(ctypes.c_int16)], ctypes.c_int),
            "mm_timing": ([vp, ctypes.c_int], ctypes.c_int),
            "mm_kernel_stats": ([vp, ctypes.c_char_p, ctypes.c_int, c_double_p, c_int64_p, ctypes.c_int],
                                ctypes.c_int),
            "mm_comm_unique_id": ([ctypes.c_char_p], ctypes.c_int),
            "mm_comm_init": ([vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p], ctypes.c_int),
            "mm_comm_destroy": ([vp], ctypes.c_int),
            "mm_allreduce_sum_f64": ([vp, c_double_p, ctypes.c_int64], ctypes.c_int),
            "mm_allgather_f64": ([vp, c_double_p, c_double_p, ctypes.c_int64], ctypes.c_int),
            "mm_allreduce_sum_f64_device": ([vp, vp, ctypes.c_int64], ctypes.c_int),
            "mm_allgather_f64_device": ([vp, vp, vp, ctypes.c_int64], ctypes.c_int),
            "mm_op_pcm_to_float": ([vp, vp, ctypes.c_int64, vp], ctypes.c_int),
            "mm_op_saturation": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_double, vp], ctypes.c_int),
            "mm_op_saturation_table": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_double,
                                        ctypes.POINTER(ctypes.c_float), vp], ctypes.c_int),
            "mm_op_stereo_width": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_double, vp], ctypes.c_int),
            "mm_op_quantize": ([vp, ctypes.c_int, vp, ctypes.c_int64, vp], ctypes.c_int),
            "mm_op_soft_limiter": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_double], ctypes.c_int),
            "mm_op_gain": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_double, vp], ctypes.c_int),
            "mm_op_sosfilt": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_int, P(MMIir), ctypes.c_int, vp],
                              ctypes.c_int),
            "mm_op_loudness": ([vp, P(MMJob), ctypes.c_int, vp, c_double_p], ctypes.c_int),
            "mm_op_multiband": ([vp, P(MMJob), vp, vp], ctypes.c_int),
            "mm_op_saturation_legacy": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_double, vp], ctypes.c_int),
            "mm_op_soft_limiter_legacy": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_double], ctypes.c_int),
            "mm_op_sosfilt_mix": ([vp, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_int, P(MMIir), ctypes.c_double,
                                   ctypes.c_double, vp], ctypes.c_int),
            "mm_op_compress_bands": ([vp, P(MMJob), vp, vp, vp, vp], ctypes.c_int),
            "mm_solve_geometry": ([P(MMJob), P(MMSolveGeom)], ctypes.c_int),
            "mm_np_sum_f32": ([P(ctypes.c_float), ctypes.c_int64, P(ctypes.c_float)], ctypes.c_int),
            "mm_check_compressor_math": ([vp, ctypes.c_int, c_double_p, c_double_p, ctypes.c_int64, c_double_p],
                                         ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.mm_version() != ABI_VERSION:  # the structs above mirror one header version
            raise RuntimeError(f"{LIB_PATH}: ABI version {lib.mm_version()}, this binding expects {ABI_VERSION}")
        _lib = lib
        return lib


class Context:
    """One HIP stream + device work buffers (mm_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        self.ptr = ctypes.c_void_p()
        rc = self.lib.mm_create(device, ctypes.byref(self.ptr))
        if rc != 0:
            raise RuntimeError(f"mm_create(device={device}) failed ({rc}): no usable MI355X/HIP device")
        self.device = device

    def check(self, rc: int, what: str):
        """Raise on a negative status: ValueError for bad arguments or input files
        (MM_ERR_ARG, like the reference's decode errors), RuntimeError otherwise."""
        if rc < 0:
            msg = self.lib.mm_last_error(self.ptr)
            text = f"{what} failed ({rc}): {msg.decode(errors='replace') if msg else ''}"
            raise ValueError(text) if rc == MM_ERR_ARG else RuntimeError(text)
        return rc

    def close(self):
        if self.ptr:
            self.lib.mm_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # timing ---------------------------------------------------------------
    def timing(self, enable: bool):
        self.check(self.lib.mm_timing(self.ptr, int(enable)), "mm_timing")

    def kernel_stats(self):
        cap = 64
        names = ctypes.create_string_buffer(8192)
        ms = (ctypes.c_double * cap)()
        n = (ctypes.c_int64 * cap)()
        k = self.check(self.lib.mm_kernel_stats(self.ptr, names, 8192, ms, n, cap), "mm_kernel_stats")
        labels = names.value.decode().split("\n") if k else []
        return {labels[i]: (ms[i], n[i]) for i in range(k)}

    def sync(self):
        self.check(self.lib.mm_sync(self.ptr), "mm_sync")


_tls = threading.local()


def context(device: int = 0) -> Context:
    """Per-thread context (the reference's GUI calls from a worker thread)."""
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    if device not in ctxs:
        ctxs[device] = Context(device)
    return ctxs[device]


def library_sha() -> str:
    """Source hash embedded in the loaded library (srcsha.library_sha at build time)."""
    return load().mm_source_sha().decode()
