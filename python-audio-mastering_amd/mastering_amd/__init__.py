"""mastering_amd — MI355X-native drop-in for the reference's mastering hot path.

Public surface (mirrors worker/audio_mastering_engine.py):
  EQ_PRESETS                   AME:15-20
  process(in, out, params)     AME:24-113 with local WAV IO instead of GCS
  master_pcm(pcm, rate, params)  the chain on an in-memory PCM array
  process_audio(settings, cb), batch_process_audio(settings, in_dir, out_dir, cb)
                               the desktop GUI's engine API (mastering_gui.py:204,220)
  apply_saturation, apply_eq_to_samples, apply_shelf_filter, apply_peak_filter,
  apply_stereo_width, apply_multiband_compressor, normalize_to_lufs, soft_limiter,
  audio_segment_to_float_array, float_array_to_audio_segment, integrated_loudness
                               the per-stage DSP helpers (AME:117-227), one HIP operator each
  worker.handle_push / worker.wsgi_app / worker.process_audio_from_gcs
                               the job worker (worker/main.py:15-50, AME:24-113) on a
                               local object tree
  legacy.master_pcm / legacy.process and main.py's helpers
                               the older monolithic engine (root main.py:46-192) as an
                               alternate DSP profile on the same HIP operators
"""
from .engine import EQ_PRESETS, Job, master_batch, master_device, master_pcm, process  # noqa: F401
from . import legacy  # noqa: F401
from .gui_compat import batch_process_audio, process_audio  # noqa: F401
from .ops import (apply_eq_to_samples, apply_multiband_compressor, apply_peak_filter, apply_saturation,  # noqa: F401
                  apply_shelf_filter, apply_stereo_width, audio_segment_to_float_array,
                  float_array_to_audio_segment, integrated_loudness, normalize_to_lufs, soft_limiter)

__all__ = ["legacy", "EQ_PRESETS", "Job", "master_pcm", "master_device", "master_batch", "process", "process_audio", "batch_process_audio",
           "apply_saturation", "apply_eq_to_samples", "apply_shelf_filter", "apply_peak_filter", "apply_stereo_width",
           "apply_multiband_compressor", "normalize_to_lufs", "soft_limiter", "audio_segment_to_float_array",
           "float_array_to_audio_segment", "integrated_loudness"]
