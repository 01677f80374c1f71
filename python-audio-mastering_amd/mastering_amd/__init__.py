"""mastering_amd — MI355X-native drop-in for the reference's mastering hot path.

Public surface (mirrors worker/audio_mastering_engine.py):
  EQ_PRESETS                   AME:15-20
  process(in, out, params)     AME:24-113 with local WAV IO instead of GCS
  master_pcm(pcm, rate, params)  the chain on an in-memory PCM array
  process_audio(settings, cb), batch_process_audio(settings, in_dir, out_dir, cb)
                               the desktop GUI's engine API (mastering_gui.py:204,220)
  worker.handle_push / worker.wsgi_app / worker.process_audio_from_gcs
                               the job worker (worker/main.py:15-50, AME:24-113) on a
                               local object tree
"""
from .engine import EQ_PRESETS, Job, master_device, master_pcm, process  # noqa: F401
from .gui_compat import batch_process_audio, process_audio  # noqa: F401

__all__ = ["EQ_PRESETS", "Job", "master_pcm", "master_device", "process", "process_audio", "batch_process_audio"]
