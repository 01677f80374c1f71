"""The desktop GUI's engine API.

`mastering_gui.py` calls `engine.process_audio(settings, update_status)` and
`engine.batch_process_audio(settings, input_folder, output_folder,
update_status)` from a daemon thread (mastering_gui.py:204, 220), but the
reference snapshot defines neither.  This module provides both
on top of `engine.process`, so the GUI runs against the MI355X engine unchanged
(`import mastering_amd.gui_compat as engine`).

Settings arrive with the GUI's keys (mastering_gui.py:181-190).  The worker
engine reads canonical keys (AME:58-86) and would ignore
the GUI's band keys; here they are mapped onto the canonical ones
(`low_band_threshold` -> `low_thresh`, ...), which is what the GUI's sliders
mean.  `compress`, `input_file` and `output_file` are not chain settings.

Status strings drive the GUI (mastering_gui.py:224-232): it re-enables its
buttons when a message contains "complete", "error" or "no audio files", and
shows a dialog for "complete" / "error".

Batches are a multi-GPU file scheduler (C3/C5 of BASELINE.json): files are
dealt to the given devices (`distributed.shard_files`), one host thread per
device, each thread with its own engine context (one HIP stream) — the same
file sharding `bench.py --gpus N` measures, without any collective.
"""
from __future__ import annotations

import os
import threading

from . import distributed, engine

GUI_KEY_MAP = {
    "low_band_threshold": "low_thresh", "low_band_ratio": "low_ratio",
    "mid_band_threshold": "mid_thresh", "mid_band_ratio": "mid_ratio",
    "high_band_threshold": "high_thresh", "high_band_ratio": "high_ratio",
}
NOT_CHAIN_KEYS = ("input_file", "output_file", "compress")
AUDIO_EXTENSIONS = (".wav", ".wave")


def chain_settings(settings: dict) -> dict:
    """GUI settings -> the engine's canonical settings."""
    out = {}
    for k, v in (settings or {}).items():
        if k in NOT_CHAIN_KEYS:
            continue
        out[GUI_KEY_MAP.get(k, k)] = v
    return out


def output_name(input_name: str) -> str:
    """Batch output file name: `<stem>_mastered.wav`."""
    stem, _ = os.path.splitext(os.path.basename(input_name))
    return f"{stem}_mastered.wav"


def _status(cb):
    return cb if cb is not None else (lambda message: None)


def process_audio(settings: dict, status_callback=None, device: int = 0):
    """Master settings['input_file'] into settings['output_file'] (mastering_gui.py:192-206).
    Reports through `status_callback`; returns the engine's info dict, or None on error."""
    cb = _status(status_callback)
    src, dst = (settings or {}).get("input_file"), (settings or {}).get("output_file")
    if not src or not dst:
        cb("Error: select both an input and an output file.")
        return None
    try:
        cb(f"Processing {os.path.basename(src)}...")
        info = engine.process(src, dst, chain_settings(settings), device=device)
    except Exception as e:  # the GUI shows the message; AME:110-113 re-raises to its caller
        cb(f"Error: {e}")
        return None
    cb(f"Processing complete: {os.path.basename(dst)}")
    return info


def list_audio_files(folder: str) -> list[str]:
    return sorted(f for f in os.listdir(folder)
                  if f.lower().endswith(AUDIO_EXTENSIONS) and os.path.isfile(os.path.join(folder, f)))


def batch_process_audio(settings: dict, input_folder: str, output_folder: str, status_callback=None,
                        devices=None) -> dict:
    """Master every WAV in `input_folder` into `output_folder` (mastering_gui.py:208-222).
    `devices`: GPU ids to spread the files over (default: GPU 0).  Returns
    {input file name: info dict or the error message}."""
    cb = _status(status_callback)
    try:
        files = list_audio_files(input_folder)
    except OSError as e:
        cb(f"Error: {e}")
        return {}
    if not files:
        cb("No audio files found in the input folder.")
        return {}
    os.makedirs(output_folder, exist_ok=True)
    devices = list(devices) if devices else [0]
    params = chain_settings(settings)
    results: dict = {}
    lock = threading.Lock()
    done = [0]

    def work(rank: int):
        for i in distributed.shard_files(len(files), len(devices), rank):
            name = files[i]
            try:
                info = engine.process(os.path.join(input_folder, name),
                                      os.path.join(output_folder, output_name(name)), params,
                                      device=devices[rank])
            except Exception as e:
                info = f"{type(e).__name__}: {e}"
            with lock:
                results[name] = info
                done[0] += 1
                cb(f"Processed {done[0]}/{len(files)}: {name}")

    threads = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(len(devices))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    failed = [n for n, v in results.items() if not isinstance(v, dict)]
    if failed:
        cb(f"Batch processing complete with errors: {len(files) - len(failed)} of {len(files)} files "
           f"mastered; failed: {', '.join(sorted(failed))}")
    else:
        cb(f"Batch processing complete: {len(files)} files mastered.")
    return results
