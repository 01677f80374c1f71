"""End-to-end file mastering time (decode WAV -> chain -> encode WAV) for the C2
track, broken down by stage.  Usage (GPU box): python tools/e2e_bench.py [seconds]"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-audio-mastering_amd"))

import numpy as np  # noqa: E402

from mastering_amd import engine, native, wavio  # noqa: E402
from mastering_amd.synth import pink_noise_pcm16  # noqa: E402

P = {"bass_boost": 4.0, "mid_cut": 3.0, "presence_boost": 1.0, "treble_boost": 3.0,
     "saturation": 30, "width": 1.3, "multiband": True, "lufs": -14.0}
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
pcm = pink_noise_pcm16(int(secs * 44100), 44100, 2, 0)
d = tempfile.mkdtemp()
src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
wavio.write_wav(src, pcm, 44100)
engine.process(src, dst, P)  # warm: context, tables, buffers
times = {}
for rep in range(3):
    t0 = time.perf_counter()
    x, rate = wavio.read_wav(src)
    t1 = time.perf_counter()
    out, info = engine.master_pcm(x, rate, P)
    t2 = time.perf_counter()
    wavio.write_wav(dst, out, rate)
    t3 = time.perf_counter()
    times = {"decode_ms": (t1 - t0) * 1e3, "master_pcm_ms": (t2 - t1) * 1e3, "encode_ms": (t3 - t2) * 1e3,
             "total_ms": (t3 - t0) * 1e3}
t0 = time.perf_counter()
engine.process(src, dst, P)
times["process_ms"] = (time.perf_counter() - t0) * 1e3
times["seconds_of_audio"] = secs
times["realtime_factor"] = secs * 1e3 / times["process_ms"]
print(json.dumps({k: round(v, 2) for k, v in times.items()}))
