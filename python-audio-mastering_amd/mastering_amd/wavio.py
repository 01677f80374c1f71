"""Minimal RIFF/WAVE codec (replaces pydub/ffmpeg decode at AME:43 and the stdlib
`wave` export at AME:98).  PCM16 and IEEE-float32, mono or stereo."""
from __future__ import annotations

import struct

import numpy as np


def read_wav(path: str):
    """Return (samples, rate); int16 [N] / [N, ch] for PCM16, float32 for fmt 3."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, rate, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: subformat GUID
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, rate, bits)
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, rate, bits = fmt
    if tag == 1 and bits == 16:
        x = np.frombuffer(payload[: len(payload) // (2 * ch) * 2 * ch], dtype="<i2").astype(np.int16)
    elif tag == 3 and bits == 32:
        x = np.frombuffer(payload[: len(payload) // (4 * ch) * 4 * ch], dtype="<f4").astype(np.float32)
    else:
        raise ValueError(f"{path}: unsupported WAV format tag={tag} bits={bits}")
    if ch > 1:
        x = x.reshape(-1, ch)
    return x, rate


def write_wav(path: str, x: np.ndarray, rate: int):
    ch = 1 if x.ndim == 1 else x.shape[1]
    if x.dtype == np.int16:
        tag, bits, payload = 1, 16, np.ascontiguousarray(x, dtype="<i2").tobytes()
    elif x.dtype == np.float32:
        tag, bits, payload = 3, 32, np.ascontiguousarray(x, dtype="<f4").tobytes()
    else:
        raise TypeError("write_wav expects int16 or float32")
    ba = ch * bits // 8
    hdr = b"RIFF" + struct.pack("<I", 36 + len(payload)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, tag, ch, rate, rate * ba, ba, bits)
    hdr += b"data" + struct.pack("<I", len(payload))
    with open(path, "wb") as f:
        f.write(hdr + payload)
