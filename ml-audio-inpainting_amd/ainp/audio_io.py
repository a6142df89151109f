"""Audio ingest on the native FLAC decoder (include/ainp.h).

read_flac replaces soundfile.read(dtype='float32') behind librosa.load
(utils.py:36): interleaved integer samples from ainp_flac_decode, scaled by
2^-(bits-1) as libsndfile normalises integer PCM to float.  Host-side: the
decoder runs on the CPU (FLAC is a serial bitstream), once per file.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import call, lib


def flac_info(data: bytes) -> dict:
    """STREAMINFO of an in-memory FLAC file."""
    sr, ch, bps, total = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    md5 = (ctypes.c_uint8 * 16)()
    call("ainp_flac_info", data, len(data), ctypes.byref(sr), ctypes.byref(ch),
         ctypes.byref(bps), ctypes.byref(total), md5)
    return {"sample_rate": sr.value, "channels": ch.value, "bits_per_sample": bps.value,
            "total_samples": total.value, "md5": bytes(md5)}


def decode_flac(data: bytes):
    """-> (int32 [frames, channels] samples exactly as encoded, STREAMINFO dict)."""
    info = flac_info(data)
    ch = info["channels"]
    cap = info["total_samples"]
    if cap == 0:  # unknown length in STREAMINFO: bound by the compressed size
        cap = max(1, len(data)) * 8 // max(1, ch)
    out = np.empty(cap * ch, dtype=np.int32)
    got = ctypes.c_int64()
    call("ainp_flac_decode", data, len(data), out.ctypes.data, cap, ctypes.byref(got))
    return out[:got.value * ch].reshape(-1, ch), info


def read_flac(path):
    """(float32 [frames, channels] in [-1, 1), sample_rate) of a FLAC file."""
    with open(path, "rb") as f:
        data = f.read()
    pcm, info = decode_flac(data)
    scale = np.float32(1.0 / float(1 << (info["bits_per_sample"] - 1)))
    return pcm.astype(np.float32) * scale, info["sample_rate"]


__all__ = ["flac_info", "decode_flac", "read_flac", "lib"]
