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


def encode_flac(pcm: np.ndarray, sample_rate: int, bits_per_sample: int = 16) -> bytes:
    """Integer samples [frames] or [frames, channels] -> FLAC file bytes
    (ainp_flac_encode: lossless, STREAMINFO MD5 set)."""
    pcm = np.asarray(pcm)
    if pcm.ndim == 1:
        pcm = pcm[:, None]
    x = np.ascontiguousarray(pcm, dtype=np.int32)
    frames, ch = x.shape
    cap = int(lib.ainp_flac_encode_bound(frames, ch, bits_per_sample))
    out = np.empty(max(cap, 1), dtype=np.uint8)
    n = ctypes.c_size_t()
    call("ainp_flac_encode", x.ctypes.data, frames, ch, int(bits_per_sample), int(sample_rate),
         out.ctypes.data, cap, ctypes.byref(n))
    return out[:n.value].tobytes()


def write_flac(path, audio: np.ndarray, sample_rate: int) -> None:
    """soundfile.write(path, float_audio, sr) with the FLAC default subtype
    PCM_16: libsndfile's conversion lrint(x * 0x7FFF) (round half to even),
    in float32 for float32 data (sf_write_float) and float64 otherwise
    (sf_write_double), then the native encoder."""
    a = np.asarray(audio)
    if a.dtype == np.float32:
        pcm = np.rint(a * np.float32(32767.0))
    else:
        pcm = np.rint(a.astype(np.float64) * 32767.0)
    pcm = np.clip(pcm, -32768, 32767).astype(np.int32)
    with open(path, "wb") as f:
        f.write(encode_flac(pcm, sample_rate, 16))


__all__ = ["flac_info", "decode_flac", "read_flac", "encode_flac", "write_flac", "lib"]
