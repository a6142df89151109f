"""Native FLAC ingest (include/ainp.h ainp_flac_*), host-only.

Fixtures: the reference's bundled LibriSpeech clips (test_samples/*.flac,
BASELINE.json configs[0]) copied as data to tests/golden/flac/.  Bit-exactness
is pinned by each file's own STREAMINFO MD5 of the decoded PCM (no reference
decoder exists in this image), plus every frame's CRC-8/CRC-16 inside the
decoder.  load_audio's contract follows the reference tests
(tests/utils_test.py:149-212): truncate or zero-pad to sr*max_len, IOError on
any failure.
"""
import glob
import hashlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
FILES = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "flac", "*.flac")))


def _pcm_bytes(pcm, bps):
    nb = (bps + 7) // 8
    if nb == 2:
        return pcm.astype("<i2").tobytes()
    v = pcm.astype("<i4").reshape(-1, 1).view(np.uint8).reshape(-1, 4)[:, :nb]
    return v.tobytes()


def test_fixture_set():
    assert len(FILES) == 9


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_decode_matches_streaminfo_md5(path):
    from ainp.audio_io import decode_flac
    data = open(path, "rb").read()
    pcm, info = decode_flac(data)
    assert info["sample_rate"] == 16000 and info["channels"] == 1
    assert pcm.shape == (info["total_samples"], 1)
    assert hashlib.md5(_pcm_bytes(pcm, info["bits_per_sample"])).digest() == info["md5"]


def test_load_audio_truncates_pads_and_scales():
    import utils
    from ainp.audio_io import decode_flac
    path = FILES[0]
    pcm, info = decode_flac(open(path, "rb").read())
    y, sr = utils.load_audio(path, sample_rate=16000, max_len=5)
    assert sr == 16000 and y.dtype == np.float32 and y.shape == (80000,)
    np.testing.assert_array_equal(y, pcm[:80000, 0].astype(np.float32) / 32768.0)
    n = info["total_samples"]
    y2, _ = utils.load_audio(path, sample_rate=16000, max_len=n / 16000 + 1)
    assert y2.shape == (n + 16000,)
    np.testing.assert_array_equal(y2[:n], pcm[:, 0].astype(np.float32) / 32768.0)
    assert not y2[n:].any()


def test_corrupt_stream_raises_ioerror(tmp_path):
    import utils
    data = bytearray(open(FILES[-1], "rb").read())
    data[len(data) // 2] ^= 0x5A          # flips bits inside a frame: CRC-16 mismatch
    bad = tmp_path / "bad.flac"
    bad.write_bytes(bytes(data))
    with pytest.raises(IOError):
        utils.load_audio(str(bad))
    with pytest.raises(IOError):
        utils.load_audio(str(tmp_path / "missing.flac"))


# ---- stream features the LibriSpeech fixtures do not exercise, from the
# ---- test-only encoder tests/flac_encode.py
def _signal(n, nch, bps, seed, step=1):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    lim = (1 << (bps - 1)) - 1
    out = []
    for c in range(nch):
        x = 0.4 * np.sin(2 * np.pi * (0.01 + 0.003 * c) * t) + 0.05 * rng.standard_normal(n)
        out.append(np.clip(np.round(x * lim / step) * step, -lim - 1, lim))
    return np.stack(out, 1).astype(np.int64)


CASES = [
    dict(bps=16, nch=2, chmode="left_side", order=2),
    dict(bps=16, nch=2, chmode="side_right", order=3, method=1),
    dict(bps=16, nch=2, chmode="mid_side", order=4, porder=3),
    dict(bps=16, nch=2, chmode="independent", order=1, escape_every=2),
    dict(bps=24, nch=1, chmode="independent", kind="verbatim"),
    dict(bps=20, nch=1, chmode="independent", order=2, method=1, escape_every=3),
    dict(bps=12, nch=1, chmode="independent", order=0),
    dict(bps=8, nch=1, chmode="independent", order=2, ss_code_in_header=False),
    dict(bps=16, nch=1, chmode="independent", order=2, step=8),          # wasted bits
    dict(bps=16, nch=2, chmode="mid_side", kind="constant"),             # constant blocks
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c['bps']}b-{c['chmode']}-{i}"
                                             for i, c in enumerate(CASES)])
def test_decoder_stream_features(case):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from flac_encode import encode
    from ainp.audio_io import decode_flac
    case = dict(case)
    bps, nch, step = case.pop("bps"), case.pop("nch"), case.pop("step", 1)
    n = 5 * 1024 + 500                                 # short final block
    pcm = _signal(n, nch, bps, seed=bps * 10 + nch, step=step)
    if case.get("kind") == "constant":
        pcm[:] = 0
        pcm[2048:, 0] = 1234
        pcm[2048:, 1] = 1234
    data = encode(pcm, 16000, bps, **case)
    out, info = decode_flac(data)
    assert info["bits_per_sample"] == bps and info["channels"] == nch
    np.testing.assert_array_equal(out, pcm)
    assert hashlib.md5(_pcm_bytes(out, bps)).digest() == info["md5"]
