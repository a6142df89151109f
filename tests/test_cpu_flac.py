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


# ----------------------------------------------------------------- encoder
@pytest.mark.parametrize("frames,ch,bits", [(80000, 1, 16), (4096, 1, 16), (4097, 2, 16),
                                             (1, 1, 16), (0, 1, 16), (12345, 2, 24),
                                             (5000, 1, 8)])
def test_encoder_roundtrip_bit_exact(frames, ch, bits):
    """ainp_flac_encode -> ainp_flac_decode returns the samples bit for bit;
    STREAMINFO carries the right MD5 (computed as FLAC defines it)."""
    import hashlib
    from ainp.audio_io import decode_flac, encode_flac
    from ainp.synth import synthetic_clip
    rng = np.random.default_rng(frames + ch + bits)
    lim = 1 << (bits - 1)
    if frames >= 4096:
        clip = synthetic_clip(frames, frames) * (lim - 1)
        pcm = np.stack([np.rint(clip * (0.5 + 0.5 * c)) for c in range(ch)], 1).astype(np.int32)
        pcm[:50] = 7                              # a constant run
        pcm[100:130] = rng.integers(-lim, lim, size=(30, ch))   # full-scale noise
    else:
        pcm = rng.integers(-lim, lim, size=(frames, ch)).astype(np.int32)
    data = encode_flac(pcm, 16000, bits)
    out, info = decode_flac(data)
    assert info["total_samples"] == frames and info["channels"] == ch
    assert info["bits_per_sample"] == bits and info["sample_rate"] == 16000
    np.testing.assert_array_equal(out, pcm)
    le = pcm.astype(f"<i{4}").view(np.uint8).reshape(-1, 4)[:, :(bits + 7) // 8].tobytes()
    assert info["md5"] == hashlib.md5(le).digest()
    if frames >= 80000:      # the predictor + Rice coder compresses (noisy) harmonic audio
        assert len(data) < 0.7 * frames * ch * 2


def test_encoder_on_librispeech_fixtures(golden_dir):
    """Re-encoding the bundled LibriSpeech clips is lossless and within 1.3x
    of the size the reference's encoder (libFLAC) produced."""
    from ainp.audio_io import decode_flac, encode_flac
    d = os.path.join(golden_dir, "flac")
    for name in sorted(os.listdir(d))[:3]:
        raw = open(os.path.join(d, name), "rb").read()
        pcm, info = decode_flac(raw)
        data = encode_flac(pcm, info["sample_rate"], info["bits_per_sample"])
        out, info2 = decode_flac(data)
        np.testing.assert_array_equal(out, pcm)
        assert info2["md5"] == info["md5"]
        assert len(data) < 1.3 * len(raw), (name, len(data), len(raw))


def test_save_audio_flac_roundtrip(tmp_path):
    """utils.save_audio(.flac) (peak-normalised, PCM_16) is read back by
    utils.load_audio as libsndfile would: x / max|x| quantised by 32767."""
    import utils
    from ainp.synth import synthetic_clip
    x = synthetic_clip(9, 16000) * 0.3
    p = tmp_path / "sub" / "a.flac"
    utils.save_audio(x, p, 16000)
    y, sr = utils.load_audio(str(p), sample_rate=16000, max_len=1)
    assert sr == 16000
    n = x / np.abs(x).max()                      # float32, as save_audio normalises it
    ref = np.rint(n * np.float32(32767.0)) / 32768.0
    np.testing.assert_array_equal(y, ref.astype(np.float32))


def test_pre_process_dataset_on_a_librispeech_tree(tmp_path, golden_dir):
    """pre_process_dataset.py:20-43 end to end on a LibriSpeech-shaped tree
    (speaker/chapter/*.flac, here two bundled clips): mirrored tree, FLAC
    output, 5 s (load_audio's max_len), one 0.1 s zero gap, peak-normalised."""
    import shutil
    import pre_process_dataset
    from ainp.audio_io import read_flac
    src = tmp_path / "LibriSpeech" / "train"
    names = sorted(os.listdir(os.path.join(golden_dir, "flac")))[:2]
    for i, name in enumerate(names):
        d = src / f"{100 + i}" / "200"
        d.mkdir(parents=True)
        shutil.copy(os.path.join(golden_dir, "flac", name), d / name)
    dst = tmp_path / "processed"
    np.random.seed(3)
    assert pre_process_dataset.process(str(src), str(dst)) == 2
    for i, name in enumerate(names):
        y, sr = read_flac(dst / f"{100 + i}" / "200" / name)
        y = y[:, 0]
        assert sr == 16000 and len(y) == 80000
        assert np.abs(y).max() == np.float32(32767 / 32768)
        z = (y == 0).astype(np.int8)
        run, best = 0, 0
        for v in z:
            run = run + 1 if v else 0
            best = max(best, run)
        assert best >= 1600


def test_add_gaps_writes_flac(tmp_path, golden_dir):
    import add_gaps
    from ainp.audio_io import read_flac
    name = sorted(os.listdir(os.path.join(golden_dir, "flac")))[0]
    out = tmp_path / "gap.flac"
    y_new = add_gaps.insert_gap_file(os.path.join(golden_dir, "flac", name), out, 1.0, 0.25)
    y, sr = read_flac(out)
    assert not np.any(y[16000:20000, 0])
    np.testing.assert_array_equal(y[:, 0], np.rint(y_new * np.float32(32767)) / 32768)
