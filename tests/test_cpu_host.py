"""CPU tests of the host-side mirror of the reference's Python surface
(utils.py, config.py, dataset file walk / RNG order) -- no kernel launches."""
import os
import wave

import numpy as np
import pytest

import config
import utils


def _write_wav(path, x, sr=16000, nch=1):
    pcm = np.clip(np.round(np.asarray(x) * 32767), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(nch)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())


@pytest.fixture
def sine_wav(tmp_path):
    t = np.linspace(0, 2, 32000)
    x = 0.5 * np.sin(2 * np.pi * 440 * t) + 0.2 * np.sin(2 * np.pi * 880 * t)
    p = tmp_path / "tone.wav"
    _write_wav(p, x)
    return p, x


def test_config_constants():
    """config.py:27-30."""
    assert (config.DEFAULT_SAMPLE_RATE, config.DEFAULT_N_FFT, config.DEFAULT_HANN_WINDOW_SIZE,
            config.DEFAULT_HANN_HOP_LENGTH) == (16000, 512, 384, 192)


def test_load_audio_pads_and_clips(sine_wav):
    """tests/utils_test.py:149-207 spec: pad/clip to sr*max_len, float32."""
    p, x = sine_wav
    a, sr = utils.load_audio(p)
    assert sr == 16000 and a.dtype == np.float32 and len(a) == 80000
    assert np.all(a[32000:] == 0)
    assert np.abs(a[:32000] - x).max() < 1e-4
    b, _ = utils.load_audio(p, max_len=1)
    assert len(b) == 16000


def test_load_audio_resamples(sine_wav):
    p, _ = sine_wav
    a, sr = utils.load_audio(p, sample_rate=8000, max_len=2)
    assert sr == 8000 and len(a) == 16000


def test_load_audio_missing_file_raises_ioerror():
    """tests/utils_test.py:209-212."""
    with pytest.raises(IOError):
        utils.load_audio("/nonexistent/file.wav")


def test_add_random_gap_contract(sine_wav):
    """tests/utils_test.py:216-243: gap length, zeros, same length, float64."""
    p, _ = sine_wav
    np.random.seed(0)
    y, (s, e) = utils.add_random_gap(p, 0.2)
    assert y.dtype == np.float64 and len(y) == 80000
    assert abs((e - s) - 0.2) < 1e-12
    k = int(round(s * 16000))
    assert np.all(y[k:k + 3200] == 0)
    # the draw is np.random.randint(0, S - g) (exclusive), utils.py:179
    np.random.seed(0)
    assert k == np.random.randint(0, 80000 - 3200)


def test_add_random_gap_too_long_raises(sine_wav):
    """tests/utils_test.py:245-255."""
    p, _ = sine_wav
    with pytest.raises(ValueError):
        utils.add_random_gap(p, 10.0)


def test_create_gap_mask_edges():
    """utils.py:120-144 edge cases and inclusive start range."""
    m, iv = utils.create_gap_mask(1000, 0.0)
    assert iv == (0, 0) and m.dtype == np.float32 and m.sum() == 1000
    m, iv = utils.create_gap_mask(1000, 1.0)
    assert iv == (0, 1000) and m.sum() == 0
    m, iv = utils.create_gap_mask(16000, 0.1, gap_start_s=0.5)
    assert iv == (8000, 9600) and m[8000:9600].sum() == 0 and m.sum() == 16000 - 1600
    np.random.seed(3)
    m, (s, e) = utils.create_gap_mask(4000, 0.1)
    np.random.seed(3)
    assert s == np.random.randint(0, 4000 - 1600 + 1) and e - s == 1600


def test_extract_spectrogram_negative_power():
    """tests/utils_test.py:300-305."""
    with pytest.raises(ValueError):
        utils.extract_spectrogram(np.zeros(100, np.float32), power=-1)


def test_save_audio_normalises_and_creates_dirs(tmp_path):
    """tests/utils_test.py:494-535 spec (WAV container)."""
    x = 0.25 * np.sin(np.linspace(0, 100, 8000))
    out = tmp_path / "a" / "b" / "x.wav"
    utils.save_audio(x, out, file_format="wav")
    y, _ = utils.load_audio(out, max_len=0.5)
    assert np.abs(np.abs(y).max() - 1.0) < 1e-3


def test_dataset_walk_and_gap_draws(tmp_path):
    """models/CNNBLSTM/dataset.py:59-69 walk (first n_files, sorted) and the
    per-gap RNG draws of utils.py:179 (same order as the reference)."""
    from models.CNNBLSTM.dataset import LibriSpeechDataset
    d = tmp_path / "root" / "train-clean-100" / "19" / "198"
    d.mkdir(parents=True)
    for i in range(5):
        _write_wav(d / f"19-198-{i:04d}.wav", np.zeros(100))
    cfg = {"data": {"root_path": str(tmp_path / "root"), "sample_rate": 16000,
                    "train_path": "train-clean-100", "test_path": "x", "max_len_s": 4.0,
                    "gap_len_s": 0.2, "n_files": 3, "gaps_per_audio": 4,
                    "spectrogram": {"n_fft": 512, "hop_length": 192, "win_length": 384}}}
    ds = LibriSpeechDataset(None, "train", device="cpu", config=cfg)
    assert len(ds) == 3 and ds.file_paths == sorted(ds.file_paths)
    assert ds.n_frames == 334
    np.random.seed(5)
    st = ds.draw_gaps(80000)
    np.random.seed(5)
    assert list(st) == [np.random.randint(0, 80000 - 3200) for _ in range(4)]
    with pytest.raises(ValueError):
        LibriSpeechDataset(None, "bogus", device="cpu", config=cfg)
