"""GPU tests of the mirrored reference API: utils.extract_spectrogram,
LibriSpeechDataset.__getitem__ and the models/CNNBLSTM/train.py loop."""
import os
import wave

import numpy as np
import pytest
import torch
import yaml

from oracle import stft_ref
from ainp import synth

pytestmark = pytest.mark.gpu


def _write_wav(path, x, sr=16000):
    pcm = np.clip(np.round(np.asarray(x) * 32767), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("center", [True, False])
def test_extract_spectrogram_vs_oracle(dtype, center):
    import utils
    y = synth.synthetic_clip(7, 9000).astype(dtype)
    X = utils.extract_spectrogram(y, n_fft=512, hop_length=192, win_length=384, center=center)
    assert X.dtype == (np.complex64 if dtype == np.float32 else np.complex128)
    if center:
        R = stft_ref.stft(y, 512, 192, 384)
    else:
        w = stft_ref.padded_window("hann", 384, 512)
        nfr = 1 + (len(y) - 512) // 192
        idx = np.arange(512)[:, None] + 192 * np.arange(nfr)[None, :]
        R = np.fft.rfft(y.astype(np.float64)[idx] * w[:, None], axis=0)
    assert X.shape == R.shape
    tol = 2e-6 if dtype == np.float32 else 1e-12
    assert np.abs(X - R).max() <= tol * np.abs(R).max()
    # torch tensor stays on the GPU
    Xt = utils.extract_spectrogram(torch.from_numpy(y).cuda(), n_fft=512, hop_length=192,
                                   win_length=384, center=center)
    assert Xt.is_cuda and np.abs(Xt.cpu().numpy() - X).max() == 0


def _tree(tmp_path, n_files, seconds):
    for split in ("train-clean-100", "test-clean"):
        d = tmp_path / "root" / split / "1" / "2"
        d.mkdir(parents=True)
        for i in range(n_files):
            _write_wav(d / f"1-2-{i:04d}.wav", synth.synthetic_clip(50 + i, int(16000 * seconds)))


def _cfg(tmp_path, n_files=2, gaps=3, max_len_s=4.0, batch=1, epochs=1):
    return {
        "data": {"dataset": "LibriSpeech", "root_path": str(tmp_path / "root"),
                 "sample_rate": 16000, "train_path": "train-clean-100", "test_path": "test-clean",
                 "max_len_s": max_len_s, "gap_len_s": 0.2, "n_files": n_files,
                 "gaps_per_audio": gaps,
                 "spectrogram": {"n_fft": 512, "hop_length": 192, "win_length": 384,
                                 "window": "hann", "normalize": True, "power": 1.0}},
        "model": {"input_dim": 334, "in_channels": 1, "num_lstm_layers": 2,
                  "lstm_hidden_dim": 64, "enc_filters": [16, 32], "dec_filters": [16, 32]},
        "training": {"batch_size": batch, "optimizer_type": "adam",
                     "starter_learning_rate": 1e-4, "lr_decay": 1.0, "max_n_epochs": epochs},
        "paths": {"tensorboard_dir": str(tmp_path / "tb"), "checkpoint_dir": str(tmp_path / "ck"),
                  "log_dir": str(tmp_path / "logs"), "sample_dir": str(tmp_path / "samples"),
                  "resume_mdl_path": None},
        "logging": {"checkpoint_interval": 1, "metric_interval": 1, "spectrogram_interval": 100,
                    "audio_interval": 500, "run_name": "t"},
    }


def test_dataset_item_matches_oracle(tmp_path):
    from models.CNNBLSTM.dataset import LibriSpeechDataset
    import utils
    _tree(tmp_path, 2, 6.0)
    cfg = _cfg(tmp_path)
    ds = LibriSpeechDataset(None, "train", device="cuda", config=cfg)
    np.random.seed(11)
    lg, gi, gm, tg = ds[0]
    assert lg.shape == (3, 257, 334) and tg.dtype == torch.complex64 and gi.shape == (3, 2)
    audio, _ = utils.load_audio(ds.file_paths[0])
    np.random.seed(11)
    starts = [np.random.randint(0, 80000 - 3200) for _ in range(3)]
    for i, s in enumerate(starts):
        rl, rt, rm = stft_ref.cnnblstm_item(audio, s, 3200, 512, 192, 384, 16000, 334)
        np.testing.assert_array_equal(gm[i].cpu().numpy(), rm)
        assert np.abs(lg[i].cpu().numpy() - rl).max() < 2e-5
        assert np.abs(tg[i].cpu().numpy() - rt).max() <= 2e-6 * np.abs(rt).max()
        assert gi[i, 0].item() == np.float32(s / 16000)


def test_train_script_runs_one_epoch(tmp_path):
    from models.CNNBLSTM import train as train_mod
    _tree(tmp_path, 3, 5.0)
    cfg = _cfg(tmp_path, n_files=3, gaps=2, batch=2, epochs=1)  # 3 files, batch 2: partial batch (Q2)
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    train_mod.main(str(p))
    ck = list((tmp_path / "ck").rglob("blstm_cnn_epoch_1.pt"))
    assert len(ck) == 1
    sd = torch.load(ck[0], weights_only=True)
    assert "lstm.weight_ih_l0_reverse" in sd and "encoder.1.running_var" in sd
    assert all(torch.isfinite(v).all() for v in sd.values() if v.is_floating_point())


# ------------------------------------------------- C1: the bundled FLAC clips
FLAC_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "flac")


def _flac_tree(tmp_path):
    import shutil
    for split in ("train-clean-100", "test-clean"):
        d = tmp_path / "root" / split / "19" / "198"
        d.mkdir(parents=True)
        for f in sorted(os.listdir(FLAC_DIR)):
            shutil.copy(os.path.join(FLAC_DIR, f), d / f)


def test_c1_flac_dataset_items_match_oracle(tmp_path):
    """Real LibriSpeech speech through the native FLAC decoder and the fused
    feature kernel vs the float64 oracle (BASELINE configs[0] shapes: 5 s,
    T = 417, 25 gaps per file)."""
    from models.CNNBLSTM.dataset import LibriSpeechDataset
    import utils
    _flac_tree(tmp_path)
    cfg = _cfg(tmp_path, n_files=9, gaps=25, max_len_s=5.0)
    ds = LibriSpeechDataset(None, "train", device="cuda", config=cfg)
    assert len(ds) == 9
    for idx in (0, 8):
        np.random.seed(100 + idx)
        lg, gi, gm, tg = ds[idx]
        assert lg.shape == (25, 257, 417)
        audio, _ = utils.load_audio(ds.file_paths[idx])
        np.random.seed(100 + idx)
        starts = [np.random.randint(0, 80000 - 3200) for _ in range(25)]
        for i in (0, 7, 24):
            rl, rt, rm = stft_ref.cnnblstm_item(audio, starts[i], 3200, 512, 192, 384, 16000, 417)
            np.testing.assert_array_equal(gm[i].cpu().numpy(), rm)
            assert np.abs(lg[i].cpu().numpy() - rl).max() < 2e-5
            assert np.abs(tg[i].cpu().numpy() - rt).max() <= 2e-6 * np.abs(rt).max()


def test_c1_train_script_on_bundled_flacs(tmp_path):
    """BASELINE configs[0]: train.py on the 9 bundled clips, batch 2 files x 25
    gaps, the reference model (3-layer BLSTM, H=128), one epoch incl. the
    partial last batch the reference crashes on."""
    from models.CNNBLSTM import train as train_mod
    _flac_tree(tmp_path)
    cfg = _cfg(tmp_path, n_files=9, gaps=25, max_len_s=5.0, batch=2, epochs=1)
    cfg["model"].update({"input_dim": 417, "num_lstm_layers": 3, "lstm_hidden_dim": 128})
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    train_mod.main(str(p))
    ck = list((tmp_path / "ck").rglob("blstm_cnn_epoch_1.pt"))
    assert len(ck) == 1
    sd = torch.load(ck[0], weights_only=True)
    assert sd["lstm.weight_ih_l0"].shape == (512, 64 * 257)
    assert all(torch.isfinite(v).all() for v in sd.values() if v.is_floating_point())


# ------------------------------------------------------------------ GAN API
def _gan_cfg(tmp_path, limit=8, batch=2, epochs=1):
    return {
        "data": {"dataset": "LibriSpeech", "root_path": str(tmp_path / "root"),
                 "sample_rate": 16000, "train_path": "train-clean-100",
                 "valid_path": "test-clean", "test_path": "test-clean", "max_len_s": 5.0,
                 "gap_len_s": 0.2, "train_limit": limit,
                 "spectrogram": {"n_fft": 512, "hop_length": 128, "win_length": 512,
                                 "window": "hann", "normalize": True, "power": 1.0}},
        "model": {"generator": {"input_channels": 1, "mask_channels": 1, "output_channels": 1},
                  "discriminator": {"input_channels": 1, "use_spectral_norm": True}},
        "training": {"batch_size": batch, "epochs": epochs, "g_lr": 2e-4, "d_lr": 2e-4,
                     "b1": 0.5, "b2": 0.999, "lambda_adv": 0.01, "lambda_l1_valid": 1.0,
                     "lambda_l1_hole": 2.0, "lambda_vgg_perceptual": 4.0,
                     "lambda_vgg_style": 500.0, "lambda_mag_weighted": 0.2,
                     "resume_from_chkpt": False},
        "paths": {"tensorboard_dir": str(tmp_path / "tb"), "checkpoint_dir": str(tmp_path / "ck"),
                  "log_dir": str(tmp_path / "logs"), "sample_dir": str(tmp_path / "samples")},
        "logging": {"log_interval": 1, "checkpoint_interval": 1, "sample_interval": 1000,
                    "num_workers": 0, "run_name": "t", "validation_interval": 1},
    }


def test_gan_dataset_item_matches_oracle(tmp_path):
    from models.GAN.dataset import SpeechInpaintingDataset
    import utils
    _tree(tmp_path, 2, 6.0)
    ds = SpeechInpaintingDataset(_gan_cfg(tmp_path), "train", device="cuda")
    np.random.seed(21)
    item = ds[0]
    assert item["original_magnitude"].shape == (1, 257, 626)
    audio, _ = utils.load_audio(ds.file_paths[0], max_len=5.0)
    np.random.seed(21)
    start = np.random.randint(0, 80000 - 3200 + 1)
    ro, ri, rp, rm = stft_ref.gan_item(audio, start, 3200, 512, 128, 512)
    np.testing.assert_array_equal(item["mask"][0].cpu().numpy(), rm)
    for k, r in (("original_magnitude", ro), ("impaired_magnitude", ri)):
        assert np.abs(item[k][0].cpu().numpy() - r).max() < 2e-5, k
    # phase: compare on the unit circle (angle wraps at +-pi)
    ph = item["original_phase"][0].cpu().numpy()
    assert np.abs(np.exp(1j * ph) - np.exp(1j * rp)).max() < 1e-3


def test_gan_train_script_runs_one_epoch(tmp_path):
    from models.GAN import train as gan_train
    _tree(tmp_path, 4, 5.0)
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(_gan_cfg(tmp_path, limit=4, batch=2, epochs=1)))
    gan_train.main(str(p))
    ck = list((tmp_path / "ck").rglob("discriminator_epoch_0001.pth"))
    assert len(ck) == 1
    sd = torch.load(ck[0], weights_only=True)
    assert "model.0.block.0.weight_orig" in sd and "model.4.weight_u" in sd
    assert all(torch.isfinite(v).all() for v in sd.values() if v.is_floating_point())
    opt = torch.load(list((tmp_path / "ck").rglob("optimizers_epoch_0001.pth"))[0],
                     weights_only=True)
    assert opt["epoch"] == 0 and opt["global_step"] == 2
