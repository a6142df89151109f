"""GPU test of models/model_eval.py: the fixed 80 ms gap at
2.0 s, model inpainting and ISTFT with the original phase, FLAC output.

Expected audio is rebuilt from the oracle (oracle/stft_ref.py: float64 STFT,
librosa gap frames, ISTFT) around the same random-init model on the GPU, then
peak-normalised and quantised like save_audio.  The two differ only by the
GPU-vs-oracle STFT rounding fed through the model: tolerance 3 LSB of 16-bit
PCM per sample, 1e-3 relative L2.  Output lengths are hop * (T - 1):
79872 (CNN-BLSTM, hop 192) and 80000 (GAN, hop 128) for a 5 s clip."""
import os
import shutil

import numpy as np
import pytest
import torch

from oracle import stft_ref as S

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ml-audio-inpainting_amd")
CLIPS = ["81-121543-0008.flac", "1241-121103-0021.flac"]
LSB = 1.0 / 32767.0


def _expected(model_type, model, audio, cfg):
    sp = cfg["data"]["spectrogram"]
    n_fft, hop, win = sp["n_fft"], sp["hop_length"], sp["win_length"]
    sr = 16000
    X = S.stft(audio.astype(np.float32), n_fft, hop, win).astype(np.complex64)
    phase = np.angle(X)
    gs, gl = int(2.0 * sr), int(0.08 * sr)
    if model_type == "gan":
        m = np.ones(len(audio), np.float32)
        m[gs:gs + gl] = 0
        Xi = S.stft((audio * m).astype(np.float32), n_fft, hop, win)
        imp = np.log1p(np.abs(Xi)).astype(np.float32)
        fs, fe = S.gan_gap_frames(gs, gl, hop, X.shape[1])
        mask = np.ones(X.shape, np.float32)
        mask[:, fs:fe] = 0
        with torch.no_grad():
            out = model(torch.from_numpy(imp).cuda()[None, None],
                        torch.from_numpy(mask).cuda()[None, None])[0, 0]
    else:
        fs, fe = S.time_to_frames(2.0, sr, hop), S.time_to_frames(2.08, sr, hop)
        mask = np.zeros(X.shape, np.float32)
        mask[:, fs:fe] = 1
        li = np.log10(np.abs(X * (1 - mask)) + 1e-9).astype(np.float32)
        with torch.no_grad():
            out = (10 ** model.reconstruct_spectrogram(torch.from_numpy(li).cuda()[None],
                                                       torch.from_numpy(mask).cuda()))[0]
    mag = out.double().cpu().numpy()
    y = S.istft(mag * np.exp(1j * phase.astype(np.float64)), hop, win, n_fft)
    y = y / np.max(np.abs(y))
    return np.clip(np.rint(y * 32767.0), -32768, 32767) / 32767.0, (fs, fe)


@pytest.mark.parametrize("model_type", ["cnnlstm", "gan"])
def test_run_evaluation(model_type, tmp_path, golden_dir):
    import yaml
    from ainp.audio_io import read_flac
    from models import model_eval as ME
    import utils

    cfg_path = os.path.join(PKG, "models", "CNNBLSTM", "cnn_blstm.yaml") if model_type == "cnnlstm" \
        else os.path.join(PKG, "models", "GAN", "config.yaml")
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f)
    torch.manual_seed(0)
    init = ME.StackedBLSTMCNN(cfg_path) if model_type == "cnnlstm" else ME.PConvUNet(1, 1, 1)
    model = ME.load_model(model_type, cfg_path, init.state_dict(), torch.device("cuda"))
    ck = tmp_path / "model.pt"
    torch.save(model.state_dict(), ck)
    src = tmp_path / "in"
    src.mkdir()
    for c in CLIPS:
        shutil.copy(os.path.join(golden_dir, "flac", c), src / c)
    outs = ME.run_evaluation(str(src), str(tmp_path / "out"), model_type, str(ck), cfg_path)
    assert [os.path.basename(o) for o in outs] == \
        [f"{os.path.splitext(c)[0]}_{model_type}_inpainted.flac" for c in sorted(CLIPS)]
    # the checkpoint round trip (weights_only=True) reloads the same weights
    reloaded = ME.load_model(model_type, cfg_path, str(ck), torch.device("cuda"))
    for (k, a), b in zip(model.state_dict().items(), reloaded.state_dict().values()):
        assert torch.equal(a, b), k
    hop = cfg["data"]["spectrogram"]["hop_length"]
    for c, o in zip(sorted(CLIPS), outs):
        got, sr = read_flac(o)
        got = got[:, 0].astype(np.float64) * (32768.0 / 32767.0)
        assert sr == 16000
        assert len(got) == hop * (80000 // hop)          # hop * (T - 1)
        audio, _ = utils.load_audio(os.path.join(golden_dir, "flac", c))
        exp, (fs, fe) = _expected(model_type, model, audio, cfg)
        if model_type == "cnnlstm":
            assert (fs, fe) == (166, 173)
        assert len(exp) == len(got)
        err = np.abs(got - exp)
        assert err.max() <= 3 * LSB + 1e-9, (c, err.max() / LSB)
        assert np.linalg.norm(got - exp) / np.linalg.norm(exp) < 1e-3


class _RecWriter:
    def __init__(self):
        self.scalars, self.audio = {}, {}

    def add_scalar(self, tag, v, step):
        self.scalars[tag] = (float(v), step)

    def add_audio(self, tag, a, step, sample_rate):
        self.audio[tag] = (np.asarray(a), step, sample_rate)


def test_gan_train_logging_and_samples(tmp_path, golden_dir):
    """models/GAN/train.py:403-504: the 12 Loss_Train/LR scalars and the three
    sample FLACs (combined log1p magnitude, original, impaired through the
    ISTFT with the original phase); the combined reconstruction matches the
    oracle ISTFT to 1e-5 relative L2."""
    import utils
    from ainp import gan as G
    from ainp.gan_train import GanTrainer
    from ainp.audio_io import read_flac
    from models.GAN import train as T
    from oracle import gan_ref as R

    n_fft, hop, win, sr = 512, 128, 512, 16000
    items = []
    for k, c in enumerate(CLIPS):
        audio, _ = utils.load_audio(os.path.join(golden_dir, "flac", c))
        items.append(S.gan_item(audio, 20000 + 7000 * k, 3200, n_fft, hop, win))
    b = {name: torch.from_numpy(np.stack([it[j] for it in items])[:, None]).cuda()
         for j, name in enumerate(("original_magnitude", "impaired_magnitude",
                                   "original_phase", "mask"))}
    torch.manual_seed(0)
    cfg = {"training": dict(R.LAMBDAS, g_lr=2e-4, d_lr=1e-4, b1=0.5, b2=0.999)}
    tr = GanTrainer(cfg, G.PConvUNet().cuda(), G.Discriminator().cuda(), vgg=None)
    out = tr.step(b["original_magnitude"], b["impaired_magnitude"], b["mask"])
    w = _RecWriter()
    T.log_train_step(w, out, tr, 100)
    assert len(w.scalars) == 12 and all(s == 100 for _, s in w.scalars.values())
    assert w.scalars["LR/Discriminator"][0] == 1e-4
    assert w.scalars["Loss_Train/Discriminator"][0] == pytest.approx(
        (w.scalars["Loss_Train/Discriminator_Real"][0]
         + w.scalars["Loss_Train/Discriminator_Fake"][0]) / 2, rel=1e-5)
    spec = {"n_fft": n_fft, "hop_length": hop, "win_length": win, "window": "hann"}
    rec = T.save_samples(w, b, out["generated"], spec, sr, tmp_path, 500)
    g = out["generated"][0, 0].double().cpu().numpy()
    m = items[0][3].astype(np.float64)
    comb = g * (1 - m) + items[0][0] * m
    ref = S.istft(comb * np.exp(1j * items[0][2].astype(np.float64)), hop, win, n_fft)
    assert len(rec) == len(ref) == 80000
    assert np.linalg.norm(rec - ref) / np.linalg.norm(ref) < 1e-5
    assert np.array_equal(w.audio["Audio/Generated_CombinedLogMag_OrigPhase"][0], rec)
    for name in ("recon_comb_origphase", "original", "impaired"):
        a, r = read_flac(tmp_path / f"step_500_{name}.flac")
        assert r == sr and a.shape == (80000, 1) and np.abs(a).max() > 0.99


def test_cnnblstm_audio_samples(tmp_path, golden_dir):
    """models/CNNBLSTM/train.py:178-189: orig / gap through the ISTFT and the
    reconstruction through Griffin-Lim, all at spectrogram_to_audio's default
    hop of 512 (the call passes only n_fft); the ISTFTs match the oracle."""
    import yaml
    import utils
    from ainp.audio_io import read_flac
    from models.CNNBLSTM import train as T
    from models.CNNBLSTM.model import StackedBLSTMCNN

    cfg_path = os.path.join(PKG, "models", "CNNBLSTM", "cnn_blstm.yaml")
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f)
    n_fft, hop, win = 512, 192, 384
    xs, ms, ts = [], [], []
    for k, c in enumerate(CLIPS):
        audio, _ = utils.load_audio(os.path.join(golden_dir, "flac", c))
        lg, tg, m = S.cnnblstm_item(audio, 24000 + 5000 * k, 1600, n_fft, hop, win, 16000, 417)
        xs.append(lg), ms.append(m), ts.append(tg)
    x = torch.from_numpy(np.stack(xs)).cuda()
    mask = torch.from_numpy(np.stack(ms)).cuda()
    target = torch.from_numpy(np.stack(ts)).cuda()
    torch.manual_seed(0)
    model = StackedBLSTMCNN(cfg_path).cuda().eval()
    w = _RecWriter()
    audio = T.save_audio_samples(w, model, cfg, x, mask, target, tmp_path, 500)
    assert sorted(w.audio) == ["Audio/Generated", "Audio/Impaired", "Audio/Original"]
    n = 512 * (417 - 1)
    for k, X in (("orig", ts[0]), ("gap", ts[0] * (1 - ms[0]))):
        ref = S.istft(X.astype(np.complex128), 512, None, n_fft)
        assert len(audio[k]) == len(ref) == n
        # hop == n_fft: no overlap, so the sum-square division amplifies float32
        # rounding by 1/w near every frame edge -> 1e-3, not the usual 1e-5
        assert np.linalg.norm(audio[k] - ref) / np.linalg.norm(ref) < 1e-3, k
    assert len(audio["reconstructed"]) == n and np.isfinite(audio["reconstructed"]).all()
    for k in ("orig", "gap", "reconstructed"):
        a, r = read_flac(tmp_path / f"{k}_audio_500.flac")
        assert r == 16000 and a.shape == (n, 1)
