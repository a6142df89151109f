"""CPU tests: pin the oracle against the reference's golden vectors and the
reference tests' known properties (no GPU needed)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import cnnblstm_ref, stft_ref
from ainp import synth


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


BN_FED = ("encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "decoder.0.bias", "decoder.3.bias")


# ------------------------------------------------------------------ STFT oracle
def test_stft_matches_direct_dft():
    y = synth.synthetic_clip(1, 1000)
    n_fft, hop, win = 64, 16, 48
    X = stft_ref.stft(y, n_fft, hop, win)
    assert X.shape == (n_fft // 2 + 1, 1 + len(y) // hop)  # center=True frame count
    w = stft_ref.padded_window("hann", win, n_fft)
    yp = np.pad(y.astype(np.float64), n_fft // 2)
    n = np.arange(n_fft)
    for t in (0, 5, X.shape[1] - 1):
        fr = yp[t * hop:t * hop + n_fft] * w
        ref = np.array([np.sum(fr * np.exp(-2j * np.pi * f * n / n_fft)) for f in range(n_fft // 2 + 1)])
        assert np.abs(X[:, t] - ref).max() < 1e-10


def test_hann_window_is_periodic():
    w = stft_ref.get_window("hann", 384)
    n = np.arange(384)
    assert np.abs(w - (0.5 - 0.5 * np.cos(2 * np.pi * n / 384))).max() < 1e-15


def test_reference_frame_count_and_bins():
    """tests/utils_test.py:260-275 spec (with center=True frame count)."""
    y = np.zeros(32000, np.float32)
    X = stft_ref.stft(y, 512, 192, 384)
    assert X.shape == (257, 1 + 32000 // 192)


def _istft(X, n_fft, hop, win, length):
    """Window-sum-square normalised overlap-add (librosa.istft semantics)."""
    w = stft_ref.padded_window("hann", win, n_fft)
    frames = np.fft.irfft(X, n=n_fft, axis=0) * w[:, None]
    T = X.shape[1]
    out = np.zeros(n_fft + hop * (T - 1))
    wss = np.zeros_like(out)
    for t in range(T):
        out[t * hop:t * hop + n_fft] += frames[:, t]
        wss[t * hop:t * hop + n_fft] += w ** 2
    nz = wss > 1e-12
    out[nz] /= wss[nz]
    return out[n_fft // 2:n_fft // 2 + length]


@pytest.mark.parametrize("n_fft,hop,win", [(512, 192, 384), (512, 128, 512), (512, 128, 384)])
def test_stft_istft_perfect_reconstruction(n_fft, hop, win):
    """tests/utils_test.py:780-809: ISTFT(STFT(x)) == x to 1e-10."""
    y = synth.synthetic_clip(4, 16000).astype(np.float64)
    X = stft_ref.stft(y, n_fft, hop, win)
    r = _istft(X, n_fft, hop, win, len(y))
    assert np.abs(r[n_fft:-n_fft] - y[n_fft:-n_fft]).max() < 1e-10


def test_add_gap_zeroes_exactly_and_keeps_length():
    """tests/utils_test.py:216-243 spec."""
    y = synth.synthetic_clip(2, 80000)
    g = stft_ref.add_gap(y, 1234, 3200)
    assert g.dtype == np.float64 and len(g) == len(y)
    assert np.all(g[1234:1234 + 3200] == 0)
    assert np.array_equal(g[:1234], y[:1234].astype(np.float64))


def test_gap_frames_known_answers(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "gap_frames.json")))
    # the four starts whose float round trip lands one frame early
    assert d["cnnblstm_hop192_sr16000_float_rule_differs_at"] == [64320, 64704, 65088, 65472]
    assert [c["fs"] for c in d["cases"][:4]] == [334, 336, 338, 340]
    for c in d["cases"]:
        if c["rule"] == "cnnblstm":
            assert stft_ref.cnnblstm_gap_frames(c["start"], c["gap"], c["sr"], c["hop"]) == (c["fs"], c["fe"])
        else:
            assert stft_ref.gan_gap_frames(c["start"], c["gap"], c["hop"], c["n_frames"]) == (c["fs"], c["fe"])


# ------------------------------------------------------------------ model oracle
def _small_cfg(g):
    n_fft, hop, win, hidden, layers, N, T = [int(v) for v in g["config"]]
    return {"data": {"spectrogram": {"n_fft": n_fft}},
            "model": {"in_channels": 1, "num_lstm_layers": layers, "lstm_hidden_dim": hidden,
                      "enc_filters": [16, 32], "dec_filters": [16, 32]}}, hidden, layers


def test_oracle_training_steps_match_reference_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "cnnblstm_small.npz"), allow_pickle=False)
    _, H, L = _small_cfg(g)
    p = {k[5:]: torch.from_numpy(np.array(g[k])).clone() for k in g.files if k.startswith("init/")}
    tr = cnnblstm_ref.Trainer(p, H, L, lr=1e-4)
    x, m, t = (torch.from_numpy(g[k]) for k in ("x", "mask", "target"))
    tr.opt.zero_grad()
    y = cnnblstm_ref.forward(tr.p, x.unsqueeze(1), H, L)
    loss = cnnblstm_ref.loss_fn(y, m, t)
    loss.backward()
    assert rel(y.detach(), g["y"]) < 1e-6
    assert abs(loss.item() - g["loss"][0]) / g["loss"][0] < 1e-6
    for k in tr.keys:
        if k in BN_FED:
            continue
        assert rel(tr.p[k].grad, g["grad/" + k]) < 1e-5, k
    tr.opt.step()
    tr.step(x, m, t)
    for k in tr.keys:
        if k in BN_FED:
            continue
        assert rel(tr.p[k].detach(), g["final/" + k]) < 1e-5, k
    for k in g.files:
        if k.startswith("final/") and ("running" in k):
            assert rel(tr.p[k[6:]], g[k]) < 1e-5, k


def test_init_parity_with_reference_construction(golden_dir):
    """torch.manual_seed(0) + the reference's construction order gives the
    reference's initial weights: for the oracle's parameter dict AND for the
    product's StackedBLSTMCNN (same submodule tree)."""
    g = np.load(os.path.join(golden_dir, "cnnblstm_full.npz"), allow_pickle=False)
    cfg = {"data": {"spectrogram": {"n_fft": 512}},
           "model": {"in_channels": 1, "num_lstm_layers": 3, "lstm_hidden_dim": 128,
                     "enc_filters": [16, 32], "dec_filters": [16, 32]}}
    p = cnnblstm_ref.init_params(cfg, seed=0)
    from ainp.cnnblstm import StackedBLSTMCNN
    torch.manual_seed(0)
    mod = StackedBLSTMCNN(config=cfg)
    sd = mod.state_dict()
    assert set(sd) == set(p)
    for k, chk in ((k[6:], g[k]) for k in g.files if k.startswith("check/")):
        assert abs(float(p[k].double().sum()) - chk[0]) <= 1e-6 * max(1, abs(chk[0])), k
        assert abs(float(sd[k].double().sum()) - chk[0]) <= 1e-6 * max(1, abs(chk[0])), k


def test_accel_deterministic_flag():
    """accel.deterministic: validated, default true, and under it the atomic
    colsum entry point refuses before launching anything (host-side check)."""
    from ainp import ops
    from ainp.cnnblstm import StackedBLSTMCNN
    cfg = {"data": {"spectrogram": {"n_fft": 64}},
           "model": {"in_channels": 1, "num_lstm_layers": 1, "lstm_hidden_dim": 8,
                     "enc_filters": [4, 8], "dec_filters": [4, 8]}}
    assert StackedBLSTMCNN(config=cfg).deterministic is True
    with pytest.raises(ValueError):
        StackedBLSTMCNN(config=dict(cfg, accel={"deterministic": "yes"}))
    assert StackedBLSTMCNN(config=dict(cfg, accel={"deterministic": False})).deterministic is False
    StackedBLSTMCNN(config=dict(cfg, accel={"deterministic": True}))
    with pytest.raises(RuntimeError, match="deterministic"):
        ops.colsum(torch.zeros(4, 4), out=torch.zeros(4), accumulate=True)


def test_state_dict_keys_match_reference_layout(golden_dir):
    g = np.load(os.path.join(golden_dir, "cnnblstm_small.npz"), allow_pickle=False)
    cfg, _, _ = _small_cfg(g)
    from ainp.cnnblstm import StackedBLSTMCNN
    keys = set(StackedBLSTMCNN(config=cfg).state_dict())
    ref_keys = {k[5:] for k in g.files if k.startswith("init/")}
    assert keys == ref_keys


def test_oracle_istft_inverts_stft():
    """tests/utils_test.py:780-849 property: ISTFT(STFT(x)) == x (to 1e-10), for
    the configurations the reference uses (CNNBLSTM 512/192/384, GAN 512/128/512,
    extract_spectrogram defaults 2048/512)."""
    rng = np.random.default_rng(5)
    for n_fft, hop, win, L in [(512, 192, 384, 9000), (512, 128, 512, 8000), (2048, 512, 2048, 22050)]:
        x = rng.standard_normal(L)
        y = stft_ref.istft(stft_ref.stft(x, n_fft, hop, win), hop, win, n_fft)
        assert len(y) == hop * (1 + L // hop - 1)
        assert np.abs(y - x[:len(y)]).max() < 1e-10


def test_oracle_griffinlim_converges_toward_magnitude():
    """Griffin-Lim restatement: consistent spectrogram error decreases with
    iterations (librosa's own test idea, tests/utils_test.py:851-905)."""
    from ainp.synth import synthetic_clip
    x = synthetic_clip(3, 8000).astype(np.float64)
    S = np.abs(stft_ref.stft(x, 512, 128, 512))
    errs = []
    for it in (1, 8):
        y = stft_ref.griffinlim(S, it, 128, 512, 512, random_state=0)
        errs.append(np.linalg.norm(np.abs(stft_ref.stft(y, 512, 128, 512)) - S) / np.linalg.norm(S))
    assert errs[1] < errs[0]
