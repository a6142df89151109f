"""GPU parity of ISTFT / Griffin-Lim (utils.spectrogram_to_audio)
against the float64 oracle (oracle/stft_ref.py istft / griffinlim, pinned by
the ISTFT(STFT(x)) = x property in test_cpu_oracle.py)."""
import numpy as np
import pytest
import torch

from oracle import stft_ref
from ainp import synth

pytestmark = pytest.mark.gpu


def _spec(n_fft, hop, win, L, seed=0, dtype=np.float32):
    x = synth.synthetic_clip(seed, L).astype(dtype)
    return x, stft_ref.stft(x, n_fft, hop, win)


@pytest.mark.parametrize("n_fft,hop,win", [(512, 192, 384), (512, 128, 512), (2048, 512, 2048)])
def test_istft_modes_match_oracle(n_fft, hop, win):
    from ainp import ops
    _, X = _spec(n_fft, hop, win, 12000, seed=n_fft + hop)
    rng = np.random.default_rng(1)
    X = X * (1 + 0.1 * rng.standard_normal(X.shape))      # not a consistent spectrogram
    ref = stft_ref.istft(X, hop, win, n_fft)
    # complex128 -> float64
    y = ops.istft(torch.from_numpy(X).cuda(), n_fft=n_fft, hop_length=hop, win_length=win)
    assert y.dtype == torch.float64
    assert np.abs(y.cpu().numpy() - ref).max() <= 1e-12 * np.abs(ref).max()
    # complex64 -> float32
    X64 = X.astype(np.complex64)
    ref64 = stft_ref.istft(X64.astype(np.complex128), hop, win, n_fft)
    y = ops.istft(torch.from_numpy(X64).cuda(), n_fft=n_fft, hop_length=hop, win_length=win)
    assert y.dtype == torch.float32
    assert np.abs(y.cpu().numpy() - ref64).max() <= 1e-6 * np.abs(ref64).max()
    # magnitude * exp(i phase)
    mag = np.abs(X).astype(np.float32)
    ph = np.angle(X).astype(np.float32)
    refp = stft_ref.istft(mag.astype(np.float64) * np.exp(1j * ph.astype(np.float64)), hop, win, n_fft)
    y = ops.istft(mag=torch.from_numpy(mag).cuda(), phase=torch.from_numpy(ph).cuda(),
                  n_fft=n_fft, hop_length=hop, win_length=win)
    assert np.abs(y.cpu().numpy() - refp).max() <= 1e-6 * np.abs(refp).max()
    # batched magnitude * unit angles
    ang = np.exp(1j * ph).astype(np.complex64)
    mb = np.stack([mag, 0.5 * mag])
    ab = np.stack([ang, ang])
    y = ops.istft(mag=torch.from_numpy(mb).cuda(), angles=torch.from_numpy(ab).cuda(),
                  n_fft=n_fft, hop_length=hop, win_length=win)
    for b in range(2):
        rb = stft_ref.istft((mb[b] * ab[b]).astype(np.complex128), hop, win, n_fft)
        assert np.abs(y[b].cpu().numpy() - rb).max() <= 1e-6 * np.abs(rb).max()


def test_gpu_stft_istft_round_trip():
    from ainp import ops
    x = torch.from_numpy(synth.synthetic_clip(9, 80000)).cuda()
    X = ops.stft(x, 512, 128, 512)
    y = ops.istft(X, n_fft=512, hop_length=128, win_length=512)
    assert y.shape[-1] == 128 * (X.shape[-1] - 1)
    err = (y - x[:y.shape[-1]]).abs().max().item()
    assert err < 1e-6 * x.abs().max().item() + 1e-7


def test_griffinlim_matches_oracle():
    from ainp import ops
    x = synth.synthetic_clip(11, 8000).astype(np.float64)
    S = np.abs(stft_ref.stft(x, 512, 128, 512)).astype(np.float32)
    for n_iter in (0, 1, 4):
        y = ops.griffinlim(torch.from_numpy(S).cuda(), n_iter=n_iter, hop_length=128,
                           win_length=512, n_fft=512, random_state=3)
        ref = stft_ref.griffinlim(S.astype(np.float64), n_iter, 128, 512, 512, random_state=3)
        rel = np.linalg.norm(y.cpu().numpy() - ref) / np.linalg.norm(ref)
        assert rel < 1e-4, (n_iter, rel)


def test_spectrogram_to_audio_paths():
    import utils
    x = synth.synthetic_clip(13, 8000)
    X = stft_ref.stft(x.astype(np.float64), 512, 128, 512).astype(np.complex64)
    mag, ph = np.abs(X), np.angle(X).astype(np.float32)
    y = utils.spectrogram_to_audio(mag, ph, n_fft=512, hop_length=128, win_length=512)
    assert isinstance(y, np.ndarray) and y.dtype == np.float32
    assert np.abs(y - x[:len(y)]).max() < 1e-5
    y2 = utils.spectrogram_to_audio(X, phase_info=True, n_fft=512, hop_length=128)
    assert np.abs(y2 - x[:len(y2)]).max() < 1e-5
    # dB input (max < 0, mean < 0) is converted back to amplitude first
    Sdb = 20 * np.log10(np.maximum(mag, 1e-6) / (mag.max() * 1.01))
    y3 = utils.spectrogram_to_audio(Sdb.astype(np.float32), ph, n_fft=512, hop_length=128)
    ref3 = stft_ref.istft(10 ** (0.05 * Sdb.astype(np.float64)) * np.exp(1j * ph), 128, 512, 512)
    assert np.abs(y3 - ref3).max() < 1e-5 * np.abs(ref3).max()
    # Griffin-Lim path, seeded as librosa(random_state=...)
    y4 = utils.spectrogram_to_audio(mag, n_fft=512, hop_length=128, n_iter=2, random_state=0)
    ref4 = stft_ref.griffinlim(mag.astype(np.float64), 2, 128, 512, 512, random_state=0)
    assert np.linalg.norm(y4 - ref4) / np.linalg.norm(ref4) < 1e-4


@pytest.mark.timeout(300)
def test_griffinlim_c5_shape_matches_oracle():
    """BASELINE C5's on-GPU reconstruction at its own shape: a batch of 8
    log1p-magnitude spectrograms of 8 s clips ([8, 257, 1001], n_fft 512,
    hop 128, win 512), 64 Griffin-Lim iterations (GAN train.py sample audio,
    utils.py:279-333) from supplied initial phases, against the float64
    oracle.  Tolerance 1e-3 relative L2 per signal: the GPU iterates in fp32
    (complex64 angles, float32 audio) over 64 momentum-0.99 iterations."""
    from ainp import ops
    B, S, hop, n_iter = 8, 128000, 128, 64
    mags = np.stack([np.abs(stft_ref.stft(synth.synthetic_clip(700 + b, S).astype(np.float64),
                                          512, hop, 512)) for b in range(B)]).astype(np.float32)
    assert mags.shape == (B, 257, 1001)
    rng = np.random.default_rng(5)
    ph = 2 * np.pi * rng.random(mags.shape)
    ang = (np.cos(ph) + 1j * np.sin(ph)).astype(np.complex64)
    y = ops.griffinlim(torch.from_numpy(mags).cuda(), n_iter=n_iter, hop_length=hop,
                       win_length=512, n_fft=512,
                       init_angles=torch.from_numpy(ang).cuda()).cpu().numpy()
    assert y.shape == (B, hop * 1000)
    errs = []
    for b in range(B):
        ref = stft_ref.griffinlim(mags[b].astype(np.float64), n_iter, hop, 512, 512,
                                  init_angles=ang[b].astype(np.complex128))
        errs.append(np.linalg.norm(y[b] - ref) / np.linalg.norm(ref))
    print("GL C5 rel errs", errs)
    assert max(errs) < 1e-3, errs


@pytest.mark.parametrize("hop,win,S", [(128, 512, 128000), (192, 384, 64000), (128, 512, 1000)])
def test_stft512_plain_mode_matches_oracle_and_generic(hop, win, S, monkeypatch):
    """ainp_stft at n_fft = 512 (float32, center) runs on the tiled n_fft=512
    kernel (F512_PLAIN mode): complex64 spectrum vs the float64 oracle
    (librosa>=0.10 stft restated) within 2e-6 of max|X|, and vs the generic
    radix-2 kernel (AINP_STFT_GENERIC=1) to fp32 rounding."""
    from ainp import ops
    B = 3
    xs = np.stack([synth.synthetic_clip(40 + b, S) for b in range(B)]).astype(np.float32)
    X = ops.stft(torch.from_numpy(xs).cuda(), 512, hop, win).cpu().numpy()
    ref = np.stack([stft_ref.stft(xs[b].astype(np.float64), 512, hop, win) for b in range(B)])
    assert X.shape == ref.shape == (B, 257, 1 + S // hop)
    assert np.abs(X - ref).max() <= 2e-6 * np.abs(ref).max()
    monkeypatch.setenv("AINP_STFT_GENERIC", "1")
    Xg = ops.stft(torch.from_numpy(xs).cuda(), 512, hop, win).cpu().numpy()
    assert np.abs(X - Xg).max() <= 1e-6 * np.abs(ref).max()


def test_gl_stft_update_equals_stft_then_update():
    """ainp_gl_stft_update (the STFT with the Griffin-Lim phase update fused
    into its write-out) == ainp_stft followed by ainp_gl_update, bit for bit,
    on the first and on a later iteration."""
    from ainp import ops
    B, S, hop = 2, 16000, 128
    x = torch.from_numpy(np.stack([synth.synthetic_clip(60 + b, S) for b in range(B)])
                         .astype(np.float32)).cuda()
    T = 1 + S // hop
    w = ops._device_window("hann", 512, 512, x.device)
    g = torch.Generator().manual_seed(3)
    tp0 = torch.randn(B, 257, T, 2, generator=g).cuda()
    tp0 = torch.view_as_complex(tp0).contiguous()
    for first in (True, False):
        tp_a, an_a = tp0.clone(), torch.empty_like(tp0)
        rebuilt = ops.stft(x, 512, hop, 512)
        torch.ops.ainp.gl_update(rebuilt, tp_a, an_a, 0.99, first)
        tp_b, an_b = tp0.clone(), torch.empty_like(tp0)
        torch.ops.ainp.gl_stft_update(x, w, hop, T, tp_b, an_b, 0.99, first)
        torch.cuda.synchronize()
        assert torch.equal(tp_a, tp_b) and torch.equal(an_a, an_b), first
