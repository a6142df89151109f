"""numpy float64 restatement of the reference's STFT / feature / gap path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows, per function:
  stft            utils.extract_spectrogram -> librosa.stft   (utils.py:192-234)
                  librosa>=0.10: window = scipy get_window(window, win, fftbins=True)
                  zero-padded to n_fft at offset (n_fft-win)//2; centre=True pads the
                  signal with n_fft//2 zeros ('constant', the >=0.10 default);
                  frame t = y_pad[t*hop : t*hop+n_fft]; X = rfft(w * frame).
  time_to_frames  librosa.time_to_frames(t, sr, hop) = (t*sr).astype(int) // hop
                  as used by models/CNNBLSTM/dataset.py:116-117.
  add_gap         utils.add_random_gap's zeroing (utils.py:179-186), float64 result.
  create_gap_mask utils.create_gap_mask (utils.py:93-144).
  cnnblstm_item   models/CNNBLSTM/dataset.py:93-119 for one gap of one clip.
  gan_item        models/GAN/dataset.py:104-152.
"""
from __future__ import annotations

import math

import numpy as np


def get_window(window: str, win_length: int) -> np.ndarray:
    import scipy.signal
    return scipy.signal.get_window(window, win_length, fftbins=True).astype(np.float64)


def padded_window(window: str, win_length: int, n_fft: int) -> np.ndarray:
    w = get_window(window, win_length)
    out = np.zeros(n_fft, dtype=np.float64)
    lpad = (n_fft - win_length) // 2
    out[lpad:lpad + win_length] = w
    return out


def stft(y: np.ndarray, n_fft: int = 2048, hop_length: int = 512,
         win_length: int | None = None, window: str = "hann") -> np.ndarray:
    """complex128 [1 + n_fft//2, 1 + len(y)//hop] (librosa>=0.10, center=True)."""
    if win_length is None:
        win_length = n_fft
    y = np.asarray(y, dtype=np.float64)
    w = padded_window(window, win_length, n_fft)
    pad = n_fft // 2
    yp = np.pad(y, (pad, pad), mode="constant")
    n_frames = 1 + (len(yp) - n_fft) // hop_length
    idx = np.arange(n_fft)[:, None] + hop_length * np.arange(n_frames)[None, :]
    frames = yp[idx] * w[:, None]
    return np.fft.rfft(frames, axis=0)


def time_to_frames(t_seconds: float, sr: int, hop: int) -> int:
    samples = int(np.asarray(t_seconds * sr).astype(int))
    return int(np.floor(samples // hop))


def gap_seconds(gap_start: int, gap_len_samples: int, sr: int):
    """utils.add_random_gap return value: (start/sr, (start+g)/sr) in Python floats."""
    return gap_start / sr, (gap_start + gap_len_samples) / sr


def cnnblstm_gap_frames(gap_start: int, gap_len_samples: int, sr: int, hop: int):
    s, e = gap_seconds(gap_start, gap_len_samples, sr)
    return time_to_frames(s, sr, hop), time_to_frames(e, sr, hop)


def gan_gap_frames(gap_start: int, gap_len_samples: int, hop: int, n_frames: int):
    fs = gap_start // hop
    fe = int(np.ceil((gap_start + gap_len_samples) / hop))
    return max(0, fs), min(n_frames, fe)


def add_gap(audio: np.ndarray, gap_start: int, gap_len_samples: int) -> np.ndarray:
    silence = np.zeros(gap_len_samples)  # float64
    return np.concatenate([audio[:gap_start], silence, audio[gap_start + gap_len_samples:]])


def cnnblstm_item(audio_f32: np.ndarray, gap_start: int, gap_len_samples: int,
                  n_fft: int, hop: int, win_length: int, sr: int, n_frames: int):
    """One (clip, gap) example: (log10 |X_gap| + 1e-9 f32, target c64, mask f32)."""
    F = n_fft // 2 + 1
    target = stft(audio_f32.astype(np.float32), n_fft, hop, win_length)
    gapped = add_gap(audio_f32.astype(np.float32), gap_start, gap_len_samples)
    gmag = np.abs(stft(gapped, n_fft, hop, win_length))
    logmag = np.log10(gmag + 1e-9)
    out_log = np.zeros((F, n_frames), dtype=np.float32)
    out_tgt = np.zeros((F, n_frames), dtype=np.complex64)
    nt = min(n_frames, target.shape[1])
    out_log[:, :nt] = logmag[:, :nt].astype(np.float32)
    out_tgt[:, :nt] = target[:, :nt].astype(np.complex64)
    mask = np.zeros((F, n_frames), dtype=np.float32)
    fs, fe = cnnblstm_gap_frames(gap_start, gap_len_samples, sr, hop)
    mask[:, fs:fe] = 1
    return out_log, out_tgt, mask


def gan_item(audio_f32: np.ndarray, gap_start: int, gap_len_samples: int,
             n_fft: int, hop: int, win_length: int):
    """(log1p|X|, log1p|X_imp|, angle X, mask 1=valid) float32 [F, T]."""
    a = audio_f32.astype(np.float32)
    m = np.ones(len(a), dtype=np.float32)
    m[gap_start:gap_start + gap_len_samples] = 0.0
    imp = a * m
    X = stft(a, n_fft, hop, win_length).astype(np.complex64)
    Xi = stft(imp, n_fft, hop, win_length).astype(np.complex64)
    orig = np.log1p(np.abs(X))
    impm = np.log1p(np.abs(Xi))
    phase = np.angle(X)
    T = X.shape[1]
    fs, fe = gan_gap_frames(gap_start, gap_len_samples, hop, T)
    mask = np.ones(X.shape, dtype=np.float32)
    if fe > fs:
        mask[:, fs:fe] = 0
    return (orig.astype(np.float32), impm.astype(np.float32),
            phase.astype(np.float32), mask)


# ------------------------------------------------------------- ISTFT / Griffin-Lim
def window_sumsquare(window: str, n_frames: int, hop: int, win_length: int, n_fft: int):
    """librosa.filters.window_sumsquare (norm=None): sum of the squared,
    centre-padded window shifted by hop, length n_fft + hop*(n_frames-1)."""
    w2 = padded_window(window, win_length, n_fft) ** 2
    n = n_fft + hop * (n_frames - 1)
    x = np.zeros(n, dtype=np.float64)
    for i in range(n_frames):
        s = i * hop
        x[s:min(n, s + n_fft)] += w2[:max(0, min(n_fft, n - s))]
    return x


def istft(X: np.ndarray, hop_length: int, win_length=None, n_fft=None,
          window: str = "hann", center: bool = True, length=None) -> np.ndarray:
    """librosa>=0.10 istft restated in float64 (utils.py:317-326 call sites):
    irfft per frame (imaginary DC/Nyquist ignored), synthesis window,
    overlap-add, division by the window sum-square where it exceeds tiny,
    n_fft/2 trimmed per side when center.  X [F, T] or [B, F, T]."""
    X = np.asarray(X)
    if X.ndim == 3:
        return np.stack([istft(x, hop_length, win_length, n_fft, window, center, length)
                         for x in X])
    F, T = X.shape
    n_fft = 2 * (F - 1) if n_fft is None else n_fft
    win_length = n_fft if win_length is None else win_length
    w = padded_window(window, win_length, n_fft)
    frames = np.fft.irfft(X.astype(np.complex128), n=n_fft, axis=0) * w[:, None]
    n = n_fft + hop_length * (T - 1)
    y = np.zeros(n, dtype=np.float64)
    for t in range(T):
        y[t * hop_length:t * hop_length + n_fft] += frames[:, t]
    wss = window_sumsquare(window, T, hop_length, win_length, n_fft)
    tiny = np.finfo(np.float32 if X.dtype == np.complex64 else np.float64).tiny
    nz = wss > tiny
    y[nz] /= wss[nz]
    if center:
        y = y[n_fft // 2:n - n_fft // 2]
    if length is not None:
        y = y[:length] if len(y) >= length else np.pad(y, (0, length - len(y)))
    return y


def griffinlim(S: np.ndarray, n_iter: int = 32, hop_length=None, win_length=None, n_fft=None,
               window: str = "hann", center: bool = True, momentum: float = 0.99,
               random_state=None, init_angles=None) -> np.ndarray:
    """librosa>=0.10 griffinlim (init='random', pad_mode='constant') restated:
    angles = exp(2 pi i U) from np.random.default_rng(random_state); per
    iteration inverse = istft(S*angles), rebuilt = stft(inverse),
    angles = rebuilt - m/(1+m) * previous rebuilt (from the 2nd iteration),
    angles /= |angles| + tiny; returns istft(S*angles).  float64 throughout."""
    S = np.asarray(S, dtype=np.float64)
    F, T = S.shape
    n_fft = 2 * (F - 1) if n_fft is None else n_fft
    win_length = n_fft if win_length is None else win_length
    hop_length = win_length // 4 if hop_length is None else hop_length
    if init_angles is None:
        rng = np.random.default_rng(seed=random_state)
        ph = 2 * np.pi * rng.random(size=S.shape)
        angles = np.cos(ph) + 1j * np.sin(ph)
    else:
        angles = np.asarray(init_angles, dtype=np.complex128)
    eps = np.finfo(np.float64).tiny
    rebuilt = None
    for _ in range(n_iter):
        tprev = rebuilt
        inv = istft(S * angles, hop_length, win_length, n_fft, window, center)
        rebuilt = stft(inv, n_fft, hop_length, win_length, window)
        angles = rebuilt.copy()
        if tprev is not None:
            angles -= (momentum / (1 + momentum)) * tprev
        angles /= np.abs(angles) + eps
    return istft(S * angles, hop_length, win_length, n_fft, window, center)
