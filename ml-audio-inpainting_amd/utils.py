"""Drop-in for the reference's utils.py (audio I/O, gap creation, STFT).

Same names, signatures, return types and error behaviour as
/root/reference/utils.py; the STFT runs on the MI355X kernel
(ainp_stft / ainp_stft_features) instead of librosa.

  load_audio            utils.py:14-52   (WAV via the stdlib, FLAC on the native
                                          decoder ainp_flac_decode; other formats
                                          through soundfile when it is installed)
  save_audio            utils.py:54-89   (peak-normalised, WAV; FLAC via soundfile)
  create_gap_mask       utils.py:93-144  (host numpy, the reference's own RNG call)
  add_random_gap        utils.py:146-188 (host numpy, float64 result)
  extract_spectrogram   utils.py:192-234 (GPU, returns the complex STFT; power is
                                          validated then ignored)
  spectrogram_to_audio  utils.py:279-333  (GPU ISTFT / Griffin-Lim)
Mel spectrograms and plotting are outside the hot path.
"""
from __future__ import annotations

import os
import wave
from pathlib import Path
from typing import Optional, Tuple, Union

import numpy as np

from config import DEFAULT_SAMPLE_RATE

# --- Audio I/O ---------------------------------------------------------------


def _read_wav(path: str) -> Tuple[np.ndarray, int]:
    with wave.open(path, "rb") as w:
        nch, width, sr, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if width == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif width == 2:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3)
        v = (b[:, 0].astype(np.int32) | (b[:, 1].astype(np.int32) << 8)
             | (b[:, 2].astype(np.int32) << 16))
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif width == 4:
        x = np.frombuffer(raw, "<i4").astype(np.float32) / float(1 << 31)
    else:
        raise ValueError(f"unsupported sample width {width}")
    return x.reshape(-1, nch), sr


def _is_flac(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            head = f.read(4)
    except OSError:
        return False
    return head == b"fLaC" or (head[:3] == b"ID3" and str(path).lower().endswith(".flac"))


def _read_any(path: str) -> Tuple[np.ndarray, int]:
    """(frames, channels) float32 in [-1, 1) and the native rate."""
    if str(path).lower().endswith(".wav"):
        try:
            return _read_wav(str(path))
        except (wave.Error, EOFError):
            pass
    if _is_flac(str(path)):
        from ainp.audio_io import read_flac   # native decoder
        return read_flac(str(path))
    try:
        import soundfile as sf  # optional dependency (not in this image)
    except ImportError as e:
        raise RuntimeError(
            f"cannot decode {path}: only PCM WAV and FLAC are readable without "
            "soundfile") from e
    data, sr = sf.read(str(path), dtype="float32", always_2d=True)
    return data, sr


def load_audio(file_path: Union[str, Path], sample_rate: int = DEFAULT_SAMPLE_RATE,
               max_len: int = 5, mono: bool = True) -> Tuple[np.ndarray, int]:
    """utils.py:14-52: decode, resample to `sample_rate`, mix to mono, truncate
    or zero-pad to int(sample_rate*max_len) samples; IOError on any failure."""
    try:
        data, sr = _read_any(file_path)
        if mono:
            data = data.mean(axis=1)          # librosa.to_mono
        else:
            data = data.T.squeeze()
        if sr != sample_rate:
            from math import gcd
            from scipy.signal import resample_poly
            g = gcd(int(sr), int(sample_rate))
            data = resample_poly(data, sample_rate // g, sr // g, axis=-1).astype(np.float32)
        audio_data = data.astype(np.float32)
        sr = sample_rate
        max_samples = int(sample_rate * max_len)
        if len(audio_data) > max_samples:
            audio_data = audio_data[:max_samples]
        else:
            audio_data = np.pad(audio_data, (0, max_samples - len(audio_data)), "constant")
        return audio_data, sr
    except Exception as e:
        raise IOError(f"Error loading audio file {file_path}: {str(e)}")


def save_audio(audio_data: np.ndarray, file_path: Union[str, Path],
               sample_rate: int = DEFAULT_SAMPLE_RATE, normalize: bool = True,
               file_format: str = "flac") -> None:
    """utils.py:54-89: create parent dirs, peak-normalise
    (librosa.util.normalize: x / max|x|), write 16-bit PCM."""
    output_dir = Path(file_path).parent
    if output_dir and not output_dir.exists():
        try:
            output_dir.mkdir(parents=True, exist_ok=True)
        except Exception as e:
            raise IOError(f"Error creating directory {output_dir}: {str(e)}")
    audio_data = np.asarray(audio_data)
    if normalize:
        peak = np.max(np.abs(audio_data)) if audio_data.size else 0.0
        if peak > np.finfo(np.float32).tiny:
            audio_data = audio_data / peak
    try:
        if file_format.lower() == "wav" or str(file_path).lower().endswith(".wav"):
            pcm = np.clip(np.round(audio_data * 32767.0), -32768, 32767).astype("<i2")
            with wave.open(str(file_path), "wb") as w:
                w.setnchannels(1 if pcm.ndim == 1 else pcm.shape[1])
                w.setsampwidth(2)
                w.setframerate(int(sample_rate))
                w.writeframes(pcm.tobytes())
        elif file_format.lower() == "flac":
            # soundfile's FLAC / PCM_16 write on the native encoder (csrc/flac.cpp)
            from ainp.audio_io import write_flac
            write_flac(str(file_path), audio_data, int(sample_rate))
        else:
            import soundfile as sf
            sf.write(file_path, audio_data, sample_rate, format=file_format)
    except Exception as e:
        raise IOError(f"Error saving audio to {file_path}: {str(e)}")


# --- Gap Processing ----------------------------------------------------------


def create_gap_mask(audio_len_samples: int, gap_len_s: float,
                    sample_rate: int = DEFAULT_SAMPLE_RATE,
                    gap_start_s: Optional[float] = None) -> Tuple[np.ndarray, Tuple[int, int]]:
    """utils.py:93-144: 1 = signal, 0 = gap; random start in [0, S-g] inclusive."""
    gap_len_samples = int(gap_len_s * sample_rate)
    if gap_len_samples <= 0:
        return np.ones(audio_len_samples, dtype=np.float32), (0, 0)
    if gap_len_samples >= audio_len_samples:
        print(f"Warning: Gap length ({gap_len_s}s) >= audio length. Returning all zeros mask.")
        return np.zeros(audio_len_samples, dtype=np.float32), (0, audio_len_samples)
    max_start_sample = audio_len_samples - gap_len_samples
    if gap_start_s is None:
        gap_start_sample = np.random.randint(0, max_start_sample + 1)
    else:
        gap_start_sample = int(gap_start_s * sample_rate)
    gap_end_sample = gap_start_sample + gap_len_samples
    mask = np.ones(audio_len_samples, dtype=np.float32)
    mask[gap_start_sample:gap_end_sample] = 0.0
    return mask, (gap_start_sample, gap_end_sample)


def draw_gap_start(audio_len: int, gap_length: int) -> int:
    """The RNG draw of utils.py:179 (exclusive of audio_len - gap_length)."""
    return int(np.random.randint(0, audio_len - gap_length))


def insert_gap(audio_data: np.ndarray, gap_start_idx: int, gap_length: int) -> np.ndarray:
    """Zero [start, start+gap) by concatenation with float64 zeros (utils.py:180-183)."""
    silence = np.zeros(gap_length)
    return np.concatenate([audio_data[:gap_start_idx], silence,
                           audio_data[gap_start_idx + gap_length:]])


def add_random_gap(file_path: Union[str, Path], gap_len: float,
                   sample_rate: int = DEFAULT_SAMPLE_RATE,
                   mono: bool = True) -> Tuple[np.ndarray, Tuple[float, float]]:
    """utils.py:146-188: reload, random start in [0, S-g) (exclusive), float64
    result; ValueError when the gap is not shorter than the audio."""
    audio_data, sr = load_audio(file_path, sample_rate=sample_rate, mono=mono)
    gap_length = int(gap_len * sample_rate)
    audio_len = len(audio_data)
    if gap_length >= audio_len:
        raise ValueError(f"Gap length ({gap_length}s) exceeds audio length ({audio_len/sample_rate}s)")
    gap_start_idx = draw_gap_start(audio_len, gap_length)
    audio_new = insert_gap(audio_data, gap_start_idx, gap_length)
    return audio_new, (gap_start_idx / sample_rate, (gap_start_idx + gap_length) / sample_rate)


# --- STFT Processing -----------------------------------------------------------


def extract_spectrogram(audio_data, n_fft: int = 2048, hop_length: int = 512,
                        win_length: Optional[int] = None, window: str = "hann",
                        center: bool = True, power: float = 1.0):
    """utils.py:192-234: the complex STFT (librosa>=0.10 semantics) computed by
    ainp_stft on the GPU.  float32 input -> complex64, float64 -> complex128
    (as librosa).  numpy in -> numpy out; a torch cuda tensor stays on the GPU.
    `power` is validated and otherwise ignored, as in the reference (Q4)."""
    if power < 0:
        raise ValueError("Power must be non-negative")
    if win_length is None:
        win_length = n_fft
    import torch
    from ainp import ops
    if isinstance(audio_data, torch.Tensor):
        return ops.stft(audio_data, n_fft, hop_length, win_length, window, center)
    a = np.asarray(audio_data)
    if a.dtype not in (np.float32, np.float64):
        a = a.astype(np.float32 if a.dtype.itemsize <= 4 else np.float64)
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return ops.stft(t, n_fft, hop_length, win_length, window, center).cpu().numpy()


def db_to_amplitude(S_db, ref: float = 1.0):
    """librosa.db_to_amplitude: ref * 10**(0.05 * S_db) (host numpy, as the reference)."""
    return ref * np.power(10.0, 0.05 * np.asarray(S_db))


def spectrogram_to_audio(spectrogram, phase=None, phase_info: bool = False, n_fft=512,
                         n_iter=64, window="hann", hop_length=512, win_length=None,
                         center=True, random_state=None):
    """utils.py:279-333 on the GPU kernels (ainp_istft / ainp_stft / ainp_gl_update):
    a dB-scaled input (max < 0 and mean < 0) is converted back to amplitude;
    phase_info: the input is a complex spectrogram -> istft; phase given ->
    istft(S * exp(i phase)); otherwise Griffin-Lim (n_iter, momentum 0.99,
    random initial phases; random_state seeds them as in librosa).
    numpy in -> numpy out (as the reference); torch cuda tensors stay on the GPU."""
    import torch
    from ainp import ops
    as_numpy = not isinstance(spectrogram, torch.Tensor)
    S = spectrogram
    if as_numpy:
        S = np.asarray(S)
        if not np.iscomplexobj(S) and np.max(S) < 0 and np.mean(S) < 0:
            S = db_to_amplitude(S)
        S = torch.from_numpy(np.ascontiguousarray(S)).cuda()
    elif not S.is_complex() and bool((S.max() < 0) & (S.mean() < 0)):
        S = torch.from_numpy(db_to_amplitude(S.cpu().numpy())).to(S.device)
    kw = dict(n_fft=n_fft, hop_length=hop_length, win_length=win_length, window=window,
              center=center)
    if phase_info:
        if not S.is_complex():
            S = S.to(torch.complex64)
        y = ops.istft(S.contiguous(), **kw)
    elif phase is not None:
        ph = torch.as_tensor(np.asarray(phase) if as_numpy else phase).to(S.device, torch.float32)
        y = ops.istft(mag=S.to(torch.float32).contiguous(), phase=ph.contiguous(), **kw)
    else:
        y = ops.griffinlim(S.to(torch.float32).contiguous(), n_iter=n_iter,
                           hop_length=hop_length, win_length=win_length, n_fft=n_fft,
                           window=window, center=center, random_state=random_state)
    return y.cpu().numpy() if as_numpy else y


def extract_mel_spectrogram(*args, **kwargs):
    raise NotImplementedError("mel spectrograms are outside the hot path (DESIGN.md §1)")


def mel_spectrogram_to_audio(*args, **kwargs):
    raise NotImplementedError("mel spectrograms are outside the hot path (DESIGN.md §1)")


def visualize_spectrogram(*args, **kwargs):
    raise NotImplementedError("plotting is outside the hot path (DESIGN.md §1)")
