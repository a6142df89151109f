"""Drop-in for models/CNNBLSTM/dataset.py: LibriSpeechDataset.

Same constructor (YAML path, 'train'|'valid'|'test'), same file walk
(first n_files FLACs of os.walk, then sorted: dataset.py:59-69), same
__getitem__ outputs (dataset.py:74-121):
  spectrogram_gaps [G, F, T] f32      log10(|STFT(gapped)| + 1e-9)
  gap_ints         [G, 2]    f32      (start, end) in seconds
  gap_masks        [G, F, T] f32      1 on the gap frames (float64 rule, Q3)
  targets          [G, F, T] complex64 STFT of the clean clip
with G = gaps_per_audio and T = ceil(sr*max_len_s/hop).  The file is
decoded once (the reference decodes it 2*G times with identical results),
the G gap starts are drawn with the reference's own np.random.randint calls
(utils.py:179, one per gap, same order), and all G examples come out of ONE
fused GPU launch (ainp_stft_features).  Tensors are returned on `device`.
"""
from __future__ import annotations

import math
import os
import sys
from pathlib import Path

import numpy as np
import torch
import yaml
from torch.utils.data import Dataset

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

import utils  # noqa: E402
from ainp import ops  # noqa: E402


def load_config(config_path):
    with open(config_path, "r") as f:
        return yaml.safe_load(f)


class LibriSpeechDataset(Dataset):
    def __init__(self, config_path, dataset_type="train", device="cuda", config=None):
        full_cfg = config if config is not None else load_config(config_path)
        data_cfg = full_cfg["data"]
        self.root_dir = data_cfg["root_path"]
        self.n_fft = data_cfg["spectrogram"]["n_fft"]
        self.hop_len = data_cfg["spectrogram"]["hop_length"]
        self.win_len = data_cfg["spectrogram"]["win_length"]
        self.window = data_cfg["spectrogram"].get("window", "hann")
        self.sr = data_cfg["sample_rate"]
        self.max_len_s = data_cfg["max_len_s"]
        self.gap_len_s = data_cfg["gap_len_s"]
        self.max_files = data_cfg["n_files"]
        self.gaps_per_audio = data_cfg["gaps_per_audio"]
        self.device = device

        if dataset_type == "train":
            data_path_key = "train_path"
        elif dataset_type == "valid":
            data_path_key = "valid_path"
        elif dataset_type == "test":
            data_path_key = "test_path"
        else:
            raise ValueError(f"Invalid dataset_type: {dataset_type}")

        self.root_path = Path(data_cfg["root_path"])
        self.dataset_dir = self.root_path / data_cfg[data_path_key]
        if not os.path.exists(self.dataset_dir):
            raise ValueError(f"Path {self.dataset_dir} does not exist")

        counter = 0
        self.file_paths = []
        for subdir, _, files in os.walk(self.dataset_dir):
            for file in files:
                # LibriSpeech ships FLAC; PCM WAV trees are accepted too
                if file.endswith((".flac", ".wav")) and counter < self.max_files:
                    self.file_paths.append(os.path.join(subdir, file))
                    counter += 1
        self.file_paths.sort()

    def __len__(self):
        return len(self.file_paths)

    @property
    def n_frames(self):
        return math.ceil(self.sr * self.max_len_s / self.hop_len)

    def draw_gaps(self, audio_len):
        """G gap starts, the reference's RNG calls (utils.py:171-179)."""
        g = int(self.gap_len_s * self.sr)
        if g >= audio_len:
            raise ValueError(f"Gap length ({g}s) exceeds audio length ({audio_len/self.sr}s)")
        return np.array([utils.draw_gap_start(audio_len, g) for _ in range(self.gaps_per_audio)],
                        dtype=np.int64)

    def features(self, audio, starts):
        """GPU stage: audio [S] f32 (numpy or tensor), starts [G] -> the 4 outputs."""
        g = int(self.gap_len_s * self.sr)
        a = torch.as_tensor(audio, dtype=torch.float32).to(self.device).reshape(1, -1)
        st = torch.as_tensor(starts, dtype=torch.int64).to(self.device)
        clip = torch.zeros(st.numel(), dtype=torch.int32, device=self.device)
        lg, tgt, mask, _ = ops.stft_features(a, st, g, self.n_fft, self.hop_len, self.win_len,
                                             n_frames=self.n_frames, sample_rate=self.sr,
                                             clip_index=clip, window=self.window)
        # (start/sr, (start+g)/sr) as Python floats -> float32 (utils.py:186, dataset.py:113)
        st_host = np.asarray(starts, dtype=np.int64)
        gap_ints = torch.tensor([[int(k) / self.sr, (int(k) + g) / self.sr] for k in st_host],
                                dtype=torch.float32).to(self.device)
        return lg, gap_ints, mask, tgt

    def __getitem__(self, idx):
        file_path = self.file_paths[idx]
        audio_data, _ = utils.load_audio(file_path)   # dataset.py:95 (default max_len=5)
        starts = self.draw_gaps(len(audio_data))
        return self.features(audio_data, starts)
