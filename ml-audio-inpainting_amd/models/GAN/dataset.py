"""Drop-in for models/GAN/dataset.py: SpeechInpaintingDataset(cfg, dataset_type).

Same file discovery (rglob '*.flac', sorted; PCM '*.wav' accepted too:
dataset.py:52-55), same RNG call for the gap (utils.create_gap_mask, inclusive
randint: dataset.py:104-108) and the same __getitem__ dict (dataset.py:161-166):
  original_magnitude [1,F,T]  log1p(|STFT(a)|)          (power 1, normalize)
  impaired_magnitude [1,F,T]  log1p(|STFT(a * gap_mask)|)
  mask               [1,F,T]  1 valid, 0 on [s//hop, min(T, ceil(e/hop)))
  original_phase     [1,F,T]  angle(STFT(a))
computed by ONE fused launch (ainp_stft_features, GAN mode) on `device`.
For training, `raw(idx)` + `features(audio[B,S], starts[B])` produce a whole
batch in one launch (the reference runs 2 librosa STFTs per item in 4 CPU
workers).
"""
from __future__ import annotations

import math
import os
import sys
from pathlib import Path
from typing import Any, Dict

import numpy as np
import torch
from torch.utils.data import Dataset

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

import utils  # noqa: E402
from ainp import ops  # noqa: E402


class SpeechInpaintingDataset(Dataset):
    def __init__(self, cfg: Dict[str, Any], dataset_type: str = "train", device="cuda") -> None:
        self.cfg = cfg
        self.data_cfg = cfg["data"]
        self.spec_cfg = self.data_cfg["spectrogram"]
        self.train_cfg = cfg["training"]
        self.sample_rate = self.data_cfg["sample_rate"]
        self.max_len_s = self.data_cfg["max_len_s"]
        self.gap_len_s = self.data_cfg["gap_len_s"]
        self.max_samples = int(self.sample_rate * self.max_len_s)
        self.spec_normalize = self.spec_cfg["normalize"]
        self.device = device
        if self.spec_cfg.get("power", 1.0) != 1.0 or not self.spec_normalize:
            raise NotImplementedError("the fused GAN feature kernel implements power=1, "
                                      "normalize=True (the reference config)")
        if dataset_type == "train":
            key = "train_path"
        elif dataset_type == "valid":
            key = "valid_path"
        elif dataset_type == "test":
            key = "test_path"
        else:
            raise ValueError(f"Invalid dataset_type: {dataset_type}")
        self.root_path = Path(self.data_cfg["root_path"])
        self.dataset_dir = self.root_path / self.data_cfg[key]
        if not self.dataset_dir.exists():
            raise FileNotFoundError(f"Dataset directory not found: {self.dataset_dir}")
        self.file_paths = sorted(list(self.dataset_dir.rglob("*.flac"))
                                 + list(self.dataset_dir.rglob("*.wav")))
        if not self.file_paths:
            raise FileNotFoundError(f"No .flac files found in {self.dataset_dir}")
        print(f"Found {len(self.file_paths)} files in {self.dataset_dir}")

    def __len__(self) -> int:
        return len(self.file_paths)

    @property
    def n_frames(self):
        return 1 + self.max_samples // self.spec_cfg["hop_length"]

    def raw(self, idx):
        """Host stage: decode + the reference's gap draw -> (audio f32 [S], start)."""
        audio, sr = utils.load_audio(self.file_paths[idx], sample_rate=self.sample_rate,
                                     max_len=self.max_len_s)
        if sr != self.sample_rate:
            raise ValueError(f"Sample rate mismatch: expected {self.sample_rate}, got {sr}")
        if len(audio) != self.max_samples:
            raise ValueError(f"Audio length mismatch: expected {self.max_samples}, got {len(audio)}")
        _, (start, _) = utils.create_gap_mask(len(audio), self.gap_len_s, self.sample_rate)
        return audio, int(start)

    def features(self, audio, starts):
        """GPU stage: audio [B, S] f32, starts [B] -> the four [B, 1, F, T] tensors."""
        a = torch.as_tensor(audio, dtype=torch.float32).to(self.device)
        if a.dim() == 1:
            a = a.unsqueeze(0)
        st = torch.as_tensor(np.asarray(starts, dtype=np.int64)).to(self.device).reshape(-1)
        g = int(self.gap_len_s * self.sample_rate)
        sc = self.spec_cfg
        orig, imp, phase, mask = ops.stft_features(
            a.contiguous(), st, g, sc["n_fft"], sc["hop_length"], sc["win_length"],
            n_frames=self.n_frames, mode=ops.FEAT_GAN, sample_rate=self.sample_rate,
            window=sc.get("window", "hann"))
        return {"original_magnitude": orig.unsqueeze(1), "impaired_magnitude": imp.unsqueeze(1),
                "mask": mask.unsqueeze(1), "original_phase": phase.unsqueeze(1)}

    def __getitem__(self, idx: int) -> Dict[str, torch.Tensor]:
        audio, start = self.raw(idx)
        out = self.features(audio, [start])
        return {k: v[0] for k, v in out.items()}
