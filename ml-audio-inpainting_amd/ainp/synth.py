"""Synthetic LibriSpeech-shaped clips for benchmarks and tests.

There is no network and no FLAC decoder in this image, so the benchmark and
tests use seeded synthetic 16 kHz mono clips of the reference dataset's shape.
"""
from __future__ import annotations

import numpy as np


def synthetic_clip(seed: int, n_samples: int, sr: int = 16000) -> np.ndarray:
    """LibriSpeech-shaped synthetic clip: voiced harmonic stack
    (f0 ~ U[90,260] Hz, 20 harmonics 1/k, slow AM) + 0.01 N(0,1), peak 0.5."""
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples) / sr
    f0 = rng.uniform(90, 260)
    x = np.zeros(n_samples)
    for k in range(1, 21):
        if k * f0 >= sr / 2:
            break
        x += np.sin(2 * np.pi * k * f0 * t + rng.uniform(0, 2 * np.pi)) / k
    am = 0.5 * (1 + np.sin(2 * np.pi * rng.uniform(2, 6) * t + rng.uniform(0, 2 * np.pi)))
    x = x * am + 0.01 * rng.standard_normal(n_samples)
    x = 0.5 * x / np.max(np.abs(x))
    return x.astype(np.float32)
