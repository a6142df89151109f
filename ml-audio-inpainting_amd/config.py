"""Drop-in for the reference's config.py constants (config.py:27-36).

The reference's machine-specific Windows dataset paths and its import-time
`os.makedirs(OUTPUT_DIR)` side effect are deliberately not reproduced;
dataset roots come from the YAML configs (or AINP_LIBRISPEECH_ROOT).
"""
import os
from pathlib import Path

PROJECT_ROOT = Path(os.path.dirname(os.path.abspath(__file__)))
LIBRISPEECH_ROOT = Path(os.environ.get("AINP_LIBRISPEECH_ROOT", "/LibriSpeech/train-clean-100"))
LIBRISPEECH_ROOT_PROCESSED = Path(os.environ.get("AINP_LIBRISPEECH_ROOT_PROCESSED",
                                                 "/LibriSpeech_PROCESSED/train-clean-100"))
OUTPUT_DIR = PROJECT_ROOT / "output"

DEFAULT_SAMPLE_RATE = 16000       # 16 kHz
DEFAULT_N_FFT = 512               # FFT points
DEFAULT_HANN_WINDOW_SIZE = 384    # 24 ms at 16 kHz
DEFAULT_HANN_HOP_LENGTH = 192     # 12 ms

DEFAULT_GAP_START_TIME = 2.0
DEFAULT_GAP_DURATION = 0.5

SUPPORTED_FORMATS = [".flac", ".wav", ".mp3"]
