"""Drop-in for add_gaps.py (add_gaps.py:15-38): insert a fixed zero gap
(start, duration in seconds) into one audio file and write it out."""
import sys

import numpy as np

from config import DEFAULT_GAP_DURATION, DEFAULT_GAP_START_TIME
from utils import insert_gap, load_audio, save_audio


def insert_gap_file(audio_path, output_path, gap_start, gap_duration, sample_rate=16000):
    """add_gaps.py:15-38 (named insert_gap there); the reference writes the
    gapped signal without normalisation (sf.write), so normalize=False."""
    y, _ = load_audio(audio_path, sample_rate)
    gap_start_idx = int(gap_start * sample_rate)
    gap_length = int(gap_duration * sample_rate)
    y_new = insert_gap(y, gap_start_idx, gap_length)
    save_audio(y_new, output_path, sample_rate, normalize=False,
               file_format="wav" if str(output_path).lower().endswith(".wav") else "flac")
    return y_new


if __name__ == "__main__":
    if len(sys.argv) < 3:
        print("usage: add_gaps.py IN OUT [gap_start_s] [gap_duration_s]")
        sys.exit(1)
    start = float(sys.argv[3]) if len(sys.argv) > 3 else DEFAULT_GAP_START_TIME
    dur = float(sys.argv[4]) if len(sys.argv) > 4 else DEFAULT_GAP_DURATION
    insert_gap_file(sys.argv[1], sys.argv[2], start, dur)
