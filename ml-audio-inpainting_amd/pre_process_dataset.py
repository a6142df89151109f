"""Drop-in for pre_process_dataset.py (:20-43): walk a LibriSpeech tree,
insert one random 0.1 s gap per file (utils.add_random_gap) and write the
peak-normalised result into a mirrored tree."""
import os
import sys
from pathlib import Path

import utils
from config import LIBRISPEECH_ROOT, LIBRISPEECH_ROOT_PROCESSED, SUPPORTED_FORMATS


def process(src_root=LIBRISPEECH_ROOT, dst_root=LIBRISPEECH_ROOT_PROCESSED, gap_s=0.1):
    n = 0
    for root, subdirs, files in os.walk(src_root, topdown=True):
        rel = os.path.relpath(root, src_root)
        dest_path = os.path.join(dst_root, rel)
        os.makedirs(dest_path, exist_ok=True)
        if len(subdirs) == 0:
            for f in files:
                audio_path = Path(root) / Path(f)
                if audio_path.suffix in SUPPORTED_FORMATS:
                    audio_new, _ = utils.add_random_gap(audio_path, gap_s)
                    out = Path(dest_path) / Path(f)
                    utils.save_audio(audio_new, out,
                                     file_format="wav" if out.suffix == ".wav" else "flac")
                    n += 1
    return n


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else LIBRISPEECH_ROOT
    dst = sys.argv[2] if len(sys.argv) > 2 else LIBRISPEECH_ROOT_PROCESSED
    print(f"processed {process(src, dst)} files")
