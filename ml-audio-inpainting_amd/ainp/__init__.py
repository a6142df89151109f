"""ainp -- MI355X-native spectrogram-inpainting training path.

Host layer over libainp.so (include/ainp.h).  Importing this package loads the
HIP library and binds every C-ABI symbol; there is no CPU fallback.
"""
from . import _lib  # noqa: F401  (fails loudly if libainp.so is missing)
from . import ops  # noqa: F401

__all__ = ["ops"]
