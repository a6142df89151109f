"""Drop-in for models/CNNBLSTM/model.py: StackedBLSTMCNN on the MI355X kernels
(implementation: ainp/cnnblstm.py)."""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from ainp.cnnblstm import StackedBLSTMCNN, load_config  # noqa: E402,F401

__all__ = ["StackedBLSTMCNN", "load_config"]
