"""Drop-in for models/GAN/networks.py: same classes, constructors and
state_dict keys, forwards on the MI355X kernels (see ainp/gan.py)."""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from ainp.gan import (DecoderBlock, Discriminator, DiscriminatorBlock,  # noqa: E402,F401
                      EncoderBlock, PartialConv2d, PConvUNet, calculate_total_downsampling,
                      get_pad_size)
