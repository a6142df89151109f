"""Drop-in for models/GAN/loss.py: VGGLoss(device) -> (perceptual, style).

VGG19_Weights.DEFAULT cannot be downloaded offline; pass weights= (a
torchvision vgg19().features state_dict or a path to one) to use them."""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from ainp.gan import VGGLoss  # noqa: E402,F401
