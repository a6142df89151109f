"""Call sites of the GAN bf16 step's layout kernels (nchw_to_nhwc16,
im2col_nhwc16, im2col16, d_prep16): one C4-shape training step with ops._T
wrapped, each op call attributed to its innermost ainp/gan*.py frame.

usage: python tools/glue_sites.py [batch]
"""
import os
import sys
import traceback
from collections import Counter

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "ml-audio-inpainting_amd"))

WATCH = ("nchw_to_nhwc16", "im2col_nhwc16", "im2col16", "d_prep16", "maxpool2")


def main():
    from ainp import ops
    from ainp import gan as G
    from ainp.gan_train import GanTrainer
    import bench

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    S, hop, n_fft, g = 80000, 128, 512, 3200
    T = 1 + S // hop
    torch.manual_seed(0)
    gen, disc, vgg = G.PConvUNet().to(dev), G.Discriminator().to(dev), G.VGGLoss(dev)
    tr = GanTrainer(dict(bench.GAN_CFG, accel={"dtype": "bf16"}), gen, disc, vgg)
    audio = torch.from_numpy(bench.synthetic_clips(B, S, 200000)).to(dev)
    starts = torch.from_numpy(np.random.default_rng(7).integers(0, S - g + 1, size=B)).to(dev)

    counts = Counter()
    real = ops._T

    class Proxy:
        def __getattr__(self, name):
            fn = getattr(real, name)
            if name not in WATCH:
                return fn

            def wrapped(*a, **k):
                site = "?"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    if "/ainp/" in fr.filename and not fr.filename.endswith("ops.py"):
                        site = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                        break
                shape = tuple(a[0].shape) if torch.is_tensor(a[0]) else ()
                counts[(name, site, shape)] += 1
                return fn(*a, **k)
            return wrapped

    def step():
        o, im, _, m = ops.stft_features(audio, starts, g, n_fft, hop, n_fft, n_frames=T,
                                        mode=ops.FEAT_GAN, outputs=(True, True, False, True))
        tr.step(o.unsqueeze(1), im.unsqueeze(1), m.unsqueeze(1))

    step()
    torch.cuda.synchronize()
    ops._T = Proxy()
    step()
    torch.cuda.synchronize()
    ops._T = real
    for (name, site, shape), n in sorted(counts.items()):
        print(f"{n:3d}  {name:16s} {site:40s} {shape}")


if __name__ == "__main__":
    main()
