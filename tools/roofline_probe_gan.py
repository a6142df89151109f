"""Launch only one of the GAN bench's roofline kernels a few times, on the
operands bench.py times: the sources captured from a G forward over the
bench's synthetic batch (bench.gan_roofline_operands; this probe uses the
first batch, the bench its last timed one -- same shapes, masks of the same
density).  The target of the rocprofv3 --pmc passes behind
profiles/traffic_conv_gen_{final,wide}_bf16[_c5].json.

  python tools/roofline_probe_gan.py <reps> <fp32|bf16> [clip_s (5 | 8)] [final|wide]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ainp import gan as G  # noqa: E402
from ainp import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
bf16 = len(sys.argv) > 2 and sys.argv[2] == "bf16"
clip_s = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
which = sys.argv[4] if len(sys.argv) > 4 else "final"
c5 = clip_s >= 8.0
B, hop, n_fft = 8, 128, 512
S = int(16000 * clip_s)
g = 1600 if c5 else 3200
T = 1 + S // hop
dev = "cuda"
torch.manual_seed(0)
gen = G.PConvUNet().to(dev).train()
G.set_compute_dtype(gen, "bf16" if bf16 else "fp32")
audio = torch.from_numpy(bench.synthetic_clips(B, S, 200000)).to(dev)
rng = np.random.default_rng(777)
starts = torch.from_numpy(rng.integers(0, S - g + 1, size=(1, B)).astype(np.int64)).to(dev)
o, im, ph, m = ops.stft_features(audio, starts[0], g, n_fft, hop, n_fft, n_frames=T,
                                 mode=ops.FEAT_GAN, outputs=(True, True, False, True))
fin, wide = bench.gan_roofline_operands(gen, im, m)
if which == "wide":
    launch, _, _, _ = bench.gan_roofline_launch(gen.decoder_blocks[3], wide, bf16, stats=True)
else:
    launch, _, _, _ = bench.gan_roofline_launch(gen.final_decoder_layer[0], fin, bf16)
for _ in range(reps):
    launch()
torch.cuda.synchronize()
print("done")
