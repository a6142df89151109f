"""A/B of the Cout=1 conv (ainp_conv_gen_fwd, Cout == 1) on the GAN C4
shapes: the generator's last PartialConv2d (64 -> 1, 3x3, mask plane, crop to
the input size) and the discriminator's logit conv (512 -> 1, 4x4).  Run once
with AINP_COUT1_TILE=0 (per-pixel kernel) and once without (LDS-tiled kernel);
prints ms per launch pair and the error against torch's fp32 conv.
Usage: python tools/cout1_ab.py [label]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "ml-audio-inpainting_amd"))
from ainp import ops  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("AINP_COUT1_TILE", "1")
g = torch.Generator().manual_seed(3)
cases = [("G final 64->1 3x3", 8, 64, 384, 640, 3, True, (257, 626)),
         ("D logit 512->1 4x4", 8, 512, 31, 77, 4, False, None)]
for name, N, C, H, W, k, masked, crop in cases:
    x = torch.randn(N, C, H, W, generator=g).cuda()
    m = (torch.rand(N, H, W, generator=g) > 0.2).float().cuda() if masked else None
    w = (torch.randn(1, C, k, k, generator=g) * 0.05).cuda()
    b = torch.randn(1, generator=g).cuda()
    y, _ = ops.conv_gen((x, m), w, pad=1, bias=b, crop=crop)
    xin = x * m[:, None] if masked else x
    yr = F.conv2d(xin, w, b, padding=1)[:, 0]
    if crop is not None:
        yr = yr[:, :crop[0], :crop[1]]
    else:
        y = y[:, 0]
    err = ((y - yr).norm() / yr.norm()).item()
    for _ in range(5):
        ops.conv_gen((x, m), w, pad=1, bias=b, crop=crop)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 50
    e0.record()
    for _ in range(it):
        ops.conv_gen((x, m), w, pad=1, bias=b, crop=crop)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    gb = x.numel() * 4 / 1e9
    print(f"[{label}] {name}: {ms:.4f} ms  ({gb / ms:.2f} TB/s over the input)  rel err {err:.2e}",
          flush=True)
