"""Diagnose the VGG19 input gradient (ainp.gan._VGGLossFn) against the
oracle restatement under torch autograd: perceptual-only and style-only,
against fp64 and fp32 CPU references (the fp32-vs-fp64 distance is the
conditioning floor of the sign() terms)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ainp import gan as G  # noqa: E402
from oracle import gan_ref as R  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


g = torch.Generator().manual_seed(9)
gen = torch.tanh(torch.randn(2, 1, 129, 100, generator=g))
tgt = torch.rand(2, 1, 129, 100, generator=g) * 3
pv = R.vgg19_init(0)
v = G.VGGLoss("cuda")
v.vgg_layers.load_state_dict({k: t for k, t in pv.items()}, strict=False)
for lp, ls in ((4.0, 0.0), (0.0, 500.0), (4.0, 500.0)):
    gg = gen.cuda().requires_grad_(True)
    perc, style = v(gg, tgt.cuda())
    (lp * perc + ls * style).backward()
    res = {}
    for dt in (torch.float64, torch.float32):
        p = {k: t.to(dt) for k, t in pv.items()}
        gr = gen.to(dt).requires_grad_(True)
        rp, rs = R.vgg_losses(p, gr, tgt.to(dt))
        (lp * rp + ls * rs).backward()
        res[dt] = gr.grad
    print(f"lp={lp} ls={ls}: ours vs fp64 {rel(gg.grad, res[torch.float64]):.3e}  "
          f"ours vs fp32 {rel(gg.grad, res[torch.float32]):.3e}  "
          f"fp32 vs fp64 {rel(res[torch.float32], res[torch.float64]):.3e}", flush=True)
