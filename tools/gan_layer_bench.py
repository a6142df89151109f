"""Per-layer timing of every conv_gen launch in the GAN step (G forward, VGG
loss, D forward) at the C4 shapes: HIP events around each call, 5 reps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch  # noqa: E402
from ainp import gan as G, ops  # noqa: E402

B, F, T = 8, 257, 626
dev = "cuda"
torch.manual_seed(0)
gen = G.PConvUNet().to(dev).train()
disc = G.Discriminator().to(dev).train()
vgg = G.VGGLoss(dev)
x = torch.rand(B, 1, F, T, device=dev) * 3
m = torch.ones(B, 1, F, T, device=dev)
m[:, :, :, 300:326] = 0

orig = ops.conv_gen
records = []


def timed(*a, **k):
    x0 = a[0][0]
    w = a[1]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = orig(*a, **k)
    e1.record()
    torch.cuda.synchronize()
    y = out[0]
    Cout, Cin, KH, KW = w.shape
    Ho, Wo = y.shape[-2:] if Cout > 1 else (y.shape[-2], y.shape[-1])
    flops = 2.0 * Cout * Cin * KH * KW * y.shape[0] * Ho * Wo
    records.append((tuple(x0.shape), tuple(w.shape), k.get("stride", 1), tuple(y.shape),
                    e0.elapsed_time(e1), flops))
    return out


ops.conv_gen = timed
for rep in range(3):
    records.clear()
    with torch.no_grad():
        g = gen(x, m)
        vgg(g, x)
        disc(x)
tot = 0.0
for xs, ws, s, ys, ms, fl in records:
    tot += ms
    print(f"{str(xs):22s} w{str(ws):20s} s{s} -> {str(ys):22s} {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF")
print(f"total conv_gen ms (G fwd + VGG + 1 D fwd): {tot:.2f}")
