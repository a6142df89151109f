"""Where does the bf16 C2 gradient error come from?  Runs the C2 batch
(cnnblstm_c2.npz) through variants of the bf16 configuration and prints, for
a few parameters, (norm rel err, sample rel err) against the reference's
fp32 gradients.  Usage: python tools/bf16_grad_diag.py <variant>
variants: fp32 | bf16 | bf16_staged_l0 | conv_bf16_only | gemm_bf16_only"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ainp import cnnblstm as C  # noqa: E402
from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss  # noqa: E402
from golden.gen_golden_r02 import c2_config, c2_inputs  # noqa: E402

var = sys.argv[1]
g = np.load(os.path.join(ROOT, "tests", "golden", "cnnblstm_c2.npz"), allow_pickle=False)
cfg = c2_config()
x, m, t, _ = c2_inputs()
if var != "fp32":
    cfg = dict(cfg, accel={"dtype": "bf16"})
if var == "bf16_staged_l0":
    C._l0_bf16_ok = lambda y: False
if var in ("conv_bf16_only", "gemm_bf16_only"):
    conv_b = var == "conv_bf16_only"
    oc, ob, op = C._ConvStackFn.apply, C._BLSTMFn.apply, C._ProjFn.apply
    C._ConvStackFn.apply = lambda x_, spec, tr, ntcf, comm, bf, box, dw, *p: oc(
        x_, spec, tr, ntcf, comm, conv_b, None, dw, *p)
    C._BLSTMFn.apply = lambda z, H, L, bf, sink, box, *p: ob(z, H, L, not conv_b, sink, None, *p)
    C._ProjFn.apply = lambda z, w, b, c, f, bf, d, sk: op(z, w, b, c, f, not conv_b, d, sk)
torch.manual_seed(0)
model = StackedBLSTMCNN(config=cfg).cuda().train()
X, M, Tg = torch.from_numpy(x).cuda(), torch.from_numpy(m).cuda(), torch.from_numpy(t).cuda()
y = model(X.unsqueeze(1))
loss = l1_pow10_loss(y, M, Tg)
loss.backward()


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


yf = y.detach().cpu().numpy().reshape(-1)
print(var, "y rel", round(rel(yf[::97], g["y_sample"]), 5), "loss rel",
      round(abs(loss.item() - g["loss"][0]) / g["loss"][0], 6))
for k, p in model.named_parameters():
    gr = p.grad.detach().cpu().double().numpy()
    gn = float(np.linalg.norm(gr))
    e_n = abs(gn - g["gnorm/" + k][0]) / g["gnorm/" + k][0]
    e_s = rel(gr.reshape(-1)[::max(1, gr.size // 4096)], g["gsample/" + k])
    if any(s in k for s in ("encoder.0.w", "encoder.6.w", "ih_l0", "hh_l0", "ih_l1", "projection.w",
                            "decoder.0.w")):
        print(f"  {k:32s} norm {e_n:.5f} sample {e_s:.5f}")
