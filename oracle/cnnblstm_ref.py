"""torch-CPU restatement of the reference CNNBLSTM training step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used by tests/ as the
checker and by bench.py's cpu_baseline leg; never imported by the product.

Follows models/CNNBLSTM/model.py and models/CNNBLSTM/train.py:
  encoder      model.py:34-44   3 x [conv3x3 p1 + BatchNorm2d(train) + ReLU]
  bridge       model.py:73-74   permute(0,3,1,2).reshape(N, T, C*F)
  lstm         model.py:46-47,77 nn.LSTM(C*F, H, L, batch_first, bidirectional)
  projection   model.py:50,80-83 Linear(2H, 16F) -> view(N,T,16,F).permute(0,2,3,1)
  decoder      model.py:53-61,87-88 conv+BN+ReLU, conv+BN+ReLU, conv, squeeze(1)
  loss         train.py:70,104  L1Loss(sum)((10**y)*m, |target|*m)
  optimizer    train.py:72,108  torch.optim.Adam(lr)
The parameters live in a plain dict keyed by the reference's state_dict names,
so the restatement is independent of the product's nn.Module.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def init_params(cfg: dict, seed: int = 0) -> dict:
    """Same parameter tensors torch's default init gives the reference module
    (construction order of model.py:34-61) for torch.manual_seed(seed)."""
    import torch.nn as nn
    torch.manual_seed(seed)
    m = cfg["model"]
    Fb = cfg["data"]["spectrogram"]["n_fft"] // 2 + 1
    cin, enc, dec, H, L = m["in_channels"], m["enc_filters"], m["dec_filters"], \
        m["lstm_hidden_dim"], m["num_lstm_layers"]
    mods = [
        ("encoder.0", nn.Conv2d(cin, enc[0], 3, padding=1)), ("encoder.1", nn.BatchNorm2d(enc[0])),
        ("encoder.3", nn.Conv2d(enc[0], enc[1], 3, padding=1)), ("encoder.4", nn.BatchNorm2d(enc[1])),
        ("encoder.6", nn.Conv2d(enc[1], H // 2, 3, padding=1)), ("encoder.7", nn.BatchNorm2d(H // 2)),
        ("lstm", nn.LSTM(Fb * H // 2, H, num_layers=L, batch_first=True, bidirectional=True)),
        ("projection", nn.Linear(2 * H, Fb * dec[0])),
        ("decoder.0", nn.Conv2d(dec[0], dec[1], 3, padding=1)), ("decoder.1", nn.BatchNorm2d(dec[1])),
        ("decoder.3", nn.Conv2d(dec[1], dec[0], 3, padding=1)), ("decoder.4", nn.BatchNorm2d(dec[0])),
        ("decoder.6", nn.Conv2d(dec[0], cin, 3, padding=1)),
    ]
    out = {}
    for name, mod in mods:
        for k, v in mod.state_dict().items():
            out[f"{name}.{k}"] = v.detach().clone()
    return out


def _conv_bn_relu(x, p, conv, bn, training, relu_masks=None):
    y = F.conv2d(x, p[conv + ".weight"], p[conv + ".bias"], padding=1)
    y = F.batch_norm(y, p[bn + ".running_mean"], p[bn + ".running_var"], p[bn + ".weight"],
                     p[bn + ".bias"], training=training, momentum=0.1, eps=1e-5)
    if training:
        p[bn + ".num_batches_tracked"] += 1
    if relu_masks is not None and bn in relu_masks:
        # branch-matched ReLU: the caller fixes which side of 0 each element is
        # on (the forward value differs from relu(y) only where y ~ 0)
        return y * relu_masks[bn].to(y.dtype)
    return F.relu(y)


def forward(p: dict, x: torch.Tensor, H: int, L: int, training: bool = True,
            relu_masks: dict | None = None) -> torch.Tensor:
    """x [N, 1, F, T] -> [N, F, T] (model.py:63-90).

    relu_masks (optional, {bn_name: bool tensor}) fixes the ReLU branch after
    each BatchNorm.  relu'(0) is a discontinuity: a 1e-7 difference in a
    BatchNorm output that sits at ~0 flips one element's gradient between
    g and 0, so two correct fp32 implementations can disagree by 1e-3 on every
    gradient upstream of the flip.  Evaluating the fp64 oracle on the branch
    the kernels took removes that and leaves the arithmetic error."""
    N, _, Fb, T = x.shape
    z = _conv_bn_relu(x, p, "encoder.0", "encoder.1", training, relu_masks)
    z = _conv_bn_relu(z, p, "encoder.3", "encoder.4", training, relu_masks)
    z = _conv_bn_relu(z, p, "encoder.6", "encoder.7", training, relu_masks)
    z = z.permute(0, 3, 1, 2).reshape(N, T, -1)
    flat = []
    for l in range(L):
        for sfx in ("", "_reverse"):
            flat += [p[f"lstm.weight_ih_l{l}{sfx}"], p[f"lstm.weight_hh_l{l}{sfx}"],
                     p[f"lstm.bias_ih_l{l}{sfx}"], p[f"lstm.bias_hh_l{l}{sfx}"]]
    h0 = torch.zeros(2 * L, N, H, dtype=x.dtype)
    z, _, _ = torch._VF.lstm(z, (h0, h0), flat, True, L, 0.0, training, True, True)
    z = F.linear(z, p["projection.weight"], p["projection.bias"])
    z = z.view(N, T, 16, Fb).permute(0, 2, 3, 1)
    z = _conv_bn_relu(z, p, "decoder.0", "decoder.1", training, relu_masks)
    z = _conv_bn_relu(z, p, "decoder.3", "decoder.4", training, relu_masks)
    z = F.conv2d(z, p["decoder.6.weight"], p["decoder.6.bias"], padding=1)
    return z.squeeze(1)


def loss_fn(y, mask, target):
    """train.py:70,104."""
    return torch.nn.L1Loss(reduction="sum")((10 ** y) * mask, torch.abs(target) * mask)


TRAINABLE_SUFFIXES = (".weight", ".bias", "weight_ih_l", "weight_hh_l", "bias_ih_l", "bias_hh_l")


def trainable_keys(p: dict):
    return [k for k in p if not (k.endswith("running_mean") or k.endswith("running_var")
                                 or k.endswith("num_batches_tracked"))]


class Trainer:
    """One reference training step per call: zero_grad, forward, loss, backward,
    Adam step (train.py:96-108)."""

    def __init__(self, params: dict, H: int, L: int, lr: float = 1e-4, frozen=()):
        """frozen: parameter names left out of Adam (they still get .grad),
        as tests/golden/gen_golden_r03.py does for the BN-fed conv biases."""
        self.p = params
        self.H, self.L = H, L
        self.keys = trainable_keys(params)
        for k in self.keys:
            self.p[k].requires_grad_(True)
        self.opt = torch.optim.Adam([self.p[k] for k in self.keys if k not in frozen], lr=lr)

    def step(self, x, mask, target):
        self.opt.zero_grad()
        y = forward(self.p, x.unsqueeze(1), self.H, self.L, training=True)
        loss = loss_fn(y, mask, target)
        loss.backward()
        self.opt.step()
        return y.detach(), loss.detach()
