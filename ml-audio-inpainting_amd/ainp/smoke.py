"""Small end-to-end CNNBLSTM training-step check used by __graft_entry__.smoke().

Loads the golden fixture produced from the reference model
(tests/golden/cnnblstm_small.npz), runs two training steps (forward, L1 loss,
backward, Adam) through the HIP path on cuda:0 and compares output, loss,
every gradient and the updated parameters against it.
"""
from __future__ import annotations

import numpy as np
import torch

from .cnnblstm import StackedBLSTMCNN, l1_pow10_loss
from .optim import Adam

# Conv biases feeding a BatchNorm have an analytically zero gradient; their fp32
# value is rounding noise in both implementations -> absolute check.
BN_FED_BIASES = ("encoder.0.bias", "encoder.3.bias", "encoder.6.bias",
                 "decoder.0.bias", "decoder.3.bias")
# the BatchNorm each of those biases feeds (model.py:34-61): its running_mean
# carries momentum x the bias's Adam step
BN_OF_BIAS = {"encoder.0.bias": "encoder.1", "encoder.3.bias": "encoder.4",
              "encoder.6.bias": "encoder.7", "decoder.0.bias": "decoder.1",
              "decoder.3.bias": "decoder.4"}


def small_config(cfgv):
    n_fft, hop, win, hidden, layers, N, T = [int(v) for v in cfgv]
    return {"data": {"spectrogram": {"n_fft": n_fft, "hop_length": hop, "win_length": win}},
            "model": {"in_channels": 1, "num_lstm_layers": layers, "lstm_hidden_dim": hidden,
                      "enc_filters": [16, 32], "dec_filters": [16, 32]}}


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def run_training_steps(g, device="cuda", steps=2):
    model = StackedBLSTMCNN(config=small_config(g["config"])).to(device)
    sd = {k[len("init/"):]: torch.from_numpy(np.array(g[k])) for k in g.files
          if k.startswith("init/")}
    model.load_state_dict(sd)
    model.train()
    opt = Adam(model.parameters(), lr=1e-4)
    x = torch.from_numpy(g["x"]).to(device)
    m = torch.from_numpy(g["mask"]).to(device)
    t = torch.from_numpy(g["target"]).to(device)
    out = {}
    for s in range(steps):
        opt.zero_grad()
        y = model(x.unsqueeze(1))
        loss = l1_pow10_loss(y, m, t)
        loss.backward()
        if s == 0:
            out["y"] = y.detach().cpu().numpy()
            out["loss"] = float(loss.item())
            out["grads"] = {k: p.grad.detach().cpu().numpy() for k, p in model.named_parameters()}
        else:
            out["loss2"] = float(loss.item())
        opt.step()
    out["final"] = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    return out


def check_against_golden(g, out, tol=1e-4):
    errs = {}
    errs["y"] = rel(out["y"], g["y"])
    errs["loss"] = abs(out["loss"] - float(g["loss"][0])) / abs(float(g["loss"][0]))
    errs["loss2"] = abs(out["loss2"] - float(g["loss2"][0])) / abs(float(g["loss2"][0]))
    for k, v in out["grads"].items():
        ref = g["grad/" + k]
        if k in BN_FED_BIASES:
            scale = max(np.abs(g["grad/" + k.replace("bias", "weight")]).max(), 1e-12)
            errs["grad/" + k] = float(np.abs(v - ref).max() / scale)
        else:
            errs["grad/" + k] = rel(v, ref)
    for k, v in out["final"].items():
        ref = g["final/" + k]
        if k.endswith("num_batches_tracked"):
            errs["final/" + k] = float(abs(int(v) - int(ref)))
            continue
        errs["final/" + k] = rel(v, ref)
    bad = {k: e for k, e in errs.items() if not e <= tol}
    # BN-fed conv biases: Adam moves them by ~lr * sign(rounding noise) per
    # step (the noise's sign is implementation-specific), so allow 2*lr*steps
    # absolutely; a following BatchNorm's running_mean holds the step-1 update
    # of that bias (a conv bias shifts its BN input mean 1:1): momentum*2*lr
    lr, steps, momentum = 1e-4, 2, 0.1
    for k in BN_FED_BIASES:
        d = float(np.abs(out["final"][k] - g["final/" + k]).max())
        errs["final/" + k] = d
        if d <= 2 * lr * steps + 1e-7:
            bad.pop("final/" + k, None)
        else:
            bad["final/" + k] = d
    for bias, bn in BN_OF_BIAS.items():
        k = f"final/{bn}.running_mean"
        if k in bad:
            ref = np.asarray(g[k], np.float64)
            d = float(np.abs(out["final"][k[len("final/"):]] - ref).max())
            if d <= momentum * 2 * lr + tol * float(np.abs(ref).max()):
                bad.pop(k)
    return errs, bad


def run_smoke(npz_path, device="cuda"):
    g = np.load(npz_path, allow_pickle=False)
    out = run_training_steps(g, device)
    errs, bad = check_against_golden(g, out)
    if bad:
        raise AssertionError(f"HIP training step disagrees with the reference: {bad}")
    return errs
