"""Diagnostic: full-config golden, print y/loss/grad errors for every parameter."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
g = np.load(os.path.join(ROOT, "tests/golden/cnnblstm_full.npz"), allow_pickle=False)
n_fft, hop, win, hidden, layers, N, T = [int(v) for v in g["config"]]
cfg = {"data": {"spectrogram": {"n_fft": n_fft}}, "model": {"in_channels": 1, "num_lstm_layers": layers,
       "lstm_hidden_dim": hidden, "enc_filters": [16, 32], "dec_filters": [16, 32]}}
torch.manual_seed(0)
model = StackedBLSTMCNN(config=cfg).cuda().train()
x = torch.from_numpy(g["x"]).cuda(); m = torch.from_numpy(g["mask"]).cuda(); t = torch.from_numpy(g["target"]).cuda()
y = model(x.unsqueeze(1)); loss = l1_pow10_loss(y, m, t); loss.backward()
rel = lambda a, b: float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))
print("y", rel(y.detach().cpu().numpy(), g["y"]), "loss", abs(loss.item() - g["loss"][0]) / g["loss"][0])
for k, p in model.named_parameters():
    flat = p.grad.detach().cpu().numpy().reshape(-1); step = max(1, flat.size // 2048)
    print(f"{k:35s} norm_rel={abs(float(p.grad.double().norm()) - g['gnorm/'+k][0]) / g['gnorm/'+k][0]:.2e} sample_rel={rel(flat[::step], g['gsample/'+k]):.2e}")
