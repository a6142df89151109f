"""Host issue rate of the CNNBLSTM train step: wall time of the step loop
before the final synchronize (host side) vs after it (GPU side), per step.
A host time close to the GPU time means the host issue is the bound.

  python tools/host_rate.py [fp32|bf16] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ainp import ops  # noqa: E402
from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss  # noqa: E402
from ainp.optim import Adam  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda", 0)
S, n_fft, hop, win, T, g, B = 64000, 512, 192, 384, 334, 3200, 32
torch.manual_seed(0)
model = StackedBLSTMCNN(config=dict(bench.CFG, accel={"dtype": dt})).to(dev).train()
opt = Adam(model.parameters(), lr=1e-4)
audio = torch.from_numpy(bench.synthetic_clips(B, S, 0)).to(dev)
starts = torch.from_numpy(np.random.default_rng(1).integers(0, S - g, size=(5 + steps, B))).to(dev)


def step(i):
    x, tgt, mask, _ = ops.stft_features(audio, starts[i], g, n_fft, hop, win, n_frames=T)
    opt.zero_grad()
    loss = l1_pow10_loss(model(x.unsqueeze(1)), mask, tgt)
    loss.backward()
    opt.step()


for i in range(5):
    step(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(5, 5 + steps):
    step(i)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"{dt}: host issue {1e3 * (t1 - t0) / steps:.3f} ms/step, GPU {1e3 * (t2 - t0) / steps:.3f} "
      f"ms/step over {steps} steps", flush=True)
