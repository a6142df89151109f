"""Launch only the fused STFT/feature/mask kernel on the bench's C2 batch
(32 synthetic 4 s clips, T=334, n_fft 512 / hop 192 / win 384) a few times:
the target of the rocprofv3 --pmc passes that give profiles/traffic_stft.json.
argv: [launches] [mode: cnnblstm|gan]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import numpy as np
import torch
from ainp import ops
from ainp.synth import synthetic_clip
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mode = sys.argv[2] if len(sys.argv) > 2 else "cnnblstm"
dev = "cuda"
if mode == "cnnblstm":
    B, S, hop, win, g, T, m = 32, 64000, 192, 384, 3200, 334, ops.FEAT_CNNBLSTM
else:
    B, S, hop, win, g, T, m = 8, 80000, 128, 512, 3200, 626, ops.FEAT_GAN
audio = torch.from_numpy(np.stack([synthetic_clip(i, S) for i in range(B)])).to(dev)
rng = np.random.default_rng(3)
gs = torch.from_numpy(rng.integers(0, S - g, size=B).astype(np.int64)).to(dev)
for _ in range(n):
    ops.stft_features(audio, gs, g, 512, hop, win, n_frames=T, mode=m)
torch.cuda.synchronize()
grids = sys.argv[3].split(",") if len(sys.argv) > 3 else [""]
for gr in grids:    # AINP_STFT_GRID: persistent-grid size ("" = one tile per workgroup)
    if gr:
        os.environ["AINP_STFT_GRID"] = gr
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.stft_features(audio, gs, g, 512, hop, win, n_frames=T, mode=m)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    nb = (4880 if mode == "cnnblstm" else 4624) * B * T
    print(f"{mode} grid={gr or 'all'}: {us:.1f} us/launch, {nb / us / 1e3:.1f} GB/s")
    os.environ.pop("AINP_STFT_GRID", None)
