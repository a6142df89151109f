#!/usr/bin/env python3
"""Per-step kernel breakdown: the bench's C2 (or C3 with --dtype bf16) train
step alone, `--steps` times after 3 warm-up steps, nothing else launched (no
roofline micro-benchmarks, eval or graph replay), so a rocprofv3 kernel-stats
table divided by (3 + steps) is the per-step cost of every kernel.

  rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/x -o run -- \
      python3 tools/step_prof.py --steps 10 [--dtype bf16]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--workload", choices=("cnnblstm", "gan"), default="cnnblstm")
    ap.add_argument("--clip-s", type=float, default=5.0)
    args = ap.parse_args()
    if args.workload == "gan":
        return gan(args)
    args.batch = args.batch or 32
    from ainp import ops
    from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
    from ainp.optim import Adam
    dev = torch.device("cuda", 0)
    CFG = bench.CFG
    S, n_fft, hop, win, T, g = 64000, 512, 192, 384, 334, 3200
    torch.manual_seed(0)
    model = StackedBLSTMCNN(config=dict(CFG, accel={"dtype": args.dtype})).to(dev).train()
    opt = Adam(model.parameters(), lr=1e-4)
    audio = torch.from_numpy(bench.synthetic_clips(args.batch, S, 0)).to(dev)
    rng = np.random.default_rng(1)
    starts = torch.from_numpy(rng.integers(0, S - g, size=(3 + args.steps, args.batch))).to(dev)
    t0 = None
    for i in range(3 + args.steps):
        if i == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        x, tgt, mask, _ = ops.stft_features(audio, starts[i], g, n_fft, hop, win, n_frames=T)
        opt.zero_grad()
        loss = l1_pow10_loss(model(x.unsqueeze(1)), mask, tgt)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    print(f"{args.dtype}: {1e3 * (time.perf_counter() - t0) / args.steps:.3f} ms/step "
          f"over {args.steps} steps; kernel tables / {3 + args.steps} = per step")


def gan(args):
    """The bench's GAN step (C4: 5 s / T=626; --clip-s 8: C5, T=1001)."""
    from ainp import ops
    from ainp import gan as G
    from ainp.gan_train import GanTrainer
    dev = torch.device("cuda", 0)
    B = args.batch or 8
    S = int(16000 * args.clip_s)
    g = 1600 if args.clip_s >= 8 else 3200
    T = 1 + S // 128
    torch.manual_seed(0)
    tr = GanTrainer(dict(bench.GAN_CFG, accel={"dtype": args.dtype}), G.PConvUNet().to(dev),
                    G.Discriminator().to(dev), G.VGGLoss(dev))
    audio = torch.from_numpy(bench.synthetic_clips(B, S, 5)).to(dev)
    rng = np.random.default_rng(2)
    starts = torch.from_numpy(rng.integers(0, S - g + 1, size=(3 + args.steps, B))).to(dev)
    t0 = None
    for i in range(3 + args.steps):
        if i == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        o, im, _, m = ops.stft_features(audio, starts[i], g, 512, 128, 512, n_frames=T,
                                        mode=ops.FEAT_GAN, outputs=(True, True, False, True))
        tr.step(o.unsqueeze(1), im.unsqueeze(1), m.unsqueeze(1))
    torch.cuda.synchronize()
    print(f"gan {args.dtype} T={T}: {1e3 * (time.perf_counter() - t0) / args.steps:.3f} ms/step "
          f"over {args.steps} steps; kernel tables / {3 + args.steps} = per step")


if __name__ == "__main__":
    main()
