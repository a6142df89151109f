"""Is a training step host-bound?  Runs bench.py's step function for K steps
and compares the host's enqueue time per step (perf_counter at each step's
return, no synchronisation) with the GPU's time per step (events recorded at
the same points).  Host ms/step >= GPU ms/step: the GPU waits for Python.

usage: python tools/host_bound.py [cnnblstm|gan] [fp32|bf16] [steps]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))


def main():
    import bench
    from ainp import ops
    work = sys.argv[1] if len(sys.argv) > 1 else "cnnblstm"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if work == "cnnblstm":
        from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
        from ainp.optim import Adam
        sp = bench.CFG["data"]["spectrogram"]
        sr = bench.CFG["data"]["sample_rate"]
        B, S = 32, int(sr * bench.CFG["data"]["max_len_s"])
        n_fft, hop, win = sp["n_fft"], sp["hop_length"], sp["win_length"]
        g, T = int(bench.CFG["data"]["gap_len_s"] * sr), -(-S // sp["hop_length"])
        cfg = dict(bench.CFG, accel={"dtype": dtype})
        torch.manual_seed(0)
        model = StackedBLSTMCNN(config=cfg).to(dev).train()
        opt = Adam(model.parameters(), lr=1e-3)
        audio = torch.from_numpy(bench.synthetic_clips(B, S, 0)).to(dev)
        starts = torch.from_numpy(np.random.default_rng(1).integers(0, S - g, size=(K + 5, B))
                                  .astype(np.int64)).to(dev)

        def step(i):
            x, tgt, mask, _ = ops.stft_features(audio, starts[i], g, n_fft, hop, win, n_frames=T)
            opt.zero_grad()
            y = model(x.unsqueeze(1))
            loss = l1_pow10_loss(y, mask, tgt)
            loss.backward()
            opt.step()
    else:
        from ainp import gan as G
        from ainp.gan_train import GanTrainer
        B, S, g, n_fft, hop = 8, 80000, 3200, 512, 128
        T = 1 + S // hop
        torch.manual_seed(0)
        tr = GanTrainer(dict(bench.GAN_CFG, accel={"dtype": dtype}), G.PConvUNet().to(dev),
                        G.Discriminator().to(dev), G.VGGLoss(dev))
        audio = torch.from_numpy(bench.synthetic_clips(B, S, 200000)).to(dev)
        starts = torch.from_numpy(np.random.default_rng(7).integers(0, S - g + 1, size=(K + 5, B))
                                  ).to(dev)

        def step(i):
            o, im, _, m = ops.stft_features(audio, starts[i], g, n_fft, hop, n_fft, n_frames=T,
                                            mode=ops.FEAT_GAN, outputs=(True, True, False, True))
            tr.step(o.unsqueeze(1), im.unsqueeze(1), m.unsqueeze(1))

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    host = [0.0] * (K + 1)
    host[0] = time.perf_counter()
    ev[0].record()
    for i in range(K):
        step(5 + i % 5)
        ev[i + 1].record()
        host[i + 1] = time.perf_counter()
    torch.cuda.synchronize()
    gpu = [ev[i].elapsed_time(ev[i + 1]) for i in range(K)]
    hst = [(host[i + 1] - host[i]) * 1e3 for i in range(K)]
    print(f"{work} {dtype}: host enqueue {np.median(hst):.3f} ms/step (median), "
          f"GPU {np.median(gpu):.3f} ms/step; host total {sum(hst):.1f} ms vs GPU {sum(gpu):.1f} ms",
          flush=True)


if __name__ == "__main__":
    main()
