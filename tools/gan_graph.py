#!/usr/bin/env python3
"""GAN step (bench C4 / C5 workload) eager vs captured in one HIP graph:
features + G forward + D step (fwd x2, bwd, capturable Adam) + G-step losses
(D forward, VGG) replayed per step after a D2D copy of the gap starts.
Prints eager and graph ms/step and checks that one replayed step equals one
eager step from the same state (d_loss, D weights).

  python3 tools/gan_graph.py [--dtype bf16] [--clip-s 5] [--steps 20]
"""
import argparse
import copy
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
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="bf16")
    ap.add_argument("--clip-s", type=float, default=5.0)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    from ainp import ops
    from ainp import gan as G
    from ainp.gan_train import GanTrainer
    dev = torch.device("cuda", 0)
    B = 8
    S = int(16000 * args.clip_s)
    g = 1600 if args.clip_s >= 8 else 3200
    T = 1 + S // 128
    torch.manual_seed(0)
    cfg = dict(bench.GAN_CFG, accel={"dtype": args.dtype, "capturable": True})
    tr = GanTrainer(cfg, G.PConvUNet().to(dev), G.Discriminator().to(dev), G.VGGLoss(dev))
    audio = torch.from_numpy(bench.synthetic_clips(B, S, 5)).to(dev)
    rng = np.random.default_rng(2)
    n = 8 + args.steps
    starts = torch.from_numpy(rng.integers(0, S - g + 1, size=(n, B))).to(dev)
    gstart = starts[0].clone()
    out_static = {}

    def body():
        o, im, _, m = ops.stft_features(audio, gstart, g, 512, 128, 512, n_frames=T,
                                        mode=ops.FEAT_GAN, outputs=(True, True, False, True))
        out = tr.step(o.unsqueeze(1), im.unsqueeze(1), m.unsqueeze(1))
        for k, v in out.items():
            if k not in out_static:
                out_static[k] = torch.empty_like(v)
            out_static[k].copy_(v)

    # eager timing
    for i in range(3):
        gstart.copy_(starts[i])
        body()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        gstart.copy_(starts[3 + i])
        body()
    torch.cuda.synchronize()
    eager = 1e3 * (time.perf_counter() - t0) / args.steps

    # capture (torch's recipe: warm-up on a side stream first)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for i in range(2):
            gstart.copy_(starts[i])
            body()
    torch.cuda.current_stream(dev).wait_stream(side)
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        body()
    # one replayed step vs one eager step from the same state
    snap = {k: v.clone() for k, v in tr.D.state_dict().items()}
    opt_snap = copy.deepcopy(tr.d_opt.state_dict())
    gsnap = {k: v.clone() for k, v in tr.G.state_dict().items()}
    gstart.copy_(starts[5])
    cg.replay()
    torch.cuda.synchronize()
    d_graph = {k: v.clone() for k, v in tr.D.state_dict().items()}
    loss_graph = float(out_static["d_loss"].item())
    # restore in place (the graph holds these buffers) and step eagerly
    with torch.no_grad():
        for k, v in tr.D.state_dict().items():
            v.copy_(snap[k])
        for k, v in tr.G.state_dict().items():
            v.copy_(gsnap[k])
        for (p, st), (_, st0) in zip(tr.d_opt.state.items(), opt_snap["state"].items()):
            for kk in ("exp_avg", "exp_avg_sq"):
                st[kk].copy_(st0[kk])
            st["step"].copy_(st0["step"])
    gstart.copy_(starts[5])
    body()
    torch.cuda.synchronize()
    loss_eager = float(out_static["d_loss"].item())
    maxdiff = max(float((tr.D.state_dict()[k].float() - d_graph[k].float()).abs().max())
                  for k in d_graph)
    print(f"replay vs eager: d_loss {loss_graph:.9g} vs {loss_eager:.9g}, "
          f"max |D state diff| {maxdiff:.3g}")
    # graph timing
    for i in range(3):
        gstart.copy_(starts[i])
        cg.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        gstart.copy_(starts[3 + i])
        cg.replay()
    torch.cuda.synchronize()
    graph = 1e3 * (time.perf_counter() - t0) / args.steps
    print(f"gan {args.dtype} T={T}: eager {eager:.3f} ms/step, graph {graph:.3f} ms/step")


if __name__ == "__main__":
    main()
