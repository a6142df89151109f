#!/usr/bin/env python3
"""Benchmark: CNNBLSTM training step (BASELINE.json configs[1], C2) on MI355X.

One "step" = one pass of the hot path over one batch of synthetic input:
on-GPU STFT + log-magnitude + gap mask from resident 4 s / 16 kHz clips
(ainp_stft_features), StackedBLSTMCNN forward, L1(sum) loss on 10**y inside
the gap, backward, (DP: SUM all-reduce of gradients + SyncBN), Adam step --
i.e. models/CNNBLSTM/train.py:83-108 with the dataset of
models/CNNBLSTM/dataset.py:93-119 moved onto the GPU.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Prints ONE JSON line (rank 0).  value = frames processed by all ranks / max
over ranks of the timed wall time.  Also reports:
  roofline     the dominant kernel (the LSTM layer-0 input-projection GEMM,
               M=N*T, N=8H, K=C*F) timed live with HIP events on its stream;
  cpu_baseline the oracle's torch-CPU restatement of the same step (the
               reference's CPU path), on a bounded sample, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "spectrogram-frames/sec/node (train step) + recon L1, CNNBLSTM @1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
HBM_PEAK_GBS = 8000.0

CFG = {
    "data": {"sample_rate": 16000, "max_len_s": 4.0, "gap_len_s": 0.2,
             "spectrogram": {"n_fft": 512, "hop_length": 192, "win_length": 384}},
    "model": {"in_channels": 1, "num_lstm_layers": 3, "lstm_hidden_dim": 128,
              "enc_filters": [16, 32], "dec_filters": [16, 32]},
    "training": {"starter_learning_rate": 1e-4},
}


def synthetic_clips(n, S, seed0):
    from ainp.synth import synthetic_clip
    return np.stack([synthetic_clip(seed0 + i, S) for i in range(n)])


def cpu_baseline(batch, T, steps=2, warmup=1):
    """Oracle (reference restatement) train step on the host cores."""
    from oracle import cnnblstm_ref, stft_ref
    from ainp.synth import synthetic_clip
    # the GPU box exposes the whole machine in os.cpu_count() but gives this job
    # OMP_NUM_THREADS cores; use (and report) that share
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(cores)
    H, L = CFG["model"]["lstm_hidden_dim"], CFG["model"]["num_lstm_layers"]
    p = cnnblstm_ref.init_params(CFG, seed=0)
    tr = cnnblstm_ref.Trainer(p, H, L, lr=1e-4)
    S = 64000
    rng = np.random.default_rng(1)
    xs, ms, ts = [], [], []
    for i in range(batch):
        clip = synthetic_clip(1000 + i, S)
        lg, tg, mk = stft_ref.cnnblstm_item(clip, int(rng.integers(0, S - 3200)), 3200,
                                            512, 192, 384, 16000, T)
        xs.append(lg); ms.append(mk); ts.append(tg)
    x = torch.from_numpy(np.stack(xs)); m = torch.from_numpy(np.stack(ms))
    t = torch.from_numpy(np.stack(ts))
    for _ in range(warmup):
        tr.step(x, m, t)
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(x, m, t)
    dt = (time.perf_counter() - t0) / steps
    return {"value": round(batch * T / dt, 2), "unit": "frames/s", "cores": cores,
            "kind": "port",
            "sample": f"oracle/cnnblstm_ref.py fp32 torch-CPU train step (fwd+L1+bwd+Adam), "
                      f"batch {batch} x T={T} of the C2 shapes, {steps} timed steps after "
                      f"{warmup} warmup; features precomputed (data path not timed)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="examples per GPU (C2: 32)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--roofline-reps", type=int, default=10)
    args = ap.parse_args()

    from ainp import ops
    from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
    from ainp.dist import Comm, GradAllReducer, init_from_env
    from ainp.optim import Adam
    import torch.distributed as dist

    rank, world, local = init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    comm = Comm() if world > 1 else None

    B = args.batch
    sr = CFG["data"]["sample_rate"]
    S = int(sr * CFG["data"]["max_len_s"])            # 64000 samples (4 s)
    sp = CFG["data"]["spectrogram"]
    n_fft, hop, win = sp["n_fft"], sp["hop_length"], sp["win_length"]
    T = -(-S // hop)                                   # ceil(sr*max_len/hop) = 334
    g = int(CFG["data"]["gap_len_s"] * sr)             # 3200

    torch.manual_seed(0)
    model = StackedBLSTMCNN(config=CFG).to(dev).train()
    model.comm = comm
    opt = Adam(model.parameters(), lr=CFG["training"]["starter_learning_rate"])
    reducer = GradAllReducer(model.parameters(), comm) if comm is not None else None

    audio = torch.from_numpy(synthetic_clips(B, S, 100000 * rank)).to(dev)
    nsteps = args.warmup + args.steps
    rng = np.random.default_rng(12345 + rank)
    starts = torch.from_numpy(rng.integers(0, S - g, size=(nsteps, B)).astype(np.int64)).to(dev)
    losses = torch.zeros(nsteps, device=dev)

    def step(i):
        x, tgt, mask, _ = ops.stft_features(audio, starts[i], g, n_fft, hop, win, n_frames=T)
        opt.zero_grad()
        y = model(x.unsqueeze(1))
        loss = l1_pow10_loss(y, mask, tgt)
        loss.backward()
        if reducer is not None:
            reducer.allreduce()
        opt.step()
        losses[i] = loss.detach()

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, nsteps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        lsum = losses.double().sum().reshape(1)
        dist.all_reduce(lsum)
    frames = B * T * args.steps * world
    value = frames / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    recon_l1 = float(losses[-1].item())

    # ---- roofline: dominant kernel (LSTM layer-0 input projection GEMM) timed live
    roof = None
    if rank == 0:
        H = CFG["model"]["lstm_hidden_dim"]
        I = (H // 2) * (n_fft // 2 + 1)
        M = B * T
        A = torch.randn(M, I, device=dev)
        lw = model.lstm
        zx = torch.empty(M, 8 * H, device=dev)
        args_g = (M, 4 * H, I, [A, A], I, 1, [lw.weight_ih_l0, lw.weight_ih_l0_reverse], 1, I,
                  [zx, zx[:, 4 * H:]], 8 * H, 1)
        kw = dict(bias1=[lw.bias_ih_l0, lw.bias_ih_l0_reverse],
                  bias2=[lw.bias_hh_l0, lw.bias_hh_l0_reverse])
        for _ in range(2):
            ops.gemm(*args_g, **kw)
        s = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.roofline_reps):
            ops.gemm(*args_g, **kw)
        e1.record(s)
        torch.cuda.synchronize()
        avg_s = e0.elapsed_time(e1) / 1000.0 / args.roofline_reps
        flops = 2.0 * M * (8 * H) * I
        achieved = flops / avg_s / 1e12
        traffic = None
        tf = os.path.join(ROOT, "profiles", "traffic_gemm_l0.json")
        if os.path.exists(tf):
            try:
                traffic = json.load(open(tf)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": traffic, "kernel": "gemm_f32_kernel (LSTM l0 input projection, "
                f"M={M} N={8 * H} K={I}, both directions)", "avg_launch_ms": round(avg_s * 1e3, 4),
                "flop_per_launch": flops}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_batch, T)

    if rank == 0:
        step_flops = 163.0e6 * B * T * world  # 163.0 MFLOP/frame fwd+bwd
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32", "data": "synthetic (4 s/16 kHz harmonic clips, seeded; random init)",
            "config": {"workload": "C2: CNNBLSTM train step (STFT features+fwd+bwd+Adam), "
                                   "fp32, 32 examples/GPU, F=257, T=334, H=128, 3-layer BLSTM",
                       "global_batch": B * world, "seq_len": T, "freq_bins": n_fft // 2 + 1,
                       "parallelism": f"dp{world}" + ("+syncbn" if world > 1 else "")},
            "recon_l1": recon_l1,
            "step_tflops": round(step_flops / (ms_step / 1e3) / 1e12, 2),
            "mfma_util_step": round(step_flops / world / (ms_step / 1e3) / 1e12
                                    / FP32_MFMA_PEAK_TFLOPS, 4),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
