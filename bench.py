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
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (~2.5 PF)
HBM_PEAK_GBS = 8000.0

CFG = {
    "data": {"sample_rate": 16000, "max_len_s": 4.0, "gap_len_s": 0.2,
             "spectrogram": {"n_fft": 512, "hop_length": 192, "win_length": 384}},
    "model": {"in_channels": 1, "num_lstm_layers": 3, "lstm_hidden_dim": 128,
              "enc_filters": [16, 32], "dec_filters": [16, 32]},
    "training": {"starter_learning_rate": 1e-4},
}


def _traffic(name):
    """HBM bytes per launch of a roofline kernel from its committed rocprofv3
    FETCH_SIZE/WRITE_SIZE passes (profiles/<name>, tools/pmc_*.sh), or None."""
    tf = os.path.join(ROOT, "profiles", name)
    try:
        return json.load(open(tf)).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def synthetic_clips(n, S, seed0):
    from ainp.synth import synthetic_clip
    return np.stack([synthetic_clip(seed0 + i, S) for i in range(n)])


def host_cpu():
    """(nproc, CPU model) of the host this runs on (lscpu's 'Model name')."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return os.cpu_count(), model


def cpu_baseline(batch, T, steps=5, warmup=1):
    """Oracle (reference restatement) train step on the host cores; the numpy
    float64 data path (STFT / log10 / mask, the librosa restatement) is timed
    separately on the same batch."""
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
    clips = [synthetic_clip(1000 + i, S) for i in range(batch)]
    d0 = time.perf_counter()
    for i in range(batch):
        lg, tg, mk = stft_ref.cnnblstm_item(clips[i], int(rng.integers(0, S - 3200)), 3200,
                                            512, 192, 384, 16000, T)
        xs.append(lg); ms.append(mk); ts.append(tg)
    data_s = time.perf_counter() - d0
    x = torch.from_numpy(np.stack(xs)); m = torch.from_numpy(np.stack(ms))
    t = torch.from_numpy(np.stack(ts))
    for _ in range(warmup):
        tr.step(x, m, t)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        tr.step(x, m, t)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    nproc, model = host_cpu()
    return {"value": round(batch * T / dt, 2), "unit": "frames/s", "cores": cores,
            "kind": "port", "nproc": nproc, "cpu_model": model,
            "data_path_frames_per_s": round(batch * T / data_s, 1),
            "sample": f"oracle/cnnblstm_ref.py fp32 torch-CPU train step (fwd+L1+bwd+Adam), "
                      f"batch {batch} x T={T} of the C2 shapes, median of {steps} timed steps "
                      f"after {warmup} warmup on {cores} threads; the numpy data path "
                      f"(oracle/stft_ref.py, single thread) is timed separately"}


def eval_recon_l1(model, n_fft, hop, win, T, S, g, dev, n_clips=64, batch=32):
    """Reference test loss (models/CNNBLSTM/train.py:128-150,192): model.eval(),
    L1(sum) of 10**y vs |target| inside the gap per batch, averaged over the
    batches of a fixed 64-clip synthetic eval set."""
    from ainp import ops
    from ainp.cnnblstm import l1_pow10_loss
    audio = torch.from_numpy(synthetic_clips(n_clips, S, 900000)).to(dev)
    rng = np.random.default_rng(424242)
    starts = torch.from_numpy(rng.integers(0, S - g, size=n_clips).astype(np.int64)).to(dev)
    model.eval()
    tot = 0.0
    with torch.no_grad():
        for i in range(0, n_clips, batch):
            x, tgt, mask, _ = ops.stft_features(audio[i:i + batch], starts[i:i + batch], g,
                                                n_fft, hop, win, n_frames=T)
            tot += float(l1_pow10_loss(model(x.unsqueeze(1)), mask, tgt).item())
    model.train()
    return tot / (n_clips // batch)


def time_kernel(fn, reps, dev):
    """Average wall time of fn() (one launch) from HIP events on the current stream."""
    for _ in range(2):
        fn()
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1000.0 / reps


def graph_replay(model, opt, audio, starts, g, n_fft, hop, win, T, args, dev, eager_med_ms):
    """The same train step (features + fwd + bwd + Adam) captured once in a HIP
    graph (torch.cuda.CUDAGraph over the torch.ops.ainp launches) and replayed:
    per step only the gap starts are copied into the graph's static input.
    Adam runs in its capturable form (device step counter, ainp_adam_ex) on a
    copy of the eager optimizer's state, so the replayed steps continue the
    same training.  Returns graph vs eager ms/step."""
    from ainp import ops
    from ainp.cnnblstm import l1_pow10_loss
    from ainp.optim import Adam
    gopt = Adam(model.parameters(), lr=CFG["training"]["starter_learning_rate"], capturable=True)
    for p in model.parameters():
        st = opt.state.get(p)
        if st:
            gopt.state[p] = {k: v.clone() for k, v in st.items()}
    gstart = starts[0].clone()
    gloss = torch.zeros((), device=dev)

    def body():
        x, tgt, mask, _ = ops.stft_features(audio, gstart, g, n_fft, hop, win, n_frames=T)
        y = model(x.unsqueeze(1))
        loss = l1_pow10_loss(y, mask, tgt)
        loss.backward()
        gopt.step()
        gloss.copy_(loss.detach())

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for i in range(3):                  # warm up on a side stream (torch's recipe)
            gstart.copy_(starts[i])
            gopt.zero_grad(set_to_none=True)
            body()
    torch.cuda.current_stream(dev).wait_stream(side)
    gopt.zero_grad(set_to_none=True)
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        body()
    n = len(starts)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    for i in range(min(args.warmup, 5)):
        gstart.copy_(starts[i % n])
        cg.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for k in range(args.steps):
        gstart.copy_(starts[k % n])
        cg.replay()
        ev[k + 1].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    step_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]
    med = float(np.median(step_ms))
    return {"ms_per_step": round(1000.0 * el / args.steps, 3), "ms_per_step_median": round(med, 3),
            "eager_ms_per_step_median": round(eager_med_ms, 3),
            "speedup_median": round(eager_med_ms / med, 4),
            "frames_per_s": round(args.batch * T * args.steps / el, 2),
            "loss_last": float(gloss.item()),
            "what": "whole train step (features+fwd+bwd+capturable Adam) in one HIP graph, "
                    "replayed per step after a D2D copy of the gap starts"}


def executed_peak(bf16):
    """TFLOP/s ceiling of the MFMA instruction stream a configuration issues:
    bf16 -> dense bf16 peak; fp32 -> the x6 split (6 x v_mfma_f32_32x32x16_bf16
    per fp32 product) = bf16 peak / 6, unless AINP_GEMM_EXACT runs the f32 MFMA."""
    from ainp import ops
    if bf16:
        return BF16_MFMA_PEAK_TFLOPS
    return FP32_MFMA_PEAK_TFLOPS if ops.GEMM_EXACT else BF16_MFMA_PEAK_TFLOPS / 6.0


def _roof(flops, avg_s, bf16, kernel, **extra):
    ach = flops / avg_s / 1e12
    peak = executed_peak(bf16)
    r = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
         "frac": round(ach / peak, 4), "kernel": kernel, "avg_launch_ms": round(avg_s * 1e3, 4),
         "flop_per_launch": flops,
         "peak_def": ("dense bf16 MFMA (MI355X_MICROARCH.md)" if bf16 else
                      "x6 instruction-stream ceiling = dense bf16 MFMA / 6 (6 bf16 MFMA "
                      "products per fp32 product)")}
    if not bf16:
        r["f32_mfma_ratio"] = round(ach / FP32_MFMA_PEAK_TFLOPS, 4)
    r.update(extra)
    return r


def l0_rooflines(model, B, T, H, I, bf16, reps, dev):
    """(projection, backward pair) roofline entries of the LSTM layer-0 GEMMs
    (M = B*T frames, 8H = both directions' gate rows, K = I = 64*257):
    the projection X W_cat^T, and the backward pair dX = dg W_cat (main
    stream) beside dW_cat = dg^T X (side stream), launched as
    cnnblstm._BLSTMFn.backward launches them (2 x 2*M*8H*I flop)."""
    from ainp import ops
    M = B * T
    lw = model.lstm
    fused = None
    bias = (lw.bias_ih_l0, lw.bias_hh_l0, lw.bias_ih_l0_reverse, lw.bias_hh_l0_reverse)
    zx = torch.empty(M, 8 * H, device=dev)
    flops = 2.0 * M * (8 * H) * I
    g = torch.Generator(device=dev).manual_seed(5)
    dg = torch.randn(M, 8 * H, device=dev, generator=g) * 1e-3
    if bf16:
        # bf16 X [M, I] (written by the encoder's BN+ReLU) x bf16 W_cat [8H, I]
        X16 = torch.randn(M, I, device=dev, generator=g).to(torch.bfloat16)
        XT16 = X16.t().contiguous()
        W16 = torch.cat([lw.weight_ih_l0, lw.weight_ih_l0_reverse]).detach().to(torch.bfloat16)
        WT16 = W16.t().contiguous()
        dg16, dgT16 = dg.to(torch.bfloat16), dg.t().contiguous().to(torch.bfloat16)
        ns = ops.b16_proj_split(M, 8 * H, I)
        fwd = lambda: ops.gemm_bf16nt(X16, W16, out=zx, bias=bias, bias_nsplit=4 * H,  # noqa: E731
                                      nsplit=ns)
        kname = ("g256::gemm_bf16nt_256_kernel" if ops.GEMM16_256 else "g16::gemm_bf16nt_kernel") \
            + (f", split {ns} + slab sum" if ns > 1 else "")
        dx_fn = lambda: ops.gemm_bf16nt(dg16, WT16)                       # noqa: E731
        dw_fn = lambda: ops.gemm_bf16nt_splitk(dgT16, XT16, M)            # noqa: E731
        bname = "dX gemm_bf16nt (dg16 x W_cat) + dW gemm_bf16nt_splitk (dg^T x X^T, side stream)"
        main_loop = ("bf16 operands in HBM (X, W_cat), 256x256x32 tiles staged by global_load_lds "
                     "into a 4-stage LDS ring, v_mfma_f32_32x32x16_bf16, f32 accumulate")
        if ops.l0_bwd_bf16_eligible(M, I, H):
            # the step's path (cnnblstm._BLSTMFn, round 5): both GEMMs in one
            # gemm_bf16nt_256_multi launch, dW from k-major dg / X (B16_KM)
            dxo16 = torch.empty(M, I, device=dev)
            gcat = torch.empty(8 * H, I, device=dev)
            km = ops.B16_KM
            fused = lambda: ops.lstm_l0_bwd_bf16(dg16, None if km else dgT16, WT16,  # noqa: E731
                                                 X16 if km else XT16, dxo16, gcat, km=km)
            bname = ("g256::gemm_bf16nt_256_multi_kernel, one launch: dW_cat = dg^T X (weight-"
                     "gradient items first" + (", k-major dg / X via ds_read_b64_tr_b16" if km
                                               else "") + ") + dX = dg W_cat "
                     "(ops.lstm_l0_bwd_bf16)")
    else:
        A = torch.randn(M, I, device=dev, generator=g)
        if not ops.GEMM_EXACT and ops.x6_256_eligible(M, 8 * H, I, 4 * H):
            gx = ops.gemm_x6r_nt if ops.X6R_FWD else ops.gemm_x6nt_256
            fwd = lambda: gx(A, lw.weight_ih_l0, lw.weight_ih_l0_reverse,  # noqa: E731
                             zx, bias=bias, bias_nsplit=4 * H)
            kname = ("x6r::gemm_x6r_kernel" if ops.X6R_FWD else
                     "x6_256::gemm_x6nt_256s_kernel (split pass)") + ", split 3 + slab sum"
        else:
            args_g = (M, 4 * H, I, [A, A], I, 1, [lw.weight_ih_l0, lw.weight_ih_l0_reverse], 1,
                      I, [zx, zx[:, 4 * H:]], 8 * H, 1)
            kw = dict(bias1=[lw.bias_ih_l0, lw.bias_ih_l0_reverse],
                      bias2=[lw.bias_hh_l0, lw.bias_hh_l0_reverse])
            fwd = lambda: ops.gemm(*args_g, **kw)  # noqa: E731
            kname = "gemm_f32_kernel (x6 loop)"
        wf, wr = lw.weight_ih_l0.detach(), lw.weight_ih_l0_reverse.detach()
        dxo = torch.empty(M, I, device=dev)
        dx_fn = lambda: ops.gemm(M, I, 4 * H, [dg, dg[:, 4 * H:]], 8 * H, 1, [wf, wr], I, 1,  # noqa: E731
                                 [dxo, dxo], I, 1, ksplit=True)
        dw_fn = lambda: ops.gemm_tn_splitk(dg, 8 * H, A, I, M, 4 * H, I, offsets_b=(0, 0))  # noqa: E731
        bname = ("dX gemm_f32_kernel x6 (dg x [W_f; W_r], both directions summed in-tile) + dW "
                 "gemm_tn_splitk x6 (dg^T x X, split-K slabs + fixed-order sum, side stream)")
        if ops.l0_bwd_x6r_eligible(M, I, H):
            # the step's path (cnnblstm._BLSTMFn): both GEMMs in one gemm_x6r launch
            dwf, dwr = torch.empty(4 * H, I, device=dev), torch.empty(4 * H, I, device=dev)
            fused = lambda: ops.lstm_l0_bwd_x6(dg, wf, wr, A, dxo, dwf, dwr)  # noqa: E731
            bname = ("x6r::gemm_x6r_kernel, one launch: dW_cat = dg^T X (k-major operands, "
                     "tiles first) + dX = dg W_cat (ops.lstm_l0_bwd_x6)")
        main_loop = ("fp32 operands split exactly into 3 bf16 pieces, 6 cross products on "
                     "v_mfma_f32_32x32x16_bf16, f32 accumulate; 256x256x16 tiles staged by "
                     "global_load_lds into a 2-stage fp32 ring, each K-tile split once per "
                     "workgroup into double-buffered LDS bf16 planes while the previous "
                     "tile's MFMAs run (one barrier per K-tile)")
    avg_s = time_kernel(fwd, reps, dev)
    # committed rocprofv3 FETCH/WRITE passes over the same kernel (tools/pmc_x6r.sh,
    # tools/pmc_gemm.sh)
    traffic = _traffic("traffic_gemm_l0_bf16.json" if bf16 else
                       "traffic_gemm_l0_x6r.json" if ops.X6R_FWD else "traffic_gemm_l0.json")
    roof = _roof(flops, avg_s, bf16, kname + f" (LSTM l0 input projection, M={M} N={8 * H} "
                 f"K={I}, both directions)", traffic=traffic, main_loop=main_loop)

    side = torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)

    def pair():
        if fused is not None:
            fused()
            return
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            dw_fn()
        dx_fn()
        done = torch.cuda.Event()
        done.record(side)
        main.wait_event(done)
    pair_s = time_kernel(pair, reps, dev)
    dx_s = time_kernel(dx_fn, reps, dev)
    dw_s = time_kernel(dw_fn, reps, dev)
    roof_bwd = _roof(2 * flops, pair_s, bf16, bname + f" (M={M}, 8H={8 * H}, K={I})",
                     two_stream_dx_alone_ms=round(dx_s * 1e3, 4),
                     two_stream_dw_alone_ms=round(dw_s * 1e3, 4),
                     traffic=(_traffic("traffic_l0_pair_x6r.json") if fused is not None
                              and not bf16 else None),
                     what=("both GEMMs in one launch, as cnnblstm._BLSTMFn.backward runs them"
                           if fused is not None else
                           "dX on the current stream beside dW on a side stream, as "
                           "cnnblstm._BLSTMFn.backward launches them; timed from the first "
                           "launch to the join"))
    return roof, roof_bwd


def spawn_ranks(n):
    """Launch this script as N ranks (torch.distributed.run, 127.0.0.1, one
    process per GPU, RCCL unless AINP_DIST_BACKEND says otherwise) with the
    same arguments, stream their output through, and check that rank 0's JSON
    line reports n_gpus == N.  Returns the launcher's exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    line_out = None
    for line in proc.stdout:
        if line.lstrip().startswith("{"):
            try:
                rec = json.loads(line)
            except ValueError:
                rec = None
            if isinstance(rec, dict) and "metric" in rec:
                line_out = rec
        sys.stdout.write(line)
        sys.stdout.flush()
    rc = proc.wait()
    if rc == 0:
        if line_out is None:
            raise SystemExit("bench.py: the ranks printed no result line")
        if line_out.get("n_gpus") != n:
            raise SystemExit(f"bench.py: launched {n} ranks, result reports "
                             f"n_gpus={line_out.get('n_gpus')}")
    return rc


# ------------------------------------------------------------- in-step kernels
# Committed rocprofv3 kernel-stats tables of the step alone (tools/step_prof.py:
# 3 warm-up + 10 timed steps, nothing else launched; per step = total / 13),
# regenerated by tools/gpu_stepprof.sh / tools/gpu_stepprof_gan.sh.  The bench reports the dominant in-step
# kernels from them with their own roofline fractions (per-step algorithmic
# work / per-step kernel time / peak), next to the live stand-alone launches.
# (table, steps it covers: tools/step_prof.py's "kernel tables / N"); under
# profiles/steps/ so they travel with gpurun / the driver's snapshot
# (.gpurunignore drops profiles/r0*)
STEP_TABLES = {
    ("cnnblstm", "fp32"): ("profiles/steps/r06z_cnn_fp32_step_kernel_stats.csv", 13),
    ("cnnblstm", "bf16"): ("profiles/steps/r06z_cnn_bf16_step_kernel_stats.csv", 13),
    ("gan", "bf16", 626): ("profiles/steps/r06z_gan_c4_step_kernel_stats.csv", 13),
    ("gan", "bf16", 1001): ("profiles/steps/r06z_gan_c5_step_kernel_stats.csv", 13),
}


# One step of the same profiled runs as a kernel trace (tools/step_timeline.py
# --extract): the main stream's critical path per phase and each stream's busy
# time -- the in-step kernel times above add up to more than the step, because
# the side stream's weight gradients overlap the main stream.
STEP_TRACES = {
    ("cnnblstm", "fp32"): "profiles/steps/r06z_cnn_fp32_step_trace.csv",
    ("cnnblstm", "bf16"): "profiles/steps/r06z_cnn_bf16_step_trace.csv",
}


def step_critical_path(key):
    """tools/step_timeline.critical_path of the committed one-step trace."""
    path = STEP_TRACES.get(key)
    if not path or not os.path.exists(os.path.join(ROOT, path)):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import step_timeline
    cp = step_timeline.critical_path(step_timeline.load_step(os.path.join(ROOT, path)))
    cp["trace"] = path
    cp["critical_path_sum_ms"] = round(sum(cp["critical_path_ms"].values()), 3)
    cp["span_ms"] = round(cp["span_ms"], 3)
    return cp


def _cnn_step_work(B=32, F=257, T=334, H=128, bf16=False):
    """(name substring, kind, per-step algorithmic work) of the CNNBLSTM step's
    kernels at the C2 / C3 per-GPU shape: FLOP for MFMA kernels, HBM bytes
    for the BatchNorm passes (every operand read / written once, at the
    storage width of the configuration: bf16 pre-BN y and BN-backward outputs
    in the bf16 step, fp32 otherwise; the incoming gradient is fp32 in both)."""
    P = B * F * T                       # pixels per channel plane set
    conv = lambda ci, co: 2.0 * 9 * ci * co * P          # noqa: E731
    l0 = 2.0 * B * T * 8 * H * 64 * F                     # one layer-0 GEMM
    proj = 2.0 * B * T * 16 * F * 2 * H                   # one output-projection GEMM
    big = 64 * P
    y = 2.0 if bf16 else 4.0            # pre-BN y storage
    gy = 2.0 if bf16 else 4.0           # BN-backward output storage
    # conv kernels: work PER LAUNCH (a template instance serves the encoder's
    # and the decoder's layer of its shape as separate table rows, or one row
    # of two launches): in_step_table multiplies by the row's launches per step
    return [
        # fp32: layer-0 projection + backward pair + the output projection's
        # dh and dW (proj_bwd_x6)
        ("gemm_x6r_kernel", "mfma", 3 * l0 + 2 * proj),
        ("gemm_bf16nt_256_multi_kernel", "mfma", 2 * l0),  # bf16 dX + dW pair
        ("gemm_bf16nt_256_kernel", "mfma", l0),           # bf16 projection
        ("conv3x3_x6p_kernel<32, 64", "mfma/launch", conv(32, 64)),
        ("conv3x3_fwd_b16dma_kernel<32, 64", "mfma/launch", conv(32, 64)),   # round 6
        ("conv3x3_fwd_b16dma_kernel<16, 32", "mfma/launch", conv(16, 32)),   # round 6
        ("conv3x3_x6_kernel<64, 32", "mfma/launch", conv(64, 32)),
        ("conv3x3_dgrad_b16dma_kernel", "mfma/launch", conv(64, 32)),   # bf16 64 -> 32 dgrad
        ("conv3x3_wgrad_x6<64", "mfma/launch", conv(32, 64)),
        ("conv3x3_wgrad_b16dma_kernel", "mfma/launch", conv(32, 64)),   # round 6
        ("conv3x3_x6p_kernel<16, 32, false", "mfma/launch", conv(16, 32)),
        ("conv3x3_x6q_kernel<32, true", "mfma/launch", conv(16, 32)),
        ("conv3x3_wgrad_x6s<16, 32", "mfma/launch", conv(16, 32)),
        ("conv3x3_wgrad_x6s<32, 16", "mfma/launch", conv(32, 16)),
        ("conv3x3_x6q_kernel<32, false", "mfma/launch", conv(32, 16)),
        ("conv3x3_x6p_kernel<16, 32, true", "mfma/launch", conv(32, 16)),
        # channel-last BatchNorm + ReLU backward of the 16/32-channel layers:
        # reduce reads y and dy, apply reads both and writes gy
        # (one instance per channel count: encoder + decoder layer each)
        ("bn_relu_bwd_reduce_cl<16", "hbm", (y + 4.0) * 32 * P),
        ("bn_relu_bwd_reduce_cl<32", "hbm", (y + 4.0) * 64 * P),
        ("bn_relu_bwd_apply_cl<16", "hbm", (y + 4.0 + gy) * 32 * P),
        ("bn_relu_bwd_apply_cl<32", "hbm", (y + 4.0 + gy) * 64 * P),
        # the encoder's last block against the NTCF gradient of the LSTM input
        ("bn_relu_bwd_ntcf_cl<false", "hbm", (y + 4.0) * big),
        ("bn_relu_bwd_ntcf_cl<true", "hbm", (y + 4.0 + gy) * big),
        # the bridge: y -> fp32 X [N, T, 64F], or bf16 X and X^T
        ("bn_relu_apply_ntcf_cl", "hbm", (2.0 + 4.0 if bf16 else 8.0) * big),
        # round 6: the 1 <-> 16 channel convs on row strips (fp32 in both
        # configurations): 16-channel side read / written once, the 1-channel
        # side once; the data gradient's fused BatchNorm reduce also reads y
        ("conv3x3_rows_16to1", "hbm", (16 * 4.0 + 4.0) * P),
        ("conv3x3_rows_1to16<false", "hbm", (4.0 + 16 * 4.0) * P),
        ("conv3x3_rows_1to16<true, false, true", "hbm", (4.0 + 16 * 4.0 + 16 * y) * P),
    ]


def in_step_table(key, bf16, top=8, families=None):
    """Dominant in-step kernels of the committed step table for `key` (None
    if absent): per-step ms, share of the step's kernel time, and for the
    kernels with a known per-step work their roofline fraction.
    families (the GAN step): {kernel-name substring: FLOP per step} measured
    by ops.WORK_TRACE over one live step; every table row whose name holds
    the substring belongs to the family (template instances of one kernel),
    whose fraction is its FLOP over the family's summed per-step time."""
    path, div = STEP_TABLES.get(key, (None, 1))
    if not path or not os.path.exists(os.path.join(ROOT, path)):
        return None
    import csv
    rows = list(csv.DictReader(open(os.path.join(ROOT, path))))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    work = _cnn_step_work(bf16=bf16) if key[0] == "cnnblstm" else []
    fam = None
    if families:
        peak = executed_peak(bf16)
        fam = []
        for sub, flop in sorted(families.items(), key=lambda kv: -kv[1]):
            ns = sum(float(r["TotalDurationNs"]) for r in rows if sub in r["Name"])
            if ns <= 0:
                continue
            ms = ns / 1e6 / div
            tf = flop / (ms / 1e3) / 1e12
            fam.append({"family": sub, "ms_per_step": round(ms, 4), "flop_per_step": flop,
                        "achieved_tflops": round(tf, 1), "peak": round(peak, 1),
                        "frac": round(tf / peak, 4),
                        "instances": sum(1 for r in rows if sub in r["Name"])})
    out = []
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        ms = float(r["TotalDurationNs"]) / 1e6 / div
        e = {"kernel": r["Name"].split("(")[0][:120], "ms_per_step": round(ms, 4),
             "launches_per_step": round(int(r["Calls"]) / div, 2),
             "share_of_kernel_time": round(float(r["TotalDurationNs"]) / total, 4)}
        for sub, kind, amount in work:
            if sub in r["Name"]:
                if kind == "mfma/launch":   # per-launch work x this row's launches per step
                    kind, amount = "mfma", amount * int(r["Calls"]) / div
                if kind == "mfma":
                    tf = amount / (ms / 1e3) / 1e12
                    peak = executed_peak(bf16)
                    e.update(bound="mfma", achieved_tflops=round(tf, 1), peak=round(peak, 1),
                             frac=round(tf / peak, 4), flop_per_step=amount)
                else:
                    gbs = amount / (ms / 1e3) / 1e9
                    e.update(bound="hbm", achieved_gbs=round(gbs, 1), peak=HBM_PEAK_GBS,
                             frac=round(gbs / HBM_PEAK_GBS, 4), bytes_per_step=amount)
                break
        for f in fam or ():
            if f["family"] in r["Name"]:
                e.update(family=f["family"], family_frac=f["frac"])
                break
        out.append(e)
    res = {"table": path, "per_step": f"rocprofv3 --kernel-trace --stats of tools/step_prof.py "
                                      f"(totals / {div})", "top": out}
    cp = step_critical_path(key[:2])
    if cp is not None:
        res["timeline"] = cp
    if fam is not None:
        res["families"] = fam
        res["family_work"] = ("FLOP per step of each kernel family from ops.WORK_TRACE over one "
                              "live step (2 * outputs * Cin * k * k per conv launch, by the "
                              "kernel the launch routes to; D weight gradients as GEMM FLOP). The split-K "
                              "epilogues (conv_gen_splitk_*) belong to no family: their time is "
                              "not in any family's ms_per_step, so a split-K layer's family "
                              "fraction excludes it (see the top table)")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="examples per GPU (C2: 32)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--roofline-reps", type=int, default=10)
    ap.add_argument("--workload", choices=("cnnblstm", "gan"), default="cnnblstm",
                    help="cnnblstm = BASELINE configs[1] (the headline metric); gan = configs[3]")
    ap.add_argument("--clip-s", type=float, default=None,
                    help="gan: clip length (5 s = C4, T=626; 8 s = C5, T=1001, 0.1 s gap)")
    ap.add_argument("--no-graph", action="store_true",
                    help="skip the HIP-graph replay measurement of the same step (N=1)")
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32",
                    help="fp32 = C2 (headline); bf16 = the C3 per-GPU shape (bf16 GEMM/conv "
                         "operands, fp32 accumulate / cell state / BN statistics / weights)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: one rank per GPU, started here before this
        # process touches the GPU (it never does); rank 0's line is passed on
        return spawn_ranks(args.gpus)
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != args.gpus and not (ws == 1 and args.gpus == 1):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    if args.workload == "gan":
        return run_gan(args)

    from ainp import ops
    from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
    from ainp.dist import Comm, GradAllReducer, init_from_env
    from ainp.optim import Adam
    from ainp.trace import phase
    import torch.distributed as dist

    rank, world, local = init_from_env()
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    comm = Comm() if world > 1 else None

    B = args.batch
    sr = CFG["data"]["sample_rate"]
    S = int(sr * CFG["data"]["max_len_s"])            # 64000 samples (4 s)
    sp = CFG["data"]["spectrogram"]
    n_fft, hop, win = sp["n_fft"], sp["hop_length"], sp["win_length"]
    T = -(-S // hop)                                   # ceil(sr*max_len/hop) = 334
    g = int(CFG["data"]["gap_len_s"] * sr)             # 3200

    bf16 = args.dtype == "bf16"
    cfg = dict(CFG, accel={"dtype": args.dtype})
    torch.manual_seed(0)
    model = StackedBLSTMCNN(config=cfg).to(dev).train()
    if comm is not None:
        comm.broadcast_module_(model)        # rank 0's initial weights everywhere
    model.comm = comm
    opt = Adam(model.parameters(), lr=CFG["training"]["starter_learning_rate"])
    reducer = GradAllReducer(model.parameters(), comm) if comm is not None else None
    model.grad_reducer = reducer             # layer-0 W_ih gradients: chunked, early

    audio = torch.from_numpy(synthetic_clips(B, S, 100000 * rank)).to(dev)
    nsteps = args.warmup + args.steps
    rng = np.random.default_rng(12345 + rank)
    starts = torch.from_numpy(rng.integers(0, S - g, size=(nsteps, B)).astype(np.int64)).to(dev)
    losses = torch.zeros(nsteps, device=dev)

    def step(i):
        with phase("data"):
            x, tgt, mask, _ = ops.stft_features(audio, starts[i], g, n_fft, hop, win, n_frames=T)
        opt.zero_grad()
        with phase("fwd"):
            y = model(x.unsqueeze(1))
            loss = l1_pow10_loss(y, mask, tgt)
        with phase("bwd"):
            loss.backward()
        if reducer is not None:
            with phase("allreduce"):
                reducer.allreduce()
        with phase("optimizer"):
            opt.step()
        losses[i] = loss.detach()

    for i in range(args.warmup):
        step(i)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(args.warmup, nsteps):
        step(i)
        ev[i - args.warmup + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]
    med_ms = float(np.median(step_ms))
    if world > 1:
        e = torch.tensor([elapsed, med_ms], device=dev, dtype=torch.float64)
        comm.allreduce_max_(e)
        elapsed, med_ms = float(e[0].item()), float(e[1].item())
    frames = B * T * args.steps * world
    value = frames / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    train_loss = float(losses[-1].item())

    # ---- DP accounting (N > 1): the gradient all-reduce alone, the step
    # without it (compute only, SyncBN kept), and how much of the all-reduce
    # the backward hid: overlap = 1 - (step - compute) / allreduce
    dp = None
    if world > 1:
        grads = [p.grad for p in model.parameters() if p.grad is not None]
        big = [g for g in grads if g.numel() * 4 >= reducer.bucket_bytes]
        small = torch.cat([g.reshape(-1) for g in grads if g.numel() * 4 < reducer.bucket_bytes])

        def ar():
            for t in big + [small]:
                comm._allreduce(t, dist.ReduceOp.SUM, group=comm.grad_group)
        ar_s = time_kernel(ar, 5, dev)
        reducer.remove_hooks()
        model.grad_reducer = None
        nc = min(args.steps, 20)
        dist.barrier()
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        for i in range(nc):
            x, tgt, mask, _ = ops.stft_features(audio, starts[i], g, n_fft, hop, win, n_frames=T)
            opt.zero_grad()
            l1_pow10_loss(model(x.unsqueeze(1)), mask, tgt).backward()
            opt.step()
        torch.cuda.synchronize()
        comp_ms = 1000.0 * (time.perf_counter() - c0) / nc
        t = torch.tensor([ar_s * 1e3, comp_ms], device=dev, dtype=torch.float64)
        comm.allreduce_max_(t)
        ar_ms, comp_ms = float(t[0]), float(t[1])
        exposed = max(0.0, ms_step - comp_ms)
        dp = {"allreduce_ms": round(ar_ms, 3), "compute_only_ms_per_step": round(comp_ms, 3),
              "exposed_comm_ms": round(exposed, 3),
              "overlap_frac": round(max(0.0, 1.0 - exposed / ar_ms), 3) if ar_ms > 0 else None,
              "grad_bytes": int(sum(g.numel() for g in grads) * 4),
              "groups": "SyncBN and gradients on separate communicators; W_ih_l0 gradient "
                        "in 8 gate chunks all-reduced as each completes",
              "backend": dist.get_backend()}
    graph = None
    if world == 1 and not args.no_graph:
        graph = graph_replay(model, opt, audio, starts, g, n_fft, hop, win, T, args, dev, med_ms)
    recon_l1 = eval_recon_l1(model, n_fft, hop, win, T, S, g, dev) if rank == 0 else None

    # ---- roofline: dominant kernel (LSTM layer-0 input projection GEMM) timed
    # live, and the layer-0 backward pair (data + weight gradient) as the step
    # runs them.  `peak` is the ceiling of the instruction stream the kernel
    # issues, so frac <= 1 by construction: bf16 -> the dense bf16 MFMA peak;
    # fp32 (x6: 6 bf16 MFMA products per fp32 product) -> bf16 peak / 6.
    roof = roof_bwd = None
    if rank == 0:
        H = CFG["model"]["lstm_hidden_dim"]
        I = (H // 2) * (n_fft // 2 + 1)
        roof, roof_bwd = l0_rooflines(model, B, T, H, I, bf16, args.roofline_reps, dev)

    # ---- STFT / feature / mask path (HBM-bound): 4880 B per frame
    roof_stft = None
    if rank == 0:
        st_s = time_kernel(lambda: ops.stft_features(audio, starts[0], g, n_fft, hop, win,
                                                     n_frames=T), args.roofline_reps, dev)
        st_bytes = 4880 * B * T
        gbs = st_bytes / st_s / 1e9
        roof_stft = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                     "traffic": _traffic("traffic_stft.json"),
                     "kernel": "stft512_kernel<CNNBLSTM> (fused STFT + log10|X_gap| + c64 "
                               f"target + gap mask, {B} x {T} frames)",
                     "avg_launch_ms": round(st_s * 1e3, 4), "bytes_per_launch": st_bytes}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_batch, T)

    if rank == 0:
        step_flops = 163.0e6 * B * T * world  # 163.0 MFLOP/frame fwd+bwd
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (4 s/16 kHz harmonic clips, seeded; random init)",
            "config": {"workload": ("C3 per-GPU shape: CNNBLSTM train step (STFT features+fwd+"
                                    "bwd+Adam), bf16 GEMM/conv operands with fp32 accumulate, "
                                    "32 examples/GPU" if bf16 else
                                    "C2: CNNBLSTM train step (STFT features+fwd+bwd+Adam), "
                                    "fp32, 32 examples/GPU") + ", F=257, T=334, H=128, 3-layer BLSTM",
                       "global_batch": B * world, "seq_len": T, "freq_bins": n_fft // 2 + 1,
                       "parallelism": f"dp{world}" + ("+syncbn" if world > 1 else "")},
            "ms_per_step_median": round(med_ms, 3),
            "value_median": round(B * T * world / (med_ms / 1e3), 2),
            "recon_l1": recon_l1,
            "recon_l1_def": "mean over the 2 batches of a fixed 64-clip eval set of "
                            "L1sum(10**y*m, |X|*m), model.eval() (train.py:128-150,192)",
            "train_loss_last": train_loss,
            "step_tflops": round(step_flops / (ms_step / 1e3) / 1e12, 2),
            # against the ceiling of the MFMA stream the step issues (fp32 runs
            # the x6 split: bf16 peak / 6); f32-MFMA ratio kept under its own name
            "mfma_util_step": round(step_flops / world / (ms_step / 1e3) / 1e12
                                    / executed_peak(bf16), 4),
            "mfma_util_step_def": ("step FLOPs (163.0 MFLOP/frame, SURVEY d4) / ms_per_step / "
                                   + ("dense bf16 peak" if bf16 else
                                      "x6 executed ceiling (bf16 peak / 6 = 416.7 TF)")),
            **({} if bf16 else {"f32_mfma_ratio_step": round(
                step_flops / world / (ms_step / 1e3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)}),
            "roofline": roof,
            "roofline_l0_bwd": roof_bwd,
            "in_step_kernels": in_step_table(("cnnblstm", args.dtype), bf16),
            "roofline_stft": roof_stft,
            "dp": dp,
            "graph": graph,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ====================================================================== GAN (C4)
GAN_CFG = {
    "training": {"g_lr": 2e-4, "d_lr": 2e-4, "b1": 0.5, "b2": 0.999, "lambda_adv": 0.01,
                 "lambda_l1_valid": 1.0, "lambda_l1_hole": 2.0, "lambda_vgg_perceptual": 4.0,
                 "lambda_vgg_style": 500.0, "lambda_mag_weighted": 0.2},
}
# G fwd + 3 D fwd + D-step bwd + 2 VGG fwd, per sample
GAN_FLOP_PER_SAMPLE = {626: 270.4e9, 1001: 388.7e9}


def gan_cpu_baseline(T, S, g, steps=1):
    """Oracle (reference restatement) GAN step on the host cores, batch 1."""
    from oracle import gan_ref, stft_ref
    from ainp.synth import synthetic_clip
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(cores)
    pg = gan_ref.init_generator(0)
    pd = gan_ref.init_discriminator(1)
    pv = gan_ref.vgg19_init(0)
    st = gan_ref.GanStep(pg, pd, pv)
    clip = synthetic_clip(4242, S)
    o, i, _, m = stft_ref.gan_item(clip, 30000, g, 512, 128, 512)
    t = lambda a: torch.from_numpy(a)[None, None]
    st.step(t(o), t(i), t(m))            # warmup
    t0 = time.perf_counter()
    for _ in range(steps):
        st.step(t(o), t(i), t(m))
    dt = (time.perf_counter() - t0) / steps
    return {"value": round(T / dt, 2), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"oracle/gan_ref.py GanStep fp32 torch-CPU (G fwd, D step, G-step losses "
                      f"incl. VGG19 and its backward into D as the reference), batch 1 x T={T}, "
                      f"{steps} timed step after 1 warmup; features precomputed"}


def gan_roofline_operands(gen, imp, mask):
    """Sources of the final PartialConv2d and of U-Net decoder block 3 as a G
    forward launches them (ainp.gan.PConvUNet.capture), on the batch given."""
    from ainp import gan as G
    from ainp import ops
    G.PConvUNet.capture = {"decoder": (3,)}
    try:
        with torch.no_grad(), ops.nhwc16_memo():
            gen._forward(imp.unsqueeze(1), mask.unsqueeze(1))
        cap = G.PConvUNet.capture
    finally:
        G.PConvUNet.capture = None
    return cap["final"], cap["decoder3"]


def gan_roofline_launch(mod, operands, bf16, stats=False):
    """(launch, flop per launch, Hout, Wout) of one PartialConv2d conv (mod:
    a PartialConv2d or an Encoder/DecoderBlock) on captured sources, with its
    own window ratio; bf16 -> the channel-last kernel alone (operands converted
    beforehand), fp32 -> the conv_gen call."""
    from ainp import ops
    pc = getattr(mod, "pconv", mod)
    srcs, Hin, Win = operands
    (x0, m0), (x1, m1) = srcs
    N = x0.shape[0]
    k, st, pd = pc.kernel_size, pc.stride, pc.padding
    ratio, _ = ops.pconv_mask((m0, x0.shape[1]), (m1, x1.shape[1]), N, Hin, Win, k, st, pd)
    w = pc.conv.weight
    Cout, Cin = w.shape[:2]
    kw = dict(src1=(x1, m1), Hin=Hin, Win=Win, stride=st, pad=pd, bias=pc.bias, ratio=ratio,
              act=ops.ACT_NONE if stats else ops.ACT_LEAKY, want_stats=stats, bf16=bf16)
    if bf16:
        launch = ops.conv_gen((x0, m0), w, launcher=True, **kw)
    else:
        launch = lambda: ops.conv_gen((x0, m0), w, **kw)  # noqa: E731
    Ho, Wo = ops.conv_out_size(Hin, k, st, pd), ops.conv_out_size(Win, k, st, pd)
    return launch, 2.0 * Cout * Cin * k * k * N * Ho * Wo, Ho, Wo


def run_gan(args):
    from ainp import ops
    from ainp import gan as G
    from ainp.dist import Comm, init_from_env
    from ainp.gan_train import GanTrainer
    from ainp.trace import phase
    import torch.distributed as dist

    rank, world, local = init_from_env()
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    comm = Comm() if world > 1 else None
    B = args.batch if args.batch != 32 else 8        # C4 / C5: batch 8 per GPU
    clip_s = args.clip_s if args.clip_s is not None else 5.0
    c5 = clip_s >= 8.0
    S, hop, n_fft = int(16000 * clip_s), 128, 512      # C4: 5 s, C5: 8 s @ 16 kHz
    g = 1600 if c5 else 3200                           # C5: 0.1 s gaps, C4: 0.2 s
    T = 1 + S // hop                                   # 626 / 1001
    bf16 = args.dtype == "bf16"
    torch.manual_seed(0)
    gen = G.PConvUNet().to(dev)
    disc = G.Discriminator().to(dev)
    vgg = G.VGGLoss(dev)
    tr = GanTrainer(dict(GAN_CFG, accel={"dtype": args.dtype}), gen, disc, vgg, comm=comm)
    audio = torch.from_numpy(synthetic_clips(B, S, 200000 + 100000 * rank)).to(dev)
    nsteps = args.warmup + args.steps
    rng = np.random.default_rng(777 + rank)
    starts = torch.from_numpy(rng.integers(0, S - g + 1, size=(nsteps, B)).astype(np.int64)).to(dev)
    hole = torch.zeros(nsteps, device=dev)

    last = {}

    def step(i):
        with phase("data"):
            o, im, ph, m = ops.stft_features(audio, starts[i], g, n_fft, hop, n_fft, n_frames=T,
                                             mode=ops.FEAT_GAN, outputs=(True, True, c5, True))
        out = tr.step(o.unsqueeze(1), im.unsqueeze(1), m.unsqueeze(1))
        hole[i] = out["g_l1_hole"]
        last.update(orig=o, imp=im, phase=ph, mask=m, gen=out["generated"])

    for i in range(args.warmup):
        step(i)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(args.warmup, nsteps):
        step(i)
        ev[i - args.warmup + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    med_ms = float(np.median([ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]))
    if world > 1:
        e = torch.tensor([elapsed, med_ms], device=dev, dtype=torch.float64)
        comm.allreduce_max_(e)
        elapsed, med_ms = float(e[0].item()), float(e[1].item())
    value = B * T * args.steps * world / elapsed
    ms_step = 1000.0 * elapsed / args.steps

    # C5: on-GPU audio reconstruction of the last batch, the sample path of
    # models/GAN/train.py:465-505: combined log-magnitude (generated in the
    # hole, original elsewhere; passed to utils.spectrogram_to_audio as the
    # magnitude, as the reference does), ISTFT with the original phase, and
    # Griffin-Lim (spectrogram_to_audio's n_iter=64, librosa>=0.10 semantics)
    # without phase; timed separately: the reference runs it every
    # sample_interval steps, not per step
    recon = None
    if c5 and rank == 0:
        mag = (last["gen"][:, 0] * (1 - last["mask"]) + last["orig"] * last["mask"]).contiguous()
        ist_s = time_kernel(lambda: ops.istft(mag=mag, phase=last["phase"], n_fft=n_fft,
                                              hop_length=hop), 5, dev)
        gl_s = time_kernel(lambda: ops.griffinlim(mag, n_iter=64, hop_length=hop, n_fft=n_fft,
                                                  random_state=0, init="device"), 3, dev)
        recon = {"istft_orig_phase_ms": round(ist_s * 1e3, 3),
                 "griffinlim64_ms": round(gl_s * 1e3, 3),
                 "griffinlim_def": "64 iterations on the batch, initial phases drawn on the "
                                   "device (init='device'), each iteration = ainp_istft + "
                                   "ainp_gl_stft_update (n_fft=512 tiled STFT with the phase "
                                   "update fused into its write-out)",
                 "batch": B, "samples_per_clip": hop * (T - 1)}

    roof = roof_wide = None
    if rank == 0:
        # the in-step launches of the two dominant conv kernels, on operands
        # captured from a G forward over the last timed batch (real masks and
        # window ratios): the final PartialConv2d (65 -> 64, 3x3) at the padded
        # 384 x 640 / 1024 resolution, and the U-Net decoder block 768 -> 256 at
        # 1/8 resolution (the wide-tile kernel's largest launch)
        ops_fin, ops_wide = gan_roofline_operands(gen, last["imp"], last["mask"])
        launch, flops, Hp, Wp = gan_roofline_launch(gen.final_decoder_layer[0], ops_fin, bf16)
        avg_s = time_kernel(launch, args.roofline_reps, dev)
        tsuf = "_c5" if c5 else ""
        kname = "conv_gen_nhwc16_kernel<64, true>" if bf16 else "conv_gen_x6_kernel<64,16>"
        roof = _roof(flops, avg_s, bf16, f"{kname} (final PartialConv2d 65->64 3x3 at "
                     f"{Hp}x{Wp}, B={B}, in-step operands)",
                     traffic=_traffic(f"traffic_conv_gen_final_bf16{tsuf}.json" if bf16
                                      else f"traffic_conv_gen_final{tsuf}.json"))
        roof["operands"] = ("captured from a G forward over the last timed batch (real mask "
                            "planes and window ratios; tools/roofline_probe_gan.py replays the "
                            "first batch for the PMC passes)")
        if bf16:
            roof["main_loop"] = ("channel-last bf16 operands (x*mask folded in; the 1-channel "
                                 "skip source expanded per pixel, 9 -> 32 k-values), "
                                 "v_mfma_f32_32x32x16_bf16, f32 accumulate")
            roof["executed_flop_per_launch"] = 2.0 * 64 * (64 * 9 + 32) * B * Hp * Wp
        else:
            roof["main_loop"] = ("fp32 operands split exactly into 3 bf16 pieces, 6 cross "
                                 "products on v_mfma_f32_32x32x16_bf16, f32 accumulate")
        if bf16:
            launch_w, flops_w, Hd, Wd = gan_roofline_launch(gen.decoder_blocks[3], ops_wide, True,
                                                            stats=True)
            avg_w = time_kernel(launch_w, args.roofline_reps, dev)
            roof_wide = _roof(flops_w, avg_w, True,
                              f"conv_gen_nhwc16_wide_kernel<256, 8, false> (U-Net decoder block "
                              f"768->256 3x3 at {Hd}x{Wd}, B={B}, BN partials, in-step operands)",
                              traffic=_traffic(f"traffic_conv_gen_wide_bf16{tsuf}.json"))
            roof_wide["main_loop"] = ("256x128 tiles, 8 waves of 64x64, 3-stage LDS-DMA ring "
                                      "(global_load_lds_dwordx4), v_mfma_f32_32x32x16_bf16")
    families = None
    if rank == 0 and world == 1:
        # per-family algorithmic work of one step, as the step routes it
        ops.WORK_TRACE = []
        step(nsteps - 1)
        torch.cuda.synchronize()
        families = {}
        for nm, fl in ops.WORK_TRACE:
            families[nm] = families.get(nm, 0.0) + fl
        ops.WORK_TRACE = None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = gan_cpu_baseline(T, S, g)
    if rank == 0:
        step_flops = GAN_FLOP_PER_SAMPLE[T] * B * world if T in GAN_FLOP_PER_SAMPLE else None
        cname = "C5" if c5 else "C4"
        out = {
            "metric": f"GAN spectrogram-frames/sec/node (train step), BASELINE configs"
                      f"[{4 if c5 else 3}]",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "ms_per_step_median": round(med_ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": f"synthetic ({clip_s:g} s/16 kHz harmonic clips, seeded; random init; VGG19 "
                    "random init: pretrained weights not downloadable offline)",
            "config": {"workload": f"{cname}: GAN step (GAN STFT features + PConvUNet fwd + D "
                                   "step + G-step losses incl. VGG19), "
                                   + ("bf16 conv/GEMM operands, fp32 accumulate"
                                      if bf16 else "fp32")
                                   + f", {B} examples/GPU, F=257, T={T}, gap {g / 16000:g} s",
                       "global_batch": B * world, "seq_len": T,
                       "freq_bins": 257, "parallelism": f"dp{world}"},
            "recon_l1_hole": float(hole[-1].item()),
            "step_tflops": (round(step_flops / (ms_step / 1e3) / 1e12, 2)
                            if step_flops else None),
            "mfma_util_step": (round(step_flops / world / (ms_step / 1e3) / 1e12
                                     / executed_peak(bf16), 4) if step_flops else None),
            "roofline": roof, "roofline_wide": roof_wide, "reconstruction": recon,
            "in_step_kernels": in_step_table(("gan", args.dtype, T), bf16, families=families),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    raise SystemExit(main() or 0)
