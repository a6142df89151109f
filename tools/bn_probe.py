"""Time the CNNBLSTM BatchNorm(+ReLU) passes alone at the C2 / C3-shape sizes
(N=32, F=257, T=334) with HIP events and report algorithmic HBM bytes / time:
the NTCF bridge kernels of the encoder's last block (C=64: backward reduce and
apply with g in the LSTM layout, the bf16 X / X^T writer) and the flat ones
(C=32), beside a plain device copy and torch's transposing copy of the same
bytes as reference rates.

  python tools/bn_probe.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch  # noqa: E402

from ainp import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
N, H, W = 32, 257, 334
dev = "cuda"
gen = torch.Generator(device=dev).manual_seed(3)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def report(name, ms, nbytes):
    print(f"{name:34s} {ms:7.3f} ms  {nbytes / 1e6:8.1f} MB  {nbytes / ms / 1e9:6.2f} TB/s", flush=True)


for C in (64, 32):
    y = torch.randn(N, C, H, W, device=dev, generator=gen)
    sc = torch.rand(C, device=dev, generator=gen) + 0.5
    sh = torch.randn(C, device=dev, generator=gen) * 0.1
    save = torch.cat([torch.randn(C, device=dev, generator=gen) * 0.1,
                      torch.rand(C, device=dev, generator=gen) + 0.5])
    gam = torch.rand(C, device=dev, generator=gen) + 0.5
    T4 = y.numel() * 4
    if C == 64:
        g = torch.randn(N, W, C * H, device=dev, generator=gen)
        sums = ops.bn_relu_bwd_reduce(g, y, sc, sh, save, ntcf=True)
        report("bwd_reduce ntcf C=64", timed(lambda: ops.bn_relu_bwd_reduce(
            g, y, sc, sh, save, ntcf=True)), 2 * T4)
        report("bwd_apply ntcf C=64", timed(lambda: ops.bn_relu_bwd_apply(
            g, y, sc, sh, gam, save, sums, N * H * W, ntcf=True)), 3 * T4)
        report("apply_ntcf_bf16 C=64", timed(lambda: ops.bn_relu_apply_ntcf_bf16(y, sc, sh)),
               T4 + T4)
        report("apply ntcf fp32 C=64", timed(lambda: ops.bn_relu_apply(y, sc, sh, ntcf=True)),
               2 * T4)
        o = torch.empty_like(y)
        report("torch copy (703 MB)", timed(lambda: o.copy_(y)), 2 * T4)
        report("torch transpose copy NTCF->NKW", timed(
            lambda: o.view(N, C * H, W).copy_(g.transpose(1, 2))), 2 * T4)
    else:
        g = torch.randn(N, C, H, W, device=dev, generator=gen)
        sums = ops.bn_relu_bwd_reduce(g, y, sc, sh, save)
        report("bwd_reduce flat C=32", timed(lambda: ops.bn_relu_bwd_reduce(
            g, y, sc, sh, save)), 2 * T4)
        report("bwd_apply flat C=32", timed(lambda: ops.bn_relu_bwd_apply(
            g, y, sc, sh, gam, save, sums, N * H * W)), 3 * T4)
    del y, g
    torch.cuda.empty_cache()
