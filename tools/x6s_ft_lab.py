"""conv3x3_wgrad_x6s tile rows (AINP_X6S_FT1 / _FT3 = 4, 8, 16): the 16 <-> 32
channel weight gradients at the C2 shape with the step's channel-last
operands (x fp32 [N, H, W, Cin] with the BN+ReLU prologue; dy [N, H, W, Cout],
bf16 in the bf16 configuration), timed with HIP events, dw / db against the
4-row tiles (another slab partition: a different fp32 summation order).

  python tools/x6s_ft_lab.py [reps]
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
g = torch.Generator(device=dev).manual_seed(3)


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


for bf16 in (True, False):
    key = "AINP_X6S_FT1" if bf16 else "AINP_X6S_FT3"
    for ci, co in ((16, 32), (32, 16)):
        x = torch.randn(N, H, W, ci, device=dev, generator=g)
        dy = torch.randn(N, H, W, co, device=dev, generator=g) * 1e-2
        if bf16:
            dy = dy.bfloat16()
        sc = torch.rand(ci, device=dev, generator=g) + 0.5
        sh = torch.randn(ci, device=dev, generator=g) * 0.1
        flops = 2.0 * 9 * ci * co * N * H * W
        ref = None
        for ft in ((4, 8, 16) if bf16 else (4, 8)):
            os.environ[key] = str(ft)
            fn = lambda: ops.conv3x3_wgrad(x, dy, sc, sh, bf16=bf16, xcl=True, gcl=True)  # noqa: E731
            dw, db = fn()
            dw2, db2 = fn()
            same = torch.equal(dw, dw2) and torch.equal(db, db2)
            if ref is None:
                ref = (dw, db)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(f"{'bf16' if bf16 else 'fp32'} {ci:2d}->{co:2d} FT={ft:2d} {ms:7.3f} ms "
                  f"{flops / ms / 1e9:7.1f} TF  dw rel {rel(dw, ref[0]):.2e} db rel "
                  f"{rel(db, ref[1]):.2e} rerun-identical {same}", flush=True)
        os.environ.pop(key)
