"""Launch the CNNBLSTM conv kernels alone at the C2 shapes (N=32, F=257,
T=334) -- forward (with the previous BN+ReLU prologue), data gradient and
weight gradient of each channel pair -- `reps` times each, timing every
group with HIP events.  Target of tools/pmc_conv.sh's SQ counter passes.

  python tools/conv_probe.py [reps] [fp32|bf16] [pairs, e.g. 16-32,32-16] [cl]

cl (round 5): the step's channel-last operands -- x [N, H, W, Cin] and dy
[N, H, W, Cout] (bf16 storage in the bf16 configuration: the pre-BN y16 and
the BatchNorm-backward gy16), y / dx written channel-last (y as bf16 in bf16).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch  # noqa: E402

from ainp import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
bf16 = len(sys.argv) > 2 and sys.argv[2] == "bf16"
pairs = [tuple(int(v) for v in p.split("-")) for p in
         (sys.argv[3] if len(sys.argv) > 3 else "16-32,32-16,32-64,64-32").split(",")]
cl = len(sys.argv) > 4 and sys.argv[4] == "cl"
N, H, W = 32, 257, 334
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
for ci, co in pairs:
    x = torch.randn(N, ci, H, W, device=dev, generator=g)
    dy = torch.randn(N, co, H, W, device=dev, generator=g) * 1e-2
    w = torch.randn(co, ci, 3, 3, device=dev, generator=g) * 0.05
    b = torch.zeros(co, device=dev)
    sc = torch.rand(ci, device=dev, generator=g) + 0.5
    sh = torch.randn(ci, device=dev, generator=g) * 0.1
    flops = 2.0 * 9 * ci * co * N * H * W
    if cl:
        x = x.permute(0, 2, 3, 1).contiguous()
        dy = dy.permute(0, 2, 3, 1).contiguous()
        if bf16:
            x, dy = x.bfloat16(), dy.bfloat16()
        ops_ = (("fwd", lambda: ops.conv3x3_fwd(x, w, b, sc, sh, want_stats=True, bf16=bf16,
                                                y16=bf16, xcl=True, ycl=True)),
                ("dgrad", lambda: ops.conv3x3_dgrad(dy, w, bf16=bf16, xcl=True, ycl=True)),
                ("wgrad", lambda: ops.conv3x3_wgrad(x, dy, sc, sh, bf16=bf16, xcl=True, gcl=True)))
    else:
        ops_ = (("fwd", lambda: ops.conv3x3_fwd(x, w, b, sc, sh, want_stats=True, bf16=bf16)),
                ("dgrad", lambda: ops.conv3x3_dgrad(dy, w, bf16=bf16)),
                ("wgrad", lambda: ops.conv3x3_wgrad(x, dy, sc, sh, bf16=bf16)))
    for nm, fn in ops_:
        try:
            fn()
        except Exception as e:      # a layout the kernels do not serve for this pair
            print(f"{ci:3d}->{co:3d} {nm:5s} skipped: {str(e)[:100]}", flush=True)
            continue
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"{ci:3d}->{co:3d} {nm:5s} {ms:7.3f} ms  {flops / ms / 1e9:7.1f} TF", flush=True)
