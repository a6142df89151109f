"""Time the fp32 layer-0 GEMMs of the C2 step (M = NT = 10688, 8H = 1024,
I = 16448) on their kernels, HIP events over `reps` launches each:
  fwd_256   projection on gemm_x6nt_256s (split 3 + slab sum)
  fwd_x6r   projection on gemm_x6r (split 3 + slab sum)
  pair_x6r  dX + dW_ih in one gemm_x6r launch (ops.lstm_l0_bwd_x6)
  pair_old  dX (128x128 x6) on the stream beside split-K dW on a side stream
usage: python tools/x6r_probe.py [reps] [only-name]   (only-name: for --pmc passes)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch  # noqa: E402

from ainp import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
only = sys.argv[2] if len(sys.argv) > 2 else None
H, NT, I = 128, 10688, 16448
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
X = torch.relu(torch.randn(NT, I, device=dev, generator=g))
wf = torch.randn(4 * H, I, device=dev, generator=g) * 0.01
wr = torch.randn(4 * H, I, device=dev, generator=g) * 0.01
b = tuple(torch.zeros(4 * H, device=dev) for _ in range(4))
dg = torch.randn(NT, 8 * H, device=dev, generator=g) * 1e-3
zx = torch.empty(NT, 8 * H, device=dev)
dx = torch.empty(NT, I, device=dev)
dwf = torch.empty(4 * H, I, device=dev)
dwr = torch.empty(4 * H, I, device=dev)
side = torch.cuda.Stream()


def pair_old():
    main = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        ops.gemm_tn_splitk(dg, 8 * H, X, I, NT, 4 * H, I, offsets_b=(0, 0))
    ops.gemm(NT, I, 4 * H, [dg, dg[:, 4 * H:]], 8 * H, 1, [wf, wr], I, 1, [dx, dx], I, 1,
             ksplit=True)
    done = torch.cuda.Event()
    done.record(side)
    main.wait_event(done)


cases = {
    "fwd_256": (lambda: ops.gemm_x6nt_256(X, wf, wr, zx, bias=b, bias_nsplit=4 * H), 1),
    "fwd_x6r": (lambda: ops.gemm_x6r_nt(X, wf, wr, zx, bias=b, bias_nsplit=4 * H), 1),
    "pair_x6r": (lambda: ops.lstm_l0_bwd_x6(dg, wf, wr, X, dx, dwf, dwr), 2),
    "pair_old": (pair_old, 2),
}
for name, (fn, mult) in cases.items():
    if only and name != only:
        continue
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = mult * 2.0 * NT * 8 * H * I / (ms / 1e3) / 1e12
    print(f"{name:10s} {ms:8.4f} ms  {tf:7.1f} fp32-TF  x6 executed {6 * tf:7.1f} TF "
          f"({6 * tf / 2500:.3f} of 2.5 PF)", flush=True)
