"""GEMM microbenchmark: TFLOP/s of ainp_gemm_f32 on the CNNBLSTM shapes."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch
from ainp import ops

def bench(name, M, N, K, akc, bkc, reps=5):
    dev = "cuda"
    A = torch.randn(M, K, device=dev) if akc else torch.randn(K, M, device=dev)
    B = torch.randn(N, K, device=dev) if bkc else torch.randn(K, N, device=dev)
    C = torch.empty(M, N, device=dev)
    sam, sak = (K, 1) if akc else (1, M)
    sbk, sbn = (1, K) if bkc else (N, 1)
    f = lambda: ops.gemm(M, N, K, [A], sam, sak, [B], sbk, sbn, [C], N, 1)
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = 2 * M * N * K / ms / 1e9
    print(f"{name:28s} M={M:6d} N={N:6d} K={K:6d} akc={akc} bkc={bkc}: {ms:8.3f} ms {tf:7.1f} TF", flush=True)

bench("square NT", 4096, 4096, 4096, True, True)
bench("square NN", 4096, 4096, 4096, True, False)
bench("square TN", 4096, 4096, 4096, False, False)
bench("L0 fwd (zx)", 10688, 1024, 16448, True, True)
bench("L0 fwd 2 rounds exact", 8192, 1024, 16448, True, True)
bench("L0 dX", 10688, 16448, 1024, True, False)
bench("L0 dW_ih", 1024, 16448, 10688, False, False)
bench("L0 dW_ih M=512", 512, 16448, 10688, False, False)
