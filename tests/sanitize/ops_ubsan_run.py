"""Run in a subprocess by tests/test_gpu_sanitize.py with
AINP_TORCH_OPS=libainp_torch_ubsan.so (the torch.ops.ainp host layer built
with -fsanitize=undefined, halt on error): two small CNNBLSTM training steps
and one GAN block through the UBSan build, then malformed arguments that the
host-side checks must reject with a RuntimeError before any launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ainp import ops, smoke  # noqa: E402

assert ops.TORCH_OPS_PATH.endswith("libainp_torch_ubsan.so"), ops.TORCH_OPS_PATH
g = np.load(os.path.join(ROOT, "tests", "golden", "cnnblstm_small.npz"), allow_pickle=False)
out = smoke.run_training_steps(g)
errs, bad = smoke.check_against_golden(g, out, tol=1e-4)
assert not bad, bad

dev = "cuda"
rejected = 0


def expect_reject(fn):
    global rejected
    try:
        fn()
    except (RuntimeError, ValueError, TypeError, AssertionError):
        rejected += 1
        return
    raise SystemExit("host check did not reject: %r" % fn)


A = torch.randn(64, 128, device=dev).to(torch.bfloat16)
B = torch.randn(32, 128, device=dev).to(torch.bfloat16)
C = torch.empty(64, 32, device=dev)
short = torch.zeros(3, device=dev)
expect_reject(lambda: torch.ops.ainp.gemm_bf16nt(A, B, C, 128, short, None, None, None, 16, 1, 128))
expect_reject(lambda: torch.ops.ainp.gemm_bf16nt(A, B, C, 128, None, None, short, None, 40, 1, 128))
expect_reject(lambda: torch.ops.ainp.gemm_bf16nt(A, B, torch.empty(63, 32, device=dev), 128,
                                                 None, None, None, None, 0, 1, 128))
expect_reject(lambda: torch.ops.ainp.gemm_bf16nt(A, B, C, 256, None, None, None, None, 0, 1, 256))
y = torch.randn(2, 3, 4, device=dev)
expect_reject(lambda: torch.ops.ainp.l1_pow10_loss(y, y[:1], y.to(torch.complex64),
                                                   torch.empty(1, device=dev, dtype=torch.float64),
                                                   None, 1.0))
expect_reject(lambda: ops.l1_pow10_loss(y.cpu(), y.cpu(), y.cpu().to(torch.complex64)))
expect_reject(lambda: torch.ops.ainp.transpose_f32(torch.randn(4, 5, device=dev),
                                                   torch.empty(4, 5, device=dev)))
torch.cuda.synchronize()
print(f"ubsan ops run OK: {rejected} malformed calls rejected", flush=True)
