"""Launch only the bench's roofline kernel (LSTM layer-0 input projection GEMM,
M=N*T=10688, N=8H=1024, K=C*F=16448) a few times: fp32 -> the x6 split on fp32
operands (the 256x256 x6r tile, split 3 + slab sum, as the step runs it;
argv[2] == fp32old: the 128x128 gemm_f32 loop; pair: the fused layer-0
backward dX + dW_ih launch); bf16 (argv[2]) -> gemm_bf16nt
on bf16 X / W_cat, as the bench times it.  The target of the rocprofv3 --pmc passes behind
profiles/traffic_gemm_l0*.json."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch
from ainp import ops
H, F, B, T = 128, 257, 32, 334
M, I = B * T, (H // 2) * F
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
bf16 = len(sys.argv) > 2 and sys.argv[2] == "bf16"
dev = "cuda"
A = torch.randn(M, I, device=dev)
W = [torch.randn(4 * H, I, device=dev) * 0.01 for _ in range(2)]
b = [torch.zeros(4 * H, device=dev) for _ in range(4)]
zx = torch.empty(M, 8 * H, device=dev)
if bf16:
    A16 = A.bfloat16()
    W16 = torch.cat(W).bfloat16()
    for _ in range(reps):
        ops.gemm_bf16nt(A16, W16, out=zx, bias=tuple(b), bias_nsplit=4 * H,
                        nsplit=ops.b16_proj_split(zx.shape[0], zx.shape[1], A16.shape[1]))
elif len(sys.argv) > 2 and sys.argv[2] == "fp32old":
    for _ in range(reps):
        ops.gemm(M, 4 * H, I, [A, A], I, 1, W, 1, I, [zx, zx[:, 4 * H:]], 8 * H, 1,
                 bias1=b[:2], bias2=b[2:])
elif len(sys.argv) > 2 and sys.argv[2] == "pair":
    # the fused layer-0 backward pair (dX + dW_ih in one x6r launch)
    dg = torch.randn(M, 8 * H, device=dev) * 1e-3
    dx = torch.empty(M, I, device=dev)
    dw = [torch.empty(4 * H, I, device=dev) for _ in range(2)]
    for _ in range(reps):
        ops.lstm_l0_bwd_x6(dg, W[0], W[1], A, dx, dw[0], dw[1])
elif len(sys.argv) > 2 and sys.argv[2] in ("pair_dw", "pair_dx"):
    # one half of the pair alone (its traffic apart from the other's)
    dg = torch.randn(M, 8 * H, device=dev) * 1e-3
    G4 = 4 * H
    if sys.argv[2] == "pair_dw":
        dw = [torch.empty(4 * H, I, device=dev) for _ in range(2)]
        p = ops.x6_problem(dg, A, dw[0], M=8 * H, N=I, K=M, lda=8 * H, ldb=I, ldc=I,
                           a_kmajor=True, b_kmajor=True, C2=dw[1], c_msplit=G4)
    else:
        dx = torch.empty(M, I, device=dev)
        p = ops.x6_problem(dg, W[0], dx, M=M, N=I, K=8 * H, lda=8 * H, ldb=I, ldc=I,
                           B2=W[1], b_ksplit=G4, b_kmajor=True)
    for _ in range(reps):
        ops.gemm_x6_multi([p])
else:
    for _ in range(reps):
        if ops.X6R_FWD:   # the step's kernel (gemm_x6r.hip), as the bench times it
            ops.gemm_x6r_nt(A, W[0], W[1], zx, bias=(b[0], b[2], b[1], b[3]), bias_nsplit=4 * H)
        else:
            ops.gemm_x6nt_256(A, W[0], W[1], zx, bias=(b[0], b[2], b[1], b[3]),
                              bias_nsplit=4 * H)
torch.cuda.synchronize()
print("done")
