"""Per-op timing of one CNNBLSTM training step at C2 (B=32, T=334; argv[1] =
bf16: the C3-shape bf16 configuration): every ainp.ops call is bracketed by HIP
events and a synchronize (after warmup), so each op runs alone, and listed
with its shapes; GEMM/conv lines also print TFLOP/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ainp import ops  # noqa: E402
from ainp import cnnblstm as CB  # noqa: E402
from ainp.optim import Adam  # noqa: E402
import bench  # noqa: E402

B = 32
DT = sys.argv[1] if len(sys.argv) > 1 else "fp32"     # fp32 (C2) or bf16 (C3 shape)
torch.manual_seed(0)
model = CB.StackedBLSTMCNN(config=dict(bench.CFG, accel={"dtype": DT})).cuda().train()
opt = Adam(model.parameters(), lr=1e-4)
audio = torch.from_numpy(bench.synthetic_clips(B, 64000, 0)).cuda()
starts = torch.randint(0, 64000 - 3200, (B,), dtype=torch.int64).cuda()

records = []
names = ["stft_features", "gemm", "gemm_tn_splitk", "conv3x3_fwd", "conv3x3_dgrad",
         "conv3x3_wgrad", "bn_stats_reduce", "bn_finalize", "bn_relu_apply", "bn_relu_bwd_reduce",
         "bn_relu_bwd_apply", "lstm_rec_fwd", "lstm_rec_bwd", "lstm_hprev", "l1_pow10_loss",
         "sum_slabs", "rowsum_batched", "colsum", "adam_step", "scale_by_scalar",
         "gemm_bf16nt", "gemm_bf16nt_splitk", "bn_relu_apply_ntcf_bf16", "cast_bf16_t",
         "gemm_x6r_nt", "lstm_l0_bwd_x6", "proj_bwd_x6"]
active = [False]


def shape_of(a):
    if isinstance(a, torch.Tensor):
        return tuple(a.shape)
    if isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
        return [tuple(t.shape) for t in a][:2]
    return a


def wrap(nm):
    f = getattr(ops, nm)

    def w(*a, **k):
        if not active[0]:
            return f(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = f(*a, **k)
        e1.record()
        torch.cuda.synchronize()
        flops = None
        if nm == "gemm":
            flops = 2.0 * a[0] * a[1] * a[2] * len(a[3]) * k.get("nstrided", 1)
        elif nm in ("conv3x3_fwd", "conv3x3_dgrad", "conv3x3_wgrad"):
            x = a[0]
            wt = a[1]
            if nm == "conv3x3_wgrad":
                N, Cin, H, W = x.shape
                Cout = wt.shape[1]
            else:
                N, _, H, W = x.shape
                Cout, Cin = wt.shape[:2]
            flops = 2.0 * 9 * Cin * Cout * N * H * W
        args = [shape_of(v) for v in a[:6] if not isinstance(v, (float,))]
        records.append((nm, str(args)[:110], e0.elapsed_time(e1), flops))
        return out
    setattr(ops, nm, w)
    setattr(CB.ops, nm, w)


for nm in names:
    if hasattr(ops, nm):
        wrap(nm)


def step():
    x, tgt, mask, _ = ops.stft_features(audio, starts, 3200, 512, 192, 384, n_frames=334)
    opt.zero_grad()
    y = model(x.unsqueeze(1))
    loss = CB.l1_pow10_loss(y, mask, tgt)
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
active[0] = True
step()
torch.cuda.synchronize()
tot = sum(r[2] for r in records)
print(f"total timed op ms: {tot:.2f}")
for nm, s, ms, fl in sorted(records, key=lambda r: -r[2]):
    extra = f"{fl / ms / 1e9:7.1f} TF" if fl else ""
    print(f"{ms:7.3f} ms  {nm:20s} {extra:10s} {s}")
