"""Time the BLSTM recurrence kernels alone at the C2 shape (N=32, T=334,
H=128): ops.lstm_rec_fwd / lstm_rec_bwd, `reps` launches each, HIP events.
With AINP_LSTM_DBG (measurement switches of lstm_fwd_kernel, wrong results)
it shows what a step's pieces cost.   python tools/lstm_lab.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch  # noqa: E402

from ainp import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N, T, H = 32, 334, 128
g = torch.Generator(device="cuda").manual_seed(0)
zx = torch.randn(N, T, 8 * H, device="cuda", generator=g) * 0.5
wf = torch.randn(4 * H, H, device="cuda", generator=g) * 0.05
wr = torch.randn(4 * H, H, device="cuda", generator=g) * 0.05
h, gates, cell = ops.lstm_rec_fwd(zx, wf, wr, H)
dh = torch.randn(N, T, 2 * H, device="cuda", generator=g) * 0.1
for nm, fn in (("fwd", lambda: ops.lstm_rec_fwd(zx, wf, wr, H)),
               ("bwd", lambda: ops.lstm_rec_bwd(dh, gates, cell, wf, wr, H))):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"dbg={os.environ.get('AINP_LSTM_DBG', '0')} {nm} {ms * 1e3:.1f} us  "
          f"{ms * 1e3 / T * 1e3:.0f} ns/step", flush=True)
