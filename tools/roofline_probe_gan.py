"""Launch only the GAN bench's roofline kernel (the final PartialConv2d,
65 -> 64 channels 3x3 at the padded 384 x 640 resolution, B=8) a few times,
with the same operands bench.py times: fp32 -> conv_gen x6 path; bf16 (argv[2])
-> the channel-last conv_gen_nhwc16 kernel alone on operands converted once.
The target of the rocprofv3 --pmc passes behind profiles/traffic_conv_gen_final*.json."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch
from ainp import ops
B, Hp, Wp = 8, 384, 640
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
bf16 = len(sys.argv) > 2 and sys.argv[2] == "bf16"
dev = "cuda"
x0 = torch.randn(B, 64, Hp // 2, Wp // 2, device=dev)
m0 = torch.ones(B, Hp // 2, Wp // 2, device=dev)
x1 = torch.randn(B, 1, Hp, Wp, device=dev)
m1 = torch.ones(B, Hp, Wp, device=dev)
w = torch.randn(64, 65, 3, 3, device=dev) * 0.05
ratio = torch.ones(B, Hp, Wp, device=dev)
bias = torch.zeros(64, device=dev)
out = torch.empty(B, 64, Hp, Wp, device=dev)
kw = dict(src1=(x1, m1), Hin=Hp, Win=Wp, stride=1, pad=1, bias=bias, ratio=ratio,
          act=ops.ACT_LEAKY, out=out, bf16=bf16)
if bf16:
    launch = ops.conv_gen((x0, m0), w, launcher=True, **kw)
else:
    launch = lambda: ops.conv_gen((x0, m0), w, **kw)  # noqa: E731
for _ in range(reps):
    launch()
torch.cuda.synchronize()
print("done")
