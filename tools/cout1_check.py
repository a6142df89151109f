import sys, os, torch
sys.path.insert(0, "ml-audio-inpainting_amd")
from ainp import ops
out = {}
for (k, s, C, H, W, N) in [(3, 1, 64, 260, 600, 4), (4, 1, 512, 31, 77, 8), (4, 2, 64, 32, 40, 2)]:
    g = torch.Generator().manual_seed(k + C)
    x = torch.randn(N, C, H, W, generator=g).cuda()
    m = (torch.rand(N, H, W, generator=g) > 0.2).float().cuda()
    w = (torch.randn(1, C, k, k, generator=g) * 0.1).cuda()
    y, _ = ops.conv_gen((x, m), w, stride=s, pad=1, act=0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.conv_gen((x, m), w, stride=s, pad=1, act=0)
    e1.record(); torch.cuda.synchronize()
    out[(k, s, C)] = y.cpu()
    print(k, s, C, H, W, N, f"{e0.elapsed_time(e1)/20*1e3:.1f} us")
torch.save(out, sys.argv[1])
