"""Discriminator weight-gradient probe: im2col16 + gemm_bf16nt_splitk vs the
implicit GEMM ainp_wgrad16_nhwc at the C4 layer shapes, several split counts.

usage: python tools/wgrad_probe.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "ml-audio-inpainting_amd"))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    from ainp import ops
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = "cuda"
    for (N, Cin, H, W, Cout, k, s, p) in [(8, 64, 128, 313, 128, 4, 2, 1),
                                          (8, 128, 64, 156, 256, 4, 2, 1),
                                          (8, 256, 32, 78, 512, 4, 1, 1)]:
        x = torch.randn(N, Cin, H, W, device=dev)
        x16 = ops.to_nhwc16(x)
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        NP = N * Ho * Wo
        ldA = -(-NP // 64) * 64
        gy = torch.randn(N, Cout, Ho, Wo, device=dev)
        gA, _ = ops.d_prep16(gy, 1, None, 0.2, N, Cout, Ho * Wo, ldA, want_gT=False)
        Ncol = Cin * k * k + 1
        S0 = ops._splitk_bf16(Cout, Ncol, ldA, max_split=512)
        col = ops.im2col16(x, k, s, p, ldA)
        t_im = timed(lambda: ops.im2col16(x, k, s, p, ldA), reps)
        t_gm = timed(lambda: ops.gemm_bf16nt_splitk(gA, col, ldA, max_split=512), reps)
        print(f"shape N{N} Cin{Cin} {H}x{W} Cout{Cout} s{s}: NP {NP}, split {S0}: "
              f"im2col16 {t_im:.1f} us, gemm_bf16nt_splitk {t_gm:.1f} us", flush=True)
        for S in sorted({1, 8, 32, S0, 2 * S0}):
            kc = -(-ldA // S // 64) * 64 if S > 1 else ldA
            Sr = -(-ldA // kc)
            G = torch.empty(Sr, Cout, Ncol, device=dev)
            t = timed(lambda: ops._T.wgrad16_nhwc(gA, x16, k, s, p, G, Sr, kc), reps)
            print(f"   wgrad16_nhwc split {Sr:4d}: {t:.1f} us (no slab sum)", flush=True)


if __name__ == "__main__":
    main()
