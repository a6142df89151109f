"""bf16 channel-last conv (conv_gen_nhwc16) per layer, every variant of its main
loop (ops.conv16_set_variant: 0 register-staged, 1 LDS-DMA ring, 2 / 3 wide-tile
ring of 4 / 8 waves): the launches of one bf16 GAN step at the C4 (T=626) or C5 (--clip-s 8)
shapes -- G forward, VGG19 over generated + target, one D forward -- recorded
as prepared-operand launchers (re-recorded per variant), then each timed alone
(HIP events, median of --reps) and compared with variant 0 (bit-identical
output and BatchNorm partials, else the worst relative difference; the
discriminator's spectral norm updates its weights in every forward, so its
last three convs differ between recordings by construction).

  python tools/conv16_lab.py [--reps 7] [--variants 0,1,2] [--clip-s 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))
import torch  # noqa: E402

from ainp import gan as G, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--variants", default="0,3")
    ap.add_argument("--clip-s", type=float, default=5.0)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--only", type=int, default=-1,
                    help="launch only recorded layer ONLY --reps times with the first "
                         "variant (a rocprofv3 --pmc target); no timing table")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    dev = "cuda"
    B, F = args.batch, 257
    T = int(args.clip_s * 16000) // 128 + 1
    torch.manual_seed(0)
    gen = G.set_compute_dtype(G.PConvUNet().to(dev).train(), "bf16")
    disc = G.set_compute_dtype(G.Discriminator().to(dev).train(), "bf16")
    vgg = G.set_compute_dtype(G.VGGLoss(dev), "bf16")
    x = torch.rand(B, 1, F, T, device=dev) * 3
    m = torch.ones(B, 1, F, T, device=dev)
    m[:, :, :, T // 2:T // 2 + 26] = 0

    orig = ops.conv_gen

    def collect(v):
        """Run one G forward + VGG + D forward under variant v, recording every
        bf16 channel-last conv as a launcher on its prepared operands (the
        weights in v's k order)."""
        recs = []

        def rec(*a, **k):
            res = orig(*a, **k)
            if k.get("bf16"):
                kk = dict(k)
                kk["out"] = None
                la = orig(*a, launcher=True, **kk)
                if callable(la):
                    w = a[1]
                    Cout, Cin, KH, KW = w.shape
                    y = la.out
                    flops = 2.0 * Cout * Cin * KH * KW * y.shape[0] * y.shape[-2] * y.shape[-1]
                    recs.append((tuple(a[0][0].shape), tuple(w.shape), k.get("stride", 1),
                                 tuple(y.shape), flops, la))
            return res

        prev = ops.conv16_set_variant(v)
        ops.conv_gen = rec
        try:
            with torch.no_grad():
                g = gen(x, m)
                vgg(g, x)
                disc(x)
        finally:
            ops.conv_gen = orig
            ops.conv16_set_variant(prev)
        torch.cuda.synchronize()
        return recs

    recs = collect(variants[0])
    print(f"{len(recs)} nhwc16 launches, B={B} T={T}")

    def time_it(fn):
        fn()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    prev = ops.conv16_set_variant(-1)
    if args.only >= 0:
        ops.conv16_set_variant(variants[0])
        for _ in range(args.reps):
            recs[args.only][5]()
        torch.cuda.synchronize()
        ops.conv16_set_variant(prev)
        xs, ws, s, ys, fl, _ = recs[args.only]
        print(f"layer {args.only}: {xs} w{ws} s{s} -> {ys} {fl / 1e9:.1f} GF x {args.reps}")
        return
    ref = {}
    r0 = collect(0)
    ops.conv16_set_variant(0)
    for i, r in enumerate(r0):
        la = r[5]
        la()
        ref[i] = (la.out.clone(), la.stats.clone() if la.stats is not None else None)
    torch.cuda.synchronize()
    res = {v: [] for v in variants}
    ident = {v: 0 for v in variants}
    worst = {v: 0.0 for v in variants}
    for v in variants:
        rv = collect(v)
        assert len(rv) == len(r0)
        ops.conv16_set_variant(v)
        for i, r in enumerate(rv):
            la = r[5]
            la.out.zero_()
            la()
            torch.cuda.synchronize()
            o, st = ref[i]
            same = torch.equal(la.out, o) and (st is None or torch.equal(la.stats, st))
            ident[v] += int(same)
            if not same:
                d = ((la.out - o).abs().max() / o.abs().max().clamp_min(1e-30)).item()
                worst[v] = max(worst[v], d)
            res[v].append(time_it(la))
    ops.conv16_set_variant(prev)
    hdr = "".join(f"  v{v} ms    TF" for v in variants)
    print(f"{'x':24s} {'w':22s} s {'y':22s} {'GF':>7s}{hdr}")
    for i, (xs, ws, s, ys, fl, _) in enumerate(recs):
        cols = "".join(f" {res[v][i]:7.3f} {fl / res[v][i] / 1e9:5.0f}" for v in variants)
        print(f"{str(xs):24s} {str(ws):22s} {s} {str(ys):22s} {fl / 1e9:7.1f}{cols}")
    tf = sum(r[4] for r in recs)
    for v in variants:
        tot = sum(res[v])
        print(f"variant {v}: total {tot:.3f} ms, {tf / tot / 1e9:.0f} TF, bit-identical "
              f"{ident[v]}/{len(recs)}, worst max|d|/max|ref| {worst[v]:.2e}")


if __name__ == "__main__":
    main()
