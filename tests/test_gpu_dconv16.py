"""The bf16 Discriminator backward (csrc/dconv16.hip, gan._d_backward16):
each kernel against a torch restatement of the same arithmetic (bit-exact for
the casts / gathers, fp64-of-bf16-operands for the implicit GEMM), and the
whole D backward of the bf16 configuration against the fp32 reference
gradients (gan_small.npz, made by the reference's networks.py)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("nslab,act,C,want_gT", [(1, True, 64, True), (3, True, 130, True),
                                                 (1, False, 1, True), (2, True, 7, False)])
def test_d_prep16_bit_exact(nslab, act, C, want_gT):
    from ainp import ops
    g = torch.Generator().manual_seed(C + nslab)
    N, H, W = 3, 9, 13
    P = H * W
    ldA = -(-N * P // 64) * 64
    gs = torch.randn(nslab, N, C, H, W, generator=g)
    y = torch.randn(N, C, H, W, generator=g)
    gA, gT = ops.d_prep16(gs.cuda(), nslab, y.cuda() if act else None, 0.2, N, C, P, ldA,
                          want_gT=want_gT)
    ref = gs[0].clone()
    for z in range(1, nslab):
        ref = ref + gs[z]
    if act:
        ref = torch.where(y > 0, ref, ref * 0.2)
    ref16 = ref.bfloat16()
    expA = torch.zeros(C, ldA, dtype=torch.bfloat16)
    expA[:, :N * P] = ref16.permute(1, 0, 2, 3).reshape(C, N * P)
    assert torch.equal(gA.cpu(), expA)
    if want_gT:
        assert torch.equal(gT.cpu(), ref16.permute(0, 2, 3, 1).reshape(N * P, C))
    else:
        assert gT is None


@pytest.mark.parametrize("C,H,W,k,s,p", [(1, 21, 30, 4, 2, 1), (5, 11, 14, 4, 1, 1),
                                         (3, 10, 9, 3, 2, 0), (2, 5, 5, 4, 2, 1),
                                         (3, 41, 700, 4, 2, 1),   # Wo > 256 (row-staged)
                                         (2, 7, 600, 3, 1, 1),
                                         (1, 9, 3000, 4, 2, 1)])  # rows too wide: per-pixel
def test_im2col16_bit_exact(C, H, W, k, s, p):
    from ainp import ops
    g = torch.Generator().manual_seed(H * W)
    N = 2
    x = torch.randn(N, C, H, W, generator=g)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    NP = N * Ho * Wo
    ldA = -(-NP // 64) * 64
    col = ops.im2col16(x.cuda(), k, s, p, ldA).cpu()
    u = F.unfold(x, k, padding=p, stride=s)                 # [N, C*k*k, Ho*Wo]
    exp = torch.zeros(C * k * k + 1, ldA, dtype=torch.bfloat16)
    exp[:-1, :NP] = u.permute(1, 0, 2).reshape(C * k * k, NP).bfloat16()
    exp[-1, :NP] = 1
    assert torch.equal(col, exp)


DGRAD_CASES = [
    # N, Cout, Cin, H, W, k, s, p, nsplit
    (2, 64, 1, 21, 30, 4, 2, 1, 1),       # D layer 1's input gradient (Cin = 1)
    (2, 128, 64, 17, 26, 4, 2, 1, 1),     # odd H: parity classes of unequal size
    (1, 256, 130, 9, 12, 4, 2, 1, 2),     # Cin % 64 != 0, split-K slabs
    (2, 512, 256, 7, 10, 4, 1, 1, 3),     # stride 1 (layer 4), split-K
    (2, 1, 512, 6, 9, 4, 1, 1, 1),        # the logit layer: Cout = 1 (gathered)
    (1, 64, 96, 8, 11, 3, 1, 1, 1),       # k3 s1 (general k % s == 0)
]


@pytest.mark.parametrize("case", DGRAD_CASES)
def test_dgrad16_matches_fp64_of_bf16_operands(case):
    from ainp import ops
    N, Cout, Cin, H, W, k, s, p, S = case
    g = torch.Generator().manual_seed(sum(case))
    w = torch.randn(Cout, Cin, k, k, generator=g) * 0.1
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    gy = torch.randn(N, Cout, Ho, Wo, generator=g)
    scale = torch.tensor([0.37])
    gT = gy.permute(0, 2, 3, 1).contiguous().bfloat16()
    wd = ops.dgrad16_weight(w.cuda(), s, p)
    out = ops.dgrad16(gT.cuda(), wd, Cin, H, W, k, s, p, scale=scale.cuda(), nsplit=S)
    dx = out.sum(0).cpu() if S > 1 else out[0].cpu()
    x = torch.zeros(N, Cin, H, W, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, w.bfloat16().double() * 0.37, stride=s, padding=p)
    y.backward(gy.bfloat16().double())
    assert rel(dx, x.grad) < 1e-5


def test_d_backward16_tracks_reference_gradients(golden_dir, monkeypatch):
    """D step of the small fixture in the bf16 configuration: every parameter
    gradient within 5e-2 relative of the reference's fp32 gradients and no
    further from them than the fp32-staged bf16 loop it replaces
    (AINP_D_BWD16=0) within 2x."""
    from ainp import gan as G
    from golden.gen_golden_gan import SMALL_D
    small = np.load(os.path.join(golden_dir, "gan_small.npz"), allow_pickle=False)

    def run(d16):
        monkeypatch.setattr(G, "D_BWD16", d16)
        D = G.Discriminator(layer_cfg=SMALL_D)
        D.load_state_dict({k[len("d_init/"):]: torch.from_numpy(np.array(small[k])).clone()
                           for k in small.files if k.startswith("d_init/")})
        D = D.cuda().train()
        D.ainp_bf16 = True
        dr = D(torch.from_numpy(small["d_real_in"]).cuda())
        df = D(torch.from_numpy(small["d_fake_in"]).cuda())
        dl = (G.bce_with_logits_const(dr, 1.0) + G.bce_with_logits_const(df, 0.0)) / 2
        dl.backward()
        return {k: p.grad.clone() for k, p in D.named_parameters()}

    new, old = run(True), run(False)
    errs = {k: (rel(new[k], small["d_grad/" + k]), rel(old[k], small["d_grad/" + k]))
            for k in new}
    print("bf16 D grads rel err (dconv16, fp32-staged):", errs)
    for k, (e_new, e_old) in errs.items():
        # bf16 operands: a few % on this small fixture, as the loop it replaces
        assert e_new < 5e-2 and e_new < 2 * e_old + 5e-3, (k, e_new, e_old)


def test_d_backward16_input_gradient(monkeypatch):
    """The input gradient (needs_input_grad[0]) of the bf16 D backward vs fp64
    autograd through the same 1/sigma, default D at a small size: no further
    from it than the fp32-staged bf16 loop (AINP_D_BWD16=0) within 2x."""
    from ainp import gan as G
    torch.manual_seed(3)
    D = G.Discriminator().cuda().eval()      # eval: no power iteration, same sigma each run
    D.ainp_bf16 = True
    x0 = torch.randn(2, 1, 40, 64, device="cuda")
    gout = None
    grads = {}
    for d16 in (True, False):
        monkeypatch.setattr(G, "D_BWD16", d16)
        x = x0.clone().requires_grad_(True)
        out = D(x)
        if gout is None:
            gout = torch.randn_like(out)
        out.backward(gout)
        grads[d16] = x.grad.clone()
    convs = D._convs()
    h = x0.double().cpu().requires_grad_(True)
    a = h
    for i, c in enumerate(convs):
        w = c.weight_orig.detach().double().cpu()
        u, v = c.weight_u.detach().double().cpu(), c.weight_v.detach().double().cpu()
        sigma = torch.dot(u, w.reshape(w.shape[0], -1) @ v)
        k, s, p, act = D._cfg[i]
        a = F.conv2d(a, w / sigma, c.bias.detach().double().cpu(), s, p)
        if act:
            a = F.leaky_relu(a, 0.2)
    a.backward(gout.double().cpu())
    e_new, e_old = rel(grads[True], h.grad), rel(grads[False], h.grad)
    print("bf16 D input grad rel err (dconv16, fp32-staged):", e_new, e_old)
    assert e_new < 2 * e_old + 5e-3, (e_new, e_old)


@pytest.mark.parametrize("case", [c for c in DGRAD_CASES if c[-1] == 1 and c[2] % 4 == 0])
@pytest.mark.parametrize("act", [True, False])
def test_dgrad16_prep_equals_dgrad16_then_d_prep16(case, act):
    """ainp_dgrad16_prep: the lower layer's gA / gT from the data gradient's
    epilogue, bit for bit what ainp_dgrad16 (nsplit 1) + ainp_d_prep16 give
    (LeakyReLU' of y, bf16 rounding, zero gA tail, gT optional)."""
    from ainp import ops
    N, Cout, Cin, H, W, k, s, p, _ = case
    g = torch.Generator().manual_seed(sum(case) + act)
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.1).cuda()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    gT = torch.randn(N, Ho, Wo, Cout, generator=g).bfloat16().cuda()
    y = torch.randn(N, Cin, H, W, generator=g).cuda() if act else None
    scale = torch.tensor([0.37]).cuda()
    wd = ops.dgrad16_weight(w, s, p)
    P = H * W
    ldA = -(-N * P // 64) * 64 + 64          # a tail past N*P
    dx = ops.dgrad16(gT, wd, Cin, H, W, k, s, p, scale=scale, nsplit=1)
    eA, eT = ops.d_prep16(dx, 1, y, 0.2, N, Cin, P, ldA, want_gT=True)
    for want in (True, False):
        gA, gTo = ops.dgrad16_prep(gT, wd, Cin, H, W, k, s, p, y, 0.2, ldA, scale=scale,
                                   want_gT=want)
        torch.cuda.synchronize()
        assert torch.equal(gA.view(torch.int16), eA.view(torch.int16))
        if want:
            assert torch.equal(gTo.view(torch.int16), eT.view(torch.int16))
        else:
            assert gTo is None


def test_d_backward16_prep_fused_is_bit_identical(monkeypatch):
    """The bf16 D backward with the fused data-gradient epilogue
    (AINP_D_PREP_FUSED) gives the same parameter and input gradients, bit for
    bit, as dgrad16 + d_prep16."""
    from ainp import gan as G
    torch.manual_seed(5)
    D = G.Discriminator().cuda().eval()
    D.ainp_bf16 = True
    x0 = torch.randn(2, 1, 64, 96, device="cuda")

    def run(fused):
        monkeypatch.setattr(G, "D_PREP_FUSED", fused)
        for q in D.parameters():
            q.grad = None
        x = x0.clone().requires_grad_(True)
        out = D(x)
        out.backward(torch.ones_like(out))
        return [q.grad.clone() for q in D.parameters()] + [x.grad.clone()]

    a, b = run(True), run(False)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("case", [
    # N, Cin, H, W, Cout, k, s, p, max_split
    (2, 64, 21, 30, 128, 4, 2, 1, 512),     # D layer 1-like, split-K
    (1, 128, 17, 26, 256, 4, 2, 1, 1),      # odd sizes, unsplit
    (2, 256, 9, 12, 200, 4, 1, 1, 512),     # stride 1, ragged Cout tile
    (1, 8, 7, 9, 64, 3, 1, 1, 4),           # 3x3, 8 channels (one chunk per tap)
])
def test_wgrad16_nhwc_equals_im2col16_gemm(case):
    """ainp_wgrad16_nhwc (implicit GEMM over the channel-last bf16 input) is
    bit-identical to im2col16 + gemm_bf16nt_splitk with the same split."""
    from ainp import ops
    N, Cin, H, W, Cout, k, s, p, ms = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(N, Cin, H, W, generator=g).cuda()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    NP = N * Ho * Wo
    ldA = -(-NP // 64) * 64
    gy = torch.randn(N, Cout, Ho, Wo, generator=g).cuda()
    gA, _ = ops.d_prep16(gy, 1, None, 0.2, N, Cout, Ho * Wo, ldA, want_gT=False)
    col = ops.im2col16(x, k, s, p, ldA)
    ref = ops.gemm_bf16nt_splitk(gA, col, ldA, max_split=ms)
    got = ops.wgrad16_nhwc(gA, ops.to_nhwc16(x), k, s, p, max_split=ms)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert torch.equal(got, ref)


def test_d_backward16_wgrad_nhwc_is_bit_identical(monkeypatch):
    """The bf16 D backward with implicit-GEMM weight gradients
    (AINP_WGRAD16_NHWC) gives the same gradients, bit for bit, as im2col16 +
    gemm_bf16nt."""
    from ainp import gan as G
    torch.manual_seed(6)
    D = G.Discriminator().cuda().eval()
    D.ainp_bf16 = True
    x0 = torch.randn(2, 1, 64, 96, device="cuda")

    def run(nhwc):
        monkeypatch.setattr(G, "WGRAD16_NHWC", nhwc)   # read by the forward too
        for q in D.parameters():
            q.grad = None
        x = x0.clone().requires_grad_(True)
        out = D(x)
        out.backward(torch.ones_like(out))
        return [q.grad.clone() for q in D.parameters()] + [x.grad.clone()]

    a, b = run(True), run(False)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_d_backward16_side_stream_weight_grads_bit_identical(monkeypatch):
    """The discriminator's weight gradients on the side stream
    (AINP_D_WGRAD_SIDE=1, opt-in) equal the in-line ones bit for bit, with the
    data gradient chain running beside them."""
    from ainp import gan as G
    torch.manual_seed(9)
    D = G.Discriminator().cuda().eval()
    D.ainp_bf16 = True
    x0 = torch.randn(3, 1, 80, 120, device="cuda")

    def run(side):
        monkeypatch.setattr(G, "D_WGRAD_SIDE", side)
        for q in D.parameters():
            q.grad = None
        x = x0.clone().requires_grad_(True)
        out = D(x)
        out.backward(torch.ones_like(out))
        return [q.grad.clone() for q in D.parameters()] + [x.grad.clone()]

    a, b = run(True), run(False)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
