"""GPU parity of the GAN path against the oracle
(oracle/gan_ref.py, pinned in test_cpu_oracle_gan.py) and the fixtures made by
the reference's networks.py.  Tolerance: 1e-4 relative L2 (fp32, north_star);
masks bit-exact."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import gan_ref as R

pytestmark = pytest.mark.gpu
TOL = 1e-4


def rel(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def small(golden_dir):
    return np.load(os.path.join(golden_dir, "gan_small.npz"), allow_pickle=False)


def _sd(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.array(g[k])).clone()
            for k in g.files if k.startswith(prefix)}


# ------------------------------------------------------------- conv_gen
CONV_CASES = [
    # N, C0, C1, Hin, Win, up0, Cout, k, s, p, masks, bias, ratio, scale, act
    (2, 64, 0, 17, 23, False, 96, 3, 1, 1, True, False, True, False, 0),      # fast, 1 source
    (2, 32, 32, 16, 20, True, 48, 3, 1, 1, True, False, True, False, 0),      # fast, up + skip
    (2, 2, 0, 33, 40, False, 64, 7, 2, 3, True, False, True, False, 0),       # generic k7 s2
    (2, 64, 1, 24, 30, True, 64, 3, 1, 1, True, True, True, False, 2),        # generic concat
    (2, 1, 0, 30, 50, False, 16, 4, 2, 1, False, True, False, True, 2),       # D layer 1
    (1, 128, 0, 13, 21, False, 70, 5, 2, 2, True, False, True, False, 0),     # k5 s2, Cout%64
    (2, 64, 0, 12, 14, False, 32, 3, 1, 1, False, True, False, False, 1),     # VGG-like
    (2, 512, 512, 6, 10, True, 512, 3, 1, 1, True, False, True, False, 0),    # U-Net bottleneck: split-K
    (3, 256, 0, 7, 9, False, 64, 3, 2, 1, True, True, True, False, 2),        # BM=64, split-K
    (1, 512, 0, 5, 7, False, 200, 3, 1, 1, True, True, True, True, 2),        # split-K, odd NP, Cout%64
]


def _conv_ref(x0, m0, x1, m1, Hin, Win, w, k, s, p, bias, ratio, scale, act):
    a = x0
    if a.shape[2] != Hin:
        a = F.interpolate(a, size=(Hin, Win), mode="nearest")
        mm = F.interpolate(m0.unsqueeze(1), size=(Hin, Win), mode="nearest") if m0 is not None else None
    else:
        mm = m0.unsqueeze(1) if m0 is not None else None
    if mm is not None:
        a = a * mm
    if x1 is not None:
        b = x1 * (m1.unsqueeze(1) if m1 is not None else 1.0)
        a = torch.cat([a, b], 1)
    y = F.conv2d(a.double(), w.double(), None, s, p)
    if scale is not None:
        y = y * scale.double()
    if ratio is not None:
        y = y * ratio.double().unsqueeze(1)
    if bias is not None:
        y = y + bias.double().view(1, -1, 1, 1)
    pre = y
    if act == 1:
        y = F.relu(y)
    elif act == 2:
        y = F.leaky_relu(y, 0.2)
    elif act == 3:
        y = torch.tanh(y)
    return y, pre


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_gen_matches_torch(case):
    from ainp import ops
    N, C0, C1, Hin, Win, up0, Cout, k, s, p, masks, hb, hr, hs, act = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    H0, W0 = (Hin // 2, Win // 2) if up0 else (Hin, Win)
    x0 = torch.randn(N, C0, H0, W0, generator=g)
    m0 = (torch.rand(N, H0, W0, generator=g) > 0.3).float() if masks else None
    x1 = torch.randn(N, C1, Hin, Win, generator=g) if C1 else None
    m1 = (torch.rand(N, Hin, Win, generator=g) > 0.3).float() if (masks and C1) else None
    w = torch.randn(Cout, C0 + C1, k, k, generator=g) * 0.1
    Ho, Wo = (Hin + 2 * p - k) // s + 1, (Win + 2 * p - k) // s + 1
    bias = torch.randn(Cout, generator=g) if hb else None
    ratio = torch.rand(N, Ho, Wo, generator=g) * 3 if hr else None
    scale = torch.tensor([0.7]) if hs else None
    d = lambda t: None if t is None else t.cuda()
    y, stats = ops.conv_gen((d(x0), d(m0)), d(w), src1=(d(x1), d(m1)) if C1 else None, Hin=Hin,
                            Win=Win, stride=s, pad=p, bias=d(bias), ratio=d(ratio),
                            scale=d(scale), act=act, want_stats=True)
    yr, pre = _conv_ref(x0, m0, x1, m1, Hin, Win, w, k, s, p, bias, ratio, scale, act)
    assert y.shape == yr.shape
    assert rel(y, yr) < 1e-5
    st = stats.double().sum(0).cpu()
    assert rel(st[0], pre.sum((0, 2, 3))) < 1e-5
    assert rel(st[1], (pre * pre).sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_gen_bf16_matches_torch(case):
    """AINP_CONV_BF16: gathered (masked, upsampled, concatenated) activations
    and weights rounded to bf16, fp32 accumulation, fp32 epilogue -- vs an
    fp64 convolution of the bf16-rounded operands."""
    from ainp import ops
    N, C0, C1, Hin, Win, up0, Cout, k, s, p, masks, hb, hr, hs, act = case
    g = torch.Generator().manual_seed(hash(case) % 1000 + 7)
    H0, W0 = (Hin // 2, Win // 2) if up0 else (Hin, Win)
    x0 = torch.randn(N, C0, H0, W0, generator=g)
    m0 = (torch.rand(N, H0, W0, generator=g) > 0.3).float() if masks else None
    x1 = torch.randn(N, C1, Hin, Win, generator=g) if C1 else None
    m1 = (torch.rand(N, Hin, Win, generator=g) > 0.3).float() if (masks and C1) else None
    w = torch.randn(Cout, C0 + C1, k, k, generator=g) * 0.1
    Ho, Wo = (Hin + 2 * p - k) // s + 1, (Win + 2 * p - k) // s + 1
    bias = torch.randn(Cout, generator=g) if hb else None
    ratio = torch.rand(N, Ho, Wo, generator=g) * 3 if hr else None
    scale = torch.tensor([0.7]) if hs else None
    d = lambda t: None if t is None else t.cuda()  # noqa: E731
    y, _ = ops.conv_gen((d(x0), d(m0)), d(w), src1=(d(x1), d(m1)) if C1 else None, Hin=Hin,
                        Win=Win, stride=s, pad=p, bias=d(bias), ratio=d(ratio), scale=d(scale),
                        act=act, bf16=True)
    bf = lambda t: None if t is None else t.bfloat16().float()  # noqa: E731
    # mask products are exact (0/1), so rounding x before or after masking agrees
    yr, _ = _conv_ref(bf(x0), m0, bf(x1), m1, Hin, Win, bf(w), k, s, p, bias, ratio, scale, act)
    assert rel(y, yr) < 2e-5
    y32, _ = _conv_ref(x0, m0, x1, m1, Hin, Win, w, k, s, p, bias, ratio, scale, act)
    assert rel(y, y32) > 1e-5          # a bf16 result, not the fp32-accurate one


SMALL_C_CASES = [
    # N, C0, C1, Hin, Win, up0, Cout, k, s, p, masks, bias, ratio, scale, act
    (2, 1, 1, 33, 40, False, 64, 7, 2, 3, True, False, True, False, 0),       # U-Net enc1
    (2, 64, 1, 24, 30, True, 64, 3, 1, 1, True, True, True, False, 2),        # final pc1
    (2, 3, 0, 20, 22, False, 64, 3, 1, 1, False, True, False, False, 1),      # VGG conv1_1
    (2, 2, 0, 30, 50, False, 16, 4, 2, 1, False, True, False, True, 2),       # D layer 1
    (1, 5, 32, 9, 11, True, 130, 3, 1, 1, True, False, True, False, 2),       # C0 small + up
    (2, 256, 1, 6, 10, True, 512, 3, 1, 1, True, False, True, False, 0),      # split-K, padded
]


@pytest.mark.parametrize("case", SMALL_C_CASES)
def test_conv_gen_nhwc16_small_channel_sources(case, monkeypatch):
    """bf16 channel-last conv with sources of C % 32 != 0 (k-values gathered
    element-wise into zero-padded tiles), forced for every case, with BN
    statistics: vs an fp64 convolution of the bf16-rounded operands."""
    from ainp import ops
    monkeypatch.setattr(ops, "CONV_NHWC16_SMALL", "all")
    N, C0, C1, Hin, Win, up0, Cout, k, s, p, masks, hb, hr, hs, act = case
    g = torch.Generator().manual_seed(hash(case) % 1000 + 11)
    H0, W0 = (Hin // 2, Win // 2) if up0 else (Hin, Win)
    x0 = torch.randn(N, C0, H0, W0, generator=g)
    m0 = (torch.rand(N, H0, W0, generator=g) > 0.3).float() if masks else None
    x1 = torch.randn(N, C1, Hin, Win, generator=g) if C1 else None
    m1 = (torch.rand(N, Hin, Win, generator=g) > 0.3).float() if (masks and C1) else None
    w = torch.randn(Cout, C0 + C1, k, k, generator=g) * 0.1
    Ho, Wo = (Hin + 2 * p - k) // s + 1, (Win + 2 * p - k) // s + 1
    bias = torch.randn(Cout, generator=g) if hb else None
    ratio = torch.rand(N, Ho, Wo, generator=g) * 3 if hr else None
    scale = torch.tensor([0.7]) if hs else None
    d = lambda t: None if t is None else t.cuda()  # noqa: E731
    y, stats = ops.conv_gen((d(x0), d(m0)), d(w), src1=(d(x1), d(m1)) if C1 else None, Hin=Hin,
                            Win=Win, stride=s, pad=p, bias=d(bias), ratio=d(ratio),
                            scale=d(scale), act=act, want_stats=True, bf16=True)
    bf = lambda t: None if t is None else t.bfloat16().float()  # noqa: E731
    yr, pre = _conv_ref(bf(x0), m0, bf(x1), m1, Hin, Win, bf(w), k, s, p, bias, ratio, scale, act)
    assert y.shape == yr.shape
    assert rel(y, yr) < 2e-5
    st = stats.double().sum(0).cpu()
    assert rel(st[0], pre.sum((0, 2, 3))) < 2e-5
    assert rel(st[1], (pre * pre).sum((0, 2, 3))) < 2e-5
    wt = ops.conv_weight_nhwc16(d(w), C0, C1)
    assert wt.shape[1] == ops.nhwc16_seg(C0, k * k) + ops.nhwc16_seg(C1, k * k)
    assert wt.shape[1] % 32 == 0


VARIANT_CASES = [
    # N, C0, C1, Hin, Win, up0, Cout, k, s, p, stats
    (2, 64, 1, 24, 30, True, 64, 3, 1, 1, True),        # final pc1 (expanded source, Cout 64)
    (2, 64, 64, 40, 52, True, 128, 3, 1, 1, True),      # decoder block, Cout 128
    (2, 128, 0, 37, 45, False, 256, 5, 2, 2, True),     # encoder 5x5 stride 2, Cout 256
    (2, 256, 256, 12, 20, True, 512, 3, 1, 1, True),    # decoder 512, two 256-row co tiles
    (1, 512, 512, 6, 10, True, 512, 3, 1, 1, True),     # split-K bottleneck
    (3, 96, 0, 19, 23, False, 100, 3, 1, 1, True),      # ragged Cout and pixel tails
    (2, 3, 0, 20, 22, False, 64, 3, 1, 1, False),       # VGG conv1_1 (expanded)
    (2, 64, 0, 28, 28, False, 200, 4, 2, 1, False),     # D-like 4x4 stride 2
]


@pytest.mark.parametrize("case", VARIANT_CASES)
def test_conv_gen_nhwc16_variants_bit_identical(case, monkeypatch):
    """The main loops of the bf16 channel-last conv (ainp_conv16_set_variant:
    register-staged, LDS-DMA ring, wide-tile ring of 4 or 8 waves) run the same per-output MFMA
    chain: outputs and BatchNorm partials are bit-identical."""
    from ainp import ops
    monkeypatch.setattr(ops, "CONV_NHWC16_SMALL", "all")
    N, C0, C1, Hin, Win, up0, Cout, k, s, p, want = case
    g = torch.Generator().manual_seed(hash(case) % 1000 + 3)
    H0, W0 = (Hin // 2, Win // 2) if up0 else (Hin, Win)
    d = lambda t: None if t is None else t.cuda()  # noqa: E731
    x0 = d(torch.randn(N, C0, H0, W0, generator=g))
    m0 = d((torch.rand(N, H0, W0, generator=g) > 0.3).float())
    x1 = d(torch.randn(N, C1, Hin, Win, generator=g)) if C1 else None
    m1 = d((torch.rand(N, Hin, Win, generator=g) > 0.3).float()) if C1 else None
    w = d(torch.randn(Cout, C0 + C1, k, k, generator=g) * 0.1)
    Ho, Wo = (Hin + 2 * p - k) // s + 1, (Win + 2 * p - k) // s + 1
    bias = d(torch.randn(Cout, generator=g))
    ratio = d(torch.rand(N, Ho, Wo, generator=g) * 3)
    outs = {}
    prev = ops.conv16_set_variant(-1)
    try:
        for v in (0, 1, 2, 3):
            ops.conv16_set_variant(v)
            y, st = ops.conv_gen((x0, m0), w, src1=(x1, m1) if C1 else None, Hin=Hin, Win=Win,
                                 stride=s, pad=p, bias=bias, ratio=ratio, act=ops.ACT_LEAKY,
                                 want_stats=want, bf16=True)
            torch.cuda.synchronize()
            outs[v] = (y.cpu(), st.cpu() if st is not None else None)
    finally:
        ops.conv16_set_variant(prev)
    for v in (1, 2, 3):
        assert torch.equal(outs[v][0], outs[0][0]), v
        if want:
            assert torch.equal(outs[v][1], outs[0][1]), v


@pytest.mark.parametrize("case", [
    (2, 64, 28, 28, 64, 3, 1, 1, 1),                  # VGG-like ReLU, Cout 64 (register-staged)
    (2, 128, 30, 26, 256, 4, 2, 1, 2),                # D-like LeakyReLU 4x4 stride 2, wide tile
    (1, 512, 6, 10, 512, 3, 1, 1, 1),                 # split-K epilogue kernel
    (2, 64, 30, 22, 128, 3, 1, 1, 2),                 # wide tile, 128 channels
    (1, 96, 17, 23, 200, 3, 1, 1, 1),                 # ragged last channel tile
    (1, 512, 5, 7, 200, 3, 1, 1, 2),                  # split-K, odd pixel count, Cout % 64
    (3, 256, 7, 9, 96, 3, 1, 1, 0),                   # split-K, Cout % 64, three images
])
def test_conv_gen_epilogue_nhwc16_copy(case):
    """out16: the conv epilogue's bf16 channel-last copy of y equals
    to_nhwc16(y) bit for bit, and inside an nhwc16_memo scope to_nhwc16(y)
    returns it (the VGG19 / discriminator chains use it as the next conv's
    source)."""
    from ainp import ops
    N, C, H, W, Cout, k, s, p, act = case
    g = torch.Generator().manual_seed(17 + Cout)
    x = torch.randn(N, C, H, W, generator=g).cuda()
    w = (torch.randn(Cout, C, k, k, generator=g) * 0.05).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    with ops.nhwc16_memo():
        y, st = ops.conv_gen((x, None), w, stride=s, pad=p, bias=b, act=act, want_stats=True,
                             bf16=True, out16=True)
        y16 = ops.to_nhwc16(y)
    ref = ops.to_nhwc16(y)
    torch.cuda.synchronize()
    assert torch.equal(y16.view(torch.int16), ref.view(torch.int16))
    y2, st2 = ops.conv_gen((x, None), w, stride=s, pad=p, bias=b, act=act, want_stats=True,
                           bf16=True)
    assert torch.equal(y, y2) and torch.equal(st, st2)   # y / stats unchanged by out16


@pytest.mark.parametrize("case", [
    (2, 1, 37, 70, 64, 4, 2, 1, 2),     # the discriminator's first conv (LeakyReLU)
    (2, 3, 20, 26, 64, 3, 1, 1, 1),     # VGG19 conv1_1 (ReLU)
    (1, 2, 9, 13, 16, 3, 1, 1, 0),      # 16 channels, no activation
])
def test_conv_gen_direct_kernel_nhwc16_copy(case):
    """out16 on the few-input-channel direct kernel (ainp_conv_gen_fwd_out16):
    its bf16 channel-last copy equals to_nhwc16(y) bit for bit, to_nhwc16
    finds it in the memo, and y is unchanged."""
    from ainp import ops
    N, C, H, W, Cout, k, s, p, act = case
    g = torch.Generator().manual_seed(5 + Cout + C)
    x = torch.randn(N, C, H, W, generator=g).cuda()
    w = (torch.randn(Cout, C, k, k, generator=g) * 0.2).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    assert ops._direct_route(C, 0, H, W, H, W, k, k, Cout, False)
    with ops.nhwc16_memo():
        y, _ = ops.conv_gen((x, None), w, stride=s, pad=p, bias=b, act=act, bf16=True, out16=True)
        key = (y.data_ptr(), tuple(y.shape), y._version, 0, -1)
        assert key in ops._NHWC_MEMO
        y16 = ops.to_nhwc16(y)
        assert y16 is ops._NHWC_MEMO[key][0]
    ref = ops.to_nhwc16(y)
    torch.cuda.synchronize()
    assert torch.equal(y16.view(torch.int16), ref.view(torch.int16))
    y2, _ = ops.conv_gen((x, None), w, stride=s, pad=p, bias=b, act=act, bf16=True)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("case", [
    # N, C, Hs, Ws, Hin, Win, k, stride, pad, mask
    (2, 1, 40, 150, 40, 150, 7, 2, 3, True),     # the U-Net's first conv (7x7 / 2)
    (2, 1, 21, 70, 21, 70, 3, 1, 1, True),       # the final PartialConv's input source
    (1, 2, 10, 33, 20, 66, 3, 1, 1, True),       # nearest x2 resampling, 2 channels
    (1, 3, 9, 14, 20, 30, 5, 2, 2, False),       # general nearest resampling, no mask
    (1, 4, 12, 300, 12, 300, 7, 2, 3, False),    # wide rows (several pixel blocks)
])
def test_im2col_nhwc16_matches_unfold(case):
    """ainp_im2col_nhwc16: bf16 rows [N*Ho*Wo][seg], k = tap*C + ci, of the
    source times its mask plane resampled to Hin x Win (index i*Hs//Hin), zero
    past KK*C -- equal bit for bit to torch's unfold of the same values."""
    from ainp import ops
    N, C, Hs, Ws, Hin, Win, k, st, pd, use_m = case
    g = torch.Generator().manual_seed(Hs * Ws + C)
    x = torch.randn(N, C, Hs, Ws, generator=g)
    m = (torch.rand(N, Hs, Ws, generator=g) > 0.3).float() if use_m else None
    Ho, Wo = (Hin + 2 * pd - k) // st + 1, (Win + 2 * pd - k) // st + 1
    KK = k * k
    seg = ops.nhwc16_seg(C, KK)
    out = torch.empty(N * Ho * Wo, seg, dtype=torch.bfloat16, device="cuda")
    ops._T.im2col_nhwc16(x.cuda(), m.cuda() if use_m else None, Hin, Win, k, k, st, pd, out)
    xm = x * m[:, None] if use_m else x
    sy, sx = (torch.arange(Hin) * Hs) // Hin, (torch.arange(Win) * Ws) // Win
    xr = xm[:, :, sy][:, :, :, sx]
    u = torch.nn.functional.unfold(xr, k, padding=pd, stride=st)       # [N, C*KK, L]
    u = u.view(N, C, KK, Ho * Wo).permute(0, 3, 2, 1).reshape(N * Ho * Wo, KK * C)
    exp = torch.zeros(N * Ho * Wo, seg, dtype=torch.bfloat16)
    exp[:, :KK * C] = u.bfloat16()
    assert torch.equal(out.cpu().view(torch.int16), exp.view(torch.int16))


@pytest.mark.parametrize("shape", [(2, 64, 24, 30), (1, 200, 9, 131), (3, 3, 5, 7)])
def test_maxpool2_nhwc16_copy(shape):
    """ainp_maxpool2_nhwc16: y equals ainp_maxpool2's, the copy equals
    to_nhwc16(y) bit for bit and is what to_nhwc16 finds in the memo (odd H / W:
    the last row / column dropped; C not a multiple of 64 / 2)."""
    from ainp import ops
    x = torch.randn(*shape, generator=torch.Generator().manual_seed(shape[1])).cuda()
    with ops.nhwc16_memo():
        y = ops.maxpool2(x, out16=True)
        y16 = ops.to_nhwc16(y)
        key = (y.data_ptr(), tuple(y.shape), y._version, 0, -1)
        assert y16 is ops._NHWC_MEMO[key][0]
    assert torch.equal(y, ops.maxpool2(x))
    assert torch.equal(y, torch.nn.functional.max_pool2d(x, 2))
    torch.cuda.synchronize()
    assert torch.equal(y16.view(torch.int16), ops.to_nhwc16(y).view(torch.int16))


@pytest.mark.parametrize("k,s,p,crop,act,C,H,W", [
    (3, 1, 1, (25, 30), 3, 64, 32, 40), (4, 1, 1, None, 0, 64, 32, 40),
    (4, 2, 1, None, 2, 64, 32, 40),
    # LDS-tiled path (stride 1, 3x3 / 4x4): ragged channel chunks and tiles
    (3, 1, 1, (37, 66), 3, 40, 37, 70), (4, 1, 1, None, 0, 200, 13, 35),
    (3, 1, 1, None, 0, 7, 17, 33),
    # large planes (the generator's last PartialConv2d is 64 x 384 x 640)
    (3, 1, 1, (257, 590), 3, 9, 260, 600), (4, 1, 1, None, 2, 12, 200, 700)])
def test_conv_gen_cout1(k, s, p, crop, act, C, H, W):
    from ainp import ops
    g = torch.Generator().manual_seed(5)
    N = 2 if H < 100 else 4
    x = torch.randn(N, C, H, W, generator=g)
    m = (torch.rand(N, H, W, generator=g) > 0.2).float()
    w = torch.randn(1, C, k, k, generator=g) * 0.1
    b = torch.randn(1, generator=g)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    ratio = torch.rand(N, Ho, Wo, generator=g) + 0.5
    sc = torch.tensor([1.3])
    y, _ = ops.conv_gen((x.cuda(), m.cuda()), w.cuda(), stride=s, pad=p, bias=b.cuda(),
                        ratio=ratio.cuda(), scale=sc.cuda(), act=act, crop=crop)
    yr, _ = _conv_ref(x, m, None, None, H, W, w, k, s, p, b, ratio, sc, act)
    yr = yr[:, 0]
    if crop is not None:
        yr = yr[:, :crop[0], :crop[1]]
    else:
        y = y[:, 0]
    assert rel(y, yr) < 1e-5


@pytest.mark.parametrize("k,s,p,C,H,W,nslab,leaky", [
    (4, 1, 1, 512, 31, 77, 1, False),     # the C4 logit conv
    (4, 2, 1, 64, 21, 33, 2, True),       # split-K slabs + LeakyReLU' folded in
    (3, 1, 1, 7, 9, 13, 1, True)])
def test_wgrad_cout1_matches_torch(k, s, p, C, H, W, nslab, leaky):
    """ainp_wgrad_cout1 against torch's fp32 conv weight/bias gradient."""
    from ainp import ops
    g = torch.Generator().manual_seed(11)
    N = 3
    x = torch.randn(N, C, H, W, generator=g)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    gs = torch.randn(nslab, N, 1, Ho, Wo, generator=g)
    y = torch.randn(N, 1, Ho, Wo, generator=g) if leaky else None
    gr = gs.sum(0)
    if leaky:
        gr = torch.where(y > 0, gr, gr * 0.2)
    w = torch.zeros(1, C, k, k, requires_grad=True)
    b = torch.zeros(1, requires_grad=True)
    torch.nn.functional.conv2d(x, w, b, stride=s, padding=p).backward(gr)
    gw = ops.wgrad_cout1(x.cuda(), gs.cuda().contiguous(), nslab,
                         None if y is None else y.cuda(), 0.2, k, s, p).cpu()
    assert rel(gw[0, :-1], w.grad.reshape(-1)) < 1e-5
    assert abs(gw[0, -1] - b.grad[0]) <= 1e-4 * max(1.0, abs(b.grad[0]))


# ------------------------------------------------------------- partial conv
def test_partial_conv_fixture_cases(small):
    from ainp import gan as G
    for ci in range(4):
        cin, cout, k, s, p, hb = [int(v) for v in small[f"pc{ci}/cfg"]]
        pc = G.PartialConv2d(cin, cout, k, s, p, bias=bool(hb))
        with torch.no_grad():
            pc.conv.weight.copy_(torch.from_numpy(small[f"pc{ci}/w"]))
            if hb:
                pc.bias.copy_(torch.from_numpy(small[f"pc{ci}/b"]))
        pc = pc.cuda()
        y, um = pc(torch.from_numpy(small[f"pc{ci}/x"]).cuda(), torch.from_numpy(small[f"pc{ci}/m"]).cuda())
        assert rel(y, small[f"pc{ci}/y"]) < TOL, ci
        np.testing.assert_array_equal(um.cpu().numpy(), small[f"pc{ci}/um"])


# ------------------------------------------------------------- generator
def test_generator_small_matches_reference(small):
    from ainp import gan as G
    from golden.gen_golden_gan import SMALL_DEC, SMALL_ENC, SMALL_FINAL
    m = G.PConvUNet(enc_layer_cfg=SMALL_ENC, dec_layer_cfg=SMALL_DEC, final_dec_cfg=SMALL_FINAL)
    m.load_state_dict(_sd(small, "g_init/"))
    m = m.cuda().train()
    y = m(torch.from_numpy(small["g_x"]).cuda(), torch.from_numpy(small["g_mask"]).cuda())
    assert y.shape == small["g_y"].shape
    assert rel(y, small["g_y"]) < TOL
    after = _sd(small, "g_after/")
    sd = m.state_dict()
    for k, v in after.items():
        if "running" in k:
            assert rel(sd[k], v) < TOL, k
        elif k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(v)
    # eval mode uses the running statistics: compare with the oracle
    m.eval()
    pe = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    ye = m(torch.from_numpy(small["g_x"]).cuda(), torch.from_numpy(small["g_mask"]).cuda())
    with torch.no_grad():
        yr = R.generator(pe, torch.from_numpy(small["g_x"]), torch.from_numpy(small["g_mask"]),
                         False, SMALL_ENC, SMALL_DEC)
    assert rel(ye, yr) < TOL


def test_generator_full_matches_reference(golden_dir):
    from ainp import gan as G
    g = np.load(os.path.join(golden_dir, "gan_full.npz"), allow_pickle=False)
    torch.manual_seed(0)
    m = G.PConvUNet().cuda().train()
    y = m(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["mask"]).cuda())
    yf = y.detach().cpu().numpy().reshape(-1)
    assert rel(yf[::97], g["y_sample"]) < TOL
    assert abs(np.linalg.norm(yf.astype(np.float64)) - g["y_norm"][0]) < TOL * g["y_norm"][0]


# ------------------------------------------------------------- discriminator
def test_discriminator_step_matches_reference(small):
    from ainp import gan as G
    from ainp.optim import Adam
    from golden.gen_golden_gan import SMALL_D
    D = G.Discriminator(layer_cfg=SMALL_D)
    D.load_state_dict(_sd(small, "d_init/"))
    D = D.cuda().train()
    opt = Adam(D.parameters(), lr=2e-4, betas=(0.5, 0.999))
    opt.zero_grad()
    dr = D(torch.from_numpy(small["d_real_in"]).cuda())
    after1 = _sd(small, "d_after_fwd1/")
    sd = D.state_dict()
    for k in after1:
        if k.endswith("weight_u") or k.endswith("weight_v"):
            assert rel(sd[k], after1[k]) < 1e-5, k
    lr_ = G.bce_with_logits_const(dr, 1.0)
    df = D(torch.from_numpy(small["d_fake_in"]).cuda())
    lf = G.bce_with_logits_const(df, 0.0)
    dl = (lr_ + lf) / 2
    dl.backward()
    assert rel(dr, small["d_real_logits"]) < 1e-5
    assert rel(df, small["d_fake_logits"]) < 1e-5
    assert abs(dl.item() - small["d_loss"][0]) < 1e-5 * abs(small["d_loss"][0])
    for k, p in D.named_parameters():
        assert rel(p.grad, small["d_grad/" + k]) < TOL, k
    opt.step()
    after = _sd(small, "d_after_step/")
    sd = D.state_dict()
    for k, v in after.items():
        assert rel(sd[k], v) < 1e-5, k


def test_discriminator_full_logits(golden_dir):
    from ainp import gan as G
    g = np.load(os.path.join(golden_dir, "gan_full.npz"), allow_pickle=False)
    torch.manual_seed(1)
    D = G.Discriminator().cuda().train()
    with torch.no_grad():
        logits = D(torch.from_numpy(g["x"]).cuda())
    assert rel(logits, g["d_logits"]) < TOL


# ------------------------------------------------------------- VGG + losses
def _vgg_pair(seed=0):
    from ainp import gan as G
    pv = R.vgg19_init(seed)
    v = G.VGGLoss("cuda")
    v.vgg_layers.load_state_dict({k: t for k, t in pv.items()}, strict=False)
    return v, pv


def test_vgg_prepare_matches_oracle():
    from ainp import gan as G
    g = torch.Generator().manual_seed(3)
    gen = torch.tanh(torch.randn(2, 1, 257, 626, generator=g))
    tgt = torch.rand(2, 1, 257, 626, generator=g) * 4 - 0.5
    v = G.VGGLoss("cuda")
    for x, is_gen in ((gen, True), (tgt, False)):
        ours = v._prepare(x.cuda(), is_gen)
        ref = R.vgg_prepare(x, is_gen)
        assert (ours.cpu() - ref).abs().max().item() < 2e-5


def test_vgg_losses_match_oracle():
    g = torch.Generator().manual_seed(4)
    gen = torch.tanh(torch.randn(2, 1, 257, 626, generator=g))
    tgt = torch.rand(2, 1, 257, 626, generator=g) * 3
    v, pv = _vgg_pair(0)
    perc, style = v(gen.cuda(), tgt.cuda())
    with torch.no_grad():
        rp, rs = R.vgg_losses(pv, gen, tgt)
    assert abs(perc.item() - rp.item()) <= TOL * abs(rp.item())
    assert abs(style.item() - rs.item()) <= TOL * abs(rs.item())


def test_calculate_losses_match_oracle():
    from ainp import gan as G
    g = torch.Generator().manual_seed(6)
    gen = torch.tanh(torch.randn(2, 1, 257, 626, generator=g))
    orig = torch.rand(2, 1, 257, 626, generator=g) * 3
    mask = torch.ones(2, 1, 257, 626)
    mask[:, :, :, 300:326] = 0
    d_fake = torch.randn(2, 1, 30, 76, generator=g)
    cfg = {"training": dict(R.LAMBDAS)}
    v, pv = _vgg_pair(1)
    ours = G.calculate_losses(cfg, gen.cuda(), orig.cuda(), mask.cuda(), d_fake.cuda(), v)
    with torch.no_grad():
        ref = R.generator_losses(gen, orig, mask, d_fake, pv)
    for k in ref:
        assert abs(ours[k].item() - ref[k].item()) <= TOL * max(abs(ref[k].item()), 1e-6), k


# ------------------------------------------------------------- full GAN step
def test_gan_step_matches_oracle(small):
    from ainp.gan_train import GanTrainer
    from golden.gen_golden_gan import SMALL_D, SMALL_DEC, SMALL_ENC, SMALL_FINAL
    from ainp import gan as G
    Gm = G.PConvUNet(enc_layer_cfg=SMALL_ENC, dec_layer_cfg=SMALL_DEC, final_dec_cfg=SMALL_FINAL)
    Gm.load_state_dict(_sd(small, "g_init/"))
    Dm = G.Discriminator(layer_cfg=SMALL_D)
    Dm.load_state_dict(_sd(small, "d_init/"))
    cfg = {"training": dict(R.LAMBDAS, g_lr=2e-4, d_lr=2e-4, b1=0.5, b2=0.999)}
    tr = GanTrainer(cfg, Gm.cuda(), Dm.cuda(), vgg=None)
    orig = torch.from_numpy(small["d_real_in"])
    imp = torch.from_numpy(small["g_x"])
    mask = torch.from_numpy(small["g_mask"])
    out = tr.step(orig.cuda(), imp.cuda(), mask.cuda())
    pg = _sd(small, "g_init/")
    pd = _sd(small, "d_init/")
    ref = R.GanStep(pg, pd, None, lr=2e-4, betas=(0.5, 0.999))
    lam = dict(R.LAMBDAS)
    ref.lam = lam
    r = ref.step(orig, imp, mask)
    assert rel(out["generated"], r["generated"]) < TOL
    for k in ("d_loss", "g_total", "g_adv", "g_l1_valid", "g_l1_hole", "g_mag_weighted"):
        assert abs(float(out[k]) - float(r[k])) <= TOL * max(abs(float(r[k])), 1e-6), k
    sd = Dm.state_dict()
    for k in R.d_trainable_keys(pd):
        assert rel(sd[k], pd[k].detach()) < 1e-5, k
    for k in [k for k in pd if k.endswith("weight_u") or k.endswith("weight_v")]:
        assert rel(sd[k], pd[k]) < 1e-5, k


# ------------------------------------------------------------- C5 shape: 8 s, T=1001
def test_generator_and_discriminator_t1001_match_reference(golden_dir):
    """Default PConvUNet / Discriminator at [1,1,257,1001] (gan_t1001.npz from
    the reference's networks.py): W pads 1001 -> 1024 (networks.py:255-261),
    output crop, BN running statistics after the train-mode forward, D logits
    [1,1,30,123] and the spectral-norm u/v after that forward."""
    from ainp import gan as G
    g = np.load(os.path.join(golden_dir, "gan_t1001.npz"), allow_pickle=False)
    torch.manual_seed(0)
    m = G.PConvUNet().cuda().train()
    y = m(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["mask"]).cuda())
    assert tuple(y.shape) == tuple(int(v) for v in g["y_shape"])
    # (with autograd on this is the generator's training forward, _PConvUNetFn)
    yf = y.detach().cpu().numpy().reshape(-1)
    assert rel(yf[::97], g["y_sample"]) < TOL
    assert abs(np.linalg.norm(yf.astype(np.float64)) - g["y_norm"][0]) < TOL * g["y_norm"][0]
    sd = m.state_dict()
    for k in g.files:
        if k.startswith("g_after/"):
            assert rel(sd[k[len("g_after/"):]], g[k]) < TOL, k
    torch.manual_seed(1)
    D = G.Discriminator().cuda().train()
    with torch.no_grad():
        logits = D(torch.from_numpy(g["x"]).cuda())
    assert tuple(logits.shape) == tuple(g["d_logits"].shape) == (1, 1, 30, 123)
    assert rel(logits, g["d_logits"]) < TOL
    sd = D.state_dict()
    for k in g.files:
        if k.startswith("d_after/"):
            assert rel(sd[k[len("d_after/"):]], g[k]) < 1e-5, k


# ------------------------------------------------------------- full-size GAN step
def _fixture_step(g, seeds, inputs, dtype=None):
    """One GanTrainer step on a reference step fixture (gan_step_full.npz /
    gan_step_t1001.npz) with the fixture's seeded G, D and VGG19 weights."""
    from ainp import gan as G
    from ainp.gan_train import GanTrainer
    from golden.gen_golden_r02 import checksum
    orig, imp, mask = inputs
    for a, k in ((orig, "orig_check"), (imp, "imp_check"), (mask, "mask_check")):
        assert np.allclose(checksum(a), g[k], rtol=1e-12, atol=0), k
    torch.manual_seed(seeds["g_seed"])
    Gm = G.PConvUNet()
    torch.manual_seed(seeds["d_seed"])
    Dm = G.Discriminator()
    v, _ = _vgg_pair(seeds["vgg_seed"])
    cfg = {"training": dict(R.LAMBDAS, g_lr=2e-4, d_lr=2e-4, b1=0.5, b2=0.999)}
    if dtype is not None:
        cfg["accel"] = {"dtype": dtype}
    tr = GanTrainer(cfg, Gm.cuda(), Dm.cuda(), vgg=v)
    if dtype == "bf16":
        assert Dm.ainp_bf16 and v.ainp_bf16
    out = tr.step(torch.from_numpy(orig).cuda(), torch.from_numpy(imp).cuda(),
                  torch.from_numpy(mask).cuda())
    return out, Gm, Dm


def _check_fp32_step(g, out, Gm, Dm, param_tol=1e-5):
    """param_tol: D parameters after Adam (samples).  Adam's first step moves
    each weight by lr * g / (|g| + eps'), so weights whose gradient is within
    a few eps of 0 carry most of the difference; 1e-5 holds at T=626, the
    north-star 1e-4 gate at T=1001 (measured 6.3e-5 on layer 0)."""
    gf = out["generated"].cpu().numpy().reshape(-1)
    assert rel(gf[::97], g["gen_sample"]) < TOL
    assert abs(np.linalg.norm(gf.astype(np.float64)) - g["gen_norm"][0]) < TOL * g["gen_norm"][0]
    dl, lr_, lf = g["d_losses"]
    for k, r in (("d_loss", dl), ("d_real", lr_), ("d_fake", lf)):
        assert abs(float(out[k]) - r) <= TOL * abs(r), k
    for k, p in Dm.named_parameters():
        gr = p.grad.detach().cpu().numpy()
        gn = np.linalg.norm(gr.astype(np.float64))
        assert abs(gn - g["d_gnorm/" + k][0]) <= TOL * g["d_gnorm/" + k][0], (k, gn)
        s = gr.reshape(-1)[::max(1, gr.size // 4096)]
        assert rel(s, g["d_gsample/" + k]) < TOL, k
    sd = Gm.state_dict()
    for k in g.files:
        if k.startswith("g_after/"):
            assert rel(sd[k[len("g_after/"):]], g[k]) < TOL, k
    sd = Dm.state_dict()
    for k in g.files:
        if k.startswith("d_after_g/"):
            # u/v after the third power iteration, on the Adam-updated weights
            assert rel(sd[k[len("d_after_g/"):]], g[k]) < TOL, k
        elif k.startswith("d_after/") and "weight_u" not in k and "weight_v" not in k:
            t = sd[k[len("d_after/"):]].cpu().numpy()
            s = t.reshape(-1)[::max(1, t.size // 4096)]
            assert rel(s, g[k]) < param_tol, (k, rel(s, g[k]))
    for k in ("g_total", "g_adv", "g_l1_valid", "g_l1_hole", "g_mag_weighted",
              "g_vgg_perceptual", "g_vgg_style"):
        r = float(g["oracle_loss/" + k][0])
        assert abs(float(out[k]) - r) <= TOL * max(abs(r), 1e-6), (k, float(out[k]), r)


# bf16 gate (bf16 cannot meet 1e-4): generated spectrogram, D loss
# and the G-step losses within BF16_STEP_TOL relative of the fp32 reference;
# every discriminator gradient (the bf16 D backward: csrc/dconv16.hip, the
# logit conv's GEMV) within BF16_DGRAD_NORM_TOL (norm) / BF16_DGRAD_SAMPLE_TOL
# (strided sample, relative L2) of the reference's fp32 gradient, and the D
# parameters after the Adam step within BF16_DPARAM_TOL.
BF16_STEP_TOL = 2e-2
# measured at T=626 / T=1001: norms <= 1.9e-3, samples <= 9.1e-3, parameters
# <= 3.4e-3 (profiles/r04a_pytest_bf16gates.log)
BF16_DGRAD_NORM_TOL = 1e-2
BF16_DGRAD_SAMPLE_TOL = 3e-2
BF16_DPARAM_TOL = 1e-2


def _check_bf16_step(g, out, tag, Dm=None):
    gf = out["generated"].cpu().numpy().reshape(-1)
    errs = {"generated": rel(gf[::97], g["gen_sample"]),
            "d_loss": abs(float(out["d_loss"]) - g["d_losses"][0]) / abs(g["d_losses"][0])}
    for k in ("g_total", "g_l1_valid", "g_l1_hole", "g_vgg_perceptual", "g_vgg_style"):
        r = float(g["oracle_loss/" + k][0])
        errs[k] = abs(float(out[k]) - r) / abs(r)
    print(tag, "bf16 GAN step rel errs", errs)
    gerrs, perrs = {}, {}
    if Dm is not None:
        for k, p in Dm.named_parameters():
            gr = p.grad.detach().cpu().double().numpy()
            assert np.isfinite(gr).all(), k
            e_n = abs(np.linalg.norm(gr) - g["d_gnorm/" + k][0]) / g["d_gnorm/" + k][0]
            e_s = rel(gr.reshape(-1)[::max(1, gr.size // 4096)], g["d_gsample/" + k])
            gerrs[k] = (round(float(e_n), 5), round(float(e_s), 5))
        sd = Dm.state_dict()
        for k in g.files:
            if k.startswith("d_after/") and "weight_u" not in k and "weight_v" not in k:
                t = sd[k[len("d_after/"):]].cpu().numpy()
                perrs[k] = round(float(rel(t.reshape(-1)[::max(1, t.size // 4096)], g[k])), 6)
        print(tag, "bf16 D grad errs (norm, sample)", gerrs)
        print(tag, "bf16 D params after Adam", perrs)
        assert len(gerrs) == sum(1 for k in g.files if k.startswith("d_gnorm/"))
    assert max(errs.values()) < BF16_STEP_TOL, errs
    for k, (e_n, e_s) in gerrs.items():
        assert e_n < BF16_DGRAD_NORM_TOL and e_s < BF16_DGRAD_SAMPLE_TOL, (k, e_n, e_s)
    for k, e in perrs.items():
        assert e < BF16_DPARAM_TOL, (k, e)


@pytest.mark.timeout(600)
def test_full_size_gan_step_matches_reference(golden_dir):
    """One full-size GAN step (train.py:341-378) at B=2, T=626 on the GAN data
    path (gan_step_full.npz from the reference's networks.py): generated
    spectrogram, D logits and losses, every D gradient (norms and samples),
    D parameters and u/v after Adam and after the G-step forward, G's
    BatchNorm running statistics; the G-step losses (incl. VGG19 with seeded
    weights, oracle/gan_ref.vgg19_init(0): pretrained weights parity-unpinned)
    vs the oracle values stored with the fixture."""
    from golden.gen_golden_r02 import GSTEP, gan_step_inputs
    g = np.load(os.path.join(golden_dir, "gan_step_full.npz"), allow_pickle=False)
    out, Gm, Dm = _fixture_step(g, GSTEP, gan_step_inputs())
    _check_fp32_step(g, out, Gm, Dm)


@pytest.mark.timeout(600)
def test_full_size_gan_step_bf16_tracks_reference(golden_dir):
    """The full-size B=2 step of gan_step_full.npz in the bf16 configuration
    (accel.dtype = bf16: bf16 conv / GEMM operands in G, D and VGG, fp32
    accumulation, BatchNorm statistics and weights): generated spectrogram,
    D losses and G-step losses within 2e-2 relative of the fp32 reference,
    every D gradient and the D parameters after Adam at the BF16_DGRAD_* /
    BF16_DPARAM_TOL gates."""
    from golden.gen_golden_r02 import GSTEP, gan_step_inputs
    g = np.load(os.path.join(golden_dir, "gan_step_full.npz"), allow_pickle=False)
    out, _, Dm = _fixture_step(g, GSTEP, gan_step_inputs(), dtype="bf16")
    _check_bf16_step(g, out, "T=626", Dm)


@pytest.mark.timeout(600)
def test_c5_shape_gan_step_matches_reference(golden_dir):
    """C5's own shape (8 s clips, T=1001, 0.1 s gaps, B=2; gan_step_t1001.npz
    from the reference's networks.py): the same checks as the T=626 step at
    the fp32 gate."""
    from golden.gen_golden_r03 import GSTEP1001, gan_step1001_inputs
    g = np.load(os.path.join(golden_dir, "gan_step_t1001.npz"), allow_pickle=False)
    out, Gm, Dm = _fixture_step(g, GSTEP1001, gan_step1001_inputs())
    assert tuple(out["generated"].shape) == (2, 1, 257, 1001)
    _check_fp32_step(g, out, Gm, Dm, param_tol=TOL)


@pytest.mark.timeout(600)
def test_c5_shape_gan_step_bf16_tracks_reference(golden_dir):
    """C5 in its own arithmetic: the bf16 configuration of the T=1001 step
    within BF16_STEP_TOL of the reference's fp32 step."""
    from golden.gen_golden_r03 import GSTEP1001, gan_step1001_inputs
    g = np.load(os.path.join(golden_dir, "gan_step_t1001.npz"), allow_pickle=False)
    out, _, Dm = _fixture_step(g, GSTEP1001, gan_step1001_inputs(), dtype="bf16")
    _check_bf16_step(g, out, "T=1001", Dm)


@pytest.mark.parametrize("N,C,H,W,masked", [(2, 64, 17, 70, True), (1, 96, 5, 130, False),
                                           (2, 512, 3, 5, True)])
def test_affine_act_nhwc16_equals_affine_then_convert(N, C, H, W, masked):
    """ainp_affine_act_nhwc16 (the bf16 U-Net blocks' BatchNorm + LeakyReLU with
    the next conv's channel-last source in the same pass) against affine_act_
    followed by to_nhwc16: the in-place fp32 result and the bf16 copy are both
    bit-identical; inside an nhwc16_memo scope to_nhwc16 returns the copy."""
    from ainp import ops
    g = torch.Generator().manual_seed(N * C + H * W)
    y0 = torch.randn(N, C, H, W, generator=g).cuda()
    sc = (torch.rand(C, generator=g) + 0.5).cuda()
    sh = torch.randn(C, generator=g).cuda()
    m = (torch.rand(N, H, W, generator=g) > 0.3).float().cuda() if masked else None
    ya = y0.clone()
    ops.affine_act_(ya, sc, sh, ops.ACT_LEAKY, 0.2)
    ref16 = ops.to_nhwc16(ya, m)
    yb = y0.clone()
    with ops.nhwc16_memo():
        _, out16 = ops.affine_act_nhwc16_(yb, sc, sh, ops.ACT_LEAKY, 0.2, m)
        again = ops.to_nhwc16(yb, m)
        assert again.data_ptr() == out16.data_ptr()
    torch.cuda.synchronize()
    assert torch.equal(ya, yb)
    assert torch.equal(ref16.view(torch.int16), out16.view(torch.int16))


# ------------------------------------------------------------- generator backward
# (opt-in fix_generator_grad; csrc/gan_bwd.hip + ainp.gan._PConvUNetFn,
# _VGGLossFn, _ReconFn)
def test_gen_bwd_kernels_match_torch_autograd():
    """The generator-backward building blocks against torch autograd (fp64 CPU):
    PartialConv2d source materialisation and its gradient (nearest x2 upsample
    + masks), BatchNorm2d(train) + LeakyReLU backward x window ratio, Tanh +
    crop backward, MaxPool2d backward, the Gram / L1 sign gradients and the
    reconstruction-loss gradient."""
    from ainp import ops
    g = torch.Generator().manual_seed(42)
    N, C0, C1, Hs, Ws = 2, 3, 2, 5, 7
    x0 = torch.randn(N, C0, Hs, Ws, generator=g, dtype=torch.float64, requires_grad=True)
    m0 = (torch.rand(N, Hs, Ws, generator=g) > 0.3).double()
    x1 = torch.randn(N, C1, 2 * Hs, 2 * Ws, generator=g, dtype=torch.float64, requires_grad=True)
    m1 = (torch.rand(N, 2 * Hs, 2 * Ws, generator=g) > 0.3).double()
    up = F.interpolate(x0 * m0.unsqueeze(1), scale_factor=2, mode="nearest")
    ref = torch.cat([up, x1 * m1.unsqueeze(1)], 1)
    d = lambda t: t.detach().float().contiguous().cuda()  # noqa: E731
    xin = ops.pconv_src_materialize((d(x0), d(m0)), (d(x1), d(m1)), 2 * Hs, 2 * Ws)
    assert rel(xin, ref) < 1e-7
    gout = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gout)
    dx0 = torch.full((N, C0, Hs, Ws), 0.5, device="cuda")
    ops.pconv_src_grad(d(gout), 0, d(m0), dx0, True)
    dx1 = torch.empty(N, C1, 2 * Hs, 2 * Ws, device="cuda")
    ops.pconv_src_grad(d(gout), C0, d(m1), dx1, False)
    assert rel(dx0 - 0.5, x0.grad) < 1e-6 and rel(dx1, x1.grad) < 1e-6

    # BatchNorm2d (train) + LeakyReLU(0.2) backward, times a window ratio
    C, H, W = 4, 6, 9
    y = torch.randn(N, C, H, W, generator=g, dtype=torch.float64, requires_grad=True)
    gam = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    bet = torch.randn(C, generator=g, dtype=torch.float64) * 0.1
    gam.requires_grad_(True); bet.requires_grad_(True)
    a = F.leaky_relu(F.batch_norm(y, None, None, gam, bet, True, 0.1, 1e-5), 0.2)
    ga = torch.randn(a.shape, generator=g, dtype=torch.float64)
    a.backward(ga)
    mean = y.detach().mean((0, 2, 3))
    rstd = 1.0 / torch.sqrt(y.detach().var((0, 2, 3), unbiased=False) + 1e-5)
    sc, sh = gam.detach() * rstd, bet.detach() - mean * gam.detach() * rstd
    save = torch.cat([mean, rstd])
    ratio = torch.rand(N, H, W, generator=g, dtype=torch.float64) * 3
    sums = ops.bn_act_bwd_reduce(d(ga), d(y), d(sc), d(sh), d(save), 0.2)
    ld = H * W + 2
    gc, dg_, db_ = ops.bn_act_bwd_apply(d(ga), d(y), d(sc), d(sh), d(save), d(gam), sums,
                                        N * H * W, 0.2, d(ratio), ld)
    want = (y.grad * ratio.unsqueeze(1)).reshape(N, C, H * W)
    assert rel(gc[:, :, :H * W], want) < 1e-5 and float(gc[:, :, H * W:].abs().max()) == 0.0
    assert rel(dg_, gam.grad) < 1e-5 and rel(db_, bet.grad) < 1e-5

    # Tanh + crop backward on the padded grid
    z = torch.randn(N, 1, H, W, generator=g, dtype=torch.float64, requires_grad=True)
    o = torch.tanh(z)[:, :, :H - 2, :W - 3]
    go = torch.randn(o.shape, generator=g, dtype=torch.float64)
    o.backward(go)
    gz, gc = ops.gen_act_bwd(d(go), d(o), ops.ACT_TANH, 0.2, d(ratio), H, W, H * W)
    assert rel(gz.view(N, 1, H, W), z.grad) < 1e-5
    assert rel(gc.view(N, 1, H, W), z.grad * ratio.unsqueeze(1)) < 1e-5

    # MaxPool2d(2, 2) backward (ties broken like torch CPU: first maximum)
    xp = torch.randn(N, C, 8, 10, generator=g, dtype=torch.float64)
    xp[0, 0, 0, :2] = 1.5                    # a tie inside one window
    xp.requires_grad_(True)
    yp = F.max_pool2d(xp, 2, 2)
    gp = torch.randn(yp.shape, generator=g, dtype=torch.float64)
    yp.backward(gp)
    assert rel(ops.maxpool2_bwd(d(gp), d(xp)), xp.grad) < 1e-6

    # L1 of Gram matrices: dF = (dG + dG^T) F / (c h w) and the L1 sign gradient
    Fm = torch.randn(N, C, 5, 6, generator=g, dtype=torch.float64, requires_grad=True)
    Ft = torch.randn(N, C, 5, 6, generator=g, dtype=torch.float64)
    gram = lambda t: torch.bmm(t.reshape(N, C, -1), t.reshape(N, C, -1).transpose(1, 2)) / (C * 30)  # noqa: E731,E501
    loss = torch.mean(torch.abs(gram(Fm) - gram(Ft))) * 3.0 + torch.mean(torch.abs(Fm - Ft))
    loss.backward()
    gs = torch.tensor([3.0], device="cuda")
    sg = ops.gram_sign_sym(d(gram(Fm)), d(gram(Ft)), gs, 1.0 / (N * C * C))
    dF = torch.empty(N, C, 5, 6, device="cuda")
    ops.gemm(C, 30, C, [sg], C, 1, [d(Fm)], 30, 1, [dF], 30, 1, alpha=1.0 / (C * 30),
             strideA=C * C, strideB=C * 30, strideC=C * 30, nstrided=N)
    ops.absdiff_grad(d(Fm), d(Ft), None, 1.0 / Fm.numel(), out=dF, accumulate=True)
    assert rel(dF, Fm.grad) < 1e-5

    # reconstruction losses Lv / Lh / Lw (train.py:49-63)
    gen = torch.tanh(torch.randn(N, 1, H, W, generator=g, dtype=torch.float64)).requires_grad_(True)
    org = torch.rand(N, 1, H, W, generator=g, dtype=torch.float64)
    msk = (torch.rand(N, 1, H, W, generator=g) > 0.4).double()
    lv = torch.sum(torch.abs(gen * msk - org * msk)) / (msk.sum() + 1e-8)
    lh = torch.sum(torch.abs(gen * (1 - msk) - org * (1 - msk))) / ((1 - msk).sum() + 1e-8)
    lw = torch.mean(torch.abs(gen - org) * torch.abs(org))
    (1.0 * lv + 2.0 * lh + 0.2 * lw).backward()
    sums = ops.gan_recon_sums(d(gen), d(org), d(msk))
    gr = ops.gan_recon_bwd(d(gen), d(org), d(msk), sums,
                           torch.tensor([1.0, 2.0, 0.2], device="cuda"), gen.numel())
    assert rel(gr, gen.grad) < 1e-6


def test_vgg_loss_input_gradient_matches_oracle():
    """d(lambda_p perceptual + lambda_s style) / d generated through VGG19
    (seeded weights; loss.py:89-131 incl. the inplace-ReLU feature quirk) and
    the input preparation, against torch autograd of the oracle restatement
    in fp64 on the CPU.  The L1 terms make the gradient a sum of sign()
    functions of feature / Gram differences, so two correct fp32
    implementations already differ by ~2e-3 (sign flips where fg ~ ft): the
    bound is 1.5 x the oracle's own fp32-vs-fp64 distance (+1e-5), i.e. the
    GPU path must be as accurate as an fp32 restatement of the reference."""
    g = torch.Generator().manual_seed(9)
    gen = torch.tanh(torch.randn(2, 1, 129, 100, generator=g))
    tgt = torch.rand(2, 1, 129, 100, generator=g) * 3
    v, pv = _vgg_pair(0)
    for lp, ls in ((4.0, 0.0), (0.0, 500.0)):
        gg = gen.clone().cuda().requires_grad_(True)
        perc, style = v(gg, tgt.cuda())
        (lp * perc if lp else ls * style).backward()     # one term at a time
        assert torch.isfinite(gg.grad).all()
        ref = {}
        for dt in (torch.float64, torch.float32):
            p = {k: t.to(dt) for k, t in pv.items()}
            gr = gen.clone().to(dt).requires_grad_(True)      # a fresh leaf per run
            rp, rs = R.vgg_losses(p, gr, tgt.to(dt))
            (lp * rp if lp else ls * rs).backward()
            assert torch.isfinite(gr.grad).all(), dt
            ref[dt] = (gr.grad, float(rp.detach()), float(rs.detach()))
        g64, rp, rs = ref[torch.float64]
        assert abs(float(perc) - rp) < 1e-4 * abs(rp)
        assert abs(float(style) - rs) < 1e-4 * abs(rs)
        e = rel(gg.grad, g64)
        floor = rel(ref[torch.float32][0], g64)
        print(f"VGG input gradient (lp={lp}, ls={ls}): rel err {e:.3e}, fp32 floor {floor:.3e}")
        assert e < 1.5 * floor + 1e-5, (e, floor)


@pytest.mark.timeout(600)
def test_generator_training_step_matches_reference(golden_dir):
    """fix_generator_grad: one GAN step with G trained, on the
    reference's reduced-channel PConvUNet / Discriminator (gan_gstep_small.npz
    from networks.py, losses through the oracle restatement with seeded VGG19):
    the G-step losses, every G parameter gradient (PartialConv2d weights and
    biases, BatchNorm gamma / beta) at the fp32 gate 1e-4, and G's parameters
    and BatchNorm statistics after its Adam step.  The default loop keeps Q1
    (G untouched), checked on the same fixture."""
    from ainp import gan as G
    from ainp.gan_train import GanTrainer
    from golden.gen_golden_gan import SMALL_D, SMALL_DEC, SMALL_ENC, SMALL_FINAL
    f = np.load(os.path.join(golden_dir, "gan_gstep_small.npz"), allow_pickle=False)

    def make(fix):
        Gm = G.PConvUNet(enc_layer_cfg=SMALL_ENC, dec_layer_cfg=SMALL_DEC,
                         final_dec_cfg=SMALL_FINAL)
        Gm.load_state_dict(_sd(f, "g_init/"))
        Dm = G.Discriminator(layer_cfg=SMALL_D)
        Dm.load_state_dict(_sd(f, "d_init/"))
        v, _ = _vgg_pair(0)
        cfg = {"training": dict(R.LAMBDAS, g_lr=2e-4, d_lr=2e-4, b1=0.5, b2=0.999,
                                fix_generator_grad=fix)}
        tr = GanTrainer(cfg, Gm.cuda(), Dm.cuda(), vgg=v)
        assert tr.fix_g == fix
        out = tr.step(*(torch.from_numpy(f[k]).cuda() for k in ("orig", "imp", "mask")))
        return out, Gm
    out, Gm = make(True)
    assert rel(out["generated"], f["r32/gen"]) < TOL
    assert abs(float(out["d_loss"]) - f["r32/d_loss"][0]) <= TOL * abs(f["r32/d_loss"][0])
    for k in ("g_total", "g_adv", "g_l1_valid", "g_l1_hole", "g_mag_weighted",
              "g_vgg_perceptual", "g_vgg_style"):
        r = float(f["r32/loss/" + k][0])
        assert abs(float(out[k]) - r) <= TOL * max(abs(r), 1e-6), (k, float(out[k]), r)
    # every G gradient vs the reference module run in fp64 (the fp32 reference
    # itself sits 4e-7 .. 1.2e-5 from it), and vs the fp32 reference run
    errs = {}
    for k, p in Gm.named_parameters():
        if not p.requires_grad:
            continue
        assert p.grad is not None, k
        errs[k] = (rel(p.grad, f["r64/g_grad/" + k]), rel(p.grad, f["r32/g_grad/" + k]))
    print("G grad rel errs (vs fp64, vs fp32)", sorted(errs.items(), key=lambda kv: -kv[1][0])[:6])
    assert len(errs) == sum(1 for k in f.files if k.startswith("r32/g_grad/"))
    for k, (e64, e32) in errs.items():
        assert e64 < TOL and e32 < TOL, (k, e64, e32)
    sd = Gm.state_dict()
    for k in f.files:
        if k.startswith("r32/g_after/"):
            name = k[len("r32/g_after/"):]
            if name.endswith("num_batches_tracked"):
                assert int(sd[name]) == int(f[k])
            else:
                assert rel(sd[name], f[k]) < TOL, name
    # default loop (fix_generator_grad off): G's parameters do not move (Q1)
    _, G0 = make(False)
    sd0 = G0.state_dict()
    for k in f.files:
        if k.startswith("g_init/") and "running" not in k and "num_batches" not in k:
            assert np.array_equal(sd0[k[len("g_init/"):]].cpu().numpy(), f[k]), k


def test_unet_bf16_forward_without_fp32_writeback_is_bit_identical(monkeypatch):
    """bf16 U-Net no-grad forward: the BatchNorm + LeakyReLU pass that writes
    only the channel-last copy (AINP_AFFINE_NO_Y) gives the same output, bit
    for bit -- no consumer reads the fp32 block outputs."""
    from ainp import gan as G
    torch.manual_seed(4)
    net = G.set_compute_dtype(G.PConvUNet().cuda().eval(), "bf16")
    x = torch.randn(2, 1, 129, 250, device="cuda")
    m = (torch.rand(2, 1, 129, 250, device="cuda") > 0.2).float()
    outs = []
    for flag in (True, False):
        monkeypatch.setattr(G, "AFFINE_NO_Y", flag)
        with torch.no_grad():
            outs.append(net(x, m).clone())
    assert torch.equal(outs[0], outs[1])
    # AINP_CONV_NHWC16_SMALL=0: the final PartialConv2d's 1-channel source
    # sends it down the fp32 NCHW gather, which reads the block output's fp32
    # planes -- the write-back must then stay on, same output
    # as with every consumer channel-last
    from ainp import ops
    monkeypatch.setattr(ops, "CONV_NHWC16_SMALL", "0")
    monkeypatch.setattr(G, "AFFINE_NO_Y", True)
    assert not G._affine_no_y_safe()
    with torch.no_grad():
        small0 = net(x, m).clone()
    monkeypatch.setattr(G, "AFFINE_NO_Y", False)
    with torch.no_grad():
        small0_y = net(x, m).clone()
    assert torch.equal(small0, small0_y)
    assert (small0 - outs[0]).abs().max().item() < 1e-1


@pytest.mark.parametrize("n,off", [(1, 0), (1003, 0), (4096 * 37 + 3, 0), (524288 * 9, 0), (70001, 1)])
def test_absdiff_mean_matches_fp64(n, off):
    """ainp_absdiff_mean (the perceptual / style L1 terms): mean |a - b| in
    double against numpy's, over vector-loaded, ragged-tail and unaligned
    (off = 1 float: the scalar loop) operands."""
    from ainp import ops
    g = torch.Generator().manual_seed(n)
    a = torch.randn(n + off, generator=g)
    b = torch.randn(n + off, generator=g)
    out = ops.absdiff_mean(a.cuda()[off:], b.cuda()[off:])
    ref = np.abs(a[off:].numpy() - b[off:].numpy()).astype(np.float64).mean()
    assert abs(out.item() - ref) <= 1e-12 * max(1.0, abs(ref))


@pytest.mark.parametrize("k,st,pd,N,H0,W0,C0,H1,W1,C1,Hin,Win", [
    (3, 1, 1, 2, 20, 33, 64, 40, 66, 1, 40, 66),     # final PartialConv: x2 source + input mask
    (7, 2, 3, 2, 37, 70, 2, 0, 0, 0, 37, 70),        # the U-Net's first conv (7x7 / 2)
    (5, 2, 2, 1, 19, 23, 64, 0, 0, 0, 19, 23),       # 5x5 / 2
    (4, 2, 1, 3, 9, 14, 3, 18, 28, 5, 18, 28),       # 4x4, two sources, x2
    (3, 1, 1, 1, 7, 10, 8, 0, 0, 0, 20, 30),         # general nearest resampling
    (2, 1, 0, 1, 9, 11, 4, 9, 11, 2, 9, 11),         # window size without an unrolled kernel
])
def test_pconv_mask_matches_window_counts(k, st, pd, N, H0, W0, C0, H1, W1, C1, Hin, Win):
    """ainp_pconv_mask (networks.py:83-104): count = C0 * win(m0) + C1 * win(m1)
    of the nearest-resampled masks, ratio = (Cin k^2) / (count + 1e-8), new
    mask = clamp(count, 0, 1) -- exact against an fp64 ones-kernel conv."""
    from ainp import ops
    g = torch.Generator().manual_seed(k * 100 + Hin)
    m0 = (torch.rand(N, H0, W0, generator=g) > 0.4).float()
    m1 = (torch.rand(N, H1, W1, generator=g) > 0.4).float() if C1 else None

    def up(m):
        Hs, Ws = m.shape[-2:]
        sy, sx = (torch.arange(Hin) * Hs) // Hin, (torch.arange(Win) * Ws) // Win
        return m[:, sy][:, :, sx].double().unsqueeze(1)

    ones = torch.ones(1, 1, k, k, dtype=torch.float64)
    cnt = C0 * F.conv2d(up(m0), ones, stride=st, padding=pd)
    if C1:
        cnt = cnt + C1 * F.conv2d(up(m1), ones, stride=st, padding=pd)
    cnt = cnt[:, 0].float()
    ratio, newm = ops.pconv_mask((m0.cuda(), C0), (m1.cuda(), C1) if C1 else None, N, Hin, Win,
                                 k, st, pd)
    exp_ratio = float((C0 + C1) * k * k) / (cnt + 1e-8)
    assert torch.equal(newm.cpu(), cnt.clamp(0, 1))
    assert torch.allclose(ratio.cpu(), exp_ratio, rtol=1e-6, atol=0)
