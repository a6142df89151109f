"""Channel-last activations (round 5): the CNNBLSTM conv / BatchNorm kernels
reading and writing [N, F, T, C] tensors (AINP_CONV_XCL / _YCL / _GCL,
AINP_BN_CL) against the NCHW kernels they replace.

The split-bf16 conv kernels stage the same values into the same LDS images
and run the same MFMA chains whichever layout they load from, so their
outputs, BatchNorm partials and weight gradients are bit-identical to the
NCHW launches.  The channel-last BatchNorm backward and the small-channel
row-strip weight gradient sum in another order (checked at 1e-6).  The model
test runs a CNNBLSTM step with AINP_CL on / off (models/CNNBLSTM/model.py:
34-61 is the reference either way)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ml-audio-inpainting_amd"))

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cl(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _data(N, cin, cout, H, W, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(N, cin, H, W, device=DEV, generator=g)
    dy = torch.randn(N, cout, H, W, device=DEV, generator=g) * 0.1
    w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.2
    b = torch.randn(cout, device=DEV, generator=g)
    sc = torch.rand(cin, device=DEV, generator=g) + 0.5
    sh = torch.randn(cin, device=DEV, generator=g) * 0.3
    return x, dy, w, b, sc, sh


PAIRS = [(16, 32), (32, 64), (32, 16)]
SHAPES = [(2, 257, 334), (1, 19, 47)]
# round 6's row-strip kernels (16 / 14 columns and 16 rows per strip): a lone
# pixel, strips narrower than one wave, exactly one strip, one row past it
EDGE_SHAPES = [(1, 1, 1), (2, 3, 5), (1, 16, 14), (3, 17, 15)]


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("N,H,W", SHAPES)
@pytest.mark.parametrize("cin,cout", PAIRS)
def test_cl_fwd_bit_identical(cin, cout, N, H, W, bf16):
    from ainp import ops
    x, dy, w, b, sc, sh = _data(N, cin, cout, H, W, cin * 100 + cout)
    y0, st0 = ops.conv3x3_fwd(x, w, b, sc, sh, want_stats=True, bf16=bf16)
    for xcl, ycl in ((True, True), (True, False), (False, True)):
        y, st = ops.conv3x3_fwd(_cl(x) if xcl else x, w, b, sc, sh, want_stats=True, bf16=bf16,
                                xcl=xcl, ycl=ycl)
        assert torch.equal(_nchw(y) if ycl else y, y0), (xcl, ycl)
        assert torch.equal(st, st0), (xcl, ycl)
    if bf16:   # bf16 storage of the source and of y (AINP_CONV_X16 / _Y16)
        x16 = x.to(torch.bfloat16)
        y0, st0 = ops.conv3x3_fwd(x16, w, b, sc, sh, want_stats=True, bf16=True, y16=True)
        y, st = ops.conv3x3_fwd(_cl(x16), w, b, sc, sh, want_stats=True, bf16=True, y16=True,
                                xcl=True, ycl=True)
        assert torch.equal(_nchw(y), y0) and torch.equal(st, st0)


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("N,H,W", SHAPES)
@pytest.mark.parametrize("cin,cout", PAIRS)
def test_cl_dgrad_wgrad_bit_identical(cin, cout, N, H, W, bf16):
    from ainp import ops
    x, dy, w, b, sc, sh = _data(N, cin, cout, H, W, cin * 7 + cout)
    dys = [dy] + ([dy.to(torch.bfloat16)] if bf16 else [])
    for d in dys:
        dx0 = ops.conv3x3_dgrad(d, w, bf16=bf16)
        for xcl, ycl in ((True, True), (True, False), (False, True)):
            dx = ops.conv3x3_dgrad(_cl(d) if xcl else d, w, bf16=bf16, xcl=xcl, ycl=ycl)
            assert torch.equal(_nchw(dx) if ycl else dx, dx0), (d.dtype, xcl, ycl)
        dw0, db0 = ops.conv3x3_wgrad(x, d, sc, sh, bf16=bf16)
        for xcl, gcl in ((True, True), (True, False), (False, True)):
            dw, db = ops.conv3x3_wgrad(_cl(x) if xcl else x, _cl(d) if gcl else d, sc, sh,
                                       bf16=bf16, xcl=xcl, gcl=gcl)
            assert torch.equal(dw, dw0) and torch.equal(db, db0), (d.dtype, xcl, gcl)


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("N,H,W", SHAPES + [(3, 20, 70)])
def test_dgrad_cfnt_bit_identical(N, H, W, bf16):
    """Round 6, AINP_CONV_YCFNT: the decoder's 16 -> 32 conv data gradient
    writing dx as [C, F, N, T] (the fp32 projection backward's operand) --
    the same values as the NCHW launch, bit for bit, from NCHW and channel-last
    dy; every element written (NaN-filled buffer)."""
    from ainp import ops
    assert ops.dgrad_cfnt_ok(N, 16, 32, H, W)
    x, dy, w, b, sc, sh = _data(N, 16, 32, H, W, 11)
    dys = [dy] + ([dy.to(torch.bfloat16)] if bf16 else [])
    for d in dys:
        dx0 = ops.conv3x3_dgrad(d, w, bf16=bf16)
        for xcl in (False, True):
            dx = ops.conv3x3_dgrad(_cl(d) if xcl else d, w, bf16=bf16, xcl=xcl, cfnt=True)
            assert dx.shape == dx0.shape and dx.permute(1, 2, 0, 3).is_contiguous()
            assert torch.equal(dx, dx0), (d.dtype, xcl)
    buf = torch.full((16, H, N, W), float("nan"), device=DEV)
    flags = ops.CONV_XCL | ops.CONV_YCFNT
    ops._T.conv3x3_dgrad(_cl(dy), w, buf, flags)
    assert torch.equal(buf.permute(2, 0, 1, 3), ops.conv3x3_dgrad(dy, w))
    with pytest.raises(RuntimeError, match="YCFNT"):
        ops.conv3x3_dgrad(_cl(torch.randn(N, 16, H, W, device=DEV)), w.transpose(0, 1).contiguous(),
                          xcl=True, cfnt=True)


@pytest.mark.parametrize("N,H,W", SHAPES + EDGE_SHAPES)
@pytest.mark.parametrize("pro", [True, False])
def test_cl_small_channel_convs(N, H, W, pro):
    """1 -> 16 and 16 -> 1 (encoder.0, decoder.6): forward and data gradient
    bit-identical, the channel-last row-strip weight gradient within 1e-6 of
    the NCHW one (another summation order) and run-to-run identical.  Round 6:
    the 16 -> 1 forward with channel-last input runs on row strips (another
    summation order): y and the summed BatchNorm partials within 1e-6 of the
    NCHW kernel and of an fp64 conv of the same act(x), run-to-run identical;
    the 1 -> 16 forward and data gradient on row strips keep each output's
    fma chain (bit-identical), their partials grouped per strip (1e-6)."""
    import torch.nn.functional as F
    from ainp import ops
    for cin, cout in ((1, 16), (16, 1)):
        x, dy, w, b, sc, sh = _data(N, cin, cout, H, W, 5 + cin)
        s_, h_ = (sc, sh) if pro else (None, None)
        y0, st0 = ops.conv3x3_fwd(x, w, b, s_, h_, want_stats=True)
        xcl, ycl = cin == 16, cout == 16
        y, st = ops.conv3x3_fwd(_cl(x) if xcl else x, w, b, s_, h_, want_stats=True, xcl=xcl,
                                ycl=ycl)
        if cin == 16:
            a = x.double()
            if pro:
                a = torch.relu(a * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1))
            ref = F.conv2d(a, w.double(), b.double(), padding=1)
            assert rel(y, ref) < 1e-6 and rel(y, y0) < 1e-6
            assert rel(st.sum(0), st0.sum(0)) < 1e-6
            y2, st2 = ops.conv3x3_fwd(_cl(x), w, b, s_, h_, want_stats=True, xcl=True)
            assert torch.equal(y2, y) and torch.equal(st2, st)
        else:   # 1 -> 16 (round 6: row strips, the same fma chain per output)
            assert torch.equal(_nchw(y) if ycl else y, y0)
            assert rel(st.sum(0), st0.sum(0)) < 1e-6
        dx0 = ops.conv3x3_dgrad(dy, w)
        dx = ops.conv3x3_dgrad(_cl(dy) if ycl else dy, w, xcl=ycl, ycl=xcl)
        assert torch.equal(_nchw(dx) if xcl else dx, dx0)
        dw0, db0 = ops.conv3x3_wgrad(x, dy, s_, h_)
        args = (_cl(x) if xcl else x, _cl(dy) if ycl else dy, s_, h_)
        dw, db = ops.conv3x3_wgrad(*args, xcl=xcl, gcl=ycl)
        dw2, db2 = ops.conv3x3_wgrad(*args, xcl=xcl, gcl=ycl)
        assert torch.equal(dw, dw2) and torch.equal(db, db2)
        assert rel(dw, dw0) < 1e-6 and rel(db, db0) < 1e-6, (cin, cout)


@pytest.mark.parametrize("gy16", [False, True])
@pytest.mark.parametrize("N,H,W", SHAPES + EDGE_SHAPES)
def test_dgrad_bnapply_fused_matches_two_pass(N, H, W, gy16):
    """Round 6: Conv2d(16, 1)'s data gradient with the decoder.5 BatchNorm
    backward -- conv3x3_dgrad_bnr(want_dx=False) gives the fused path's sums
    bit for bit, and conv3x3_dgrad_bnapply (dx recomputed, never written)
    gives the apply's gy within 1e-6 (fp32; bf16 storage: within one bf16
    rounding) and its dgamma / dbeta exactly; run-to-run identical."""
    from ainp import ops
    g_ = torch.Generator(device=DEV).manual_seed(N + H + W)
    dy = torch.randn(N, 1, H, W, device=DEV, generator=g_)
    w = torch.randn(1, 16, 3, 3, device=DEV, generator=g_) * 0.2
    y = torch.randn(N, H, W, 16, device=DEV, generator=g_)
    sc = torch.rand(16, device=DEV, generator=g_) + 0.5
    sh = torch.randn(16, device=DEV, generator=g_) * 0.3
    gamma = torch.rand(16, device=DEV, generator=g_) + 0.5
    save = torch.stack([torch.randn(16, device=DEV, generator=g_) * 0.1,
                        torch.rand(16, device=DEV, generator=g_) + 0.5])
    cnt = N * H * W
    dx0, s0 = ops.conv3x3_dgrad_bnr(dy, w, y, sc, sh, save)
    gy0, dg0, db0 = ops.bn_relu_bwd_apply(dx0, y, sc, sh, gamma, save, s0, cnt, gy16=gy16, cl=True)
    none, s1 = ops.conv3x3_dgrad_bnr(dy, w, y, sc, sh, save, want_dx=False)
    assert none is None and torch.equal(s1, s0)
    gy, dg, db = ops.conv3x3_dgrad_bnapply(dy, w, y, sc, sh, gamma, save, s1, cnt, gy16=gy16)
    assert gy.dtype == gy0.dtype and gy.shape == gy0.shape
    assert rel(gy.float(), gy0.float()) < (4e-3 if gy16 else 1e-6)
    assert torch.equal(dg, dg0) and torch.equal(db, db0)
    gy2, _, _ = ops.conv3x3_dgrad_bnapply(dy, w, y, sc, sh, gamma, save, s1, cnt, gy16=gy16)
    assert torch.equal(gy2, gy)


@pytest.mark.parametrize("N,H,W", SHAPES + EDGE_SHAPES)
def test_wgrad_bnapply_fused_matches_two_pass(N, H, W):
    """Round 6, ops.conv3x3_wgrad_bnapply: the encoder's first conv (1 -> 16)
    weight gradient forming gy from g and y itself against the apply pass +
    the channel-last strip weight gradient over the gy it wrote: dw / db within
    1e-6 (the same terms; only fp contraction may differ), dgamma / dbeta the
    apply's bit for bit, run-to-run identical; with and without a SyncBN-style
    count in sums."""
    from ainp import ops
    g_ = torch.Generator(device=DEV).manual_seed(H + W)
    x = torch.randn(N, 1, H, W, device=DEV, generator=g_)
    g = torch.randn(N, H, W, 16, device=DEV, generator=g_)
    y = torch.randn(N, H, W, 16, device=DEV, generator=g_)
    sc = torch.rand(16, device=DEV, generator=g_) + 0.5
    sh = torch.randn(16, device=DEV, generator=g_) * 0.3
    gamma = torch.rand(16, device=DEV, generator=g_) + 0.5
    save = torch.stack([torch.randn(16, device=DEV, generator=g_) * 0.1,
                        torch.rand(16, device=DEV, generator=g_) + 0.5])
    sums = ops.bn_relu_bwd_reduce(g, y, sc, sh, save, cl=True)
    cnt = N * H * W
    for s_, c_ in ((sums, cnt), (torch.cat([sums, torch.tensor([float(cnt)], device=DEV,
                                                               dtype=torch.float64)]), 0)):
        gy, dg0, db0 = ops.bn_relu_bwd_apply(g, y, sc, sh, gamma, save, s_, c_, cl=True)
        dw0, dbias0 = ops.conv3x3_wgrad(x, gy, gcl=True)
        dw, dbias, dg, db = ops.conv3x3_wgrad_bnapply(x, None, None, g, y, sc, sh, gamma, save,
                                                      s_, c_)
        assert rel(dw, dw0) < 1e-6 and rel(dbias, dbias0) < 1e-6
        assert torch.equal(dg, dg0) and torch.equal(db, db0)
        dw2, dbias2, _, _ = ops.conv3x3_wgrad_bnapply(x, None, None, g, y, sc, sh, gamma, save,
                                                      s_, c_)
        assert torch.equal(dw2, dw) and torch.equal(dbias2, dbias)


@pytest.mark.parametrize("C", [16, 32, 64])
@pytest.mark.parametrize("store", ["f32", "y16", "g16", "gy16"])
def test_cl_bn_relu_backward(C, store):
    """Channel-last BatchNorm+ReLU backward (reduce + apply) against the NCHW
    kernels: sums within 1e-6 (fixed-order partials of another grouping),
    gy within 1e-6, dgamma / dbeta the sums; bf16 storage of y / g / gy."""
    from ainp import ops
    N, H, W = 3, 57, 110
    g = torch.Generator(device=DEV).manual_seed(C)
    y = torch.randn(N, C, H, W, device=DEV, generator=g)
    gr = torch.randn(N, C, H, W, device=DEV, generator=g)
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.3
    save = torch.stack([torch.randn(C, device=DEV, generator=g) * 0.1,
                        torch.rand(C, device=DEV, generator=g) + 0.5])
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    if store == "y16":
        y = y.to(torch.bfloat16)
    gin = gr.to(torch.bfloat16).float() if store == "g16" else gr
    s0 = ops.bn_relu_bwd_reduce(gin, y, sc, sh, save)
    gy0, dg0, db0 = ops.bn_relu_bwd_apply(gin, y, sc, sh, gamma, save, s0, N * H * W,
                                          gy16=store == "gy16")
    gcl = _cl(gr.to(torch.bfloat16)) if store == "g16" else _cl(gr)
    s1 = ops.bn_relu_bwd_reduce(gcl, _cl(y), sc, sh, save, cl=True)
    assert rel(s1, s0) < 1e-6
    gy1, dg1, db1 = ops.bn_relu_bwd_apply(gcl, _cl(y), sc, sh, gamma, save, s0, N * H * W,
                                          gy16=store == "gy16", cl=True)
    assert gy1.dtype == gy0.dtype
    if store == "gy16":   # the same fp32 values rounded once
        assert rel(_nchw(gy1).float(), gy0.float()) < 4e-3
    else:
        assert rel(_nchw(gy1), gy0) < 1e-6
    assert torch.equal(dg1, dg0) and torch.equal(db1, db0)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_cnnblstm_step_channel_last_matches_nchw(monkeypatch, dtype):
    """One training step of the CNNBLSTM at the C2 plane (N=4) with the
    channel-last conv stacks (default) and with NCHW (AINP_CL=0): the loss
    within 1e-6 (fp32) / 1e-4 (bf16), every gradient within 2e-4 (fp32) /
    5e-2 (bf16, see below)."""
    from ainp import cnnblstm
    cfg = {"data": {"sample_rate": 16000, "spectrogram": {"n_fft": 512, "hop_length": 192,
                                                          "win_length": 384}},
           "model": {"in_channels": 1, "num_lstm_layers": 2, "lstm_hidden_dim": 128,
                     "enc_filters": [16, 32], "dec_filters": [16, 32]},
           "accel": {"dtype": dtype}}
    g = torch.Generator().manual_seed(3)
    N, F, T = 4, 257, 334
    x = (torch.randn(N, 1, F, T, generator=g) - 2.0).to(DEV)
    mask = torch.zeros(N, F, T)
    for i in range(N):
        mask[i, :, 40 + 30 * i:57 + 30 * i] = 1.0
    mask = mask.to(DEV)
    tgt = torch.complex(torch.rand(N, F, T, generator=g), torch.rand(N, F, T, generator=g)).to(DEV)
    res = []
    for cl in (True, False):
        monkeypatch.setattr(cnnblstm, "CL", cl)
        torch.manual_seed(0)
        m = cnnblstm.StackedBLSTMCNN(config=cfg).to(DEV).train()
        loss = cnnblstm.l1_pow10_loss(m(x), mask, tgt)
        loss.backward()
        torch.cuda.synchronize()
        res.append((float(loss.detach()),
                    {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    # the forward: the split-bf16 convs are bit-identical (same staging and
    # MFMA chains, same BatchNorm partials); since round 6 the 1 <-> 16
    # channel convs run on row strips in the channel-last layout (the 16 -> 1
    # output and the 1 -> 16 BatchNorm partials summed in another order), so
    # the loss agrees to fp32 rounding (bf16: to the bf16 rounding points'
    # flips downstream of those ulps, 1e-4).  The BatchNorm backward sums in
    # another order, which the cancellation in gamma*rstd*(gz - mean(gz) -
    # xhat*mean(gz*xhat)) amplifies towards the encoder's first conv (5e-5
    # there in fp32).  bf16: with the forward no longer bit-identical, a
    # perturbation of a few fp32 ulps flips single bf16 roundings, and the
    # pow10 loss concentrates the gradient on its largest outputs, so one flip
    # there moves whole gradients by up to ~4 % at this N=4 shape (measured
    # 3.7e-2 max; AINP_SMALL_ROWS=0, the tile kernels on both layouts: within
    # 2e-3 as before) -- bf16 against the fp32 reference is gated in
    # test_gpu_model.py
    tol = 2e-4 if dtype == "fp32" else 5e-2
    assert abs(res[0][0] - res[1][0]) <= (1e-6 if dtype == "fp32" else 1e-4) * abs(res[1][0])
    errs = {}
    for n, g1 in res[1][1].items():
        if n in ("encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "decoder.0.bias",
                 "decoder.3.bias"):
            continue   # BatchNorm-fed conv biases: exact gradient 0
        errs[n] = rel(res[0][1][n], g1)
    bad = {n: e for n, e in errs.items() if e >= tol}
    assert not bad, (bad, max(errs.values()))


@pytest.mark.parametrize("y16", [False, True])
@pytest.mark.parametrize("H,W", [(257, 334), (130, 70)])
def test_cl_ntcf_bridge_and_backward(y16, H, W):
    """The encoder's last block with y channel-last: the bridge to the LSTM
    layout (fp32 X, bf16 X / X^T) bit-identical to the NCHW bridges; the
    BatchNorm backward from the NTCF gradient within 1e-6 (sums) / bit-level
    (apply of the same sums)."""
    from ainp import ops
    N, C = 2, 64
    g = torch.Generator(device=DEV).manual_seed(H + W)
    y = torch.randn(N, C, H, W, device=DEV, generator=g)
    if y16:
        y = y.to(torch.bfloat16)
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.3
    save = torch.stack([torch.randn(C, device=DEV, generator=g) * 0.1,
                        torch.rand(C, device=DEV, generator=g) + 0.5])
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    X0 = ops.bn_relu_apply(y.float(), sc, sh, ntcf=True)
    X1, x16 = ops.bn_relu_apply_ntcf_cl(_cl(y), sc, sh, out32=True, out16=True)
    assert torch.equal(X1, X0)
    X16_0, XT16_0 = ops.bn_relu_apply_ntcf_bf16(y, sc, sh)
    assert torch.equal(x16[0], X16_0) and torch.equal(x16[1], XT16_0)
    gr = torch.randn(N, W, C * H, device=DEV, generator=g)
    s0 = ops.bn_relu_bwd_reduce(gr, y, sc, sh, save, ntcf=True)
    s1 = ops.bn_relu_bwd_reduce(gr, _cl(y), sc, sh, save, ntcf=True, cl=True)
    assert rel(s1, s0) < 1e-6
    for gy16 in (False, True):
        gy0, dg0, db0 = ops.bn_relu_bwd_apply(gr, y, sc, sh, gamma, save, s0, N * H * W,
                                              ntcf=True, gy16=gy16)
        gy1, dg1, db1 = ops.bn_relu_bwd_apply(gr, _cl(y), sc, sh, gamma, save, s0, N * H * W,
                                              ntcf=True, gy16=gy16, cl=True)
        assert rel(_nchw(gy1).float(), gy0.float()) < (4e-3 if gy16 else 1e-6)
        assert torch.equal(dg1, dg0) and torch.equal(db1, db0)


def test_cnnblstm_bf16_step_kmajor_weight_gradient_bit_identical(monkeypatch):
    """bf16 CNNBLSTM step with the layer-0 weight gradient read from k-major
    dg / X (ops.B16_KM: no X^T from the bridge, no dg^T copy) against the
    transposed-copy path: the same MFMAs in the same k order, so the loss and
    every gradient are bit-identical (models/CNNBLSTM/model.py:46-47,77)."""
    from ainp import cnnblstm, ops
    cfg = {"data": {"sample_rate": 16000, "spectrogram": {"n_fft": 512, "hop_length": 192,
                                                          "win_length": 384}},
           "model": {"in_channels": 1, "num_lstm_layers": 2, "lstm_hidden_dim": 128,
                     "enc_filters": [16, 32], "dec_filters": [16, 32]},
           "accel": {"dtype": "bf16"}}
    g = torch.Generator().manual_seed(5)
    N, F, T = 4, 257, 336            # N*T % 32 == 0: the pair's k-major operand rule
    x = (torch.randn(N, 1, F, T, generator=g) - 2.0).to(DEV)
    mask = torch.zeros(N, F, T)
    for i in range(N):
        mask[i, :, 40 + 30 * i:57 + 30 * i] = 1.0
    mask = mask.to(DEV)
    tgt = torch.complex(torch.rand(N, F, T, generator=g), torch.rand(N, F, T, generator=g)).to(DEV)
    res = []
    for km in (True, False):
        monkeypatch.setattr(ops, "B16_KM", km)
        torch.manual_seed(0)
        m = cnnblstm.StackedBLSTMCNN(config=cfg).to(DEV).train()
        loss = cnnblstm.l1_pow10_loss(m(x), mask, tgt)
        loss.backward()
        torch.cuda.synchronize()
        res.append((float(loss.detach()),
                    {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    assert res[0][0] == res[1][0]
    for n, g1 in res[1][1].items():
        assert torch.equal(res[0][1][n], g1), n


# (conv Cin, Cout) whose data gradient feeds a BatchNorm+ReLU in the model:
# encoder 32 -> 64 (64 -> 32 dgrad, 8-row tiles / the bf16 LDS-DMA kernel),
# encoder 16 -> 32 and decoder 32 -> 16 (persistent x6q / x6p), decoder
# 16 -> 1 (small conv: the unfused two-pass path)
BNR_PAIRS = [(32, 64), (16, 32), (32, 16), (16, 1)]


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("N,H,W", SHAPES)
@pytest.mark.parametrize("cin,cout", BNR_PAIRS)
def test_dgrad_bnr_fused_reduce(cin, cout, N, H, W, bf16):
    """ops.conv3x3_dgrad_bnr (round 5): dx bit-identical to the channel-last
    data gradient, and the fused BatchNorm-backward sums within 1e-6 of the
    separate channel-last reduce over that dx (the same fp32 terms
    gz = dx * [y*scale+shift > 0], gz * (y - mean) * rstd, summed in another
    fixed order); y in fp32 and in bf16 storage; run-to-run identical."""
    from ainp import ops
    x, dy, w, b, sc, sh = _data(N, cin, cout, H, W, cin * 11 + cout)
    g = torch.Generator(device=DEV).manual_seed(cin + cout + H)
    y = torch.randn(N, H, W, cin, device=DEV, generator=g)
    bsc = torch.rand(cin, device=DEV, generator=g) + 0.5
    bsh = torch.randn(cin, device=DEV, generator=g) * 0.3
    save = torch.stack([torch.randn(cin, device=DEV, generator=g) * 0.1,
                        torch.rand(cin, device=DEV, generator=g) + 0.5])
    small = cout == 1
    dys = [_cl(dy)] + ([_cl(dy).to(torch.bfloat16)] if bf16 and not small else [])
    for d in dys:
        dx0 = ops.conv3x3_dgrad(d, w, bf16=bf16, xcl=True, ycl=True)
        for yy in (y, y.to(torch.bfloat16)):
            dx, s = ops.conv3x3_dgrad_bnr(d, w, yy, bsc, bsh, save, bf16=bf16, xcl=True)
            assert torch.equal(dx, dx0), (d.dtype, yy.dtype)
            s0 = ops.bn_relu_bwd_reduce(dx0, yy, bsc, bsh, save, cl=True)
            assert rel(s, s0) < 1e-6, (d.dtype, yy.dtype, rel(s, s0))
            dx2, s2 = ops.conv3x3_dgrad_bnr(d, w, yy, bsc, bsh, save, bf16=bf16, xcl=True)
            assert torch.equal(dx2, dx) and torch.equal(s2, s)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_cnnblstm_step_bn_apply_fusions_match_unfused(monkeypatch, dtype):
    """Round 6: a CNNBLSTM step with the BatchNorm+ReLU backward applies of
    the 16-channel layers fused into the 1 <-> 16 convs (cnnblstm.FUSE_BNA0:
    encoder.0's weight gradient forms gy itself; FUSE_BNA6: decoder.6's data
    gradient is recomputed into decoder.5's apply) against the unfused passes:
    the same loss, every gradient within 2e-4 (fp32) / 2e-3 (bf16) -- the
    same terms, only fp contraction may differ."""
    from ainp import cnnblstm
    cfg = {"data": {"sample_rate": 16000, "spectrogram": {"n_fft": 512, "hop_length": 192,
                                                          "win_length": 384}},
           "model": {"in_channels": 1, "num_lstm_layers": 2, "lstm_hidden_dim": 128,
                     "enc_filters": [16, 32], "dec_filters": [16, 32]},
           "accel": {"dtype": dtype}}
    g = torch.Generator().manual_seed(9)
    N, F, T = 4, 257, 334
    x = (torch.randn(N, 1, F, T, generator=g) - 2.0).to(DEV)
    mask = torch.zeros(N, F, T)
    for i in range(N):
        mask[i, :, 40 + 30 * i:57 + 30 * i] = 1.0
    mask = mask.to(DEV)
    tgt = torch.complex(torch.rand(N, F, T, generator=g), torch.rand(N, F, T, generator=g)).to(DEV)
    res = []
    for fused in (True, False):
        monkeypatch.setattr(cnnblstm, "FUSE_BNA0", fused)
        monkeypatch.setattr(cnnblstm, "FUSE_BNA6", fused)
        torch.manual_seed(0)
        m = cnnblstm.StackedBLSTMCNN(config=cfg).to(DEV).train()
        loss = cnnblstm.l1_pow10_loss(m(x), mask, tgt)
        loss.backward()
        torch.cuda.synchronize()
        res.append((float(loss.detach()),
                    {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    tol = 2e-4 if dtype == "fp32" else 2e-3
    assert res[0][0] == res[1][0]
    bad = {}
    for n, g1 in res[1][1].items():
        if n in ("encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "decoder.0.bias",
                 "decoder.3.bias"):
            continue   # BatchNorm-fed conv biases: exact gradient 0
        e = rel(res[0][1][n], g1)
        if e >= tol:
            bad[n] = e
    assert not bad, bad


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_cnnblstm_step_dgrad_bnr_matches_two_pass(monkeypatch, dtype):
    """A CNNBLSTM step with the fused data-gradient + BatchNorm reduce
    (cnnblstm.DGRAD_BNR, default) against the two-pass backward: the same
    loss, every gradient within 2e-4 (fp32) / 2e-3 (bf16) -- only the
    summation order of the BatchNorm-backward sums differs."""
    from ainp import cnnblstm
    cfg = {"data": {"sample_rate": 16000, "spectrogram": {"n_fft": 512, "hop_length": 192,
                                                          "win_length": 384}},
           "model": {"in_channels": 1, "num_lstm_layers": 2, "lstm_hidden_dim": 128,
                     "enc_filters": [16, 32], "dec_filters": [16, 32]},
           "accel": {"dtype": dtype}}
    g = torch.Generator().manual_seed(7)
    N, F, T = 4, 257, 334
    x = (torch.randn(N, 1, F, T, generator=g) - 2.0).to(DEV)
    mask = torch.zeros(N, F, T)
    for i in range(N):
        mask[i, :, 40 + 30 * i:57 + 30 * i] = 1.0
    mask = mask.to(DEV)
    tgt = torch.complex(torch.rand(N, F, T, generator=g), torch.rand(N, F, T, generator=g)).to(DEV)
    res = []
    for fused in (True, False):
        monkeypatch.setattr(cnnblstm, "DGRAD_BNR", fused)
        torch.manual_seed(0)
        m = cnnblstm.StackedBLSTMCNN(config=cfg).to(DEV).train()
        loss = cnnblstm.l1_pow10_loss(m(x), mask, tgt)
        loss.backward()
        torch.cuda.synchronize()
        res.append((float(loss.detach()),
                    {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    tol = 2e-4 if dtype == "fp32" else 2e-3
    assert res[0][0] == res[1][0]
    errs = {}
    for n, g1 in res[1][1].items():
        if n in ("encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "decoder.0.bias",
                 "decoder.3.bias"):
            continue   # BatchNorm-fed conv biases: exact gradient 0
        errs[n] = rel(res[0][1][n], g1)
    bad = {n: e for n, e in errs.items() if e >= tol}
    assert not bad, (bad, max(errs.values()))


@pytest.mark.parametrize("pro", [True, False])
@pytest.mark.parametrize("N,H,W", SHAPES + [(3, 70, 50)])
def test_wgrad16_dma_matches_register_kernel(N, H, W, pro):
    """Round 6: the bf16 channel-last 32 -> 64 weight gradient on the LDS-DMA
    kernel (conv3x3_wgrad_b16dma_kernel: bf16 x and dy channel-last, the
    BatchNorm+ReLU prologue applied in LDS) stages the same bf16 operands as
    the register kernel (conv3x3_wgrad_x6, NCHW launch of the same tensors) and
    sums the same products in another fixed order: dw / db within 1e-6 of it,
    within 2e-5 of an fp64 weight gradient of the bf16-rounded operands, and
    run-to-run identical."""
    from ainp import ops
    import torch.nn.functional as Fnn  # noqa: F401
    x, dy, w, b, sc, sh = _data(N, 32, 64, H, W, 321 + H)
    x16, dy16 = x.to(torch.bfloat16), dy.to(torch.bfloat16)
    s_, h_ = (sc, sh) if pro else (None, None)
    dw0, db0 = ops.conv3x3_wgrad(x16, dy16, s_, h_, bf16=True)                 # register kernel
    dw, db = ops.conv3x3_wgrad(_cl(x16), _cl(dy16), s_, h_, bf16=True, xcl=True, gcl=True)
    dw2, db2 = ops.conv3x3_wgrad(_cl(x16), _cl(dy16), s_, h_, bf16=True, xcl=True, gcl=True)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    assert rel(dw, dw0) < 1e-6 and rel(db, db0) < 1e-6, (rel(dw, dw0), rel(db, db0))
    xa = x16.double()
    if pro:   # the kernels' fp32 prologue, rounded to bf16 once
        xa = torch.relu(torch.addcmul(sh.view(1, -1, 1, 1).float(), x16.float(),
                                      sc.view(1, -1, 1, 1))).to(torch.bfloat16).double()
    dwr = torch.nn.grad.conv2d_weight(xa, w.shape, dy16.double(), padding=1)
    assert rel(dw, dwr) < 2e-5, rel(dw, dwr)
    assert rel(db, dy16.double().sum((0, 2, 3))) < 1e-6


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("N,H,W", SHAPES + [(3, 17, 15), (1, 1, 1)])
@pytest.mark.parametrize("cin,cout", [(16, 32), (32, 16)])
def test_wgrad_x6s_tile_rows(monkeypatch, cin, cout, N, H, W, bf16):
    """Round 6: conv3x3_wgrad_x6s (the 16 <-> 32 channel weight gradients) on
    4-, 8- and 16-row tiles (AINP_X6S_FT3 / _FT1; NP = 3 defaults to 8 rows,
    NP = 1 to 4, 16 rows only with one plane).  Another tile partition sums
    the slabs in another fixed order: dw / db within 1e-5 of the 4-row tiles,
    run-to-run identical, and within 1e-5 (fp32) / 2e-5 (bf16 operands) of an
    fp64 weight gradient; channel-last and NCHW launches bit-identical."""
    from ainp import ops
    x, dy, w, b, sc, sh = _data(N, cin, cout, H, W, 77 + cin + H)
    if bf16:
        dy = dy.to(torch.bfloat16)
    key, fts = ("AINP_X6S_FT1", (4, 8, 16)) if bf16 else ("AINP_X6S_FT3", (4, 8))
    xa = torch.relu(torch.addcmul(sh.view(1, -1, 1, 1), x, sc.view(1, -1, 1, 1)))
    if bf16:   # the kernels stage act(x) rounded to bf16
        xa = xa.to(torch.bfloat16)
    dwr = torch.nn.grad.conv2d_weight(xa.double(), w.shape, dy.double(), padding=1)
    dbr = dy.double().sum((0, 2, 3))
    ref = None
    for ft in fts:
        monkeypatch.setenv(key, str(ft))
        dw, db = ops.conv3x3_wgrad(_cl(x), _cl(dy), sc, sh, bf16=bf16, xcl=True, gcl=True)
        dw2, db2 = ops.conv3x3_wgrad(_cl(x), _cl(dy), sc, sh, bf16=bf16, xcl=True, gcl=True)
        dwn, dbn = ops.conv3x3_wgrad(x, dy, sc, sh, bf16=bf16)
        assert torch.equal(dw, dw2) and torch.equal(db, db2), ft
        assert torch.equal(dw, dwn) and torch.equal(db, dbn), ft
        assert rel(dw, dwr) < (2e-5 if bf16 else 1e-5), (ft, rel(dw, dwr))
        assert rel(db, dbr) < 1e-6, (ft, rel(db, dbr))
        if ref is None:
            ref = (dw, db)
        assert rel(dw, ref[0]) < 1e-5 and rel(db, ref[1]) < 1e-5, ft


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_cnnblstm_step_blstm_issue_order_bit_identical(monkeypatch, dtype):
    """Round 6, cnnblstm.SIDE_LAG: the BLSTM backward issues each layer's
    side-stream weight-gradient launches after the next layer's recurrence
    launch (default), right after the layer's data gradient (SIDE_LAG off), or
    before it (ops.MAIN_FIRST off) -- the same kernels on the same streams, so
    the loss and every gradient are bit-identical."""
    from ainp import cnnblstm, ops
    cfg = {"data": {"sample_rate": 16000, "spectrogram": {"n_fft": 512, "hop_length": 192,
                                                          "win_length": 384}},
           "model": {"in_channels": 1, "num_lstm_layers": 3, "lstm_hidden_dim": 128,
                     "enc_filters": [16, 32], "dec_filters": [16, 32]},
           "accel": {"dtype": dtype}}
    g = torch.Generator().manual_seed(13)
    N, F, T = 3, 257, 96
    x = (torch.randn(N, 1, F, T, generator=g) - 2.0).to(DEV)
    mask = torch.zeros(N, F, T)
    for i in range(N):
        mask[i, :, 10 + 20 * i:27 + 20 * i] = 1.0
    mask = mask.to(DEV)
    tgt = torch.complex(torch.rand(N, F, T, generator=g), torch.rand(N, F, T, generator=g)).to(DEV)
    res = []
    for lag, main_first in ((True, True), (False, True), (False, False)):
        monkeypatch.setattr(cnnblstm, "SIDE_LAG", lag)
        monkeypatch.setattr(ops, "MAIN_FIRST", main_first)
        torch.manual_seed(0)
        m = cnnblstm.StackedBLSTMCNN(config=cfg).to(DEV).train()
        loss = cnnblstm.l1_pow10_loss(m(x), mask, tgt)
        loss.backward()
        torch.cuda.synchronize()
        res.append((float(loss.detach()),
                    {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    for loss_k, grads_k in res[1:]:
        assert loss_k == res[0][0]
        diff = [n for n, g0 in res[0][1].items() if not torch.equal(g0, grads_k[n])]
        assert not diff, diff
