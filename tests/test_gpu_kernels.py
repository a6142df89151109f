"""Kernel-level parity: each libainp entry point vs its CPU reference.

STFT/features/masks are checked against the oracle (oracle/stft_ref.py; masks
bit-exact, floats to the stated tolerance).  Floating-point NN kernels (GEMM,
conv, BatchNorm, LSTM, loss, Adam) are checked against a float64 PyTorch-CPU
evaluation of the same op (the reference's own backend), relative L2 <= 1e-5
unless stated.
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as Fnn

from oracle import stft_ref
from ainp import synth

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def ops():
    from ainp import ops as _ops
    return _ops


# ------------------------------------------------------------------ STFT
@pytest.mark.parametrize("S,n_fft,hop,win,n_frames", [
    (8000, 512, 192, 384, None),
    (80000, 512, 192, 384, 334),     # dataset: 5 s load, slice to 4 s of frames
    (64000, 512, 192, 384, 334),
    (4000, 64, 16, 48, None),
    (80000, 512, 192, 384, 420),     # more frames than the STFT has -> zeros
])
def test_stft_cnnblstm_vs_oracle(ops, S, n_fft, hop, win, n_frames):
    B = 3
    clips = np.stack([synth.synthetic_clip(10 + i, S) for i in range(B)])
    g = 3200 if S > 8000 else S // 20
    rng = np.random.default_rng(5)
    starts = rng.integers(0, S - g, size=B)
    starts[0] = 0                      # gap touching the start
    starts[-1] = S - g - 1             # gap at the very end
    T = n_frames if n_frames is not None else 1 + S // hop
    a = torch.from_numpy(clips).to(DEV)
    gs = torch.from_numpy(starts.astype(np.int64)).to(DEV)
    lg, tg, mk, _ = ops.stft_features(a, gs, g, n_fft, hop, win, n_frames=T)
    torch.cuda.synchronize()
    for b in range(B):
        rl, rt, rm = stft_ref.cnnblstm_item(clips[b], int(starts[b]), g, n_fft, hop, win,
                                            16000, T)
        np.testing.assert_array_equal(mk[b].cpu().numpy(), rm)
        assert np.max(np.abs(lg[b].cpu().numpy() - rl)) < 2e-5
        tt = tg[b].cpu().numpy()
        assert np.max(np.abs(tt - rt)) <= 2e-6 * max(1.0, np.abs(rt).max())


@pytest.mark.parametrize("S,n_fft,hop,win", [(80000, 512, 128, 512), (128000, 512, 128, 512),
                                             (3000, 64, 16, 64)])
def test_stft_gan_vs_oracle(ops, S, n_fft, hop, win):
    B = 2
    clips = np.stack([synth.synthetic_clip(20 + i, S) for i in range(B)])
    g = 3200 if S >= 80000 else 200
    starts = np.array([0, S - g], dtype=np.int64)  # inclusive max (utils.py:134)
    a = torch.from_numpy(clips).to(DEV)
    gs = torch.from_numpy(starts).to(DEV)
    o0, o1, o2, o3 = ops.stft_features(a, gs, g, n_fft, hop, win, mode=ops.FEAT_GAN)
    torch.cuda.synchronize()
    for b in range(B):
        r0, r1, r2, r3 = stft_ref.gan_item(clips[b], int(starts[b]), g, n_fft, hop, win)
        np.testing.assert_array_equal(o3[b].cpu().numpy(), r3)
        assert np.max(np.abs(o0[b].cpu().numpy() - r0)) < 1e-5
        assert np.max(np.abs(o1[b].cpu().numpy() - r1)) < 1e-5
        ph = o2[b].cpu().numpy()
        d = np.abs(np.angle(np.exp(1j * (ph - r2))))  # wrap-aware
        mag = np.expm1(r0)
        assert np.max(d[mag > 1e-3]) < 1e-4


def _feat_generic(ops, *a, **k):
    """The generic (one-wave-per-frame radix-2) kernel, for cross-checks of the
    n_fft=512 tiled kernel."""
    os.environ["AINP_STFT_GENERIC"] = "1"
    try:
        return ops.stft_features(*a, **k)
    finally:
        del os.environ["AINP_STFT_GENERIC"]


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("S,hop,win,n_frames,g", [
    (64000, 192, 384, 334, 3200),      # C2
    (80000, 128, 512, None, 3200),     # C4
    (128000, 128, 512, None, 1600),    # C5
    (9001, 193, 384, 60, 700),         # odd hop and length: scalar-load variant
    (8000, 192, 384, 50, 0),           # no gap
    (6000, 160, 400, 45, 5999),        # gap covering almost everything, frames past the end
])
def test_stft512_tiled_vs_generic_and_oracle(ops, mode, S, hop, win, n_frames, g):
    """Tiled n_fft=512 kernel vs the generic kernel and the oracle: masks
    bit-exact, log-magnitudes / complex target / phase to the oracle tolerance;
    several examples per clip through clip_index; gaps at the edges."""
    n_clips, B = 2, 5
    clips = np.stack([synth.synthetic_clip(70 + i, S) for i in range(n_clips)])
    ci = np.array([0, 1, 0, 1, 1], np.int32)
    hi = S - g + (1 if mode == 1 else 0)
    starts = np.array([0, max(hi - 1, 0), 1234 % max(hi, 1), 77 % max(hi, 1), hi // 2], np.int64)
    a = torch.from_numpy(clips).to(DEV)
    gs = torch.from_numpy(starts).to(DEV)
    cidx = torch.from_numpy(ci).to(DEV)
    T = n_frames if n_frames is not None else 1 + S // hop
    kw = dict(n_frames=T, mode=mode, clip_index=cidx)
    new = ops.stft_features(a, gs, g, 512, hop, win, **kw)
    old = _feat_generic(ops, a, gs, g, 512, hop, win, **kw)
    torch.cuda.synchronize()
    mi = 2 if mode == 0 else 3
    np.testing.assert_array_equal(new[mi].cpu().numpy(), old[mi].cpu().numpy())
    for b in range(B):
        clip = clips[ci[b]]
        if mode == 0:
            rl, rt, rm = stft_ref.cnnblstm_item(clip, int(starts[b]), g, 512, hop, win, 16000, T)
            np.testing.assert_array_equal(new[2][b].cpu().numpy(), rm)
            assert np.max(np.abs(new[0][b].cpu().numpy() - rl)) < 2e-5
            tt = new[1][b].cpu().numpy()
            assert np.max(np.abs(tt - rt)) <= 2e-6 * max(1.0, np.abs(rt).max())
        else:
            r0, r1, r2, r3 = stft_ref.gan_item(clip, int(starts[b]), g, 512, hop, win)
            Tc = min(T, r0.shape[1])       # frames past 1 + S//hop are zero
            o = [new[i][b].cpu().numpy() for i in range(4)]
            np.testing.assert_array_equal(o[3][:, :Tc], r3[:, :Tc])
            assert np.max(np.abs(o[0][:, :Tc] - r0[:, :Tc])) < 1e-5
            assert np.max(np.abs(o[1][:, :Tc] - r1[:, :Tc])) < 1e-5
            d = np.abs(np.angle(np.exp(1j * (o[2][:, :Tc] - r2[:, :Tc]))))
            assert np.max(d[np.expm1(r0[:, :Tc]) > 1e-3]) < 1e-4
            assert not np.any(o[0][:, Tc:]) and not np.any(o[1][:, Tc:])
    # partial output requests (null planes) give the same values
    part = ops.stft_features(a, gs, g, 512, hop, win, outputs=(True, False, False, True), **kw)
    torch.cuda.synchronize()
    assert torch.equal(part[0], new[0])
    if mode == 1:
        assert torch.equal(part[3], new[3])


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("grid", [1, 7, 64])
def test_stft512_persistent_walk_bit_identical(ops, mode, grid, monkeypatch):
    """The persistent n_fft=512 kernel loads a tile's clean frames before the
    previous tile's write-out: with a grid of 1, 7 or 64 workgroups every
    workgroup walks many tiles (edge, gap and interior ones, odd tile counts),
    and the result must equal the one-tile-per-workgroup launch bit for bit."""
    S, hop, win, T, g, B = 64000, 192, 384, 334, 3200, 6
    clips = np.stack([synth.synthetic_clip(90 + i, S) for i in range(B)])
    starts = np.array([0, S - g - 1, 5000, 17001, 40000, 33333], np.int64)
    a = torch.from_numpy(clips).to(DEV)
    gs = torch.from_numpy(starts).to(DEV)
    kw = dict(n_frames=T, mode=mode)
    ref = ops.stft_features(a, gs, g, 512, hop, win, **kw)
    monkeypatch.setenv("AINP_STFT_GRID", str(grid))
    got = ops.stft_features(a, gs, g, 512, hop, win, **kw)
    part = ops.stft_features(a, gs, g, 512, hop, win, outputs=(True, False, False, True), **kw)
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(got, ref)):
        if x is not None:
            assert torch.equal(x, y), (mode, grid, i)
    assert torch.equal(part[0], ref[0])


def test_gap_frames_known_answers_n512(ops, golden_dir):
    """The Q3 known answers through the tiled n_fft=512 kernel (mask-only launch)."""
    cases = json.load(open(os.path.join(golden_dir, "gap_frames.json")))["cases"]
    for c in cases:
        rule = c["rule"]
        hop = c["hop"]
        if rule == "gan":
            T = c["n_frames"]
            S = T * hop - 1
        else:
            T = max(c["fe"], 1) + 2
            S = max(c["start"] + c["gap"] + 1, 1000)
        a = torch.zeros(1, S, device=DEV)
        gs = torch.tensor([c["start"]], device=DEV, dtype=torch.int64)
        mode = ops.FEAT_CNNBLSTM if rule == "cnnblstm" else ops.FEAT_GAN
        out = ops.stft_features(a, gs, c["gap"], 512, hop, 512, n_frames=T, mode=mode,
                                outputs=(False, False, rule == "cnnblstm", rule == "gan"))
        m = (out[2] if rule == "cnnblstm" else out[3])[0, 0].cpu().numpy()
        if rule == "cnnblstm":
            exp = np.zeros(T, np.float32)
            exp[c["fs"]:c["fe"]] = 1
        else:
            exp = np.ones(T, np.float32)
            if c["fe"] > c["fs"]:
                exp[c["fs"]:c["fe"]] = 0
        np.testing.assert_array_equal(m, exp, err_msg=str(c))


def test_gap_frames_known_answers(ops, golden_dir):
    """bit-exact frame indices incl. the float64 round-trip quirk."""
    cases = json.load(open(os.path.join(golden_dir, "gap_frames.json")))["cases"]
    for rule in ("cnnblstm", "gan"):
        sel = [c for c in cases if c["rule"] == rule]
        # one batch per hop (kernel takes one hop per launch)
        for hop in sorted({c["hop"] for c in sel}):
            cs = [c for c in sel if c["hop"] == hop]
            for c in cs:
                if rule == "gan":
                    T = c["n_frames"]
                    S = T * hop - 1          # 1 + S//hop == n_frames
                else:
                    T = max(c["fe"], 1) + 2
                    S = max(c["start"] + c["gap"] + 1, 1000)
                a = torch.zeros(1, S, device=DEV)
                gs = torch.tensor([c["start"]], device=DEV, dtype=torch.int64)
                mode = ops.FEAT_CNNBLSTM if rule == "cnnblstm" else ops.FEAT_GAN
                out = ops.stft_features(a, gs, c["gap"], 64, hop, 64, n_frames=T, mode=mode,
                                        outputs=(False, False, rule == "cnnblstm",
                                                 rule == "gan"))
                m = (out[2] if rule == "cnnblstm" else out[3])[0, 0].cpu().numpy()
                if rule == "cnnblstm":
                    exp = np.zeros(T, np.float32)
                    exp[c["fs"]:c["fe"]] = 1
                else:
                    exp = np.ones(T, np.float32)
                    if c["fe"] > c["fs"]:
                        exp[c["fs"]:c["fe"]] = 0
                np.testing.assert_array_equal(m, exp, err_msg=str(c))


# ------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("M,N,K", [(333, 130, 77), (256, 512, 1024), (1, 5, 3), (129, 4112, 256)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("ccol", [False, True])
def test_gemm_layouts(ops, M, N, K, ta, tb, exact, ccol):
    """Every operand layout; ccol: C column-major (computed as C^T = B^T A^T
    since round 5, the bias moving to the rows), with a bias and beta."""
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, N, generator=g, dtype=torch.float64)
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    ref = A @ B
    Ad = (A.t().contiguous() if ta else A).float().to(DEV)
    Bd = (B.t().contiguous() if tb else B).float().to(DEV)
    sam, sak = (1, M) if ta else (K, 1)
    sbk, sbn = (1, K) if tb else (N, 1)
    if not ccol:
        C = torch.empty(M, N, device=DEV)
        ops.gemm(M, N, K, [Ad], sam, sak, [Bd], sbk, sbn, [C], N, 1, exact=exact)
        assert rel(C.cpu(), ref) < 1e-5
        return
    Ct = C0.t().contiguous().float().to(DEV)       # [N, M]: C[m][n] at n*M + m
    ops.gemm(M, N, K, [Ad], sam, sak, [Bd], sbk, sbn, [Ct], 1, M, exact=exact, beta=0.5,
             bias1=[bias.float().to(DEV)])
    assert rel(Ct.cpu().t(), ref + bias + 0.5 * C0) < 1e-5


def test_gemm_x6_is_fp32_accurate(ops):
    """The default (three-piece bf16 split) path against fp64 on the CNNBLSTM
    layer-0 reduction length: its error is that of an fp32 GEMM, within 2x of
    the exact f32 MFMA path on the same fp32 inputs."""
    g = torch.Generator().manual_seed(5)
    M, N, K = 256, 384, 16448
    A = torch.randn(M, K, generator=g, dtype=torch.float64).float()
    B = (torch.randn(K, N, generator=g, dtype=torch.float64) * 0.01).float()
    ref = A.double() @ B.double()
    Ad, Bd = A.to(DEV), B.to(DEV)
    errs = {}
    for exact in (False, True):
        C = torch.empty(M, N, device=DEV)
        ops.gemm(M, N, K, [Ad], K, 1, [Bd], N, 1, [C], N, 1, exact=exact)
        errs[exact] = rel(C.cpu(), ref)
    # fp32 accumulation over K=16448 random terms: ~u*sqrt(K) ~ 1e-6 relative
    assert errs[True] < 1e-5 and errs[False] < 1e-5, errs
    # a bf16x3 split (dropping the 2^-16 terms) would sit ~4x above exact f32
    assert errs[False] < 2 * errs[True] + 1e-7, errs


@pytest.mark.parametrize("M,K,H", [(2304, 1024, 128), (700, 160, 64), (10688, 16448, 128)])
def test_gemm_x6nt_256_matches_x6_path(ops, M, K, H):
    """The fp32 layer-0 projection on the 256x256 LDS-DMA tile
    (ainp_gemm_x6nt_256): unsplit it is bit-identical to ainp_gemm_f32's
    default x6 loop (same split, products and order); split 3 (what the model
    uses) is an fp32 GEMM against fp64 (models/CNNBLSTM/model.py:46-47,77:
    x W_ih^T + b_ih + b_hh for both directions).  Row tails (M % 256) and the
    C2 shape included."""
    g = torch.Generator().manual_seed(11)
    A = torch.relu(torch.randn(M, K, generator=g)).to(DEV)
    wf = (torch.randn(4 * H, K, generator=g) * 0.02).to(DEV)
    wr = (torch.randn(4 * H, K, generator=g) * 0.02).to(DEV)
    b = [(torch.randn(4 * H, generator=g) * 0.1).to(DEV) for _ in range(4)]
    ref = torch.empty(M, 8 * H, device=DEV)
    ops.gemm(M, 4 * H, K, [A, A], K, 1, [wf, wr], 1, K, [ref, ref[:, 4 * H:]], 8 * H, 1,
             bias1=[b[0], b[2]], bias2=[b[1], b[3]], exact=False)
    y1 = torch.full((M, 8 * H), float("nan"), device=DEV)
    ops.gemm_x6nt_256(A, wf, wr, y1, bias=(b[0], b[1], b[2], b[3]), bias_nsplit=4 * H, nsplit=1)
    assert torch.equal(y1, ref)
    y3 = torch.empty(M, 8 * H, device=DEV)
    ops.gemm_x6nt_256(A, wf, wr, y3, bias=(b[0], b[1], b[2], b[3]), bias_nsplit=4 * H, nsplit=3)
    W = torch.cat([wf, wr]).double().cpu()
    bias = torch.cat([b[0] + b[1], b[2] + b[3]]).double().cpu()
    r64 = A.double().cpu() @ W.T + bias
    # an fp32 GEMM over K terms (~u*sqrt(K) relative): the split changes only
    # the summation order, so its error stays at the unsplit loop's level
    e3, e1 = rel(y3.cpu(), r64), rel(ref.cpu(), r64)
    assert e3 < 1e-5 and e1 < 1e-5, (e3, e1)
    assert e3 < 2 * e1 + 1e-7, (e3, e1)


@pytest.mark.parametrize("R,C", [(512, 16448), (77, 130), (1, 65)])
def test_transpose_f32_exact(ops, R, C):
    """ainp_transpose_f32 into a strided destination (the half of W_cat^T one
    direction's W_ih fills) is an exact copy."""
    g = torch.Generator().manual_seed(R + C)
    x = torch.randn(R, C, generator=g).to(DEV)
    out = torch.full((C, 2 * R), float("nan"), device=DEV)
    ops.transpose_f32(x, out=out[:, R:])
    assert torch.equal(out[:, R:], x.t())
    assert torch.isnan(out[:, :R]).all()


@pytest.mark.parametrize("M,N,H", [(2304, 1088, 128), (10688, 16448, 128)])
def test_layer0_dx_on_x6_256(ops, M, N, H):
    """The fp32 layer-0 data gradient dX = dg [M, 8H] . [W_f; W_r] (backward of
    models/CNNBLSTM/model.py:46-47) on the 256x256 split-pass tile with the
    transposed W_cat^T (bsplit == N, N % 256 != 0 tail tile) against fp64 and
    within 2x the error of the 128x128 x6 path it replaces."""
    g = torch.Generator().manual_seed(M + N)
    dg = (torch.randn(M, 8 * H, generator=g) * 0.1).to(DEV)
    wf = (torch.randn(4 * H, N, generator=g) * 0.02).to(DEV)
    wr = (torch.randn(4 * H, N, generator=g) * 0.02).to(DEV)
    wt = torch.empty(N, 8 * H, device=DEV)
    ops.transpose_f32(wf, out=wt[:, :4 * H])
    ops.transpose_f32(wr, out=wt[:, 4 * H:])
    dx = torch.full((M, N), float("nan"), device=DEV)
    ops.gemm_x6nt_256(dg, wt, wt[:0], dx, nsplit=1)
    old = torch.empty(M, N, device=DEV)
    ops.gemm(M, N, 4 * H, [dg, dg[:, 4 * H:]], 8 * H, 1, [wf, wr], N, 1, [old, old], N, 1,
             ksplit=True)
    r64 = dg.double().cpu() @ torch.cat([wf, wr]).double().cpu()
    e_new, e_old = rel(dx.cpu(), r64), rel(old.cpu(), r64)
    assert e_new < 1e-5 and e_old < 1e-5, (e_new, e_old)
    assert e_new < 2 * e_old + 1e-7, (e_new, e_old)


def _bf(t):
    """fp64 copy of t rounded to fp32, then to bf16 (nearest-even)."""
    return t.float().bfloat16().double()


@pytest.mark.parametrize("M,N,K", [(333, 130, 77), (256, 512, 1024), (129, 4112, 256),
                                   (1, 5, 3)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm_bf16_layouts(ops, M, N, K, ta, tb):
    """AINP_GEMM_BF16: operands rounded to bf16 (as torch autocast does),
    fp32 accumulation -> equal to the fp64 product of the bf16 operands up to
    fp32 accumulation error."""
    g = torch.Generator().manual_seed(M * 11 + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, N, generator=g, dtype=torch.float64)
    ref = _bf(A) @ _bf(B)
    Ad = (A.t().contiguous() if ta else A).float().to(DEV)
    Bd = (B.t().contiguous() if tb else B).float().to(DEV)
    C = torch.empty(M, N, device=DEV)
    sam, sak = (1, M) if ta else (K, 1)
    sbk, sbn = (1, K) if tb else (N, 1)
    ops.gemm(M, N, K, [Ad], sam, sak, [Bd], sbk, sbn, [C], N, 1, bf16=True)
    assert rel(C.cpu(), ref) < 1e-5
    # and it is a bf16 product: far from the fp32 one on random data
    assert rel(C.cpu(), A @ B) > 1e-4


@pytest.mark.parametrize("N,Cin,Cout,H,W,pro", [
    (2, 32, 64, 257, 334, True), (2, 16, 32, 257, 334, True), (2, 32, 16, 257, 334, True),
    (2, 64, 32, 40, 70, False), (1, 32, 64, 19, 47, False)])
def test_conv3x3_bf16(ops, N, Cin, Cout, H, W, pro):
    """AINP_CONV_BF16 on the 16/32/64-channel pairs: act(x) (BatchNorm+ReLU
    prologue in fp32), weights and dy rounded to bf16, fp32 accumulation; fp32
    bias, outputs and BatchNorm partials.  Checked against fp64 convolutions
    of the bf16-rounded operands."""
    g = torch.Generator().manual_seed(N * 1000 + Cin * 10 + Cout)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).float().double()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) * 0.2).float().double()
    b = torch.randn(Cout, generator=g, dtype=torch.float64).float().double()
    sc = (torch.rand(Cin, generator=g, dtype=torch.float64) + 0.5).float().double() if pro else None
    sh = (torch.randn(Cin, generator=g, dtype=torch.float64) * 0.3).float().double() if pro else None
    xa = _act(x, sc, sh).float().double()        # fp32 prologue (fmaf: one rounding)
    yr = Fnn.conv2d(_bf(xa), _bf(w), b, padding=1)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64).float().double()
    d = lambda t: None if t is None else t.float().to(DEV)  # noqa: E731
    y, stats = ops.conv3x3_fwd(d(x), d(w), d(b), d(sc), d(sh), want_stats=True, bf16=True)
    assert rel(y.cpu(), yr) < 2e-5
    st = stats.sum(0).cpu()
    assert rel(st[:Cout], yr.sum((0, 2, 3))) < 2e-5
    dxr = torch.nn.grad.conv2d_input(xa.shape, _bf(w), _bf(dy), padding=1)
    dx = ops.conv3x3_dgrad(d(dy), d(w), bf16=True)
    assert rel(dx.cpu(), dxr) < 2e-5
    dw, db = ops.conv3x3_wgrad(d(x), d(dy), d(sc), d(sh), bf16=True)
    if (Cin, Cout) in ((32, 64), (16, 32), (32, 16)):   # the model's weight gradients
        dwr = torch.nn.grad.conv2d_weight(_bf(xa), w.shape, _bf(dy), padding=1)
        assert rel(dw.cpu(), dwr) < 2e-5
    else:   # no bf16 weight-gradient kernel for this pair: the fp32-accurate one serves it
        dwr = torch.nn.grad.conv2d_weight(xa, w.shape, dy, padding=1)
        assert rel(dw.cpu(), dwr) < 1e-5
    assert rel(db.cpu(), dy.sum((0, 2, 3))) < 1e-5
    # genuinely bf16 (not the fp32-accurate path)
    assert rel(y.cpu(), Fnn.conv2d(xa, w, b, padding=1)) > 1e-5


def test_gemm_batched_bias_ksplit(ops):
    g = torch.Generator().manual_seed(3)
    M, N, K, nb = 100, 96, 40, 3
    A = torch.randn(nb, M, K, generator=g, dtype=torch.float64)
    B = torch.randn(nb, K, N, generator=g, dtype=torch.float64)
    b1 = torch.randn(N, generator=g, dtype=torch.float64)
    b2 = torch.randn(N, generator=g, dtype=torch.float64)
    Ad, Bd = A.float().to(DEV), B.float().to(DEV)
    # strided batches with bias, output column-major
    C = torch.empty(nb, N, M, device=DEV)
    ops.gemm(M, N, K, [Ad], K, 1, [Bd], N, 1, [C], 1, M, strideA=M * K, strideB=K * N,
             strideC=M * N, nstrided=nb, bias1=[b1.float().to(DEV)], bias2=[b2.float().to(DEV)])
    ref = A @ B + b1 + b2
    assert rel(C.cpu().transpose(1, 2), ref) < 1e-5
    # k-split over strided batches: sum_b A_b B_b
    C2 = torch.empty(M, N, device=DEV)
    ops.gemm(M, N, K, [Ad], K, 1, [Bd], N, 1, [C2], N, 1, strideA=M * K, strideB=K * N,
             nstrided=nb, ksplit=True)
    assert rel(C2.cpu(), (A @ B).sum(0)) < 1e-5
    # pointer batches with alpha/beta
    C3 = torch.ones(2, M, N, device=DEV)
    ops.gemm(M, N, K, [Ad[0], Ad[1]], K, 1, [Bd[0], Bd[1]], N, 1, [C3[0], C3[1]], N, 1,
             alpha=0.5, beta=2.0)
    assert rel(C3.cpu(), 0.5 * (A[:2] @ B[:2]) + 2.0) < 1e-5


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm_streamk(ops, ta, tb):
    """Shapes whose 128x128 grid fills the resident slots unevenly take the
    stream-K path (split tiles summed from the workspace in fixed order):
    ragged edges, two pointer batches sharing A, bias + alpha/beta, and
    bit-identical results on repeat (deterministic)."""
    from ainp import _lib
    g = torch.Generator().manual_seed(11)
    M, N, K = 2000, 700, 2100            # 16 x 6 tiles x 2 batches = 192, nk = 66
    assert _lib.lib.ainp_gemm_f32_workspace(M, N, K, 2, 1, 0) > 0
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(2, K, N, generator=g, dtype=torch.float64) * 0.5
    bias = torch.randn(2, N, generator=g, dtype=torch.float64)
    C0 = torch.randn(2, M, N, generator=g, dtype=torch.float64)
    Ad = (A.t().contiguous() if ta else A).float().to(DEV)
    Bd = [(B[i].t().contiguous() if tb else B[i]).float().to(DEV) for i in range(2)]
    sam, sak = (1, M) if ta else (K, 1)
    sbk, sbn = (1, K) if tb else (N, 1)
    outs = []
    for _ in range(2):
        C = C0.float().to(DEV)
        ops.gemm(M, N, K, [Ad, Ad], sam, sak, Bd, sbk, sbn, [C[0], C[1]], N, 1,
                 alpha=0.75, beta=-0.5, bias1=[bias[0].float().to(DEV), bias[1].float().to(DEV)],
                 exact=True)   # stream-K serves the exact f32 loop
        outs.append(C.cpu())
    ref = 0.75 * (A @ B) - 0.5 * C0 + bias.view(2, 1, N)
    assert rel(outs[0], ref) < 1e-5
    assert torch.equal(outs[0], outs[1])


# ------------------------------------------------------------------ conv
def _act(x, sc, sh):
    if sc is None:
        return x
    return torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))


@pytest.mark.parametrize("N,Cin,Cout,H,W,pro", [
    (2, 1, 16, 33, 24, False), (2, 16, 32, 33, 50, True), (1, 32, 64, 40, 100, True),
    (2, 32, 16, 17, 49, True), (2, 16, 1, 20, 30, True), (1, 64, 32, 9, 7, False),
    (1, 8, 48, 11, 13, True),
    # small-channel kernels (1-2 channels on one side, 16 on the other), multi-tile
    (2, 1, 16, 41, 100, False), (3, 16, 1, 19, 97, True), (1, 2, 16, 12, 50, True),
    (1, 16, 2, 25, 60, False),
    # the row-strip weight gradient: several 32-row strips and 62-column blocks
    (2, 16, 1, 70, 130, True), (1, 1, 16, 65, 125, False),
    # split-bf16 weight gradient (32-channel passes x 64 outputs): the model's
    # plane, two passes without a prologue, tiles smaller than one 2 x 48 tile
    (2, 32, 64, 257, 334, True), (1, 64, 64, 19, 47, False), (3, 32, 64, 5, 3, True),
    # its 16x16x32 variant: (32 -> 16) and (16 -> 32) on the model's plane
    (2, 32, 16, 257, 334, True), (2, 16, 32, 257, 334, False)])
def test_conv3x3_fwd_dgrad_wgrad(ops, N, Cin, Cout, H, W, pro):
    g = torch.Generator().manual_seed(N * 100 + Cin * 10 + Cout)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) * 0.2
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    sc = torch.rand(Cin, generator=g, dtype=torch.float64) + 0.5 if pro else None
    sh = torch.randn(Cin, generator=g, dtype=torch.float64) * 0.3 if pro else None
    xa = _act(x, sc, sh).requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = Fnn.conv2d(xa, wr, br, padding=1)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    d = lambda t: None if t is None else t.float().to(DEV)  # noqa: E731
    y, stats = ops.conv3x3_fwd(d(x), d(w), d(b), d(sc), d(sh), want_stats=True)
    assert rel(y.cpu(), yr.detach()) < 1e-5
    st = stats.sum(0).cpu()
    assert rel(st[:Cout], yr.detach().sum((0, 2, 3))) < 1e-5
    assert rel(st[Cout:], (yr.detach() ** 2).sum((0, 2, 3))) < 1e-5
    dx = ops.conv3x3_dgrad(d(dy), d(w))
    assert rel(dx.cpu(), xa.grad) < 1e-5
    dw, db = ops.conv3x3_wgrad(d(x), d(dy), d(sc), d(sh))
    assert rel(dw.cpu(), wr.grad) < 1e-5
    assert rel(db.cpu(), br.grad) < 1e-5


@pytest.mark.parametrize("Cin,Cout,pro", [(16, 1, True), (1, 16, False), (2, 16, True),
                                           (16, 2, False)])
def test_small_wgrad_strip_matches_tile_kernel(ops, monkeypatch, Cin, Cout, pro):
    """The row-strip weight gradient of the 1-2-channel-sided convs against
    the 8 x 48-tile kernel it replaced (AINP_SMALL_WGRAD_TILE=1), at the C2
    plane: the same sums in another order, and run-to-run bit-identical."""
    g = torch.Generator().manual_seed(Cin * 7 + Cout)
    N, H, W = 3, 257, 334
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV)
    dy = torch.randn(N, Cout, H, W, generator=g).to(DEV)
    sc = (torch.rand(Cin, generator=g) + 0.5).to(DEV) if pro else None
    sh = (torch.randn(Cin, generator=g) * 0.3).to(DEV) if pro else None
    dw, db = ops.conv3x3_wgrad(x, dy, sc, sh)
    dw2, db2 = ops.conv3x3_wgrad(x, dy, sc, sh)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    monkeypatch.setenv("AINP_SMALL_WGRAD_TILE", "1")
    tw, tb = ops.conv3x3_wgrad(x, dy, sc, sh)
    assert rel(dw.cpu().double(), tw.cpu().double()) < 1e-6
    # the bias: a sum of 2.7M random terms with heavy cancellation -- against fp64
    ref = dy.double().sum((0, 2, 3)).cpu()
    assert rel(db.cpu().double(), ref) < 1e-5 and rel(tb.cpu().double(), ref) < 1e-5


# ------------------------------------------------------------------ BN
@pytest.mark.parametrize("ntcf,H,W", [(False, 37, 70), (True, 37, 70), (False, 37, 71),
                                       (False, 65, 130),
                                       # C*H % 64 == 0, even W: the flattened-k NTCF kernels
                                       (True, 48, 70), (True, 16, 134), (True, 8, 6),
                                       # H >= 64 as well: the ntcf2 backward statistics
                                       # (64-row k-tiles spanning two channels)
                                       (True, 72, 70), (True, 264, 66)])
def test_bn_relu_fwd_bwd(ops, ntcf, H, W):
    g = torch.Generator().manual_seed(9)
    N, C = 3, 8
    y = torch.randn(N, C, H, W, generator=g, dtype=torch.float64) * 2 + 0.5
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(C, generator=g, dtype=torch.float64) * 0.1
    rm = torch.randn(C, generator=g, dtype=torch.float64)
    rv = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    yq = y.clone().requires_grad_(True)
    gq = gamma.clone().requires_grad_(True)
    bq = beta.clone().requires_grad_(True)
    rm_r, rv_r = rm.clone(), rv.clone()
    z = torch.relu(Fnn.batch_norm(yq, rm_r, rv_r, gq, bq, training=True, momentum=0.1,
                                  eps=1e-5))
    if ntcf:
        zr = z.permute(0, 3, 1, 2).reshape(N, W, C * H)
    else:
        zr = z
    gz = torch.randn(zr.shape, generator=g, dtype=torch.float64)
    zr.backward(gz)
    # our path: stats from the conv epilogue layout (one partial row)
    yd = y.float().to(DEV)
    stats = torch.cat([y.sum((0, 2, 3)), (y ** 2).sum((0, 2, 3))]).view(1, -1).to(DEV)
    rmd, rvd = rm.float().to(DEV), rv.float().to(DEV)
    sums = ops.bn_stats_reduce(stats, C)
    sc, sh, save = ops.bn_finalize(sums, N * H * W, gamma.float().to(DEV),
                                   beta.float().to(DEV), rmd, rvd, 0.1, 1e-5)
    out = ops.bn_relu_apply(yd, sc, sh, ntcf=ntcf)
    assert rel(out.cpu(), zr.detach()) < 1e-5
    assert rel(rmd.cpu(), rm_r) < 1e-6 and rel(rvd.cpu(), rv_r) < 1e-6
    gy, dgam, dbet = ops.bn_relu_bwd(gz.float().to(DEV), yd, sc, sh, gamma.float().to(DEV),
                                     save, ntcf=ntcf)
    assert rel(gy.cpu(), yq.grad) < 1e-4
    assert rel(dgam.cpu(), gq.grad) < 1e-5
    assert rel(dbet.cpu(), bq.grad) < 1e-5


# ------------------------------------------------------------------ LSTM
@pytest.mark.parametrize("H,N,T", [(32, 3, 37), (128, 2, 50), (64, 1, 5)])
def test_lstm_recurrence(ops, H, N, T):
    g = torch.Generator().manual_seed(H + T)
    I = 24
    lstm = torch.nn.LSTM(I, H, num_layers=1, batch_first=True, bidirectional=True).double()
    with torch.no_grad():
        for p in lstm.parameters():
            p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float64) * 0.3)
    x = torch.randn(N, T, I, generator=g, dtype=torch.float64, requires_grad=True)
    out, _ = lstm(x)
    dh = torch.randn(out.shape, generator=g, dtype=torch.float64)
    out.backward(dh)
    # zx = x W_ih^T + b_ih + b_hh for both directions
    zf = x.detach() @ lstm.weight_ih_l0.detach().t() + lstm.bias_ih_l0.detach() + lstm.bias_hh_l0.detach()
    zr = (x.detach() @ lstm.weight_ih_l0_reverse.detach().t() + lstm.bias_ih_l0_reverse.detach()
          + lstm.bias_hh_l0_reverse.detach())
    zx = torch.cat([zf, zr], dim=2).float().to(DEV).contiguous()
    wf = lstm.weight_hh_l0.detach().float().to(DEV).contiguous()
    wr = lstm.weight_hh_l0_reverse.detach().float().to(DEV).contiguous()
    h, gates, cell = ops.lstm_rec_fwd(zx, wf, wr, H)
    assert rel(h.cpu(), out.detach()) < 1e-5
    dg = ops.lstm_rec_bwd(dh.float().to(DEV), gates, cell, wf, wr, H)
    # dgates -> dx through W_ih, compare with autograd
    dgc = dg.cpu().double()
    dx = dgc[..., :4 * H] @ lstm.weight_ih_l0.detach() + dgc[..., 4 * H:] @ lstm.weight_ih_l0_reverse.detach()
    assert rel(dx, x.grad) < 1e-4
    db = dgc[..., :4 * H].sum((0, 1))
    assert rel(db, lstm.bias_ih_l0.grad) < 1e-4
    hp = ops.lstm_hprev(h, H).cpu().double()
    dwhh = dgc[..., :4 * H].reshape(-1, 4 * H).t() @ hp[..., :H].reshape(-1, H)
    assert rel(dwhh, lstm.weight_hh_l0.grad) < 1e-4
    dwhh_r = dgc[..., 4 * H:].reshape(-1, 4 * H).t() @ hp[..., H:].reshape(-1, H)
    assert rel(dwhh_r, lstm.weight_hh_l0_reverse.grad) < 1e-4


# ------------------------------------------------------------------ loss / adam
def test_l1_pow10_loss(ops):
    g = torch.Generator().manual_seed(1)
    n = (5, 33, 40)
    y = (torch.randn(n, generator=g) * 0.5).double().requires_grad_(True)
    m = (torch.rand(n, generator=g) > 0.7).double()
    t = torch.complex(torch.randn(n, generator=g), torch.randn(n, generator=g))
    loss = torch.nn.L1Loss(reduction="sum")((10 ** y) * m, torch.abs(t).double() * m)
    loss.backward()
    l, dy = ops.l1_pow10_loss(y.detach().float().to(DEV), m.float().to(DEV), t.to(DEV))
    assert abs(l.item() - loss.item()) / loss.item() < 1e-6
    assert rel(dy.cpu(), y.grad) < 1e-6


def test_l1_pow10_loss_is_bit_reproducible(ops):
    """The loss scalar is a fixed-order two-pass reduction (no fp64 atomics):
    repeated evaluations at the C2 size (N=32, F=257, T=334; 2048 workgroup
    partials) agree bit for bit; an empty input gives 0."""
    g = torch.Generator().manual_seed(2)
    n = (32, 257, 334)
    y = (torch.randn(n, generator=g) * 0.5).to(DEV)
    m = (torch.rand(n, generator=g) > 0.9).float().to(DEV)
    t = torch.complex(torch.randn(n, generator=g), torch.randn(n, generator=g)).to(DEV)
    vals = {ops.l1_pow10_loss(y, m, t, want_grad=False)[0].item() for _ in range(20)}
    assert len(vals) == 1, vals
    ref = ((10 ** y.double().cpu()) * m.double().cpu()
           - t.abs().double().cpu() * m.double().cpu()).abs().sum().item()
    assert abs(vals.pop() - ref) / ref < 1e-6
    e = torch.empty(0, device=DEV)
    l0, _ = ops.l1_pow10_loss(e, e, e.to(torch.complex64), want_grad=False)
    assert l0.item() == 0.0


@pytest.mark.parametrize("rows,cols,ld", [(10688, 1024, 1024), (10688, 512, 1024), (37, 130, 131),
                                           (5, 3, 3)])
def test_colsum_fixed_order(ops, rows, cols, ld):
    """LSTM bias gradients (sum of the gate gradients over N*T rows): row
    slabs in fixed order + sum_slabs, bit-identical across runs."""
    g = torch.Generator().manual_seed(rows + cols)
    x = torch.randn(rows, ld, generator=g, dtype=torch.float64)
    xd = x.float().to(DEV)[:, :cols]
    a = ops.colsum(xd).cpu()
    b = ops.colsum(xd).cpu()
    assert torch.equal(a, b)
    assert rel(a, x[:, :cols].sum(0)) < 1e-6


def test_adam_matches_torch(ops):
    g = torch.Generator().manual_seed(2)
    shapes = [(7, 5), (1000,), (3, 3, 3, 3), (4097,)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.Adam(ref, lr=1e-3)
    dp = [p.to(DEV) for p in ps]
    m = [torch.zeros_like(p) for p in dp]
    v = [torch.zeros_like(p) for p in dp]
    for step in range(1, 4):
        grads = [torch.randn(s, generator=g) for s in shapes]
        for r, gg in zip(ref, grads):
            r.grad = gg.clone()
        opt.step()
        ops.adam_step(dp, [gg.to(DEV) for gg in grads], m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, step)
    for r, p in zip(ref, dp):
        assert torch.allclose(p.cpu(), r.detach(), rtol=1e-6, atol=1e-7)


# ------------------------------------------------------------------ im2col / col2im
# The Discriminator backward's unfold / fold (4x4 kernels at stride 2 and 1;
# 3x3 exercises the generic col2im).  im2col is a copy: bit-exact against
# torch's unfold.  col2im sums up to k*k terms: float64 fold, 1e-6.
@pytest.mark.parametrize("N,C,H,W,k,s,pad,ones,pad4", [
    (2, 3, 17, 30, 4, 2, 1, False, True),
    (2, 5, 16, 33, 4, 1, 1, True, True),
    (1, 4, 13, 21, 4, 2, 1, True, False),
    (2, 3, 12, 19, 3, 1, 1, False, True),
    (1, 2, 9, 14, 3, 2, 1, False, False),
])
def test_im2col_col2im(ops, N, C, H, W, k, s, pad, ones, pad4):
    g = torch.Generator().manual_seed(N * 1000 + C * 10 + H + k)
    x = torch.randn(N, C, H, W, generator=g)
    Ho, Wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    P = Ho * Wo
    ldp = (P + 3) // 4 * 4 if pad4 else None
    col = ops.im2col(x.to(DEV), k, s, pad, ones_row=ones, ldp=ldp).cpu()
    ref = Fnn.unfold(x, k, padding=pad, stride=s)           # [N, C*k*k, P]
    L = ldp or P
    assert col.shape == (N, C * k * k + int(ones), L)
    assert torch.equal(col[:, :C * k * k, :P], ref)
    if ones:
        assert torch.equal(col[:, -1, :P], torch.ones(N, P))
    if L > P:
        assert torch.count_nonzero(col[:, :, P:]) == 0
    dcol = torch.randn(N, C * k * k, L, generator=g)
    dx = ops.col2im(dcol.to(DEV), N, C, H, W, k, s, pad).cpu()
    want = Fnn.fold(dcol[:, :, :P].double(), (H, W), k, padding=pad, stride=s)
    assert dx.shape == (N, C, H, W)
    assert rel(dx, want) < 1e-6


# ------------------------------------------------- bf16-operand GEMM (gemm16.hip)
def _tobf16(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,S", [(300, 200, 520, 1), (128, 256, 1024, 1), (257, 130, 4096, 3),
                                     (1000, 77, 5376, 2), (1000, 1024, 2080, 1),
                                     (777, 600, 1056, 1)])
def test_gemm_bf16nt_matches_fp64_of_bf16_operands(M, N, K, S):
    """ainp_gemm_bf16nt vs fp64 products of the same bf16 operands: bf16 x bf16
    products are exact in fp32, so only the fp32 accumulation differs (<= 1e-5
    relative); ragged M / N tiles, K % 64 != 0, split-K slabs, bias segments.
    The last two shapes are routed to the 256x256 LDS-DMA tile (g256: unsplit,
    M, N >= 512), ragged in M and N with ld > K."""
    from ainp import ops
    g = torch.Generator().manual_seed(M + N + K)
    A = _tobf16(torch.randn(M, K, generator=g)).cuda()
    B = _tobf16(torch.randn(N, K + 16, generator=g)).cuda()[:, :K]     # ld > K
    ref = A.double().cpu() @ B.double().cpu().T
    if S == 1:
        nb = N // 2
        bias = [torch.randn(n, generator=g).cuda() for n in (nb, nb, N - nb, N - nb)]
        C = ops.gemm_bf16nt(A, B, K=K, bias=tuple(bias), bias_nsplit=nb)
        bref = torch.cat([bias[0] + bias[1], bias[2] + bias[3]]).double().cpu()
        ref = ref + bref
    else:
        C = torch.empty(M, N, device="cuda")
        kc = -(-K // S // 64) * 64
        slabs = torch.empty(S, M, N, device="cuda")
        torch.ops.ainp.gemm_bf16nt(A, B, slabs, K, None, None, None, None, 0, S, kc)
        ops.sum_slabs(slabs, S, out=C.view(-1))
    torch.cuda.synchronize()
    err = (C.double().cpu() - ref).norm() / ref.norm()
    assert err < 1e-5, float(err)


@pytest.mark.parametrize("M,N,K,S", [(10688, 1024, 16448, 3), (4100, 512, 1088, 2),
                                     (4100, 300, 1088, 3)])
def test_gemm_bf16nt_split_projection_with_bias(M, N, K, S):
    """The bf16 layer-0 projection split over K (ops.gemm_bf16nt nsplit > 1;
    M >= 8N runs split on the 256x256 tile, N < 512 on the 128 tile): the two
    directions' biases land once (slab 0 only) and the result is the unsplit
    one up to fp32 summation order (models/CNNBLSTM/model.py:46-47,77)."""
    from ainp import ops
    g = torch.Generator().manual_seed(M + N + K + S)
    A = _tobf16(torch.randn(M, K, generator=g)).cuda()
    B = _tobf16(torch.randn(N, K, generator=g)).cuda()
    nb = N // 2
    bias = tuple(torch.randn(n, generator=g).cuda() for n in (nb, nb, N - nb, N - nb))
    C1 = ops.gemm_bf16nt(A, B, bias=bias, bias_nsplit=nb)
    CS = torch.full((M, N), float("nan"), device="cuda")
    ops.gemm_bf16nt(A, B, out=CS, bias=bias, bias_nsplit=nb, nsplit=S)
    torch.cuda.synchronize()
    err = (CS.double() - C1.double()).norm() / C1.double().norm()
    assert err < 1e-6, float(err)
    # the slabs themselves: slab 0 = its K range + the bias, every other slab
    # = the bias-free GEMM over its K range, bit for bit (same kernel, same k
    # order), so the bias lands exactly once and exactly in slab 0
    kc = -(-K // S // 64) * 64
    slabs = torch.full((S, M, N), float("nan"), device="cuda")
    torch.ops.ainp.gemm_bf16nt(A, B, slabs, K, *bias, nb, S, kc)
    for s_ in range(S):
        k0, k1 = s_ * kc, min(K, (s_ + 1) * kc)
        part = ops.gemm_bf16nt(A[:, k0:], B[:, k0:], K=k1 - k0,
                               bias=bias if s_ == 0 else (None,) * 4, bias_nsplit=nb)
        torch.cuda.synchronize()
        assert torch.equal(slabs[s_], part), s_


def test_gemm_bf16nt_multi_problems_match_single_launches():
    """ainp_gemm_bf16nt_multi: three problems in one grid (ragged tiles, one
    split-K with slabs, ld > K) give exactly what each gives alone on the
    256 x 256 tile / the 128 x 128 tile (same MFMA, same k order), and the
    products of the bf16 operands to fp32 accumulation order."""
    from ainp import ops
    g = torch.Generator().manual_seed(7)
    shapes = [(1024, 700, 2112, 3), (777, 600, 1056, 1), (300, 520, 96, 1)]
    probs, refs, outs = [], [], []
    for M, N, K, S in shapes:
        A = _tobf16(torch.randn(M, K + 8, generator=g)).cuda()[:, :K]
        B = _tobf16(torch.randn(N, K, generator=g)).cuda()
        kc = -(-K // S // 32) * 32 if S > 1 else K
        C = torch.full((S, M, N) if S > 1 else (M, N), float("nan"), device="cuda")
        probs.append((A, B, C, K, S, kc))
        refs.append(A.double().cpu() @ B.double().cpu().T)
    ops.gemm_bf16nt_multi(probs)
    for (A, B, C, K, S, kc), ref in zip(probs, refs):
        if S > 1:
            for s_ in range(S):
                k0, k1 = s_ * kc, min(K, (s_ + 1) * kc)
                part = ops.gemm_bf16nt(A[:, k0:], B[:, k0:], K=k1 - k0)
                torch.cuda.synchronize()
                assert torch.equal(C[s_], part), s_
            C = C.sum(0)
        else:
            alone = ops.gemm_bf16nt(A, B, K=K)
            torch.cuda.synchronize()
            assert torch.equal(C, alone)
        err = (C.double().cpu() - ref).norm() / ref.norm()
        assert err < 1e-5, float(err)


@pytest.mark.parametrize("akm,bkm", [(True, True), (True, False), (False, True)])
def test_gemm_bf16nt_multi_kmajor_operands_bit_identical(akm, bkm):
    """ainp_gemm_bf16nt_multi with k-major A and / or B (the operand read as it
    lies, [K][ld], transposed in LDS by ds_read_b64_tr_b16) equals the
    k-contiguous launch on the transposed copies bit for bit: ragged M / N
    tiles, ld > M / N, split-K slabs."""
    from ainp import ops
    g = torch.Generator().manual_seed(11)
    for M, N, K, S in ((1024, 520, 2112, 3), (264, 776, 1056, 1), (40, 1000, 96, 1)):
        A = _tobf16(torch.randn(M, K, generator=g)).cuda()
        B = _tobf16(torch.randn(N, K, generator=g)).cuda()
        Akm = torch.zeros(K, M + 16, dtype=torch.bfloat16, device="cuda")[:, :M]
        Akm.copy_(A.T)
        Bkm = torch.zeros(K, N + 8, dtype=torch.bfloat16, device="cuda")[:, :N]
        Bkm.copy_(B.T)
        kc = -(-K // S // 32) * 32 if S > 1 else K
        shape = (S, M, N) if S > 1 else (M, N)
        C0 = torch.full(shape, float("nan"), device="cuda")
        C1 = torch.full(shape, float("nan"), device="cuda")
        ops.gemm_bf16nt_multi([(A, B, C0, K, S, kc)])
        ops.gemm_bf16nt_multi([(Akm if akm else A, Bkm if bkm else B, C1, K, S, kc, akm, bkm)])
        torch.cuda.synchronize()
        assert torch.equal(C0, C1), (M, N, K, S)
        ref = A.double() @ B.double().T
        got = C1.sum(0) if S > 1 else C1
        assert float((got.double() - ref).norm() / ref.norm()) < 1e-5


@pytest.mark.parametrize("akm,bkm", [(False, False), (True, True), (False, True)])
def test_gemm_bf16nt_multi_bk64_matches_bk32(akm, bkm):
    """Round 6: the 64-deep K-tile variant of the 256 x 256 tile (gemm16.hip
    tile256b, taken when 64 divides every problem's K and kc) against the
    32-deep ring (forced by a second problem with K % 64 != 0 in the same job):
    bit-identical -- the same MFMAs in the same k order -- for k-contiguous
    and k-major operands, ragged tiles, split-K slabs."""
    from ainp import ops
    g = torch.Generator().manual_seed(21)
    M, N, K, S = 1000, 776, 2112, 3
    A = _tobf16(torch.randn(M, K, generator=g)).cuda()
    B = _tobf16(torch.randn(N, K, generator=g)).cuda()
    Akm = A.T.contiguous() if akm else A
    Bkm = B.T.contiguous() if bkm else B
    kc = -(-K // S // 64) * 64
    A2 = _tobf16(torch.randn(300, 1056, generator=g)).cuda()
    B2 = _tobf16(torch.randn(520, 1056, generator=g)).cuda()
    C64 = torch.full((S, M, N), float("nan"), device="cuda")
    C32 = torch.full((S, M, N), float("nan"), device="cuda")
    C2 = torch.full((300, 520), float("nan"), device="cuda")
    ops.gemm_bf16nt_multi([(Akm, Bkm, C64, K, S, kc, akm, bkm)])
    ops.gemm_bf16nt_multi([(Akm, Bkm, C32, K, S, kc, akm, bkm), (A2, B2, C2, 1056, 1, 1056)])
    torch.cuda.synchronize()
    assert torch.equal(C64, C32)
    ref = A.double() @ B.double().T
    assert float((C64.sum(0).double() - ref).norm() / ref.norm()) < 1e-5


def test_lstm_l0_bwd_bf16_pair_kmajor_bit_identical():
    """ops.lstm_l0_bwd_bf16(km=True) -- dW_cat from dg [NT, 8H] and X [NT, I]
    k-major -- equals the transposed-copy pair bit for bit."""
    from ainp import ops
    NT, H, I = 10688, 128, 16448
    g = torch.Generator().manual_seed(13)
    dg16 = _tobf16(torch.randn(NT, 8 * H, generator=g) * 1e-3).cuda()
    x16 = _tobf16(torch.randn(NT, I, generator=g)).cuda()
    wT16 = _tobf16(torch.randn(I, 8 * H, generator=g) * 0.01).cuda()
    out = []
    for km in (False, True):
        dx = torch.full((NT, I), float("nan"), device="cuda")
        gcat = torch.full((8 * H, I), float("nan"), device="cuda")
        ops.lstm_l0_bwd_bf16(dg16, None if km else dg16.T.contiguous(), wT16,
                             x16 if km else x16.T.contiguous(), dx, gcat, km=km)
        torch.cuda.synchronize()
        out.append((dx, gcat))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("NT,H,I", [(10688, 128, 16448), (1024, 64, 520)])
def test_lstm_l0_bwd_bf16_pair(NT, H, I):
    """The bf16 layer-0 backward pair in one launch (ops.lstm_l0_bwd_bf16,
    models/CNNBLSTM/model.py:46-47,77 backward) equals dX and dW_cat from
    separate ainp_gemm_bf16nt launches with the same splits, bit for bit."""
    from ainp import ops
    g = torch.Generator().manual_seed(NT + H)
    dg = torch.randn(NT, 8 * H, generator=g).cuda() * 1e-3
    x = torch.randn(NT, I, generator=g).cuda()
    w = torch.randn(8 * H, I, generator=g).cuda() * 0.01
    dg16, dgT16, xT16, wT16 = _tobf16(dg), _tobf16(dg.T.contiguous()), _tobf16(x.T.contiguous()), \
        _tobf16(w.T.contiguous())
    dx = torch.full((NT, I), float("nan"), device="cuda")
    gcat = torch.full((8 * H, I), float("nan"), device="cuda")
    ops.lstm_l0_bwd_bf16(dg16, dgT16, wT16, xT16, dx, gcat)
    (Sw, kcw), (Sx, kcx) = ops.g256_splits(((8 * H, I, NT), (NT, I, 8 * H)))

    def alone(A, B, K, S, kc):
        if S == 1:
            return ops.gemm_bf16nt(A, B)
        slabs = torch.empty(S, A.shape[0], B.shape[0], device="cuda")
        torch.ops.ainp.gemm_bf16nt(A, B, slabs, K, None, None, None, None, 0, S, kc)
        return ops.sum_slabs(slabs, S).view(A.shape[0], B.shape[0])
    want_dx = alone(dg16, wT16, 8 * H, Sx, kcx)
    want_dw = alone(dgT16, xT16, NT, Sw, kcw)
    torch.cuda.synchronize()
    assert torch.equal(dx, want_dx)
    assert torch.equal(gcat, want_dw)
    ref = dg16.double() @ wT16.double().T
    assert float((dx.double() - ref).norm() / ref.norm()) < 1e-5


def test_cast_bf16_t_and_ntcf_bf16_bridge_bit_exact():
    """The bf16 operand producers round to nearest-even exactly as torch's
    .to(bfloat16): cast (+ transpose into a strided view) and the encoder's
    BN+ReLU writing X [N, W, C*H] and X^T [C*H, N*W]."""
    from ainp import ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn(300, 200, generator=g).cuda()
    out, outT = ops.cast_bf16_t(x, out=True, outT=True)
    wide = torch.zeros(200, 640, device="cuda", dtype=torch.bfloat16)
    ops.cast_bf16_t(x, outT=wide[:, 320:620])
    ref = x.to(torch.bfloat16)
    assert torch.equal(out, ref) and torch.equal(outT, ref.T)
    assert torch.equal(wide[:, 320:620], ref.T) and not wide[:, :320].any()
    # k / w tails of both tilings (64 x 64 and 128 x 128): C*H = 576 and 320,
    # W = 12 and 134, odd N (X^T rows start at odd multiples of W)
    for N, C, H, W in ((2, 64, 9, 12), (3, 64, 5, 134)):
        y = torch.randn(N, C, H, W, generator=g).cuda()
        sc = torch.rand(C, generator=g).cuda() + 0.5
        sh = torch.randn(C, generator=g).cuda() * 0.1
        X16, XT16 = ops.bn_relu_apply_ntcf_bf16(y, sc, sh)
        z = torch.relu(y * sc[None, :, None, None] + sh[None, :, None, None])
        # fmaf vs torch's separate mul+add can differ by one fp32 rounding: compare
        # against both roundings of the fused value
        zf = torch.relu(torch.addcmul(sh[None, :, None, None], y, sc[None, :, None, None]))
        # and the single rounding of fmaf itself (the fp32 product is exact in
        # float64): near-cancelling y*sc + sh differ by more than one ulp
        zd = torch.relu(y.double() * sc.double()[None, :, None, None]
                        + sh.double()[None, :, None, None]).float()
        xr = z.permute(0, 3, 1, 2).reshape(N, W, C * H)
        xf = zf.permute(0, 3, 1, 2).reshape(N, W, C * H)
        xd = zd.permute(0, 3, 1, 2).reshape(N, W, C * H)
        ok = ((X16 == xr.to(torch.bfloat16)) | (X16 == xf.to(torch.bfloat16))
              | (X16 == xd.to(torch.bfloat16)))
        assert bool(ok.all())
        assert torch.equal(XT16, X16.reshape(N * W, C * H).T)


def test_bf16_layer0_operand_path_matches_staged_bf16_path(monkeypatch):
    """The bf16 configuration's layer-0 path on bf16 operands in HBM (bridge +
    cast + gemm_bf16nt) against the fp32-staged bf16 GEMM loop it replaces, on
    a C2-shaped batch (N*T % 8 == 0): both round every operand to bf16 once, so
    only the fp32 accumulation order differs -- output, loss and every
    gradient within 1e-4 relative (ReLU-branch flips aside).  The pre-BN bf16
    storage point (cnnblstm.Y16) of the encoder's last block exists only on
    the bf16-operand path (its bridge reads bf16 y), so it is off for both."""
    import ainp.cnnblstm as CB
    monkeypatch.setattr(CB, "Y16", False)
    from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
    cfg = {"data": {"spectrogram": {"n_fft": 512}},
           "model": {"in_channels": 1, "num_lstm_layers": 2, "lstm_hidden_dim": 128,
                     "enc_filters": [16, 32], "dec_filters": [16, 32]},
           "accel": {"dtype": "bf16"}}
    g = torch.Generator().manual_seed(11)
    N, F, T = 4, 257, 90
    x = (torch.randn(N, F, T, generator=g) - 2).cuda()
    m = torch.zeros(N, F, T)
    m[:, :, 40:48] = 1
    m = m.cuda()
    tgt = torch.polar(torch.rand(N, F, T, generator=g) * 5, torch.rand(N, F, T, generator=g)).to(
        torch.complex64).cuda()
    res = []
    for use16 in (True, False):
        torch.manual_seed(0)
        model = StackedBLSTMCNN(config=cfg).cuda().train()
        orig = CB._l0_bf16_ok
        if not use16:
            CB._l0_bf16_ok = lambda y: False
        try:
            y = model(x.unsqueeze(1))
            loss = l1_pow10_loss(y, m, tgt)
            loss.backward()
        finally:
            CB._l0_bf16_ok = orig
        res.append((y.detach().double().cpu(), float(loss),
                    {k: p.grad.double().cpu() for k, p in model.named_parameters()}))
    from ainp.smoke import BN_FED_BIASES
    (y1, l1, g1), (y0, l0, g0) = res
    assert (y1 - y0).norm() / y0.norm() < 1e-4
    assert abs(l1 - l0) / abs(l0) < 1e-4
    for k in g0:
        if k in BN_FED_BIASES:
            continue   # BN-fed conv biases: exact gradient 0
        e = float((g1[k] - g0[k]).norm() / max(g0[k].norm(), 1e-30))
        assert e < 1e-3, (k, e)


# ------------------------------------------------------- x6r (csrc/gemm_x6r.hip)
@pytest.mark.parametrize("M,K,H", [(2304, 1024, 128), (700, 160, 64), (10688, 16448, 128)])
def test_gemm_x6r_projection_bit_identical_to_x6nt_256(ops, M, K, H):
    """The layer-0 projection on the split-plane tile (ainp_gemm_x6_multi,
    one problem, k-contiguous operands, B split by rows at 4H) is bit-identical
    to ainp_gemm_x6nt_256 unsplit and split 3 (same split, products, k order;
    bias in slab 0)."""
    g = torch.Generator().manual_seed(12)
    A = torch.relu(torch.randn(M, K, generator=g)).to(DEV)
    wf = (torch.randn(4 * H, K, generator=g) * 0.02).to(DEV)
    wr = (torch.randn(4 * H, K, generator=g) * 0.02).to(DEV)
    b = tuple((torch.randn(4 * H, generator=g) * 0.1).to(DEV) for _ in range(4))
    for S in (1, 3):
        y0 = torch.full((M, 8 * H), float("nan"), device=DEV)
        ops.gemm_x6nt_256(A, wf, wr, y0, bias=b, bias_nsplit=4 * H, nsplit=S)
        y1 = torch.full((M, 8 * H), float("nan"), device=DEV)
        ops.gemm_x6r_nt(A, wf, wr, y1, bias=b, bias_nsplit=4 * H, nsplit=S)
        torch.cuda.synchronize()
        assert torch.equal(y0, y1), S


@pytest.mark.parametrize("NT,H,I", [(1200, 64, 1088), (2048, 128, 520), (10688, 128, 16448)])
def test_lstm_l0_bwd_x6_pair(ops, NT, H, I):
    """The fp32 layer-0 backward pair in one launch (ops.lstm_l0_bwd_x6:
    dW_cat = dg^T X with both operands k-major, rows split into the two
    directions; dX = dg W_cat with W_cat's k-halves from W_f / W_r): an fp32
    GEMM against fp64 (within 1e-6 relative, a few times torch's blocked fp32
    GEMM on the CPU, at the small shapes), and at the C2 shape within 1e-6 of the two-stream 128 x 128
    x6 path it replaces (models/CNNBLSTM/model.py:46-47 backward)."""
    g = torch.Generator().manual_seed(NT + I)
    dg = (torch.randn(NT, 8 * H, generator=g) * 1e-2).to(DEV)
    x = torch.relu(torch.randn(NT, I, generator=g)).to(DEV)
    wf = (torch.randn(4 * H, I, generator=g) * 0.05).to(DEV)
    wr = (torch.randn(4 * H, I, generator=g) * 0.05).to(DEV)
    dx = torch.full((NT, I), float("nan"), device=DEV)
    dwf = torch.full((4 * H, I), float("nan"), device=DEV)
    dwr = torch.full((4 * H, I), float("nan"), device=DEV)
    ops.lstm_l0_bwd_x6(dg, wf, wr, x, dx, dwf, dwr)
    torch.cuda.synchronize()
    dW = torch.cat([dwf, dwr]).cpu()
    if NT * I <= 4 * 2 ** 20:
        d64, x64 = dg.double().cpu(), x.double().cpu()
        W64 = torch.cat([wf, wr]).double().cpu()
        rw, rx = d64.T @ x64, d64 @ W64
        fw = (dg.cpu().T @ x.cpu()).double()
        fx = (dg.cpu() @ torch.cat([wf, wr]).cpu()).double()
        # one fp32 accumulator per output over the whole K (no split-K slabs):
        # within 1e-6, a few times the CPU's blocked fp32 sum
        assert rel(dW, rw) < max(4 * rel(fw, rw), 1e-6), (rel(dW, rw), rel(fw, rw))
        assert rel(dx.cpu(), rx) < max(4 * rel(fx, rx), 1e-6), (rel(dx.cpu(), rx), rel(fx, rx))
    else:
        # the two-stream path (cnnblstm._BLSTMFn with AINP_L0_BWD_X6R=0)
        ox = torch.empty(NT, I, device=DEV)
        dg2 = dg.contiguous()
        ops.gemm(NT, I, 4 * H, [dg2, dg2[:, 4 * H:]], 8 * H, 1, [wf, wr], I, 1, [ox, ox], I, 1,
                 ksplit=True)
        ow = ops.gemm_tn_splitk(dg2, 8 * H, x, I, NT, 4 * H, I, offsets_b=(0, 0))
        torch.cuda.synchronize()
        assert rel(dx.cpu(), ox.cpu()) < 1e-6
        assert rel(dW, torch.cat([ow[0], ow[1]]).cpu()) < 1e-6


@pytest.mark.parametrize("N,T,C,F,K", [(2, 48, 4, 20, 64), (3, 112, 16, 33, 256),
                                       (32, 528, 16, 257, 256)])
def test_proj_bwd_x6(ops, N, T, C, F, K):
    """The fp32 output-projection backward on the x6r tile (ops.proj_bwd_x6,
    nn.Linear(2H, C*F) of models/CNNBLSTM/model.py:48,78): dh = g^T w and
    dW = g h from the gradient permuted to [C*F, N*T], against fp64 (a few
    times torch's fp32 CPU GEMM, floor 2e-6: split-K slabs at the C2 shape),
    and the joint launch bit-identical to the two separate ones."""
    g = torch.Generator().manual_seed(N * T + K)
    NO, NT = C * F, N * T
    gr = (torch.randn(N, NO, T, generator=g) * 1e-2).to(DEV)
    h = torch.tanh(torch.randn(NT, K, generator=g)).to(DEV)
    w = (torch.randn(NO, K, generator=g) * 0.05).to(DEV)
    gp = gr.transpose(0, 1).contiguous().view(NO, NT)
    dh = torch.full((NT, K), float("nan"), device=DEV)
    dw = torch.full((NO, K), float("nan"), device=DEV)
    ops.proj_bwd_x6(gp, h, w, dh=dh, dw=dw)
    dh1 = torch.full((NT, K), float("nan"), device=DEV)
    dw1 = torch.full((NO, K), float("nan"), device=DEV)
    ops.proj_bwd_x6(gp, h, w, dh=dh1)
    ops.proj_bwd_x6(gp, h, w, dw=dw1)
    torch.cuda.synchronize()
    assert torch.equal(dh, dh1) and torch.equal(dw, dw1)
    g64, h64, w64 = gp.double().cpu(), h.double().cpu(), w.double().cpu()
    rh, rw = g64.T @ w64, g64 @ h64
    fh = (gp.cpu().T @ w.cpu()).double()
    fw = (gp.cpu() @ h.cpu()).double()
    assert rel(dh.cpu(), rh) < max(4 * rel(fh, rh), 2e-6), (rel(dh.cpu(), rh), rel(fh, rh))
    assert rel(dw.cpu(), rw) < max(4 * rel(fw, rw), 2e-6), (rel(dw.cpu(), rw), rel(fw, rw))


def test_gemm_x6_multi_equals_separate_launches(ops):
    """Problems launched together (one grid) give bit-identical results to the
    same problems launched one by one; a split-K problem writes its slabs."""
    g = torch.Generator().manual_seed(21)
    NT, H, I = 1200, 64, 1088
    dg = torch.randn(NT, 8 * H, generator=g).to(DEV)
    x = torch.randn(NT, I, generator=g).to(DEV)
    wf, wr = (torch.randn(4 * H, I, generator=g).to(DEV) for _ in range(2))

    def probs(outs):
        dx, dwf, dwr, sl = outs
        return [ops.x6_problem(dg, x, dwf, M=8 * H, N=I, K=NT, lda=8 * H, ldb=I, ldc=I,
                               a_kmajor=True, b_kmajor=True, C2=dwr, c_msplit=4 * H),
                ops.x6_problem(dg, wf, dx, M=NT, N=I, K=8 * H, lda=8 * H, ldb=I, ldc=I, B2=wr,
                               b_ksplit=4 * H, b_kmajor=True),
                ops.x6_problem(x, wf, sl, M=NT, N=4 * H, K=I, lda=I, ldb=I, ldc=4 * H, nsplit=2,
                               kc=544, strideC=NT * 4 * H)]

    def fresh():
        return (torch.full((NT, I), float("nan"), device=DEV),
                torch.full((4 * H, I), float("nan"), device=DEV),
                torch.full((4 * H, I), float("nan"), device=DEV),
                torch.full((2, NT, 4 * H), float("nan"), device=DEV))
    a, b = fresh(), fresh()
    ops.gemm_x6_multi(probs(a))
    for p in probs(b):
        ops.gemm_x6_multi([p])
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert not torch.isnan(u).any()
        assert torch.equal(u, v)
    ref = (x.double().cpu() @ wf.double().cpu().T)
    assert rel(a[3].sum(0).cpu(), ref) < 1e-6


def test_gemm_x6_multi_rejects_bad_extents(ops):
    """Host checks before the launch: an operand shorter than its extent, a
    split off the tile grid, more than 3 problems."""
    A = torch.randn(300, 64, device=DEV)
    B = torch.randn(256, 64, device=DEV)
    C = torch.empty(300, 256, device=DEV)
    with pytest.raises(RuntimeError):
        ops.gemm_x6_multi([ops.x6_problem(A, B, C, M=300, N=256, K=128, lda=64, ldb=64, ldc=256)])
    with pytest.raises(RuntimeError):
        ops.gemm_x6_multi([ops.x6_problem(A, B, C, M=300, N=256, K=64, lda=64, ldb=64, ldc=256,
                                          C2=C, c_msplit=100)])
    p = ops.x6_problem(A, B, C, M=300, N=256, K=64, lda=64, ldb=64, ldc=256)
    with pytest.raises(RuntimeError):
        ops.gemm_x6_multi([p] * 4)



@pytest.mark.parametrize("Cin,Cout,H,W", [(16, 32, 37, 70), (32, 16, 37, 70), (32, 64, 37, 70)])
def test_conv3x3_grads_take_bf16_dy_bit_exact(ops, Cin, Cout, H, W):
    """bf16 configuration: the data / weight gradients read a bf16-stored dy
    (AINP_CONV_DY16) and give exactly what they give for the same values in
    fp32 (they round dy to bf16 when staging it), incl. the bias gradient."""
    N = 3
    g = torch.Generator(device=DEV).manual_seed(Cin + 7 * Cout)
    dy16 = torch.randn(N, Cout, H, W, device=DEV, generator=g).to(torch.bfloat16)
    dy32 = dy16.float()
    x = torch.randn(N, Cin, H, W, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) * 0.2
    sc = torch.rand(Cin, device=DEV, generator=g) + 0.5
    sh = torch.randn(Cin, device=DEV, generator=g) * 0.3
    assert ops.dy16_ok(N, Cin, Cout, H, W)
    assert torch.equal(ops.conv3x3_dgrad(dy16, w, bf16=True), ops.conv3x3_dgrad(dy32, w, bf16=True))
    dw16, db16 = ops.conv3x3_wgrad(x, dy16, sc, sh, bf16=True)
    dw32, db32 = ops.conv3x3_wgrad(x, dy32, sc, sh, bf16=True)
    torch.cuda.synchronize()
    assert torch.equal(dw16, dw32) and torch.equal(db16, db32)
    with pytest.raises(ValueError):
        ops.conv3x3_dgrad(dy16, w)          # bf16 storage needs the bf16 arithmetic


def test_conv3x3_bf16_dy_refused_where_no_kernel_reads_it(ops):
    """The exact fp32 small-channel kernels have no bf16-dy path: an error, not
    a silent misread."""
    dy16 = torch.zeros(1, 16, 8, 8, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(16, 1, 3, 3, device=DEV)
    assert not ops.dy16_ok(1, 1, 16, 8, 8)
    with pytest.raises(RuntimeError, match="DY16"):
        ops.conv3x3_dgrad(dy16, w, bf16=True)


@pytest.mark.parametrize("ntcf,C,H,W", [(False, 8, 37, 70), (True, 64, 37, 70), (True, 8, 37, 70)])
def test_bn_relu_bwd_apply_bf16_output_is_rounded_fp32(ops, ntcf, C, H, W):
    """AINP_BN_GY16: gy written as bf16 equals the fp32 gy rounded to nearest
    even (flat, NTCF v2 (C*H % 64 == 0) and NTCF tile paths)."""
    N = 2
    g = torch.Generator(device=DEV).manual_seed(H + W)
    y = torch.randn(N, C, H, W, device=DEV, generator=g) * 2 + 0.5
    gg = torch.randn((N, W, C * H) if ntcf else (N, C, H, W), device=DEV, generator=g)
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.1
    gam = torch.rand(C, device=DEV, generator=g) + 0.5
    save = torch.cat([y.mean((0, 2, 3)), 1.0 / (y.var((0, 2, 3)) + 1e-5).sqrt()])
    sums = ops.bn_relu_bwd_reduce(gg, y, sc, sh, save, ntcf)
    gy32, dg32, db32 = ops.bn_relu_bwd_apply(gg, y, sc, sh, gam, save, sums, N * H * W, ntcf)
    gy16, dg16, db16 = ops.bn_relu_bwd_apply(gg, y, sc, sh, gam, save, sums, N * H * W, ntcf,
                                             gy16=True)
    torch.cuda.synchronize()
    assert gy16.dtype == torch.bfloat16
    assert torch.equal(gy16, gy32.to(torch.bfloat16))
    assert torch.equal(dg16, dg32) and torch.equal(db16, db32)


@pytest.mark.parametrize("Cin,Cout,H,W", [(16, 32, 37, 70), (32, 16, 37, 70), (32, 64, 37, 70)])
def test_conv3x3_bf16_activation_storage(ops, Cin, Cout, H, W):
    """bf16 configuration, pre-BN activations in bf16 storage: a forward with
    AINP_CONV_Y16 writes round(y) of the fp32-output forward bit for bit, its
    BatchNorm partials sum the stored values; a forward / weight gradient
    reading a bf16 act(x) source (AINP_CONV_X16) equals the one reading the
    same values in fp32; BatchNorm backward and the NTCF bridge likewise."""
    N = 3
    g = torch.Generator(device=DEV).manual_seed(3 * Cin + Cout)
    x16 = (torch.randn(N, Cin, H, W, device=DEV, generator=g) * 2).to(torch.bfloat16)
    x32 = x16.float()
    w = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) * 0.2
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    sc = torch.rand(Cin, device=DEV, generator=g) + 0.5
    sh = torch.randn(Cin, device=DEV, generator=g) * 0.3
    assert ops.io16_ok(N, Cin, Cout, H, W)
    y32, st32 = ops.conv3x3_fwd(x32, w, b, sc, sh, want_stats=True, bf16=True)
    y16, st16 = ops.conv3x3_fwd(x16, w, b, sc, sh, want_stats=True, bf16=True, y16=True)
    y32b, _ = ops.conv3x3_fwd(x16, w, b, sc, sh, want_stats=True, bf16=True)
    torch.cuda.synchronize()
    assert y16.dtype == torch.bfloat16
    assert torch.equal(y32b, y32)                       # X16 read == fp32 read of the values
    assert torch.equal(y16, y32.to(torch.bfloat16))     # Y16 == round(fp32 output)
    s = st16.sum(0).double().cpu()
    yd = y16.double().cpu()
    assert rel(s[:Cout], yd.sum((0, 2, 3))) < 1e-6
    assert rel(s[Cout:], (yd ** 2).sum((0, 2, 3))) < 1e-6
    dy = torch.randn(N, Cout, H, W, device=DEV, generator=g)
    dw16, db16 = ops.conv3x3_wgrad(x16, dy, sc, sh, bf16=True)
    dw32, db32 = ops.conv3x3_wgrad(x32, dy, sc, sh, bf16=True)
    torch.cuda.synchronize()
    assert torch.equal(dw16, dw32) and torch.equal(db16, db32)
    # BatchNorm backward over the bf16-stored y (same values as fp32)
    scb = torch.rand(Cout, device=DEV, generator=g) + 0.5
    shb = torch.randn(Cout, device=DEV, generator=g) * 0.1
    save = torch.cat([yd.float().mean((0, 2, 3)), 1.0 / (yd.float().var((0, 2, 3)) + 1e-5).sqrt()]).cuda()
    gam = torch.rand(Cout, device=DEV, generator=g) + 0.5
    gg = torch.randn(N, Cout, H, W, device=DEV, generator=g)
    r16 = ops.bn_relu_bwd_reduce(gg, y16, scb, shb, save)
    r32 = ops.bn_relu_bwd_reduce(gg, y16.float(), scb, shb, save)
    a16 = ops.bn_relu_bwd_apply(gg, y16, scb, shb, gam, save, r32, N * H * W, gy16=True)
    a32 = ops.bn_relu_bwd_apply(gg, y16.float(), scb, shb, gam, save, r32, N * H * W, gy16=True)
    torch.cuda.synchronize()
    assert torch.equal(r16, r32)
    for u, v in zip(a16, a32):
        assert torch.equal(u, v)


def test_ntcf_bridge_and_backward_read_bf16_y(ops):
    """The encoder's last block with its pre-BN output in bf16 storage: the
    bf16 X / X^T bridge and the NTCF BatchNorm backward (reduce + apply) give
    what they give for the same values in fp32."""
    N, C, H, W = 2, 64, 37, 70
    g = torch.Generator(device=DEV).manual_seed(11)
    y16 = (torch.randn(N, C, H, W, device=DEV, generator=g) * 2).to(torch.bfloat16)
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.1
    X16, XT16 = ops.bn_relu_apply_ntcf_bf16(y16, sc, sh)
    X32, XT32 = ops.bn_relu_apply_ntcf_bf16(y16.float(), sc, sh)
    gg = torch.randn(N, W, C * H, device=DEV, generator=g)
    save = torch.cat([y16.float().mean((0, 2, 3)), 1.0 / (y16.float().var((0, 2, 3)) + 1e-5).sqrt()])
    gam = torch.rand(C, device=DEV, generator=g) + 0.5
    r16 = ops.bn_relu_bwd_reduce(gg, y16, sc, sh, save, ntcf=True)
    r32 = ops.bn_relu_bwd_reduce(gg, y16.float(), sc, sh, save, ntcf=True)
    a16 = ops.bn_relu_bwd_apply(gg, y16, sc, sh, gam, save, r32, N * H * W, ntcf=True, gy16=True)
    a32 = ops.bn_relu_bwd_apply(gg, y16.float(), sc, sh, gam, save, r32, N * H * W, ntcf=True,
                                gy16=True)
    torch.cuda.synchronize()
    assert torch.equal(X16, X32) and torch.equal(XT16, XT32) and torch.equal(r16, r32)
    for u, v in zip(a16, a32):
        assert torch.equal(u, v)


@pytest.mark.parametrize("nslabs,n", [(512, 1088), (100, 37), (64, 4000), (3, 10), (70, 4096 * 4 + 3)])
def test_sum_slabs_orders(nslabs, n):
    """ainp_sum_slabs: sequential slab order on its main kernel; for few
    elements over >= 64 slabs, 32 slab groups (g, g+32, ...) each summed in
    order and the group partials added in order -- both reproduced exactly."""
    from ainp import ops
    g = torch.Generator().manual_seed(nslabs + n)
    x = torch.randn(nslabs, n, generator=g)
    out = ops.sum_slabs(x.cuda().contiguous(), nslabs).cpu()
    grid = -(-(-(-n // 4)) // 256)
    if grid < 16 and nslabs >= 64:
        parts = []
        for q in range(32):
            a = torch.zeros(n)
            for s in range(q, nslabs, 32):
                a = a + x[s]
            parts.append(a)
        ref = parts[0].clone()
        for q in range(1, 32):
            ref = ref + parts[q]
    else:
        ref = x[0].clone()
        for s in range(1, nslabs):
            ref = ref + x[s]
    assert torch.equal(out, ref)


@pytest.mark.parametrize("C,parts,running", [(64, 300, True), (16, 7, False), (512, 1, True)])
def test_bn_reduce_finalize_equals_two_calls(C, parts, running):
    """ainp_bn_reduce_finalize: scale / shift / save and the running statistics
    bit for bit those of ainp_bn_stats_reduce + ainp_bn_finalize."""
    from ainp import ops
    g = torch.Generator().manual_seed(C + parts)
    stats = (torch.randn(parts, 2 * C, generator=g, dtype=torch.float64).abs() * 50).cuda()
    gamma = torch.randn(C, generator=g).cuda()
    beta = torch.randn(C, generator=g).cuda()
    rm1 = torch.randn(C, generator=g).cuda() if running else None
    rv1 = torch.rand(C, generator=g).cuda() + 0.5 if running else None
    rm2 = rm1.clone() if running else None
    rv2 = rv1.clone() if running else None
    count = 1000 * parts
    sums = ops.bn_stats_reduce(stats, C)
    a = ops.bn_finalize(sums, count, gamma, beta, rm1, rv1, 0.1, 1e-5)
    b = ops.bn_reduce_finalize(stats, C, count, gamma, beta, rm2, rv2, 0.1, 1e-5)
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    if running:
        assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2)


def test_adam_bumps_parameter_versions():
    """The device weight caches keyed on tensor._version (conv_weight_nhwc16,
    dgrad16_weight) see every ainp Adam update: the op's mutable-argument
    schema makes the dispatcher bump the parameters' version counters."""
    from ainp.optim import Adam
    p = torch.nn.Parameter(torch.randn(64, 32, 3, 3, device=DEV))
    opt = Adam([p], lr=1e-3)
    p.grad = torch.randn_like(p)
    v0 = p._version
    opt.step()
    torch.cuda.synchronize()
    assert p._version > v0
