"""Tensor-level wrappers over the libainp kernels.

Each function validates its torch tensors (device, dtype, layout), allocates
outputs through PyTorch's caching allocator and launches the gfx950 kernel on
the current HIP stream through the PyTorch custom operators torch.ops.ainp.*
(csrc/torch_ops.cpp: the TORCH_LIBRARY registration of every GPU entry point
of include/ainp.h, out= style; the operator re-checks shapes on the host
before the launch).  These are the only entry points the rest of the package
uses to compute; nothing here falls back to ATen or the CPU, and importing
this module fails when libainp_torch.so is missing.  Host-only queries
(workspace sizes) use the plain C ABI through ctypes (_lib).
"""
from __future__ import annotations

import atexit
import functools
import heapq
import itertools
import math
import os
import weakref

import numpy as np
import torch

from . import _lib

# AINP_TORCH_OPS: another build of the same registration (e.g. the UBSan build
# libainp_torch_ubsan.so that tests/test_gpu_sanitize.py loads)
TORCH_OPS_PATH = os.environ.get("AINP_TORCH_OPS") or \
    os.path.join(os.path.dirname(_lib.LIB_PATH), "libainp_torch.so")
if not os.path.exists(TORCH_OPS_PATH):
    raise ImportError(f"torch ops library not found at {TORCH_OPS_PATH}; build it with "
                      "`make -C ml-audio-inpainting_amd/csrc` (or __graft_entry__.build())")
torch.ops.load_library(TORCH_OPS_PATH)
_T = torch.ops.ainp


def _release_device_caches():
    """atexit: drop the module-level device tensors (windows, GEMM workspaces,
    bf16 weight copies) while the HIP runtime is still up, so nothing of ours
    is freed from a static destructor during __cxa_finalize, after the runtime
    (and a profiler's tool library) has been torn down -- the failure mode of
    round 2's dropped CU-masked-stream variant."""
    try:
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:   # noqa: BLE001 -- best effort at interpreter exit
        pass
    for c in (_WIN_CACHE, _GEMM_WS, _EMPTY, _WT_CACHE, _WT16_CACHE, _RED_WS):
        c.clear()


atexit.register(_release_device_caches)

FEAT_CNNBLSTM = 0
FEAT_GAN = 1


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _req(t: torch.Tensor, name: str, dtype=torch.float32, contiguous=True):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} must live on the GPU (got {t.device}); the ainp "
                           "kernels have no CPU path")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


# --------------------------------------------------------------------- STFT
@functools.lru_cache(maxsize=None)
def analysis_window(window: str, win_length: int, n_fft: int) -> np.ndarray:
    """librosa.filters.get_window(window, win_length, fftbins=True) centred in
    n_fft (librosa.util.pad_center), float64 -- the window librosa.stft uses."""
    import scipy.signal
    w = scipy.signal.get_window(window, win_length, fftbins=True).astype(np.float64)
    out = np.zeros(n_fft, dtype=np.float64)
    lpad = (n_fft - win_length) // 2
    out[lpad:lpad + win_length] = w
    return out


_WIN_CACHE: dict = {}


def _device_window(window, win_length, n_fft, device):
    key = (window, win_length, n_fft, str(device))
    w = _WIN_CACHE.get(key)
    if w is None:
        w = torch.from_numpy(analysis_window(window, win_length, n_fft)).to(device)
        _WIN_CACHE[key] = w
    return w


def stft_features(audio: torch.Tensor, gap_start: torch.Tensor, gap_len: int,
                  n_fft: int, hop: int, win_length: int | None = None,
                  n_frames: int | None = None, mode: int = FEAT_CNNBLSTM,
                  sample_rate: int = 16000, clip_index: torch.Tensor | None = None,
                  window: str = "hann", outputs=(True, True, True, True)):
    """Fused STFT + features + gap mask (include/ainp.h ainp_stft_features).

    audio [n_clips, S] f32 cuda; gap_start [B] int64 cuda.
    Returns (out0, out1, out2, out3); CNNBLSTM: (log10 |X_gap| + 1e-9,
    complex64 target, mask 1=gap, None); GAN: (log1p|X|, log1p|X_imp|,
    angle X, mask 1=valid).
    """
    _req(audio, "audio")
    if audio.dim() == 1:
        audio = audio.unsqueeze(0)
    _req(gap_start, "gap_start", torch.int64)
    if clip_index is not None:
        _req(clip_index, "clip_index", torch.int32)
        batch = clip_index.numel()
    else:
        batch = audio.shape[0]
    if gap_start.numel() != batch:
        raise ValueError("gap_start must have one entry per example")
    n_clips, S = audio.shape
    win_length = n_fft if win_length is None else win_length
    n_avail = 1 + S // hop
    n_frames = n_avail if n_frames is None else int(n_frames)
    F = n_fft // 2 + 1
    dev = audio.device
    w = _device_window(window, win_length, n_fft, dev)
    o = [None, None, None, None]
    if outputs[0]:
        o[0] = torch.empty(batch, F, n_frames, device=dev, dtype=torch.float32)
    if outputs[1]:
        o[1] = (torch.empty(batch, F, n_frames, device=dev, dtype=torch.complex64)
                if mode == FEAT_CNNBLSTM else
                torch.empty(batch, F, n_frames, device=dev, dtype=torch.float32))
    if outputs[2]:
        o[2] = torch.empty(batch, F, n_frames, device=dev, dtype=torch.float32)
    if outputs[3] and mode == FEAT_GAN:
        o[3] = torch.empty(batch, F, n_frames, device=dev, dtype=torch.float32)
    _T.stft_features(audio, clip_index, gap_start, int(gap_len), int(sample_rate), w,
                     int(n_fft), int(hop), n_frames, int(mode), o[0], o[1], o[2], o[3])
    return tuple(o)


def stft(audio: torch.Tensor, n_fft: int = 2048, hop_length: int = 512,
         win_length: int | None = None, window: str = "hann", center: bool = True):
    """librosa>=0.10 stft on the GPU: audio [..., S] float32/float64 cuda ->
    complex64/complex128 [..., n_fft/2+1, n_frames] (ainp_stft)."""
    _req(audio, "audio", dtype=None)
    if audio.dtype not in (torch.float32, torch.float64):
        raise TypeError("stft input must be float32 or float64")
    lead = audio.shape[:-1]
    S = audio.shape[-1]
    x = audio.reshape(-1, S).contiguous()
    win_length = n_fft if win_length is None else win_length
    if center:
        n_frames = 1 + S // hop_length
    else:
        if S < n_fft:
            raise ValueError(f"n_fft={n_fft} is too large for input signal of length={S}")
        n_frames = 1 + (S - n_fft) // hop_length
    F = n_fft // 2 + 1
    cdt = torch.complex64 if audio.dtype == torch.float32 else torch.complex128
    out = torch.empty(x.shape[0], F, n_frames, device=audio.device, dtype=cdt)
    w = _device_window(window, win_length, n_fft, audio.device)
    _T.stft(x, w, int(n_fft), int(hop_length), bool(center), n_frames, out)
    return out.reshape(*lead, F, n_frames)


# ------------------------------------------------------------ work accounting
# bench.py's in-step roofline table for the GAN step: while WORK_TRACE is a
# list, the GAN conv / D-backward launches below append (kernel-name
# substring, algorithmic FLOP) -- the name of the kernel the C side routes the
# launch to (include/ainp.h; default variants), the FLOP of the layer's
# product (2 * outputs * Cin * k * k).  Off (None) otherwise.
WORK_TRACE = None


def _work(name, flop):
    if WORK_TRACE is not None:
        WORK_TRACE.append((name, float(flop)))


# --------------------------------------------------------------------- GEMM
# ainp_gemm_f32_ex precision: False (default) = fp32-accurate three-piece bf16
# split on the bf16 MFMA (include/ainp.h); True = exact f32 MFMA.  The
# AINP_GEMM_EXACT=1 environment variable selects the exact path process-wide.
GEMM_EXACT = os.environ.get("AINP_GEMM_EXACT", "0") == "1"
GEMM_EXACT_F32 = 1
GEMM_BF16 = 2          # include/ainp.h AINP_GEMM_BF16
CONV_BF16 = 2          # include/ainp.h AINP_CONV_BF16
CONV_DY16 = 4          # AINP_CONV_DY16: dy in bf16 storage (data / weight gradients)
CONV_X16 = 8           # AINP_CONV_X16: the act(x) source in bf16 storage (fwd / wgrad)
CONV_Y16 = 16          # AINP_CONV_Y16: forward output y in bf16 storage
BN_GY16 = 1            # AINP_BN_GY16: BatchNorm-backward output gy in bf16 storage
BN_Y16 = 2             # AINP_BN_Y16: the pre-BN input y in bf16 storage
# round 5: channel-last activations [N, H, W, C] (include/ainp.h)
CONV_XCL = 32          # AINP_CONV_XCL: input channel-last (fwd x, dgrad dy, wgrad x)
CONV_YCL = 64          # AINP_CONV_YCL: output channel-last (fwd y, dgrad dx)
CONV_GCL = 128         # AINP_CONV_GCL: the weight gradient's dy channel-last
CONV_YCFNT = 256       # AINP_CONV_YCFNT: the data gradient's dx as [C][H][N][W]
BN_CL = 4              # AINP_BN_CL: g / y / gy channel-last
BN_G16 = 8             # AINP_BN_G16: g in bf16 storage (with BN_CL)


def gemm(M, N, K, A, sam, sak, B, sbk, sbn, C, scm, scn, *, alpha=1.0, beta=0.0,
         strideA=0, strideB=0, strideC=0, bias1=None, bias2=None, nstrided=1,
         ksplit=False, stream_of=None, exact=None, bf16=False):
    """Raw strided/batched GEMM (ainp_gemm_f32_ex).  A, B, C, bias1, bias2 are
    lists (pointer batches) of cuda float32 tensors (views allowed) or None.
    exact: None -> GEMM_EXACT; True -> exact f32 MFMA; False -> bf16x6 split.
    bf16=True: bf16-rounded operands, f32 accumulation (the bf16 configs)."""
    A = list(A); B = list(B); C = list(C)
    nptr = len(A)
    assert len(B) == nptr and len(C) == nptr and 1 <= nptr <= 8
    ref = C[0]
    if stream_of is not None and stream_of.device != ref.device:
        raise ValueError("gemm: stream_of must be on the operands' device")
    exact = False if bf16 else (GEMM_EXACT if exact is None else bool(exact))
    ws = (_gemm_workspace(ref.device, _stream(ref), int(M), int(N), int(K), nptr,
                          int(nstrided), int(ksplit)) if exact else None)
    flags = GEMM_BF16 if bf16 else (GEMM_EXACT_F32 if exact else 0)
    _T.gemm(int(M), int(N), int(K), float(alpha), A, int(sam), int(sak), int(strideA),
            B, int(sbk), int(sbn), int(strideB), float(beta), C, int(scm), int(scn),
            int(strideC), list(bias1) if bias1 is not None else [],
            list(bias2) if bias2 is not None else [], int(nstrided), int(ksplit), flags, ws)


_GEMM_WS: dict = {}


def _gemm_workspace(device, stream: int, M, N, K, nptr, nstrided, ksplit):
    """Stream-K workspace (ainp_gemm_f32_workspace bytes), one buffer per
    (device, stream) so concurrent streams never share it; (None, 0) when the
    plain tile grid is used."""
    need = int(_lib.lib.ainp_gemm_f32_workspace(M, N, K, nptr, nstrided, ksplit))
    if need == 0:
        return None
    key = (device.index, stream)
    buf = _GEMM_WS.get(key)
    if buf is None or buf.numel() * 4 < need:
        buf = torch.empty((need + 3) // 4, device=device, dtype=torch.float32)
        _GEMM_WS[key] = buf
    return buf


def _chunks_for(K, tiles, target_blocks=512, min_rows=64):
    """Split count S (a divisor of K) so tiles*S ~ target workgroups."""
    want = max(1, min(K // min_rows, target_blocks // max(1, tiles)))
    for s in range(want, 0, -1):
        if K % s == 0:
            return s
    return 1


def gemm_tn_splitk(a, lda, b, ldb, K, M, N, offsets_b=(0, 0), bf16=False):
    """Two-direction weight-gradient GEMM C[d] = A_d^T B_d for the BLSTM:
    A_d = a[:, d*M:(d+1)*M] ([K, M] row-major view, row stride lda),
    B_d = b[:, off_d:off_d+N] ([K, N], row stride ldb); returns [C_0, C_1]
    ([M, N] each).  K (= N*T rows) is split into S strided chunks computed
    by independent workgroups into slabs, then summed in fixed order."""
    tiles = -(-M // 128) * -(-N // 128) * 2
    S = _chunks_for(K, tiles)
    kc = K // S
    slabs = torch.empty(2, S, M, N, device=a.device, dtype=torch.float32)
    gemm(M, N, kc, [a, a[:, M:]], 1, lda, [b[:, offsets_b[0]:], b[:, offsets_b[1]:]], ldb, 1,
         [slabs[0], slabs[1]], N, 1, strideA=kc * lda, strideB=kc * ldb, strideC=M * N,
         nstrided=S, bf16=bf16)
    if S == 1:
        return [slabs[0, 0], slabs[1, 0]]
    return [sum_slabs(slabs[0], S).view(M, N), sum_slabs(slabs[1], S).view(M, N)]


# ------------------------------------------------------- bf16-operand GEMM (C3)
def bn_relu_apply_ntcf_bf16(y, scale, shift):
    """ainp_bn_relu_apply_ntcf_bf16: relu(y*scale+shift) of the encoder's last
    block as bf16 X [N, W, C*H] and X^T [C*H, N*W] (row stride rounded up to 8
    elements, so every row starts 16-byte aligned)."""
    _req(y, "y", None)
    N, C, H, W = y.shape
    K, NW = C * H, N * W
    out = torch.empty(N, W, K, device=y.device, dtype=torch.bfloat16)
    ldt = -(-NW // 8) * 8
    outT = torch.empty(K, ldt, device=y.device, dtype=torch.bfloat16)[:, :NW]
    _T.bn_relu_apply_ntcf_bf16(y, scale, shift, out, outT, _y_flag(y))
    return out, outT


def bn_relu_apply_ntcf_cl(y, scale, shift, out32=True, out16=False, outT=True):
    """ainp_bn_relu_apply_ntcf_cl (round 5): relu(y*scale+shift) of a
    channel-last y [N, H, W, 64] as the LSTM input: fp32 X [N, W, 64*H]
    (out32) and / or the bf16 X [N, W, 64*H] and (outT) X^T [64*H, N*W] (out16,
    row stride rounded up to 8 elements).  Returns (X or None, (X16, XT16 or
    None) or None)."""
    _req(y, "y", None)
    N, H, W, C = y.shape
    K, NW = C * H, N * W
    out = torch.empty(N, W, K, device=y.device, dtype=torch.float32) if out32 else None
    o16 = oT = None
    if out16:
        o16 = torch.empty(N, W, K, device=y.device, dtype=torch.bfloat16)
        if outT:
            ldt = -(-NW // 8) * 8
            oT = torch.empty(K, ldt, device=y.device, dtype=torch.bfloat16)[:, :NW]
    _T.bn_relu_apply_ntcf_cl(y, scale, shift, out, o16, oT, _y_flag(y))
    return out, ((o16, oT) if out16 else None)


def cast_bf16_t(x, out=None, outT=None):
    """ainp_cast_bf16_t: fp32 [R, C] (unit-stride rows) -> bf16 out [R, C] and/or
    outT [C, R] (views with unit-stride rows; allocated when True is passed)."""
    R, Cc = x.shape
    if out is True:
        out = torch.empty(R, Cc, device=x.device, dtype=torch.bfloat16)
    if outT is True:
        outT = torch.empty(Cc, R, device=x.device, dtype=torch.bfloat16)
    _T.cast_bf16_t(x, out, outT)
    return out, outT


# bf16 layer-0 projection split count (M >= 8N, M,N >= 512: ainp_gemm_bf16nt runs
# a split tall GEMM on the 256 x 256 tile, 168 -> 504 workgroups): inside the
# C3-shape step 483 -> 368 us + a 22 us slab sum, 9.92 -> 9.83 ms/step
# (profiles/r02_s14_b16_proj_split_ab.txt); AINP_B16_PROJ_SPLIT=1 = unsplit
B16_PROJ_SPLIT = int(os.environ.get("AINP_B16_PROJ_SPLIT", "3"))


GEMM16_256 = os.environ.get("AINP_GEMM16_256", "1")[:1] != "0"


def b16_proj_split(M, N, K):
    """Split count the bf16 layer-0 projection [M, N] x K uses (cnnblstm,
    bench): B16_PROJ_SPLIT only where ainp_gemm_bf16nt routes the split GEMM
    to the 256 x 256 tile (gemm16.hip: M >= 8N, M, N >= 512, at most 1536
    128 x 128 tiles, K % 32 == 0, AINP_GEMM16_256 on); else unsplit."""
    tiles128 = -(-M // 128) * -(-N // 128)
    ok = (GEMM16_256 and M >= 8 * N and M >= 512 and N >= 512 and tiles128 <= 1536
          and K % 32 == 0)
    return B16_PROJ_SPLIT if ok else 1


def gemm_bf16nt(A, B, K=None, out=None, bias=(None, None, None, None), bias_nsplit=0,
                nsplit=1):
    """C [M, N] = A [M, >=K] . B [N, >=K]^T + bias on bf16 operands (ainp_gemm_bf16nt);
    bias = (a1, a2, b1, b2): a1 + a2 for columns < bias_nsplit, b1 + b2 after.
    nsplit > 1: K split over slabs (bias in slab 0) summed in fixed order."""
    M, N = A.shape[0], B.shape[0]
    K = A.shape[1] if K is None else int(K)
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=torch.float32)
    S = int(nsplit)
    kc = -(-K // S // 64) * 64 if S > 1 else K
    if S > 1 and (-(-K // kc) != S or not out.is_contiguous()):
        S, kc = 1, K
    if S == 1:
        _T.gemm_bf16nt(A, B, out, K, *bias, int(bias_nsplit), 1, K)
        return out
    slabs = torch.empty(S, M, N, device=A.device, dtype=torch.float32)
    _T.gemm_bf16nt(A, B, slabs, K, *bias, int(bias_nsplit), S, kc)
    sum_slabs(slabs, S, out=out.view(-1))
    return out


# fp32 layer-0 projection on the 256 x 256 LDS-DMA tile (ainp_gemm_x6nt_256):
# split 3 fills the 256 CUs with the 168 tiles of M = 10688, N = 1024
# (2.28 -> 2.09 ms, tools/x6_256_lab.cpp); AINP_X6_256=0 keeps ainp_gemm_f32.
X6_256 = os.environ.get("AINP_X6_256", "1") != "0"
# layer-0 fp32 data gradient on the same tile (W_ih^T transposed per step).  Off:
# inside the step it ran 4.11 ms against the 128 x 128 x6 kernel's 3.10 ms, as
# the side-stream weight-gradient GEMM cannot co-reside with its 144 KB of LDS
# (profiles/r02_s11_dx_x6_256_ab.txt); AINP_DX_X6_256=1 turns it on.
DX_X6_256 = os.environ.get("AINP_DX_X6_256", "0") == "1"
_X6_SPLIT = 3


def x6_256_eligible(M, N, K, bsplit):
    return X6_256 and M >= 2048 and K % 16 == 0 and (bsplit % 256 == 0 or bsplit == N) \
        and N >= 512


def transpose_f32(x, out=None):
    """ainp_transpose_f32: fp32 x [R, C] (unit-stride rows) -> out [C, R]."""
    R, Cc = x.shape
    if out is None:
        out = torch.empty(Cc, R, device=x.device, dtype=torch.float32)
    _T.transpose_f32(x, out)
    return out


def gemm_x6nt_256(A, B1, B2, out, bias=(None, None, None, None), bias_nsplit=0, nsplit=None):
    """out [M, N1+N2] = A [M, K] . [B1; B2]^T + bias, fp32 on the three-piece
    bf16 split (ainp_gemm_x6nt_256); split-K slabs summed in fixed order."""
    M, K = A.shape
    N = B1.shape[0] + B2.shape[0]
    S = _X6_SPLIT if nsplit is None else int(nsplit)
    if S == 1:
        _T.gemm_x6nt_256(A, B1, B2, out, *bias, int(bias_nsplit), 1, K)
        return out
    kc = -(-K // S // 16) * 16
    slabs = torch.empty(S, M, N, device=A.device, dtype=torch.float32)
    _T.gemm_x6nt_256(A, B1, B2, slabs, *bias, int(bias_nsplit), S, kc)
    sum_slabs(slabs, S, out=out.view(-1))
    return out


# bf16 MFMA rate per resident workgroup slot and the HBM rate, for the split-K
# choice below (measured orders of magnitude, not limits)
_B16_TILE_RATE = 700e12 / 768
_SLAB_RATE = 4e12


@functools.lru_cache(maxsize=256)
def _splitk_bf16(M, N, K, slots=768, max_split=16):
    """Split count S for a bf16 GEMM over a small M x N: minimise the wave-quantised
    MFMA time ceil(tiles*S/slots) * tile_time(K/S) plus the slab round trip."""
    tiles = -(-M // 128) * -(-N // 128)
    best, best_t = 1, None
    for S in range(1, max_split + 1):
        kc = -(-K // S // 64) * 64
        if kc < 64:
            break
        Sr = -(-K // kc)
        if Sr != S:
            continue
        t = -(-tiles * S // slots) * 2.0 * 128 * 128 * kc / _B16_TILE_RATE
        if S > 1:
            t += 2.0 * S * M * N * 4 / _SLAB_RATE
        if best_t is None or t < best_t:
            best, best_t = S, t
    return best


def x6_problem(A, B, C, M, N, K, lda, ldb, ldc, *, A2=None, a_ksplit=0, a_kmajor=False,
               B2=None, b_nsplit=0, b_ksplit=0, b_kmajor=False, C2=None, c_msplit=0,
               bias=(None, None, None, None), bias_nsplit=0, nsplit=1, kc=0, strideC=0):
    """One problem of ainp_gemm_x6_multi (include/ainp.h: element maps, splits)."""
    return {"ins": [A, A2, B, B2, *bias], "outs": [C, C2],
            "ints": [int(a_ksplit), int(bool(a_kmajor)), int(b_nsplit), int(b_ksplit),
                     int(bool(b_kmajor)), int(c_msplit), int(bias_nsplit), int(M), int(N), int(K),
                     int(nsplit), int(kc), int(strideC), int(lda), int(ldb), int(ldc)]}


_EMPTY = {}


def gemm_x6_multi(problems):
    """fp32-accurate GEMMs, 1..3 problems in one launch (ainp_gemm_x6_multi,
    csrc/gemm_x6r.hip)."""
    ins, outs, ints = [], [], []
    for p in problems:
        ins += p["ins"]
        for t in p["outs"]:
            if t is None:
                dev = p["outs"][0].device
                t = _EMPTY.get(dev)
                if t is None:
                    t = _EMPTY[dev] = torch.empty(0, device=dev)
            outs.append(t)
        ints += p["ints"]
    _T.gemm_x6_multi(ins, outs, ints)


# AINP_L0_BWD_X6R=0 keeps the layer-0 backward pair on two streams (128 x 128
# x6 kernels: dX on the current stream, the split-K weight gradient beside it)
L0_BWD_X6R = os.environ.get("AINP_L0_BWD_X6R", "1") != "0"
# AINP_PAIR_JOIN=1 (measured slower, 16.6 vs 16.1 ms C2 step, profiles/r03_ab1_*): the pair waits for the side stream's weight gradients
PAIR_JOIN = os.environ.get("AINP_PAIR_JOIN", "0") == "1"
# AINP_MAIN_FIRST=0: the BLSTM backward issues each layer's data gradient after
# the side stream's weight-gradient launches (the round-3 order); default: before
MAIN_FIRST = os.environ.get("AINP_MAIN_FIRST", "1") != "0"
# the fp32 layer-0 projection on the split-plane tile (AINP_X6R_FWD=0: on
# gemm_x6nt_256; 1.73 vs 2.15 ms alone, profiles/r03_x6r_probe.log)
# (bit-identical to gemm_x6nt_256)
X6R_FWD = os.environ.get("AINP_X6R_FWD", "1") != "0"


def l0_bwd_x6r_eligible(NT, I, H):
    """Shapes ops.lstm_l0_bwd_x6 takes: K of the weight gradient (= NT) and of
    the data gradient (= 8H) in whole 16-deep K-tiles, the direction split on
    the 256-row tile grid, 4-row groups of the k-major operands."""
    return (L0_BWD_X6R and NT % 16 == 0 and I % 4 == 0 and (4 * H) % 256 == 0 and NT >= 256)


def lstm_l0_bwd_x6(dg, wf, wr, x, dx, dwf, dwr):
    """The fp32 layer-0 LSTM backward pair in ONE launch (nn.LSTM backward,
    models/CNNBLSTM/model.py:46-47,77):
        dW_cat [8H, I] = dg^T [8H, NT] . X [NT, I]   (rows < 4H -> dwf, rest -> dwr)
        dX [NT, I]     = dg [NT, 8H] . W_cat [8H, I] (k < 4H from wf, rest from wr)
    dg [NT, 8H], x [NT, I] (row-major, read as they lie: k-major operands of the
    weight gradient), wf / wr [4H, I]; the weight-gradient tiles (long K = NT)
    are scheduled first, the data-gradient tiles fill in behind them."""
    NT, G8 = dg.shape
    I = x.shape[1]
    G4 = G8 // 2
    for t in (dg, x, wf, wr, dx, dwf, dwr):
        _req(t, "operand")
    pw = x6_problem(dg, x, dwf, M=G8, N=I, K=NT, lda=G8, ldb=I, ldc=I, a_kmajor=True,
                    b_kmajor=True, C2=dwr, c_msplit=G4)
    px = x6_problem(dg, wf, dx, M=NT, N=I, K=G8, lda=G8, ldb=I, ldc=I, B2=wr, b_ksplit=G4,
                    b_kmajor=True)
    gemm_x6_multi([pw, px])


def gemm_x6r_nt(A, B1, B2, out, bias=(None, None, None, None), bias_nsplit=0, nsplit=None):
    """The fp32 layer-0 projection on the split-plane tile: drop-in for
    gemm_x6nt_256 (same split-K rule, bias in slab 0, bit-identical slabs)."""
    M, K = A.shape
    N1 = B1.shape[0]
    N = N1 + B2.shape[0]
    S = _X6_SPLIT if nsplit is None else int(nsplit)
    kc = -(-K // S // 16) * 16 if S > 1 else K
    if S > 1 and -(-K // kc) != S:
        S, kc = 1, K
    kw = dict(B2=B2 if B2.shape[0] else None, b_nsplit=N1 if B2.shape[0] else 0,
              bias=bias, bias_nsplit=bias_nsplit)
    if S == 1:
        gemm_x6_multi([x6_problem(A, B1, out, M=M, N=N, K=K, lda=A.stride(0), ldb=B1.stride(0),
                                  ldc=out.stride(0), **kw)])
        return out
    slabs = torch.empty(S, M, N, device=A.device, dtype=torch.float32)
    gemm_x6_multi([x6_problem(A, B1, slabs, M=M, N=N, K=K, lda=A.stride(0), ldb=B1.stride(0),
                              ldc=N, nsplit=S, kc=kc, strideC=M * N, **kw)])
    sum_slabs(slabs, S, out=out.view(-1))
    return out


# AINP_PROJ_X6R=0 keeps the fp32 output-projection backward on gemm_f32
# (pointer-batched FMA GEMMs over the [N, C*F, T] gradient as it lies)
PROJ_X6R = os.environ.get("AINP_PROJ_X6R", "1") != "0"
# AINP_PROJ_JOINT=1: dh and dW in one launch even when the weight gradient
# could be deferred to the side stream (A/B)
PROJ_JOINT = os.environ.get("AINP_PROJ_JOINT", "0") == "1"
_X6R_SLOTS = 256        # one 160 KB-LDS workgroup per CU


def _x6r_makespan(items_kt, slots=_X6R_SLOTS):
    """Finish time (in K-tiles) of work items dispatched in grid order onto
    `slots` CUs, each taking the next item when it frees (items_kt: K-tiles
    per item)."""
    free = [0] * slots
    heapq.heapify(free)
    end = 0
    for kt in items_kt:
        t = heapq.heappop(free) + kt
        end = max(end, t)
        heapq.heappush(free, t)
    return end


@functools.lru_cache(maxsize=64)
def x6r_splits(shapes, max_split=16):
    """Split-K counts for problems (M, N, K) launched together on the x6r tile:
    minimise the estimated makespan plus the slab traffic (each split > 1 writes
    S slabs that ainp_sum_slabs reads back).  Returns ((S, kc), ...)."""
    def opts(M, N, K):
        out = []
        for S in range(1, max_split + 1):
            kc = -(-K // S // 16) * 16 if S > 1 else K
            if S > 1 and -(-K // kc) != S:
                continue
            out.append((S, kc))
        return out
    best, best_t = None, None
    for combo in itertools.product(*(opts(*s) for s in shapes)):
        items = []
        slab = 0.0
        for (M, N, K), (S, kc) in zip(shapes, combo):
            tiles = -(-M // 256) * -(-N // 256)
            items += [kc // 16] * (tiles * S)
            if S > 1:
                slab += (S + 1) * M * N * 4
        # K-tile of a 256 x 256 x16 x6 item ~ 4.5 us at the measured rate
        t = _x6r_makespan(items) * 4.5e-6 + slab / _SLAB_RATE
        if best_t is None or t < best_t:
            best, best_t = combo, t
    return best


def proj_bwd_x6_eligible(NT, NO, K):
    """Output projection shapes the x6r backward takes: whole 16-deep K-tiles
    (K of dW = N*T, of dh = C*F) and 4-row groups of the k-major operands."""
    return PROJ_X6R and NT % 16 == 0 and NO % 16 == 0 and K % 4 == 0


def proj_bwd_x6(gp, h, w, dh=None, dw=None):
    """The fp32 output-projection gradients of nn.Linear(2H, C*F)
    (models/CNNBLSTM/model.py:48,78) on the x6r tile, from the gradient
    permuted to gp [C*F, N*T] (row c*... = output column, k = n*T + t):
        dh [NT, K] = gp^T [NT, NO] . w [NO, K]   (both operands k-major)
        dW [NO, K] = gp   [NO, NT] . h [NT, K]   (h k-major)
    Either output may be None; both given -> ONE launch.  Rows of gp are the
    C*F output columns, its columns k = n*T + t."""
    NO, NT = gp.shape
    K = h.shape[-1]
    for t in (gp, h, w):
        _req(t, "operand")
    # each problem's split-K is chosen for it alone, so the joint launch and
    # two separate ones (side-stream deferral) give bit-identical gradients
    probs, outs = [], []
    if dh is not None:
        (S, kc), = x6r_splits(((NT, K, NO),))
        C = dh if S == 1 else torch.empty(S, NT, K, device=gp.device)
        probs.append(x6_problem(gp, w, C, M=NT, N=K, K=NO, lda=NT, ldb=K, ldc=K, a_kmajor=True,
                                b_kmajor=True, nsplit=S, kc=kc, strideC=NT * K))
        outs.append((dh, C, S))
    if dw is not None:
        (S, kc), = x6r_splits(((NO, K, NT),))
        C = dw if S == 1 else torch.empty(S, NO, K, device=gp.device)
        probs.append(x6_problem(gp, h, C, M=NO, N=K, K=NT, lda=NT, ldb=K, ldc=K, b_kmajor=True,
                                nsplit=S, kc=kc, strideC=NO * K))
        outs.append((dw, C, S))
    gemm_x6_multi(probs)
    for o, C, S in outs:
        if S > 1:
            sum_slabs(C, S, out=o.view(-1))


# AINP_B16_PAIR=0: the bf16 layer-0 backward keeps dX (128 x 128 tiles) on the
# current stream beside a split-K dW on the side stream, instead of the pair in
# one 256 x 256 launch (ops.lstm_l0_bwd_bf16)
B16_PAIR = os.environ.get("AINP_B16_PAIR", "1") != "0"
# AINP_B16_KM=1: the pair's weight gradient reads dg [NT, 8H] and X [NT, I] as
# they lie (k-major operands, ds_read_b64_tr_b16), so the bridge writes no X^T
# and the BPTT gradient no dg^T copy
# (C3-shape 8.21 -> 7.90 ms/step A/B, profiles/r05s_ab_b16_kmajor.txt)
B16_KM = os.environ.get("AINP_B16_KM", "1") != "0"


@functools.lru_cache(maxsize=64)
def g256_splits(shapes, max_split=16):
    """Split-K counts for bf16 problems (M, N, K) launched together by
    ainp_gemm_bf16nt_multi (256 x 256 tiles, 32-deep K-tiles, one workgroup per
    CU): minimise the estimated makespan plus the slab round trip, as
    x6r_splits does for the x6r tile.  Returns ((S, kc), ...)."""
    def opts(M, N, K):
        out = []
        # 64-deep K-tiles where K allows (gemm16.hip tile256b needs 64 | kc)
        g = 64 if K % 64 == 0 else 32
        for S in range(1, max_split + 1):
            kc = -(-K // S // g) * g if S > 1 else K
            if S > 1 and -(-K // kc) != S:
                continue
            out.append((S, kc))
        return out
    best, best_t = None, None
    for combo in itertools.product(*(opts(*sh) for sh in shapes)):
        items = []
        slab = 0.0
        for (M, N, K), (S, kc) in zip(shapes, combo):
            tiles = -(-M // 256) * -(-N // 256)
            items += [kc // 32] * (tiles * S)
            if S > 1:
                slab += (S + 1) * M * N * 4
        # a 256 x 256 x 32 bf16 K-tile ~ 1.1 us at the measured per-CU rate
        t = _x6r_makespan(items) * 1.1e-6 + slab / _SLAB_RATE
        if best_t is None or t < best_t:
            best, best_t = combo, t
    return best


def gemm_bf16nt_multi(problems):
    """Up to 3 bf16 GEMMs C = A . B^T in ONE launch (ainp_gemm_bf16nt_multi,
    256 x 256 tiles): problems = [(A, B, C, K, nsplit, kc[, a_kmajor, b_kmajor])],
    A [M, >=K] or k-major [>=K, M], B [N, >=K] or k-major [>=K, N], C [M, N]
    (nsplit 1) or slabs [nsplit, M, N]."""
    ints = []
    for pr in problems:
        A, B, C, K, S, kc = pr[:6]
        akm, bkm = (pr[6], pr[7]) if len(pr) > 6 else (False, False)
        _work("gemm_bf16nt", 2.0 * C.shape[-2] * C.shape[-1] * K)
        ints += [int(K), int(S), int(kc), int(bool(akm)), int(bool(bkm))]
    _T.gemm_bf16nt_multi([p[0] for p in problems], [p[1] for p in problems],
                         [p[2] for p in problems], ints)


def wgrad_bf16_km(dg16_cols, x16, NT, out):
    """out [rows, I] = dg16_cols^T . X on the 256 x 256 tile from k-major
    operands (dg16_cols: [NT, rows] column view of dg [NT, 8H]; x16 [NT, I]),
    split over K by the makespan model, slabs summed in fixed order."""
    rows, I = out.shape
    (S, kc), = g256_splits(((rows, I, NT),))
    C = out if S == 1 else torch.empty(S, rows, I, device=out.device)
    gemm_bf16nt_multi([(dg16_cols, x16, C, NT, S, kc, True, True)])
    if S > 1:
        sum_slabs(C, S, out=out.view(-1))
    return out


def l0_bwd_bf16_eligible(NT, I, H):
    """Shapes ops.lstm_l0_bwd_bf16 takes: both reductions (N*T, 8H) in whole
    32-deep K-tiles, 16-byte operand rows."""
    return B16_PAIR and NT % 32 == 0 and (8 * H) % 32 == 0 and I % 8 == 0


def lstm_l0_bwd_bf16(dg16, dgT16, wT16, xB16, dx, gcat, km=False):
    """The bf16 layer-0 LSTM backward pair in ONE launch (nn.LSTM backward,
    models/CNNBLSTM/model.py:46-47,77):
        dW_cat [8H, I] = dg^T . X   from dgT16 [8H, >=NT] and xB16 = X^T [I, >=NT]
                                    (km: from dg16 and xB16 = X [NT, I], k-major)
        dX [NT, I]     = dg . W_cat from dg16 [NT, 8H] and wT16 = W_cat^T [I, 8H]
    the weight-gradient items (long K = N*T) first, the data-gradient items
    behind them; dW split over K only where the makespan model asks for it."""
    NT, G8 = dg16.shape
    I = xB16.shape[1] if km else xB16.shape[0]
    (Sw, kcw), (Sx, kcx) = g256_splits(((G8, I, NT), (NT, I, G8)))
    Cw = gcat if Sw == 1 else torch.empty(Sw, G8, I, device=dg16.device)
    Cx = dx if Sx == 1 else torch.empty(Sx, NT, I, device=dg16.device)
    pw = (dg16, xB16, Cw, NT, Sw, kcw, True, True) if km else (dgT16, xB16, Cw, NT, Sw, kcw)
    gemm_bf16nt_multi([pw, (dg16, wT16, Cx, G8, Sx, kcx)])
    if Sw > 1:
        sum_slabs(Cw, Sw, out=gcat.view(-1))
    if Sx > 1:
        sum_slabs(Cx, Sx, out=dx.view(-1))


def gemm_bf16nt_splitk(A, B, K, out=None, max_split=16):
    """A [M, >=K] . B [N, >=K]^T (bf16, no bias) with the long K split over
    slabs summed in fixed order (ainp_sum_slabs) -- the weight gradients."""
    M, N = A.shape[0], B.shape[0]
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=torch.float32)
    if not out.is_contiguous():
        raise ValueError("gemm_bf16nt_splitk: out must be contiguous")
    S = _splitk_bf16(M, N, K, max_split=max_split)
    _work("gemm_bf16nt", 2.0 * M * N * K)
    if S == 1:
        _T.gemm_bf16nt(A, B, out, int(K), None, None, None, None, 0, 1, int(K))
        return out
    kc = -(-K // S // 64) * 64
    slabs = torch.empty(S, M, N, device=A.device, dtype=torch.float32)
    _T.gemm_bf16nt(A, B, slabs, int(K), None, None, None, None, 0, S, kc)
    sum_slabs(slabs, S, out=out.view(-1))
    return out


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """y = x @ w^T + b for x [M, K] row-major (nn.Linear semantics)."""
    _req(x, "x"); _req(w, "w")
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N, device=x.device, dtype=torch.float32)
    gemm(M, N, K, [x], K, 1, [w], 1, K, [y], N, 1,
         bias1=[b] if b is not None else None)
    return y


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a [M,K] @ b [K,N] for 2-D float32 cuda tensors (any unit-stride layout)."""
    _req(a, "a", contiguous=False); _req(b, "b", contiguous=False)
    M, K = a.shape
    K2, N = b.shape
    assert K == K2
    c = torch.empty(M, N, device=a.device, dtype=torch.float32)
    sam, sak = a.stride()
    sbk, sbn = b.stride()
    if sam != 1 and sak != 1:
        a = a.contiguous(); sam, sak = a.stride()
    if sbk != 1 and sbn != 1:
        b = b.contiguous(); sbk, sbn = b.stride()
    gemm(M, N, K, [a], sam, sak, [b], sbk, sbn, [c], N, 1)
    return c


# --------------------------------------------------------------------- conv
def conv_stat_parts(N, H, W) -> int:
    return _lib.lib.ainp_conv3x3_fwd_stat_parts(N, H, W)


def _x_flag(x, bf16, name="x"):
    if x.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"{name} must be float32 or bfloat16, got {x.dtype}")
    if x.dtype == torch.bfloat16 and not bf16:
        raise ValueError(f"a bf16 {name} needs the bf16 conv arithmetic (bf16=True)")
    return CONV_X16 if x.dtype == torch.bfloat16 else 0


def conv3x3_fwd(x, w, b=None, in_scale=None, in_shift=None, want_stats=False, bf16=False,
                y16=False, xcl=False, ycl=False):
    """x fp32, or bf16 storage with bf16=True (AINP_CONV_X16); y16: y written
    as bf16 (AINP_CONV_Y16, BatchNorm partials of the stored values).  Both
    where io16_ok says so (the bf16 configuration's pre-BN activations).
    xcl / ycl (round 5): x given / y returned channel-last, [N, H, W, C]
    (AINP_CONV_XCL / _YCL; cl_ok says for which convs)."""
    _req(x, "x", None); _req(w, "w")
    if xcl:
        N, H, W, Cin = x.shape
    else:
        N, Cin, H, W = x.shape
    Cout = w.shape[0]
    assert tuple(w.shape) == (Cout, Cin, 3, 3)
    flags = (CONV_BF16 if bf16 else 0) | _x_flag(x, bf16)
    flags |= (CONV_XCL if xcl else 0) | (CONV_YCL if ycl else 0)
    if y16:
        if not bf16:
            raise ValueError("y16 needs the bf16 conv arithmetic (bf16=True)")
        flags |= CONV_Y16
    shape = (N, H, W, Cout) if ycl else (N, Cout, H, W)
    y = torch.empty(shape, device=x.device, dtype=torch.bfloat16 if y16 else torch.float32)
    stats = None
    if want_stats:
        stats = torch.empty(_lib.lib.ainp_conv3x3_fwd_stat_rows_ex(N, Cin, Cout, H, W,
                                                                   CONV_BF16 if bf16 else 0),
                            2 * Cout,
                            device=x.device, dtype=torch.float64)
    _T.conv3x3_fwd(x, w, b, in_scale, in_shift, y, stats, flags)
    return y, stats


def cl_ok(N, Cin, Cout, H, W) -> bool:
    """ainp_conv3x3_cl_ok: every entry point of Conv2d(Cin, Cout) takes
    channel-last activations."""
    return bool(_lib.lib.ainp_conv3x3_cl_ok(N, Cin, Cout, H, W))


def io16_ok(N, Cin, Cout, H, W) -> bool:
    """ainp_conv3x3_io16_ok: Conv2d(Cin, Cout)'s forward takes a bf16 act(x)
    source and writes a bf16 y, and its weight gradient takes the bf16 source."""
    return bool(_lib.lib.ainp_conv3x3_io16_ok(N, Cin, Cout, H, W))


def _dy_flags(dy, bf16):
    if dy.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"dy must be float32 or bfloat16, got {dy.dtype}")
    if dy.dtype == torch.bfloat16:
        if not bf16:
            raise ValueError("a bf16 dy needs the bf16 conv arithmetic (bf16=True)")
        return CONV_BF16 | CONV_DY16
    return CONV_BF16 if bf16 else 0


def conv3x3_dgrad(dy, w, bf16=False, xcl=False, ycl=False, cfnt=False):
    """dy fp32, or bf16 storage with bf16=True (AINP_CONV_DY16).  xcl / ycl:
    dy given / dx returned channel-last [N, H, W, C].  cfnt (AINP_CONV_YCFNT,
    see dgrad_cfnt_ok): dx written [C, H, N, W], returned as its [N, C, H, W]
    view (permute(2, 0, 1, 3) of that buffer)."""
    _req(dy, "dy", None); _req(w, "w")
    if xcl:
        N, H, W, Cout = dy.shape
    else:
        N, Cout, H, W = dy.shape
    Cin = w.shape[1]
    if cfnt:
        if ycl:
            raise ValueError("conv3x3_dgrad: cfnt and ycl are exclusive")
        buf = torch.empty((Cin, H, N, W), device=dy.device, dtype=torch.float32)
        _T.conv3x3_dgrad(dy, w, buf, _dy_flags(dy, bf16) | (CONV_XCL if xcl else 0) | CONV_YCFNT)
        return buf.permute(2, 0, 1, 3)
    dx = torch.empty((N, H, W, Cin) if ycl else (N, Cin, H, W), device=dy.device,
                     dtype=torch.float32)
    _T.conv3x3_dgrad(dy, w, dx, _dy_flags(dy, bf16) | (CONV_XCL if xcl else 0)
                     | (CONV_YCL if ycl else 0))
    return dx


def dgrad_cfnt_ok(N, Cin, Cout, H, W) -> bool:
    """ainp_conv3x3_dgrad_cfnt_ok: the data gradient of Conv2d(Cin, Cout) can
    write dx as [Cin, H, N, W] (conv3x3_dgrad(cfnt=True))."""
    return bool(_lib.lib.ainp_conv3x3_dgrad_cfnt_ok(N, Cin, Cout, H, W))


def conv3x3_dgrad_bnr(dy, w, y, scale, shift, save, bf16=False, xcl=False, want_dx=True):
    """The data gradient (dx channel-last [N, H, W, Cin]) and the reduce step
    of the BatchNorm+ReLU backward it feeds (ainp_conv3x3_dgrad_bnr): y is that
    layer's pre-BatchNorm output [N, H, W, Cin] (fp32 or bf16 storage).
    Returns (dx, sums) -- sums as bn_relu_bwd_reduce(dx, y, ..., cl=True).
    want_dx=False (Conv2d(16, 1), round 6): dx is not written (returned None);
    conv3x3_dgrad_bnapply recomputes it into the apply."""
    _req(dy, "dy", None); _req(w, "w"); _req(y, "y", None)
    if xcl:
        N, H, W, Cout = dy.shape
    else:
        N, Cout, H, W = dy.shape
    Cin = w.shape[1]
    dx = torch.empty((N, H, W, Cin) if want_dx else (0,), device=dy.device,
                     dtype=torch.float32)
    ws = torch.empty(_lib.lib.ainp_conv3x3_dgrad_bnr_workspace(N, Cin, Cout, H, W),
                     device=dy.device, dtype=torch.uint8)
    sums = torch.empty(2 * Cin, device=dy.device, dtype=torch.float64)
    _T.conv3x3_dgrad_bnr(dy, w, dx, _dy_flags(dy, bf16) | (CONV_XCL if xcl else 0) | CONV_YCL,
                         y, scale, shift, save, ws, sums, _y_flag(y))
    return (dx if want_dx else None), sums


def conv3x3_dgrad_bnapply(dy, w, y, scale, shift, gamma, save, sums, count, gy16=False):
    """Round 6 (ainp_conv3x3_dgrad_bnapply): Conv2d(16, 1)'s data gradient
    (dy [N, 1, H, W]) recomputed and fed through the BatchNorm+ReLU backward
    apply of the 16-channel layer (y fp32 [N, H, W, 16], sums from
    conv3x3_dgrad_bnr(want_dx=False)).  Returns (gy, dgamma, dbeta) as
    bn_relu_bwd_apply(dx, y, ..., cl=True) would (gy16: bf16 storage)."""
    _req(dy, "dy"); _req(w, "w"); _req(y, "y")
    N, _, H, W = dy.shape
    gy = torch.empty(N, H, W, 16, device=dy.device,
                     dtype=torch.bfloat16 if gy16 else torch.float32)
    dgamma = torch.empty(16, device=dy.device, dtype=torch.float32)
    dbeta = torch.empty(16, device=dy.device, dtype=torch.float32)
    _T.conv3x3_dgrad_bnapply(dy, w, y, scale, shift, gamma, save, sums, int(count), gy, dgamma,
                             dbeta)
    return gy, dgamma, dbeta


def conv3x3_wgrad(x, dy, in_scale=None, in_shift=None, want_bias=True, bf16=False, out=None,
                  xcl=False, gcl=False):
    """out: optional preallocated (dw, db) to write.  dy fp32, or bf16 storage
    with bf16=True (AINP_CONV_DY16).  xcl / gcl: x / dy channel-last."""
    _req(x, "x", None); _req(dy, "dy", None)
    if xcl:
        N, H, W, Cin = x.shape
    else:
        N, Cin, H, W = x.shape
    Cout = dy.shape[3] if gcl else dy.shape[1]
    if out is not None:
        dw, db = out
    else:
        dw = torch.empty(Cout, Cin, 3, 3, device=x.device, dtype=torch.float32)
        db = torch.empty(Cout, device=x.device, dtype=torch.float32) if want_bias else None
    ws_bytes = _lib.lib.ainp_conv3x3_wgrad_workspace(N, Cin, Cout, H, W)
    ws = torch.empty(ws_bytes, device=x.device, dtype=torch.uint8)
    _T.conv3x3_wgrad(x, in_scale, in_shift, dy, dw, db, ws,
                     _dy_flags(dy, bf16) | _x_flag(x, bf16) | (CONV_XCL if xcl else 0)
                     | (CONV_GCL if gcl else 0))
    return dw, db


# --------------------------------------------------------------------- BN
def bn_stats_reduce(stats, C, count=None):
    """conv epilogue partials [parts, 2C] -> per-channel [sum y | sum y^2] (f64).
    count (data parallel): appended as sums[2C], so that all-reducing the
    vector also sums the element counts; then pass count=0 to bn_finalize /
    bn_relu_bwd_apply (include/ainp.h)."""
    sums = torch.empty(2 * C + (1 if count is not None else 0), device=stats.device,
                       dtype=torch.float64)
    _T.bn_stats_reduce(stats, sums, int(C))
    if count is not None:
        sums[2 * C:].fill_(float(count))
    return sums


def bn_finalize(sums, count, gamma, beta, running_mean, running_var, momentum, eps):
    """count == 0: the count is sums[2C] (see bn_stats_reduce)."""
    C = sums.numel() // 2
    dev = sums.device
    scale = torch.empty(C, device=dev, dtype=torch.float32)
    shift = torch.empty(C, device=dev, dtype=torch.float32)
    save = torch.empty(2, C, device=dev, dtype=torch.float32)
    _T.bn_finalize(sums, int(count), gamma, beta, running_mean, running_var, float(momentum),
                   float(eps), scale, shift, save)
    return scale, shift, save


def bn_reduce_finalize(stats, C, count, gamma, beta, running_mean, running_var, momentum, eps):
    """bn_stats_reduce + bn_finalize in one launch (single process, count > 0):
    (scale, shift, save), bit for bit those of the two calls."""
    dev = stats.device
    scale = torch.empty(C, device=dev, dtype=torch.float32)
    shift = torch.empty(C, device=dev, dtype=torch.float32)
    save = torch.empty(2, C, device=dev, dtype=torch.float32)
    _T.bn_reduce_finalize(stats, int(count), gamma, beta, running_mean, running_var,
                          float(momentum), float(eps), scale, shift, save)
    return scale, shift, save


def bn_eval_affine(gamma, beta, running_mean, running_var, eps):
    C = running_mean.numel()
    dev = running_mean.device
    scale = torch.empty(C, device=dev, dtype=torch.float32)
    shift = torch.empty(C, device=dev, dtype=torch.float32)
    _T.bn_eval_affine(gamma, beta, running_mean, running_var, float(eps), scale, shift)
    return scale, shift


def bn_relu_apply(x, scale, shift, ntcf=False):
    _req(x, "x")
    N, C, H, W = x.shape
    if ntcf:
        out = torch.empty(N, W, C * H, device=x.device, dtype=torch.float32)
    else:
        out = torch.empty_like(x)
    _T.bn_relu_apply(x, scale, shift, out, bool(ntcf))
    return out


def _y_flag(y):
    if y.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"y must be float32 or bfloat16, got {y.dtype}")
    return BN_Y16 if y.dtype == torch.bfloat16 else 0


def bn_relu_bwd_reduce(g, y, scale, shift, save, ntcf=False, cl=False):
    """y fp32 or bf16 storage (AINP_BN_Y16).  cl (round 5): g and y
    channel-last [N, H, W, C] (AINP_BN_CL), g fp32 or bf16 (AINP_BN_G16)."""
    _req(y, "y", None)
    if cl:
        N, H, W, C = y.shape
        flags = BN_CL | (BN_G16 if g.dtype == torch.bfloat16 else 0)
    else:
        _req(g, "g")
        N, C, H, W = y.shape
        flags = 0
    ws = torch.empty(_lib.lib.ainp_bn_relu_bwd_workspace(N, C, H, W), device=y.device,
                     dtype=torch.uint8)
    sums = torch.empty(2 * C, device=y.device, dtype=torch.float64)
    _T.bn_relu_bwd_reduce(g, y, scale, shift, save, ws, sums, bool(ntcf), _y_flag(y) | flags)
    return sums


def bn_relu_bwd_apply(g, y, scale, shift, gamma, save, sums, count, ntcf=False, gy16=False,
                      cl=False):
    """gy16: gy in bf16 storage (AINP_BN_GY16) -- for the bf16 configuration's
    data / weight gradients, which round gy to bf16 anyway (conv3x3_dgrad /
    conv3x3_wgrad take it with bf16=True; dy16_ok says for which convs).
    cl: g, y and gy channel-last [N, H, W, C]."""
    if cl:
        N, H, W, C = y.shape
        flags = BN_CL | (BN_G16 if g.dtype == torch.bfloat16 else 0)
    else:
        N, C, H, W = y.shape
        flags = 0
    gy = torch.empty(y.shape, device=y.device, dtype=torch.bfloat16 if gy16 else torch.float32)
    dgamma = torch.empty(C, device=y.device, dtype=torch.float32)
    dbeta = torch.empty(C, device=y.device, dtype=torch.float32)
    _T.bn_relu_bwd_apply(g, y, scale, shift, gamma, save, sums, int(count), gy, dgamma, dbeta,
                         bool(ntcf), (BN_GY16 if gy16 else 0) | _y_flag(y) | flags)
    return gy, dgamma, dbeta


def conv3x3_wgrad_bnapply(x, in_scale, in_shift, g, y, scale, shift, gamma, save, sums, count):
    """Round 6 (ainp_conv3x3_wgrad_bnapply): the Conv2d(1, 16) weight gradient
    (x [N, 1, H, W]) whose dy is the BatchNorm+ReLU backward apply of its
    output -- g, y channel-last [N, H, W, 16] fp32 -- formed per element and
    never written.  Returns (dw, db, dgamma, dbeta): conv3x3_wgrad(x, gy, ...,
    gcl=True) and bn_relu_bwd_apply(g, y, ..., cl=True)'s dgamma / dbeta."""
    _req(x, "x"); _req(g, "g"); _req(y, "y")
    N, _, H, W = x.shape
    dw = torch.empty(16, 1, 3, 3, device=x.device, dtype=torch.float32)
    db = torch.empty(16, device=x.device, dtype=torch.float32)
    dgamma = torch.empty(16, device=x.device, dtype=torch.float32)
    dbeta = torch.empty(16, device=x.device, dtype=torch.float32)
    ws = torch.empty(_lib.lib.ainp_conv3x3_wgrad_workspace(N, 1, 16, H, W), device=x.device,
                     dtype=torch.uint8)
    _T.conv3x3_wgrad_bnapply(x, in_scale, in_shift, g, y, scale, shift, gamma, save, sums,
                             int(count), dw, db, dgamma, dbeta, ws)
    return dw, db, dgamma, dbeta


def dy16_ok(N, Cin, Cout, H, W) -> bool:
    """ainp_conv3x3_dy16_ok: the data and weight gradients of Conv2d(Cin, Cout)
    take a bf16 dy (bf16 configuration)."""
    return bool(_lib.lib.ainp_conv3x3_dy16_ok(N, Cin, Cout, H, W))


def bn_relu_bwd(g, y, scale, shift, gamma, save, ntcf=False):
    N, C, H, W = y.shape
    sums = bn_relu_bwd_reduce(g, y, scale, shift, save, ntcf)
    return bn_relu_bwd_apply(g, y, scale, shift, gamma, save, sums, N * H * W, ntcf)


# --------------------------------------------------------------------- LSTM
def lstm_rec_fwd(zx, whh_f, whh_r, H, save=True):
    _req(zx, "zx"); _req(whh_f, "whh_f"); _req(whh_r, "whh_r")
    N, T, G = zx.shape
    assert G == 8 * H
    dev = zx.device
    h_out = torch.empty(N, T, 2 * H, device=dev, dtype=torch.float32)
    gates = torch.empty(N, T, 8 * H, device=dev, dtype=torch.float32) if save else None
    cell = torch.empty(N, T, 2 * H, device=dev, dtype=torch.float32) if save else None
    _T.lstm_rec_fwd(zx, whh_f, whh_r, h_out, gates, cell, int(H))
    return h_out, gates, cell


def lstm_rec_bwd(dh_out, gates, cell, whh_f, whh_r, H):
    _req(dh_out, "dh_out")
    N, T, _ = dh_out.shape
    dgates = torch.empty(N, T, 8 * H, device=dh_out.device, dtype=torch.float32)
    _T.lstm_rec_bwd(dh_out, gates, cell, whh_f, whh_r, dgates, int(H))
    return dgates


def lstm_hprev(h_out, H):
    N, T, _ = h_out.shape
    hp = torch.empty_like(h_out)
    _T.lstm_hprev(h_out, hp, int(H))
    return hp


# --------------------------------------------------------------------- loss
def l1_pow10_loss(y, mask, target, want_grad=True, grad_scale=1.0):
    """sum |10^y*m - |target|*m| -> (loss float64 [1], dy or None).  The sum
    is a fixed-order two-pass reduction (bit-reproducible run to run)."""
    _req(y, "y"); _req(mask, "mask"); _req(target, "target", torch.complex64)
    n = y.numel()
    assert mask.numel() == n and target.numel() == n
    ws = torch.empty(int(_lib.lib.ainp_l1_pow10_loss_slots(n)), device=y.device,
                     dtype=torch.float64)
    dy = torch.empty_like(y) if want_grad else None
    _T.l1_pow10_loss(y, mask, target, ws, dy, float(grad_scale))
    return ws[:1], dy


def scale_by_scalar(x, s):
    """x * s for a 0-dim/1-element float32 cuda tensor s (no host sync)."""
    s = s.reshape(1).to(torch.float32).contiguous()
    out = torch.empty_like(x)
    _T.scale_by_dev(x, out, s)
    return out


def sum_slabs(x, nslabs, out=None):
    n = x.numel() // nslabs
    if out is None:
        out = torch.empty(n, device=x.device, dtype=torch.float32)
    _T.sum_slabs(x, int(nslabs), int(n), out)
    return out


def rowsum_batched(x3d, out=None):
    nb, rows, cols = x3d.shape
    if out is None:
        out = torch.empty(rows, device=x3d.device, dtype=torch.float32)
    _T.rowsum_batched(x3d, out)
    return out


_DETERMINISTIC = True


def set_deterministic(on: bool) -> None:
    """accel.deterministic: forbid the atomic-accumulating entry points (the
    only non-fixed-order reductions; nothing on the training path uses them)."""
    global _DETERMINISTIC
    _DETERMINISTIC = bool(on)


def colsum(x2d, out=None, accumulate=False):
    """Column sums of a row-major [rows, cols] view.  Default: fixed-order row
    slabs combined by sum_slabs (deterministic);
    accumulate=True adds into `out` with float atomics (refused under
    accel.deterministic)."""
    rows, cols = x2d.shape
    ld = x2d.stride(0)
    assert x2d.stride(1) == 1
    if accumulate:
        if _DETERMINISTIC:
            raise RuntimeError("ops.colsum(accumulate=True) uses float atomics; "
                               "accel.deterministic is set")
        _T.colsum(x2d, rows, cols, ld, out, True)
        return out
    # ~256 workgroups of column sums; the slab combine then reads nslabs*cols
    nslabs = max(1, min(64, rows // 16, 256 // -(-cols // 256)))
    part = torch.empty(nslabs, cols, device=x2d.device, dtype=torch.float32)
    _T.colsum_slabs(x2d, rows, cols, ld, nslabs, part)
    return sum_slabs(part, nslabs, out)


def adam_step(params, grads, exp_avgs, exp_avg_sqs, lr, beta1, beta2, eps,
              weight_decay, step, step_dev=None, scalars_dev=None):
    """Multi-tensor Adam (ainp_adam_ex).  step_dev (float32 [1] device tensor,
    with scalars_dev float32 [2] scratch): the step counter lives on the device
    and is advanced by the launch (HIP-graph capturable); else host `step`."""
    if not params:
        return
    _T.adam(list(params), list(grads), list(exp_avgs), list(exp_avg_sqs), float(lr),
            float(beta1), float(beta2), float(eps), float(weight_decay),
            int(step) if step_dev is None else 0, step_dev, scalars_dev)


# ===================================================================== GAN
ACT_NONE, ACT_RELU, ACT_LEAKY, ACT_TANH = 0, 1, 2, 3


def conv_out_size(n, k, stride, pad):
    return (n + 2 * pad - k) // stride + 1


_WT_CACHE: dict = {}


def conv_weight_kmajor(w, C0, C1):
    """k-major copy of a conv weight for ainp_conv_gen_fwd, cached per weight
    tensor (id + weakref identity check) and invalidated by any in-place
    update (tensor._version) or reallocation (data_ptr)."""
    key = (w._version, C0, C1, w.data_ptr())
    ent = _WT_CACHE.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == key:
        return ent[2]
    Cout, Cin, KH, KW = w.shape
    wt = torch.empty(Cin * KH * KW, Cout, device=w.device, dtype=torch.float32)
    _T.conv_weight_kmajor(w, int(C0), int(C1), wt)
    wid = id(w)
    _WT_CACHE[wid] = (weakref.ref(w, lambda _r, wid=wid: _WT_CACHE.pop(wid, None)), key, wt)
    return wt


_WT16_CACHE: dict = {}
# bf16 convs run channel-last (ainp_conv_gen_fwd_nhwc16); AINP_CONV_NHWC16=0
# keeps the NCHW gather.  Sources with C % 32 != 0 (the U-Net's 1-channel
# planes) are gathered element-wise inside it unless AINP_CONV_NHWC16_SMALL=0;
# the plain few-channel first layers (D's, VGG's) keep the direct kernel
# (ainp_conv_gen_fwd_ex) unless AINP_CONV_NHWC16_SMALL=all.
CONV_NHWC16 = os.environ.get("AINP_CONV_NHWC16", "1") != "0"
# conv_gen(out16=True): the epilogue writes the next conv's channel-last bf16
# source (AINP_CONV_OUT16=0: a separate nchw_to_nhwc16 pass, as before)
CONV_OUT16 = os.environ.get("AINP_CONV_OUT16", "1") != "0"
CONV_NHWC16_SMALL = os.environ.get("AINP_CONV_NHWC16_SMALL", "1")
# the same copy from the few-input-channel direct conv and from the max-pool
# (AINP_OUT16_DIRECT=0: separate nchw_to_nhwc16 passes for those, A/B)
OUT16_DIRECT = os.environ.get("AINP_OUT16_DIRECT", "1") != "0"


def nhwc16_seg(C, KK):
    """k-values a source contributes to an nhwc16 weight row (gan.hip)."""
    return -(-KK * C // 32) * 32 if C % 32 else KK * C


def _direct_route(C0, C1, H0, W0, Hin, Win, KH, KW, Cout, want_stats):
    """ainp_conv_gen_fwd_ex's few-input-channel kernel (gan.hip
    conv_gen_smallcin_kernel) takes this conv (AINP_CONV_SMALLCIN unset)."""
    return (os.environ.get("AINP_CONV_SMALLCIN", "1") != "0" and C1 == 0
            and (H0, W0) == (Hin, Win) and not want_stats and 1 < Cout <= 64
            and C0 * KH * KW <= 160 and C0 <= 4)


def _nhwc16_route(C0, C1, H0, W0, Hin, Win, KH, KW, Cout, want_stats):
    if not CONV_NHWC16:
        return False
    if C0 % 32 == 0 and C1 % 32 == 0:
        return True
    if CONV_NHWC16_SMALL == "0":
        return False
    direct = (C1 == 0 and (H0, W0) == (Hin, Win) and not want_stats and Cout <= 64
              and C0 * KH * KW <= 160 and C0 <= 4)
    return CONV_NHWC16_SMALL == "all" or not direct


def conv_weight_nhwc16(w, C0, C1):
    """bf16 [Cout][K] weights for ainp_conv_gen_fwd_nhwc16, cached like
    conv_weight_kmajor (invalidated by in-place updates / reallocation)."""
    key = (w._version, C0, C1, w.data_ptr())
    ent = _WT16_CACHE.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == key:
        return ent[2]
    KK = w.shape[2] * w.shape[3]
    wt = torch.empty(w.shape[0], nhwc16_seg(C0, KK) + nhwc16_seg(C1, KK), device=w.device,
                     dtype=torch.bfloat16)
    _T.conv_weight_nhwc16(w, int(C0), int(C1), wt)
    wid = id(w)
    _WT16_CACHE[wid] = (weakref.ref(w, lambda _r, wid=wid: _WT16_CACHE.pop(wid, None)), key, wt)
    return wt


_NHWC_MEMO = None   # dict while an nhwc16_memo scope is active


class nhwc16_memo:
    """Scope in which to_nhwc16 reuses its result for an unchanged (x, mask)
    pair: PConvUNet converts each encoder output once for the next encoder
    conv and finds it again as the decoder's skip source.  The memo holds the
    sources, so their storage cannot be reused inside the scope; an in-place
    update bumps the tensor version and misses."""

    def __enter__(self):
        global _NHWC_MEMO
        self._prev = _NHWC_MEMO
        _NHWC_MEMO = {}
        return self

    def __exit__(self, *exc):
        global _NHWC_MEMO
        _NHWC_MEMO = self._prev
        return False


def to_nhwc16(x, m=None):
    """x [N,C,H,W] fp32 (x mask plane m) -> bf16 [N,H,W,C] (ainp_nchw_to_nhwc16)."""
    memo = _NHWC_MEMO
    key = None
    if memo is not None:
        key = (x.data_ptr(), tuple(x.shape), x._version,
               m.data_ptr() if m is not None else 0, m._version if m is not None else -1)
        hit = memo.get(key)
        if hit is not None:
            return hit[0]
    N, C, H, W = x.shape
    out = torch.empty(N, H, W, C, device=x.device, dtype=torch.bfloat16)
    _T.nchw_to_nhwc16(x, m, out)
    if memo is not None:
        memo[key] = (out, x, m)
    return out


def conv16_set_variant(v):
    """Main loop of the bf16 channel-last conv (ainp_conv16_set_variant): 0
    register-staged tiles, 1 LDS-DMA ring, 2 / 3 wide-tile ring of 4 / 8 waves
    (3, the default: Cout > 64, else 0); same sums in all, bit for bit.  Returns
    the previous variant (v outside 0..3 only queries)."""
    return int(_lib.lib.ainp_conv16_set_variant(int(v)))


def conv_gen(src0, w, *, src1=None, Hin=None, Win=None, stride=1, pad=0, bias=None, ratio=None,
             scale=None, act=ACT_NONE, slope=0.2, want_stats=False, crop=None, out=None,
             bf16=False, launcher=False, out16=False):
    """ainp_conv_gen_fwd.  src0/src1 = (x [N,C,Hs,Ws], mask plane [N,Hs,Ws] or None);
    the conv's input is cat(src0 nearest-resampled to (Hin, Win), src1) * masks.
    Returns (y [N,Cout,Ho,Wo] (or [N,crop_h,crop_w] for Cout=1 with crop), stats).
    out16 (bf16 channel-last route, inside an nhwc16_memo scope): the epilogue
    also writes y's bf16 channel-last copy (ainp_conv_gen_fwd_nhwc16_ex), which
    to_nhwc16(y) then returns -- for a next conv with no mask plane."""
    x0, m0 = src0
    _req(x0, "x0"); _req(w, "w")
    N, C0, H0, W0 = x0.shape
    x1 = m1 = None
    C1 = H1 = W1 = 0
    if src1 is not None:
        x1, m1 = src1
        _req(x1, "x1")
        _, C1, H1, W1 = x1.shape
    if Hin is None:
        Hin, Win = (H1, W1) if src1 is not None else (H0, W0)
    Cout, Cin, KH, KW = w.shape
    if Cin != C0 + C1:
        raise ValueError(f"conv_gen: weight expects {Cin} input channels, sources give {C0 + C1}")
    for m, (h, ww) in ((m0, (H0, W0)), (m1, (H1, W1))):
        if m is not None:
            _req(m, "mask")
            if m.numel() != N * h * ww:
                raise ValueError("conv_gen: mask plane must be [N, Hs, Ws] of its source")
    Ho, Wo = conv_out_size(Hin, KH, stride, pad), conv_out_size(Win, KW, stride, pad)
    ch, cw = (0, 0) if crop is None else crop
    if WORK_TRACE is not None and not launcher:
        flop = 2.0 * N * Cout * Cin * KH * KW * ((ch * cw) if (Cout == 1 and crop) else Ho * Wo)
        if bf16 and Cout > 1 and crop is None and _nhwc16_route(C0, C1, H0, W0, Hin, Win, KH, KW,
                                                                 Cout, want_stats):
            nm = ("conv_gen_nhwc16_wide_kernel<256" if Cout > 128 else
                  "conv_gen_nhwc16_wide_kernel<128" if Cout > 64 else "conv_gen_nhwc16_kernel<64")
        elif Cout == 1:
            # both Cout = 1 kernels: conv_cout1_partial_kernel and the batched-
            # tap conv_cout1_partial_b_kernel<KT, CG> (round 6)
            nm = "conv_cout1_partial"
        elif _direct_route(C0, C1, H0, W0, Hin, Win, KH, KW, Cout, want_stats):
            nm = "conv_gen_smallcin_kernel"
        else:
            # exact kernel names: a bare "conv_gen" would also match the nhwc16,
            # few-channel, wide and split-K epilogue rows of the step table
            nm = "conv_gen_x6_kernel" if not bf16 else "conv_gen_fwd_kernel"
        _work(nm, flop)
    if out is None:
        if Cout == 1 and crop is not None:
            out = torch.empty(N, ch, cw, device=x0.device, dtype=torch.float32)
        else:
            out = torch.empty(N, Cout, Ho, Wo, device=x0.device, dtype=torch.float32)
    stats = None
    if want_stats:
        parts = _lib.lib.ainp_conv_gen_stat_parts(N, Cin, KH, KW, Cout, Ho, Wo)
        stats = torch.empty(parts, 2, Cout, device=x0.device, dtype=torch.float64)
    for t, nm in ((bias, "bias"), (ratio, "ratio"), (scale, "scale")):
        if t is not None:
            _req(t, nm)
    ws = wt = None
    if bf16 and Cout > 1 and crop is None and _nhwc16_route(C0, C1, H0, W0, Hin, Win, KH, KW,
                                                             Cout, want_stats):
        nb = int(_lib.lib.ainp_conv_gen_workspace(N, Cin, KH, KW, Cout, Ho, Wo))
        if nb:
            ws = torch.empty(-(-nb // 4), device=x0.device)
        def src16(x, m, C):
            if C % 32:   # few channels: expanded per output pixel
                e = torch.empty(N * Ho * Wo, nhwc16_seg(C, KH * KW), device=x.device,
                                dtype=torch.bfloat16)
                _T.im2col_nhwc16(x, m, int(Hin), int(Win), int(KH), int(KW), int(stride),
                                 int(pad), e)
                return e
            return to_nhwc16(x, m)
        a16 = src16(x0, m0, C0)
        b16 = src16(x1, m1, C1) if src1 is not None else None
        wt16 = conv_weight_nhwc16(w, C0, C1)
        y16 = None
        if out16 and CONV_OUT16 and _NHWC_MEMO is not None:
            y16 = torch.empty(N, Ho, Wo, Cout, device=x0.device, dtype=torch.bfloat16)

        def launch():
            _T.conv_gen_fwd_nhwc16(a16, b16, wt16, int(Cout), int(KH), int(KW), bias, ratio,
                                   scale, out, stats, int(Hin), int(Win), int(stride), int(pad),
                                   int(act), float(slope), ws,
                                   [int(N), int(C0), int(H0), int(W0), int(C1), int(H1), int(W1)],
                                   y16)
        if launcher:   # bench / profiling: the conv kernel alone on prepared operands
            launch.out, launch.stats, launch.y16 = out, stats, y16
            return launch
        launch()
        if y16 is not None:
            _NHWC_MEMO[(out.data_ptr(), tuple(out.shape), out._version, 0, -1)] = (y16, out, None)
        return out, stats
    if Cout == 1:
        nb = int(_lib.lib.ainp_conv_gen_workspace(N, Cin, KH, KW, Cout, ch or Ho, cw or Wo))
    else:
        nb = int(_lib.lib.ainp_conv_gen_workspace(N, Cin, KH, KW, Cout, Ho, Wo))
        wt = conv_weight_kmajor(w, C0, C1)
    if nb:
        ws = torch.empty(-(-nb // 4), device=x0.device)
    y16 = None
    if (out16 and bf16 and CONV_OUT16 and OUT16_DIRECT and _NHWC_MEMO is not None
            and Cout % 8 == 0 and _direct_route(C0, C1, H0, W0, Hin, Win, KH, KW, Cout, want_stats)):
        # the few-input-channel kernel writes the next conv's channel-last source
        y16 = torch.empty(N, Ho, Wo, Cout, device=x0.device, dtype=torch.bfloat16)
    _T.conv_gen_fwd(x0, m0, x1, m1, w, wt, bias, ratio, scale, out, stats, int(Hin), int(Win),
                    int(stride), int(pad), int(act), float(slope), int(ch), int(cw),
                    CONV_BF16 if bf16 else 0, ws, y16)
    if y16 is not None:
        _NHWC_MEMO[(out.data_ptr(), tuple(out.shape), out._version, 0, -1)] = (y16, out, None)
    return out, stats


def pconv_mask(src0, src1, N, Hin, Win, k, stride, pad, want_ratio=True, want_mask=True,
               winsize=0.0):
    """ainp_pconv_mask: src = (mask plane [N,Hs,Ws], channels).  Returns
    (ratio [N,Ho,Wo], newmask [N,Ho,Wo])."""
    m0, C0 = src0
    _req(m0, "m0")
    H0, W0 = m0.shape[-2:]
    m1, C1 = src1 if src1 is not None else (None, 0)
    H1, W1 = (m1.shape[-2:] if m1 is not None else (0, 0))
    Ho, Wo = conv_out_size(Hin, k, stride, pad), conv_out_size(Win, k, stride, pad)
    ratio = torch.empty(N, Ho, Wo, device=m0.device) if want_ratio else None
    newm = torch.empty(N, Ho, Wo, device=m0.device) if want_mask else None
    _T.pconv_mask(m0, int(C0), m1, int(C1), int(N), int(Hin), int(Win), int(k), int(stride),
                  int(pad), float(winsize), ratio, newm)
    return ratio, newm


def gan_pad_input(x, m, Hp, Wp):
    _req(x, "x"); _req(m, "mask")
    N, _, H, W = x.shape
    xp = torch.empty(N, Hp, Wp, device=x.device)
    mp = torch.empty(N, Hp, Wp, device=x.device)
    _T.gan_pad_input(x, m, xp, mp)
    return xp, mp


def affine_act_(y, scale, shift, act, slope=0.2):
    _req(y, "y")
    N, C = y.shape[:2]
    _T.affine_act(y, scale, shift, int(act), float(slope))
    return y


def affine_act_nhwc16_(y, scale, shift, act, slope=0.2, m=None, keep_y=True):
    """affine_act_ in place and, in the same pass, the bf16 channel-last copy of
    the result times the mask plane m (ainp_affine_act_nhwc16); inside an
    nhwc16_memo scope the copy is what to_nhwc16(y, m) returns afterwards.
    keep_y=False: y keeps its input values (AINP_AFFINE_NO_Y) -- only for
    callers whose every consumer reads the copy."""
    _req(y, "y")
    N, C, H, W = y.shape
    out = torch.empty(N, H, W, C, device=y.device, dtype=torch.bfloat16)
    _T.affine_act_nhwc16(y, scale, shift, int(act), float(slope), m, out, bool(keep_y))
    memo = _NHWC_MEMO
    if memo is not None:
        key = (y.data_ptr(), tuple(y.shape), y._version,
               m.data_ptr() if m is not None else 0, m._version if m is not None else -1)
        memo[key] = (out, y, m)
    return y, out


def maxpool2(x, out16=False):
    """2x2 / stride-2 max-pool.  out16 (inside an nhwc16_memo scope): the same
    pass writes y's bf16 channel-last copy (ainp_maxpool2_nhwc16), which
    to_nhwc16(y) then returns -- the next VGG19 conv's source."""
    _req(x, "x")
    N, C, H, W = x.shape
    y = torch.empty(N, C, H // 2, W // 2, device=x.device)
    y16 = None
    if out16 and CONV_OUT16 and OUT16_DIRECT and _NHWC_MEMO is not None:
        y16 = torch.empty(N, H // 2, W // 2, C, device=x.device, dtype=torch.bfloat16)
    _T.maxpool2(x, y, y16)
    if y16 is not None:
        _NHWC_MEMO[(y.data_ptr(), tuple(y.shape), y._version, 0, -1)] = (y16, y, None)
    return y


_RED_WS: dict = {}


def _reduce_ws(device):
    key = str(device)
    ws = _RED_WS.get(key)
    if ws is None:
        ws = torch.empty(-(-int(_lib.lib.ainp_reduce_workspace()) // 8), device=device,
                         dtype=torch.float64)
        _RED_WS[key] = ws
    return ws


def absdiff_mean(a, b, out=None):
    """mean |a - b| as a float64 device scalar (nn.L1Loss()); out: a float64
    0-d tensor (e.g. one element of a loss vector) to write it to."""
    _req(a, "a"); _req(b, "b")
    assert a.numel() == b.numel()
    if out is None:
        out = torch.empty((), device=a.device, dtype=torch.float64)
    _T.absdiff_mean(a, b, _reduce_ws(a.device), out)
    return out


def bce_logits(x, target, want_grad=False, grad_scale=None):
    """mean BCEWithLogits(x, const target) (float64 scalar), optional
    gradient grad_scale * (sigmoid(x) - target) (default scale 1/numel)."""
    _req(x, "logits")
    n = x.numel()
    out = torch.empty((), device=x.device, dtype=torch.float64)
    grad = torch.empty_like(x) if want_grad else None
    gs = 1.0 / n if grad_scale is None else grad_scale
    _T.bce_logits(x, float(target), grad, float(gs), _reduce_ws(x.device), out)
    return out, grad


def gan_recon_losses(g, o, m):
    """(Lv, Lh, Lw) of calculate_losses as a float64 [3] device tensor."""
    for t, nm in ((g, "generated"), (o, "original"), (m, "mask")):
        _req(t, nm)
    out = torch.empty(3, device=g.device, dtype=torch.float64)
    _T.gan_recon_losses(g, o, m, _reduce_ws(g.device), out)
    return out


def gan_recon_sums(g, o, m):
    """Raw fp64 sums [sum|(g-o)m|, sum m, sum|(g-o)(1-m)|, sum(1-m), sum|g-o||o|]
    behind gan_recon_losses (ainp_gan_recon_sums), for a SUM all-reduce."""
    for t, nm in ((g, "generated"), (o, "original"), (m, "mask")):
        _req(t, nm)
    out = torch.empty(5, device=g.device, dtype=torch.float64)
    _T.gan_recon_sums(g, o, m, _reduce_ws(g.device), out)
    return out


def gan_recon_from_sums(sums, n):
    """(Lv, Lh, Lw) from the (all-reduced) sums with the kernel's rounding:
    fp32 sums / (fp32 sum + 1e-8), Lw = fp32(sum / n)."""
    f = sums.to(torch.float32)
    lv = f[0] / (f[1] + 1e-8)
    lh = f[2] / (f[3] + 1e-8)
    lw = (sums[4] / float(n)).to(torch.float32)
    return torch.stack([lv, lh, lw]).to(torch.float64)


def sn_power(weights, us, vs, update=True, eps=1e-12):
    """Spectral norm for several layers: power iteration (in place on us/vs)
    when update, then inv_sigma [nl] (device float32)."""
    nl = len(weights)
    hs = [w.shape[0] for w in weights]
    wds = [w[0].numel() for w in weights]
    maxdim = max(hs + wds)
    dev = weights[0].device
    ws = torch.empty(-(-int(_lib.lib.ainp_sn_workspace(nl, maxdim)) // 4), device=dev)
    inv = torch.empty(nl, device=dev)
    _T.sn_power(list(weights), list(us), list(vs), float(eps), ws, inv, bool(update))
    return inv


def sn_weight_grad(G, w_orig, u, v, inv_sigma, with_bias=False, ws=None):
    """G [h, ldg] (ldg >= wd, +1 with the bias column) -> (dW_orig, dbias or None).
    ws: a reduction workspace (default: the device's shared one; a side stream
    passes its own)."""
    _req(G, "G"); _req(w_orig, "w_orig")
    out = torch.empty_like(w_orig)
    h = w_orig.shape[0]
    ob = torch.empty(h, device=G.device) if with_bias else None
    _T.sn_weight_grad(G, w_orig, u, v, inv_sigma, _reduce_ws(G.device) if ws is None else ws,
                      out, ob)
    return out, ob


def im2col(x, k, stride, pad, ones_row=False, ldp=None):
    """[N, C*k*k (+1), ldp] (ldp >= Ho*Wo; columns past Ho*Wo are zero)."""
    _req(x, "x")
    N, C, H, W = x.shape
    Ho, Wo = conv_out_size(H, k, stride, pad), conv_out_size(W, k, stride, pad)
    ldp = Ho * Wo if ldp is None else int(ldp)
    col = torch.empty(N, C * k * k + int(ones_row), ldp, device=x.device)
    _T.im2col_ld(x, int(k), int(stride), int(pad), bool(ones_row), ldp, col)
    return col


def largest_divisor_at_most(n, cap):
    for s in range(max(1, min(n, cap)), 0, -1):
        if n % s == 0:
            return s
    return 1


def gemm_batched_splitk(M, N, Kd, As, sam, sak, Bs, sbk, sbn, out, *, alpha=1.0,
                        per_batch_out=False, target_blocks=768, min_k=256, bf16=False):
    """C = alpha * sum_b A_b B_b (or C_b = alpha * A_b B_b when per_batch_out),
    with the long reduction Kd split into S strided chunks per batch so the
    small-M/N products still fill the chip.  A_b / B_b: tensors whose element
    (m, k) / (k, n) sits at m*sam + k*sak / k*sbk + n*sbn (k-chunks advance by
    chunk*sak / chunk*sbk).  Partial products go to slabs summed in fixed order."""
    nb = len(As)
    tiles = -(-M // 128) * -(-N // 128)
    want = max(1, min(Kd // min_k, target_blocks // max(1, tiles * nb)))
    # chunks of a multiple of 4 when Kd allows (16-byte aligned chunk starts)
    q = 4 if Kd % 4 == 0 else 1
    S = largest_divisor_at_most(Kd // q, want)
    kc = Kd // S
    # slab layout [S, nb, M, N]: the per-batch results are one sum over S
    # slabs of nb*M*N, the batch total one sum over S*nb slabs of M*N
    slabs = torch.empty(S, nb, M, N, device=out.device, dtype=torch.float32)
    for g0 in range(0, nb, 8):
        g1 = min(nb, g0 + 8)
        gemm(M, N, kc, As[g0:g1], sam, sak, Bs[g0:g1], sbk, sbn,
             [slabs[0, i] for i in range(g0, g1)], N, 1, alpha=alpha, strideA=kc * sak,
             strideB=kc * sbk, strideC=nb * M * N, nstrided=S, bf16=bf16)
    if per_batch_out:
        sum_slabs(slabs, S, out=out.reshape(-1))
    else:
        sum_slabs(slabs, nb * S, out=out.reshape(-1))
    return out


def d_prep16(g, nslab, y, slope, N, C, P, ldA, want_gT=True):
    """ainp_d_prep16: sum of nslab slabs of g [N, C, P] (x LeakyReLU'(y)) ->
    (gA bf16 [C, ldA] pixel-contiguous, gT bf16 [N*P, C] or None)."""
    gA = torch.empty(C, ldA, device=g.device, dtype=torch.bfloat16)
    gT = torch.empty(N * P, C, device=g.device, dtype=torch.bfloat16) if want_gT else None
    _T.d_prep16(g, int(nslab), y, float(slope), int(N), int(C), int(P), gA, gT)
    return gA, gT


def wgrad_cout1(x, g, nslab, y, slope, k, stride, pad):
    """ainp_wgrad_cout1: [dW | db] [1, Cin*k*k + 1] of a Cout = 1 conv from the
    fp32 input x [N, Cin, H, W] and nslab slabs of g [N, 1, Ho, Wo]."""
    _req(x, "x"); _req(g, "g")
    _work("wgrad_cout1_kernel", 2.0 * x.shape[0] * g.shape[-2] * g.shape[-1] * x.shape[1] * k * k)
    gw = torch.empty(1, x.shape[1] * k * k + 1, device=x.device)
    ws = torch.empty(_lib.lib.ainp_wgrad_cout1_workspace(x.shape[1], k) // 4, device=x.device)
    _T.wgrad_cout1(x, g, int(nslab), y, float(slope), int(k), int(stride), int(pad), gw, ws)
    return gw


def im2col16(x, k, stride, pad, ldA, ones_row=True):
    """ainp_im2col16: bf16 [C*k*k (+1), ldA] columns, all images' pixels in a row."""
    C = x.shape[1]
    col = torch.empty(C * k * k + int(ones_row), ldA, device=x.device, dtype=torch.bfloat16)
    _T.im2col16(x, int(k), int(stride), int(pad), bool(ones_row), col)
    return col


_WD16_CACHE: dict = {}


def dgrad16_weight(w, stride, pad):
    """ainp_dgrad16_weight: bf16 [s*s, Cin, Kc] parity-class weights; reused
    while w's storage and version are unchanged (the discriminator's real and
    fake backward passes of one step share them)."""
    key = (w.data_ptr(), w._version, tuple(w.shape), int(stride), int(pad), w.device)
    hit = _WD16_CACHE.get(key)
    if hit is not None:
        return hit[1]
    Cout, Cin, k, _ = w.shape
    nt = k // stride
    wd = torch.empty(stride * stride, Cin, nhwc16_seg(Cout, nt * nt), device=w.device,
                     dtype=torch.bfloat16)
    _T.dgrad16_weight(w, int(stride), int(pad), wd)
    if len(_WD16_CACHE) >= 64:
        _WD16_CACHE.clear()
    # the entry holds w: its storage cannot be freed and its address reused by
    # another tensor while the entry exists
    _WD16_CACHE[key] = (w, wd)
    return wd


def dgrad16_nsplit(N, Cin, H, W, k, stride, Cout):
    """Split-K count of ainp_dgrad16: ~768 workgroups, >= 8 K-tiles a split."""
    BM = 128 if Cin > 64 else 64
    tiles = -(-(N * -(-H // stride) * -(-W // stride)) // (16384 // BM))
    blocks = tiles * -(-Cin // BM) * stride * stride
    nkt = nhwc16_seg(Cout, (k // stride) ** 2) // 32
    if blocks >= 512 or nkt < 16:
        return 1
    return max(1, min(-(-768 // blocks), nkt // 8))


def dgrad16(gT, wd, Cin, H, W, k, stride, pad, scale=None, nsplit=1):
    """ainp_dgrad16: gT bf16 [N, Ho, Wo, Cout] -> dx fp32 [nsplit, N, Cin, H, W]
    (split-K partial slabs; nsplit == 1: the data gradient itself)."""
    N = gT.shape[0]
    _work("dgrad16_kernel", 2.0 * gT.numel() * Cin * k * k)
    out = torch.empty(nsplit, N, Cin, H, W, device=gT.device, dtype=torch.float32)
    _T.dgrad16(gT, wd, int(Cin), int(H), int(W), int(k), int(stride), int(pad), scale, out,
               int(nsplit))
    return out


def wgrad16_nhwc(gA, x16, k, stride, pad, max_split=512):
    """ainp_wgrad16_nhwc: [dW | db] [Cout, Cin*k*k + 1] from gA bf16 [Cout, ldA]
    and the layer input's channel-last bf16 copy x16 [N, H, W, Cin] -- what
    gemm_bf16nt_splitk(gA, im2col16(x, ...), ldA) gives, bit for bit."""
    Cout, ldA = gA.shape[0], gA.shape[1]
    Cin = x16.shape[3]
    Ncol = Cin * k * k + 1
    S = _splitk_bf16(Cout, Ncol, ldA, max_split=max_split)
    kc = -(-ldA // S // 64) * 64 if S > 1 else ldA
    G = torch.empty(S, Cout, Ncol, device=gA.device, dtype=torch.float32)
    _T.wgrad16_nhwc(gA, x16, int(k), int(stride), int(pad), G, int(S), int(kc))
    if S == 1:
        return G[0]
    out = torch.empty(Cout, Ncol, device=gA.device, dtype=torch.float32)
    sum_slabs(G, S, out=out.view(-1))
    return out


def nhwc16_memo_get(x):
    """The channel-last bf16 copy of x (no mask plane) held by the active
    nhwc16_memo scope, or None."""
    memo = _NHWC_MEMO
    if memo is None:
        return None
    hit = memo.get((x.data_ptr(), tuple(x.shape), x._version, 0, -1))
    return hit[0] if hit is not None else None


def dgrad16_prep(gT, wd, Cin, H, W, k, stride, pad, y, slope, ldA, scale=None, want_gT=True):
    """ainp_dgrad16_prep: dgrad16 (nsplit 1) then d_prep16 of its dx in one
    pass -> (gA bf16 [Cin, ldA], gT bf16 [N*H*W, Cin] or None), the lower
    layer's gradient operands, bit for bit those of the two calls."""
    N = gT.shape[0]
    _work("dgrad16_kernel", 2.0 * gT.numel() * Cin * k * k)
    gA = torch.empty(Cin, ldA, device=gT.device, dtype=torch.bfloat16)
    gTo = (torch.empty(N * H * W, Cin, device=gT.device, dtype=torch.bfloat16)
           if want_gT else None)
    _T.dgrad16_prep(gT, wd, int(Cin), int(H), int(W), int(k), int(stride), int(pad), scale, y,
                    float(slope), gA, gTo)
    return gA, gTo


def col2im(dcol, N, C, H, W, k, stride, pad):
    """dcol [N, C*k*k, ldp] (ldp >= Ho*Wo) -> dx [N, C, H, W]."""
    _req(dcol, "dcol")
    dx = torch.empty(N, C, H, W, device=dcol.device)
    _T.col2im_ld(dcol, int(k), int(stride), int(pad), dx)
    return dx


def leaky_bwd(g, y, slope=0.2, ldo=None):
    """LeakyReLU backward; with ldo, g/y [N, C, H, W] -> [N, C, ldo] rows of
    H*W zero-padded to ldo."""
    _req(g, "g"); _req(y, "y")
    if ldo is None:
        out = torch.empty_like(g)
        _T.leaky_bwd(g, y, float(slope), out)
        return out
    N, C = g.shape[:2]
    P = g.numel() // (N * C)
    out = torch.empty(N, C, int(ldo), device=g.device, dtype=torch.float32)
    _T.leaky_bwd_ld(g, y, N * C, float(slope), int(ldo), out)
    return out


def aa_bilinear_weights(in_size, out_size, start, count):
    """Separable weights of torch's antialiased bilinear resize
    (aten/src/ATen/native/cpu/UpSampleKernel.cpp, _compute_indices_min_size_weights_aa,
    align_corners=False) for output indices [start, start+count): returns
    (first input index [count] int32, taps [count] int32, weights [count][max_taps] f32)."""
    scale = np.float32(in_size) / np.float32(out_size)
    support = np.float32(scale) if scale >= 1.0 else np.float32(1.0)
    invscale = np.float32(1.0) / scale if scale >= 1.0 else np.float32(1.0)
    x0s, ns, ws = [], [], []
    for i in range(start, start + count):
        center = np.float32(scale * np.float32(i + 0.5))
        xmin = max(int(center - support + np.float32(0.5)), 0)
        xsize = min(int(center + support + np.float32(0.5)), in_size) - xmin
        w = []
        for j in range(xsize):
            x = np.float32((j + xmin - center + np.float32(0.5)) * invscale)
            w.append(np.float32(1.0) - abs(x) if abs(x) < 1.0 else np.float32(0.0))
        w = np.array(w, dtype=np.float32)
        tot = w.sum(dtype=np.float32)
        if tot != 0:
            w = w / tot
        x0s.append(xmin); ns.append(xsize); ws.append(w)
    taps = max(ns)
    W = np.zeros((count, taps), np.float32)
    for i, w in enumerate(ws):
        W[i, :len(w)] = w
    return np.array(x0s, np.int32), np.array(ns, np.int32), W


def vgg_target_max(x):
    """Batch max of clamp(x, 0) as its float bits in an int32 [1] device tensor
    (ainp_vgg_target_max); non-negative floats order like their bits, so a MAX
    all-reduce of this tensor is the global batch max (loss.py:78)."""
    _req(x, "x")
    mx = torch.empty(1, device=x.device, dtype=torch.int32)
    _T.vgg_target_max(x, mx)
    return mx


def vgg_prep(x, generated, tables, S=224, target_max=None):
    """ainp_vgg_prep: x [N,1,H,W] -> [N,3,S,S] normalised VGG input.
    target_max: precomputed (e.g. all-reduced) vgg_target_max for a target."""
    _req(x, "x")
    N, _, H, W = x.shape
    ry0, rn, rw, cx0, cn, cw = tables
    out = torch.empty(N, 3, S, S, device=x.device)
    if target_max is not None and not generated:
        mx, mode = target_max, 2
    else:
        mx, mode = torch.empty(1, device=x.device, dtype=torch.int32), int(bool(generated))
    _T.vgg_prep(x, mode, mx, ry0, rn, rw, cx0, cn, cw, int(S), out)
    return out


def mul(a, b):
    _req(a, "a"); _req(b, "b")
    out = torch.empty_like(a)
    _T.mul(a, b, out)
    return out


def channel_sum(m):
    _req(m, "mask")
    N, C, H, W = m.shape
    out = torch.empty(N, H, W, device=m.device)
    _T.channel_sum(m, out)
    return out


# ============================================================ generator backward
# (csrc/gan_bwd.hip; the opt-in fix_generator_grad path of ainp.gan)
def affine_leaky_out(y, scale, shift, slope=0.2):
    """LeakyReLU(y * scale[c] + shift[c]) into a new tensor (y kept)."""
    _req(y, "y")
    out = torch.empty_like(y)
    _T.affine_leaky_out(y, scale, shift, float(slope), out)
    return out


def pconv_src_materialize(src0, src1, Hin, Win):
    """cat(nearest(x0) * m0, x1 * m1) [N, C0+C1, Hin, Win]: the input a
    PartialConv2d convolves (src = (x, mask plane or None))."""
    x0, m0 = src0
    _req(x0, "x0")
    x1, m1 = src1 if src1 is not None else (None, None)
    C1 = x1.shape[1] if x1 is not None else 0
    out = torch.empty(x0.shape[0], x0.shape[1] + C1, int(Hin), int(Win), device=x0.device)
    _T.pconv_src_materialize(x0, m0, x1, m1, int(Hin), int(Win), out)
    return out


def pconv_src_grad(dxin, c_off, ms, dxs, accumulate):
    """dxs (+)= ms * block-sum of dxin[:, c_off:c_off+C] (the gradient of one
    PartialConv2d source from that of the materialised input)."""
    _req(dxin, "dxin"); _req(dxs, "dxs")
    _T.pconv_src_grad(dxin, int(c_off), ms, bool(accumulate), dxs)
    return dxs


def gen_act_bwd(g, a, act, slope, ratio, H, W, ldo, want_gz=True):
    """(gz [N,C,H*W] = g * act'(a) on the conv grid, gc [N,C,ldo] = gz * ratio)."""
    _req(g, "g")
    N, C = g.shape[:2]
    gz = torch.empty(N, C, H * W, device=g.device) if want_gz else None
    gc = torch.empty(N, C, int(ldo), device=g.device)
    _T.gen_act_bwd(g, a, int(act), float(slope), ratio, int(H), int(W), int(ldo), gz, gc)
    return gz, gc


def bn_act_bwd_reduce(ga, y, scale, shift, save, slope=0.2, count=None):
    """[sum g' | sum g' xhat] (f64; + the element count when `count` is given,
    for a SyncBN all-reduce, see bn_stats_reduce)."""
    _req(ga, "ga"); _req(y, "y")
    N, C = y.shape[:2]
    P = y.shape[2] * y.shape[3]
    ws = torch.empty(-(-int(_lib.lib.ainp_bn_act_bwd_workspace(N, C, P)) // 8),
                     device=y.device, dtype=torch.float64)
    sums = torch.empty(2 * C + (1 if count is not None else 0), device=y.device,
                       dtype=torch.float64)
    _T.bn_act_bwd_reduce(ga, y, scale, shift, save, float(slope), ws, sums)
    if count is not None:
        sums[2 * C:].fill_(float(count))
    return sums


def bn_act_bwd_apply(ga, y, scale, shift, save, gamma, sums, count, slope, ratio, ldo):
    """(gc [N, C, ldo] = BN(+LeakyReLU) data gradient x ratio, dgamma, dbeta)."""
    N, C = y.shape[:2]
    gc = torch.empty(N, C, int(ldo), device=y.device)
    dgamma = torch.empty(C, device=y.device) if gamma is not None else None
    dbeta = torch.empty(C, device=y.device)
    _T.bn_act_bwd_apply(ga, y, scale, shift, save, gamma, sums, int(count), float(slope), ratio,
                        int(ldo), gc, dgamma, dbeta)
    return gc, dgamma, dbeta


def maxpool2_bwd(g, x):
    _req(g, "g"); _req(x, "x")
    gx = torch.empty_like(x)
    _T.maxpool2_bwd(g, x, gx)
    return gx


def vgg_prep_bwd(g, x, tables, S=224):
    """Gradient of vgg_prep(x, generated=True) w.r.t. x [N,1,H,W]."""
    _req(g, "g"); _req(x, "x")
    N, _, H, W = x.shape
    ry0, rn, rw, cx0, cn, cw = tables
    ws = torch.empty(-(-int(_lib.lib.ainp_vgg_prep_bwd_workspace(N, W, S)) // 4),
                     device=x.device)
    gx = torch.empty_like(x)
    _T.vgg_prep_bwd(g, x, ry0, rn, rw, cx0, cn, cw, int(S), ws, gx)
    return gx


def absdiff_grad(a, b, gscale=None, scale=1.0, out=None, accumulate=False):
    """nn.L1Loss backward: out (+)= gscale * scale * sign(a - b)."""
    _req(a, "a"); _req(b, "b")
    if out is None:
        out = torch.empty_like(a)
        accumulate = False
    _T.absdiff_grad(a, b, gscale, float(scale), bool(accumulate), out)
    return out


def gram_sign_sym(Ga, Gb, gscale=None, scale=1.0):
    out = torch.empty_like(Ga)
    _T.gram_sign_sym(Ga, Gb, gscale, float(scale), out)
    return out


def gan_recon_bwd(g, o, m, sums5, gout3, n_total):
    """d(Lv, Lh, Lw) . gout3 / d generated (ainp_gan_recon_bwd)."""
    out = torch.empty_like(g)
    _T.gan_recon_bwd(g, o, m, sums5, gout3, float(n_total), out)
    return out


def conv_weight_flip_t(w):
    """w [Cout, Cin, K, K] -> [Cin, Cout, K, K] spatially flipped."""
    _req(w, "w")
    Cout, Cin, K, _ = w.shape
    out = torch.empty(Cin, Cout, K, K, device=w.device)
    _T.conv_weight_flip_t(w, out)
    return out


# ============================================================ ISTFT / Griffin-Lim
IST_C64, IST_C128, IST_MAG_ANGLES, IST_MAG_PHASE = 0, 1, 2, 3


def istft(spec=None, *, mag=None, angles=None, phase=None, n_fft=None, hop_length=512,
          win_length=None, window="hann", center=True):
    """librosa>=0.10 istft on the GPU (ainp_istft).  Either a complex spectrum
    spec [..., F, T] (complex64 -> float32, complex128 -> float64), or
    mag [..., F, T] float32 with unit complex64 `angles` or float32 `phase`.
    Returns [..., hop*(T-1)] (center) or [..., n_fft + hop*(T-1)]."""
    if spec is not None:
        _req(spec, "spec", dtype=None)
        if spec.dtype not in (torch.complex64, torch.complex128):
            raise TypeError("spec must be complex64 or complex128")
        lead, (F, T) = spec.shape[:-2], spec.shape[-2:]
        mode = IST_C64 if spec.dtype == torch.complex64 else IST_C128
        in0, in1 = spec.contiguous(), None
        odt = torch.float32 if mode == IST_C64 else torch.float64
    else:
        _req(mag, "mag")
        lead, (F, T) = mag.shape[:-2], mag.shape[-2:]
        if angles is not None:
            _req(angles, "angles", dtype=torch.complex64)
            mode, in1 = IST_MAG_ANGLES, angles
        else:
            _req(phase, "phase")
            mode, in1 = IST_MAG_PHASE, phase
        in0 = mag
        odt = torch.float32
    n_fft = 2 * (F - 1) if n_fft is None else n_fft
    win_length = n_fft if win_length is None else win_length
    nsig = int(np.prod(lead)) if len(lead) else 1
    dev = in0.device
    w = _device_window(window, win_length, n_fft, dev)
    full = n_fft + hop_length * (T - 1)
    out_len = full - 2 * (n_fft // 2) if center else full
    out = torch.empty(*lead, out_len, device=dev, dtype=odt)
    ws = torch.empty(-(-int(_lib.lib.ainp_istft_workspace(nsig, T, n_fft)) // 8), device=dev,
                     dtype=torch.float64)
    _T.istft(in0, in1, mode, F, T, w, int(n_fft), int(hop_length), bool(center), ws, out)
    return out


def griffinlim(S, n_iter=32, hop_length=None, win_length=None, n_fft=None, window="hann",
               center=True, momentum=0.99, random_state=None, init_angles=None, init="numpy"):
    """librosa>=0.10 griffinlim (init='random') on the GPU: S [F, T] or [B, F, T]
    float32 magnitudes.  Initial phases: init_angles (complex64, any device),
    else init="numpy" draws them exactly as librosa does
    (np.random.default_rng(random_state).random(S.shape), on the host, then one
    copy), or init="device" draws them on the GPU (torch.rand with a
    torch.Generator seeded by random_state: same distribution, different
    stream -- no host work).  Each iteration = ainp_istft (S * angles) + the
    STFT with the phase update fused into its write-out (ainp_gl_stft_update,
    n_fft = 512 center float32; ainp_stft + ainp_gl_update otherwise)."""
    _req(S, "S")
    F, T = S.shape[-2:]
    n_fft = 2 * (F - 1) if n_fft is None else n_fft
    win_length = n_fft if win_length is None else win_length
    hop_length = win_length // 4 if hop_length is None else hop_length
    if momentum > 1:
        raise ValueError("momentum > 1 is not a stable algorithm (librosa)")
    if momentum < 0:
        raise ValueError("momentum must be non-negative")
    if init_angles is None:
        if init == "device":
            gen = torch.Generator(device=S.device)
            gen.manual_seed(0 if random_state is None else int(random_state))
            ph = (2 * np.pi) * torch.rand(tuple(S.shape), device=S.device, generator=gen,
                                          dtype=torch.float64)
            init_angles = torch.polar(torch.ones_like(ph), ph).to(torch.complex64)
        elif init == "numpy":
            rng = np.random.default_rng(seed=random_state)
            ph = 2 * np.pi * rng.random(size=tuple(S.shape))
            init_angles = torch.from_numpy((np.cos(ph) + 1j * np.sin(ph)).astype(np.complex64))
        else:
            raise ValueError("init must be 'numpy' or 'device'")
    angles = init_angles.to(S.device, torch.complex64).contiguous().clone()
    tprev = torch.empty_like(angles)
    fused = n_fft == 512 and center and window == "hann"
    w = _device_window(window, win_length, n_fft, S.device) if fused else None
    nsig = int(np.prod(S.shape[:-2])) if S.dim() > 2 else 1
    for it in range(n_iter):
        inv = istft(mag=S, angles=angles, n_fft=n_fft, hop_length=hop_length,
                    win_length=win_length, window=window, center=center)
        if fused:
            _T.gl_stft_update(inv.reshape(nsig, -1), w, int(hop_length), T, tprev, angles,
                              float(momentum), it == 0)
        else:
            rebuilt = stft(inv, n_fft, hop_length, win_length, window, center)
            _T.gl_update(rebuilt, tprev, angles, float(momentum), it == 0)
    return istft(mag=S, angles=angles, n_fft=n_fft, hop_length=hop_length,
                 win_length=win_length, window=window, center=center)
