"""GAN inpainting path on the MI355X kernels.

Modules keep the reference's constructors, submodule trees, state_dict keys
and default-init RNG draw order (models/GAN/networks.py, models/GAN/loss.py),
so checkpoints move between the two unchanged; only the arithmetic moves onto
libainp (ainp.ops):

  PartialConv2d / EncoderBlock / DecoderBlock  networks.py:10-168
  PConvUNet       networks.py:173-345  under torch.no_grad (the reference
                  loop) the forward-only path; with autograd on
                  (fix_generator_grad) _PConvUNetFn adds the generator
                  backward (csrc/gan_bwd.hip).  Every PartialConv2d is ONE
                  implicit-GEMM launch whose gather reads the upsampled decoder
                  input and the skip directly (no torch.cat / nn.Upsample
                  tensors) times their 0/1 mask planes, plus one mask-count
                  launch; BatchNorm2d statistics come from the conv epilogue.
  Discriminator   networks.py:352-409  spectral norm (one power iteration per
                  train-mode forward, torch.nn.utils.spectral_norm semantics),
                  forward = conv_gen with 1/sigma, bias and LeakyReLU fused;
                  backward = im2col + MFMA GEMMs + the spectral-norm weight-grad
                  correction.
  VGGLoss         loss.py:6-131  VGG19.features[0..30] (frozen); the input
                  gradient of the generated batch under autograd (_VGGLossFn).
  calculate_losses train.py:33-88.
"""
from __future__ import annotations

import os
import re
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch.nn.utils import spectral_norm

from . import ops

SLOPE = 0.2


def _need_cuda(t, what):
    if t.device.type != "cuda":
        raise RuntimeError(f"ainp {what} runs on the MI355X kernels only; move it to a GPU")


_NBT_PENDING = None   # list while a _nbt_batch scope is active


class _nbt_batch:
    """Scope in which the BatchNorm layers' num_batches_tracked += 1 are
    collected and applied by one multi-tensor add at exit (the U-Net's 13
    BatchNorms: one launch instead of 13 single-element kernels)."""

    def __enter__(self):
        global _NBT_PENDING
        self._prev = _NBT_PENDING
        if self._prev is None:
            _NBT_PENDING = []
        return self

    def __exit__(self, *exc):
        global _NBT_PENDING
        if self._prev is None:
            pend, _NBT_PENDING = _NBT_PENDING, None
            if pend:
                torch._foreach_add_(pend, 1)
        return False


def _bn_affine(bn: nn.BatchNorm2d, stats, count, C, want_save=False):
    """BatchNorm2d train (batch stats + running update) or eval -> (scale, shift)
    (+ save = [mean | rstd] of the batch with want_save, for the backward).
    A data-parallel trainer sets `bn.ainp_comm`: the (sum, sum of squares)
    are then all-reduced (SyncBN), so every rank normalises with the statistics
    of the global batch, as the single-process reference does."""
    if bn.training or not bn.track_running_stats:
        comm = getattr(bn, "ainp_comm", None)
        rm = bn.running_mean if bn.track_running_stats else None
        rv = bn.running_var if bn.track_running_stats else None
        mom = bn.momentum if bn.momentum is not None else 0.1
        if comm is not None and comm.world_size > 1:
            # the local count rides in sums[2C]: uneven shards get the true global count
            sums = comm.allreduce_sum_(ops.bn_stats_reduce(stats, C, count=count))
            sc, sh, save = ops.bn_finalize(sums, 0, bn.weight, bn.bias, rm, rv, mom, bn.eps)
        else:
            # one launch: partials -> sums -> scale / shift / running statistics
            sc, sh, save = ops.bn_reduce_finalize(stats, C, count, bn.weight, bn.bias, rm, rv,
                                                  mom, bn.eps)
        if bn.track_running_stats:
            if _NBT_PENDING is not None:
                _NBT_PENDING.append(bn.num_batches_tracked)
            else:
                bn.num_batches_tracked.add_(1)
        return (sc, sh, save) if want_save else (sc, sh)
    sc, sh = ops.bn_eval_affine(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps)
    if want_save:
        # eval mode under autograd: the running statistics are constants
        # (ainp_bn_act_bwd_apply count = -1); [mean | rstd] for xhat
        save = torch.cat([bn.running_mean.float(),
                          torch.rsqrt(bn.running_var.float() + bn.eps)])
        return sc, sh, save
    return sc, sh


# ------------------------------------------------------------ partial conv
class PartialConv2d(nn.Module):
    """networks.py:10-106 (multi_channel=False)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, multi_channel=False):
        super().__init__()
        if dilation != 1 or groups != 1 or multi_channel:
            raise NotImplementedError("the reference only uses dilation=1, groups=1, "
                                      "multi_channel=False")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.dilation, self.groups, self.multi_channel = dilation, groups, multi_channel
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, dilation,
                              groups, bias=False)
        self.mask_kernel = torch.ones(1, in_channels, kernel_size, kernel_size)
        self.mask_conv = nn.Conv2d(in_channels, 1, kernel_size, stride, padding, dilation,
                                   groups=groups, bias=False)
        self.mask_conv.weight.data.fill_(1.0)
        for p in self.mask_conv.parameters():
            p.requires_grad = False
        self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None
        self.window_size = float(in_channels * kernel_size * kernel_size)
        self.ainp_bf16 = False   # set_compute_dtype(): bf16 conv operands (C4 / C5)

    # plane-level entry used by the U-Net: srcs = [(x, mask_plane [N,H,W]), ...]
    def run(self, srcs, Hin, Win, act=ops.ACT_NONE, want_stats=False, crop=None,
            with_ratio=False):
        k, s, p = self.kernel_size, self.stride, self.padding
        (x0, m0) = srcs[0]
        src1 = srcs[1] if len(srcs) > 1 else None
        N = x0.shape[0]
        ratio, newm = ops.pconv_mask((m0, x0.shape[1]),
                                     (src1[1], src1[0].shape[1]) if src1 is not None else None,
                                     N, Hin, Win, k, s, p)
        y, stats = ops.conv_gen(srcs[0], self.conv.weight, src1=src1, Hin=Hin, Win=Win, stride=s,
                                pad=p, bias=self.bias, ratio=ratio, act=act, slope=SLOPE,
                                want_stats=want_stats, crop=crop, bf16=self.ainp_bf16)
        if with_ratio:
            return y, newm, stats, ratio
        return y, newm, stats

    def run_full_mask(self, x, mask, want_stats=False):
        """PartialConv2d with a per-channel mask [N, Cin, H, W]."""
        N, C, H, W = x.shape
        xm = ops.mul(x, mask)
        msum = ops.channel_sum(mask)
        k, s, p = self.kernel_size, self.stride, self.padding
        # the window sum of the channel-summed plane is the full count; the
        # ratio's numerator stays Cin*k*k
        ratio, newm = ops.pconv_mask((msum, 1), None, N, H, W, k, s, p, winsize=self.window_size)
        y, stats = ops.conv_gen((xm, None), self.conv.weight, stride=s, pad=p, bias=self.bias,
                                ratio=ratio, want_stats=want_stats, bf16=self.ainp_bf16)
        return y, newm, stats

    def forward(self, x: torch.Tensor, mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """networks.py:63-106: (output, updated mask repeated to out_channels)."""
        _need_cuda(x, "PartialConv2d")
        x = x.contiguous().float()
        mask = mask.contiguous().float()
        N, C, H, W = x.shape
        if mask.shape[1] == 1:
            y, newm, _ = self.run([(x, mask.reshape(N, H, W))], H, W)
        elif mask.shape[1] == C:
            y, newm, _ = self.run_full_mask(x, mask)
        else:
            raise ValueError("mask must have 1 or in_channels channels")
        Ho, Wo = y.shape[2:]
        return y, newm.reshape(N, 1, Ho, Wo).expand(N, self.out_channels, Ho, Wo).contiguous()


# bf16 no-grad U-Net: the BatchNorm + LeakyReLU pass writes only the next
# convs' channel-last bf16 copy, not the fp32 block output back
# (AINP_AFFINE_NO_Y=0: both, A/B)
AFFINE_NO_Y = os.environ.get("AINP_AFFINE_NO_Y", "1") != "0"


def _affine_no_y_safe():
    """The fp32 write-back may be skipped only while every consumer of a U-Net
    block output reads the channel-last copy: the 32-multiple-channel convs
    always take the nhwc16 route, but the final PartialConv2d's (64 + 1 -> 64)
    second source is the 1-channel padded input, which reaches that route only
    through the CONV_NHWC16_SMALL branch (ops._nhwc16_route); with
    AINP_CONV_NHWC16_SMALL=0 it runs the NCHW fp32 gather, which reads the
    block output's fp32 planes, so they must be written."""
    return AFFINE_NO_Y and ops.CONV_NHWC16 and ops.CONV_NHWC16_SMALL != "0"


class EncoderBlock(nn.Module):
    """networks.py:139-152: PartialConv -> BatchNorm2d -> LeakyReLU(0.2)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding,
                 norm_layer=nn.BatchNorm2d, activation=None):
        super().__init__()
        self.pconv = PartialConv2d(in_channels, out_channels, kernel_size, stride, padding,
                                   bias=False)
        self.norm = norm_layer(out_channels) if norm_layer else nn.Identity()
        self.activation = activation if activation is not None else nn.LeakyReLU(SLOPE, True)

    def _finish(self, y, stats):
        N, C, Ho, Wo = y.shape
        if isinstance(self.norm, nn.BatchNorm2d):
            sc, sh = _bn_affine(self.norm, stats, N * Ho * Wo, C)
        else:
            sc = torch.ones(C, device=y.device)
            sh = torch.zeros(C, device=y.device)
        ops.affine_act_(y, sc, sh, ops.ACT_LEAKY, SLOPE)
        return y

    def _want_stats(self):
        return isinstance(self.norm, nn.BatchNorm2d) and (
            self.norm.training or not self.norm.track_running_stats)

    def run(self, srcs, Hin, Win, keep_y=True):
        """keep_y=False (the U-Net's own no-grad forward): in the channel-last
        bf16 path the fp32 block output is not written back -- its consumers
        read the copy."""
        y, newm, stats = self.pconv.run(srcs, Hin, Win, want_stats=self._want_stats())
        if (self.pconv.ainp_bf16 and ops._NHWC_MEMO is not None and ops.CONV_NHWC16
                and y.shape[1] % 32 == 0):
            # bf16 U-Net: the next conv's channel-last source in the same pass
            N, C, Ho, Wo = y.shape
            if isinstance(self.norm, nn.BatchNorm2d):
                sc, sh = _bn_affine(self.norm, stats, N * Ho * Wo, C)
            else:
                sc = torch.ones(C, device=y.device)
                sh = torch.zeros(C, device=y.device)
            # the block output's consumers (the next encoder conv, the decoder's
            # skip / upsampled sources) read the channel-last copy: in the U-Net's
            # forward the fp32 write-back is skipped unless a profiling capture
            # reads the planes
            ops.affine_act_nhwc16_(y, sc, sh, ops.ACT_LEAKY, SLOPE, newm,
                                   keep_y=keep_y or not _affine_no_y_safe()
                                   or PConvUNet.capture is not None)
            return y, newm
        return self._finish(y, stats), newm

    def forward(self, x, mask):
        _need_cuda(x, "EncoderBlock")
        x = x.contiguous().float()
        mask = mask.contiguous().float()
        N, C, H, W = x.shape
        if mask.shape[1] == 1:
            y, newm = self.run([(x, mask.reshape(N, H, W))], H, W)
        else:
            y, newm, stats = self.pconv.run_full_mask(x, mask, want_stats=self._want_stats())
            y = self._finish(y, stats)
        Ho, Wo = y.shape[2:]
        return y, newm.reshape(N, 1, Ho, Wo).expand(N, y.shape[1], Ho, Wo).contiguous()


class DecoderBlock(EncoderBlock):
    """networks.py:154-168."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1,
                 norm_layer=nn.BatchNorm2d, activation=None):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, norm_layer,
                         activation)


def get_pad_size(input_size: int, factor: int) -> int:
    """networks.py:111-115."""
    return 0 if input_size % factor == 0 else factor - (input_size % factor)


def calculate_total_downsampling(layers) -> int:
    """networks.py:117-134 (for EncoderBlock lists)."""
    f = 1
    for layer in layers:
        conv = getattr(layer, "pconv", None) or getattr(layer, "conv", None)
        if conv is not None:
            s = conv.stride[0] if isinstance(conv.stride, tuple) else conv.stride
            if s > 1:
                f *= s
    return f


class PConvUNet(nn.Module):
    """networks.py:173-345."""

    def __init__(self, input_channels=1, mask_channels=1, output_channels=1,
                 enc_layer_cfg=((64, 7, 2, 3), (128, 5, 2, 2), (256, 5, 2, 2), (512, 3, 2, 1),
                                (512, 3, 2, 1), (512, 3, 2, 1), (512, 3, 2, 1)),
                 dec_layer_cfg=((512, 3, 1, 1), (512, 3, 1, 1), (512, 3, 1, 1), (256, 3, 1, 1),
                                (128, 3, 1, 1), (64, 3, 1, 1)),
                 final_dec_cfg=None, norm_layer=nn.BatchNorm2d, activation=None,
                 final_activation=None, upsample_mode="nearest"):
        super().__init__()
        if final_dec_cfg is None:
            final_dec_cfg = {"interim_ch": 64, "out_ch": 1, "kernel": 3, "padding": 1}
        if input_channels != 1 or mask_channels != 1:
            raise NotImplementedError("the reference's skip logic assumes 1 input / mask channel")
        if upsample_mode != "nearest":
            raise NotImplementedError("upsample_mode must be 'nearest' (the reference default)")
        self.input_channels, self.mask_channels = input_channels, mask_channels
        self.upsample = nn.Upsample(scale_factor=2, mode=upsample_mode)
        self.final_activation = final_activation if final_activation is not None else nn.Tanh()
        act = activation if activation is not None else nn.LeakyReLU(SLOPE, inplace=True)
        self.encoder_blocks = nn.ModuleList()
        in_c = input_channels + mask_channels
        self.enc_output_channels = []
        for out_c, k, s, p in enc_layer_cfg:
            self.encoder_blocks.append(EncoderBlock(in_c, out_c, k, s, p, norm_layer, act))
            self.enc_output_channels.append(out_c)
            in_c = out_c
        self._total_downsampling = calculate_total_downsampling(self.encoder_blocks)
        self.decoder_blocks = nn.ModuleList()
        skip_rev = self.enc_output_channels[::-1]
        up_c = skip_rev[0]
        for i, (out_c, k, s, p) in enumerate(dec_layer_cfg):
            self.decoder_blocks.append(DecoderBlock(up_c + skip_rev[i + 1], out_c, k, s, p,
                                                    norm_layer, act))
            up_c = out_c
        fk, fp = final_dec_cfg["kernel"], final_dec_cfg["padding"]
        self.final_decoder_layer = nn.Sequential(
            PartialConv2d(up_c + input_channels, final_dec_cfg["interim_ch"], fk, 1, fp, bias=True),
            act,
            PartialConv2d(final_dec_cfg["interim_ch"], final_dec_cfg["out_ch"], fk, 1, fp, bias=True),
        )
        if final_dec_cfg["out_ch"] != 1:
            raise NotImplementedError("out_ch must be 1 (the reference's configuration)")

    def forward(self, x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        """networks.py:247-345.  Under torch.no_grad() (the reference training
        loop, train.py:349-350: G is never trained) the forward-only
        path; with autograd on and trainable parameters (fix_generator_grad,
        or any caller that back-propagates into G as the reference module
        allows) the output carries G's gradient: _PConvUNetFn keeps each
        block's pre-BN conv output, window ratio and batch statistics and its
        backward runs the kernels of csrc/gan_bwd.hip plus the MFMA GEMMs."""
        params = [p for p in self.parameters()]
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            with _nbt_batch():
                return _PConvUNetFn.apply(x.contiguous().float(), mask.contiguous().float(),
                                          self, *params)
        with torch.no_grad(), ops.nhwc16_memo(), _nbt_batch():
            return self._forward(x, mask)

    # profiling hook: a dict set here collects the sources of the final
    # PartialConv2d ("final") and of the decoder blocks listed under "decoder"
    # during the next no-grad forward (bench.py's in-step roofline launches)
    capture = None

    def _check_inputs(self, x, mask):
        if x.shape[1] != self.input_channels:
            raise ValueError(f"Input x channels ({x.shape[1]}) != expected ({self.input_channels})")
        if mask.shape[1] != self.mask_channels:
            raise ValueError(f"Input mask channels ({mask.shape[1]}) != expected ({self.mask_channels})")
        if x.shape[2:] != mask.shape[2:]:
            raise ValueError("x and mask spatial dims must match")
        _need_cuda(x, "PConvUNet")

    def _forward_tape(self, x, mask):
        """The training forward of _PConvUNetFn: the same launches as _forward
        (no channel-last memo: the pre-BN outputs must survive), recording what
        the backward needs.  Returns (output [N,1,H,W], tape)."""
        self._check_inputs(x, mask)
        N, _, H, W = x.shape
        f = self._total_downsampling
        Hp, Wp = H + get_pad_size(H, f), W + get_pad_size(W, f)
        xp, mp = ops.gan_pad_input(x, mask, Hp, Wp)
        xp4, mp4 = xp.view(N, 1, Hp, Wp), mp.view(N, 1, Hp, Wp)
        tape = {"Hp": Hp, "Wp": Wp, "H": H, "W": W, "blocks": []}

        def block(blk, srcs, Hin, Win):
            pc = blk.pconv
            y, newm, stats, ratio = pc.run(srcs, Hin, Win, want_stats=blk._want_stats(),
                                           with_ratio=True)
            Nn, C, Ho, Wo = y.shape
            if isinstance(blk.norm, nn.BatchNorm2d):
                sc, sh, save = _bn_affine(blk.norm, stats, Nn * Ho * Wo, C, want_save=True)
            else:
                sc = torch.ones(C, device=y.device)
                sh = torch.zeros(C, device=y.device)
                save = None
            a = ops.affine_leaky_out(y, sc, sh, SLOPE)
            ev = isinstance(blk.norm, nn.BatchNorm2d) and not (
                blk.norm.training or not blk.norm.track_running_stats)
            tape["blocks"].append({"blk": blk, "srcs": srcs, "Hin": Hin, "Win": Win, "y": y,
                                   "ratio": ratio, "sc": sc, "sh": sh, "save": save, "a": a,
                                   "eval": ev})
            return a, newm

        srcs = [(xp4, mp), (mp4, mp)]
        Hc, Wc = Hp, Wp
        feats, masks = [], []
        for blk in self.encoder_blocks:
            a, m = block(blk, srcs, Hc, Wc)
            feats.append(a)
            masks.append(m)
            Hc, Wc = a.shape[2:]
            srcs = [(a, m)]
        d, dm = feats[-1], masks[-1]
        for i, blk in enumerate(self.decoder_blocks):
            j = len(feats) - 2 - i
            Hs, Ws = feats[j].shape[2:]
            if (2 * d.shape[2], 2 * d.shape[3]) != (Hs, Ws):
                raise RuntimeError("decoder/skip size mismatch")
            d, dm = block(blk, [(d, dm), (feats[j], masks[j])], Hs, Ws)
        if (2 * d.shape[2], 2 * d.shape[3]) != (Hp, Wp):
            raise RuntimeError(f"Size mismatch before final layer. Dec: {d.shape[2:]}, "
                               f"Skip: {(Hp, Wp)}")
        pc1, pc2 = self.final_decoder_layer[0], self.final_decoder_layer[2]
        s1 = [(d, dm), (xp4, mp)]
        y1, m1, _, r1 = pc1.run(s1, Hp, Wp, act=ops.ACT_LEAKY, with_ratio=True)
        s2 = [(y1, m1)]
        out, _, _, r2 = pc2.run(s2, Hp, Wp, act=ops.ACT_TANH, crop=(H, W), with_ratio=True)
        tape["pc1"] = {"pc": pc1, "srcs": s1, "ratio": r1, "a": y1}
        tape["pc2"] = {"pc": pc2, "srcs": s2, "ratio": r2, "a": out.view(N, 1, H, W)}
        tape["n_enc"] = len(self.encoder_blocks)
        return out.view(N, 1, H, W), tape

    def _forward(self, x, mask):
        self._check_inputs(x, mask)
        x = x.contiguous().float()
        mask = mask.contiguous().float()
        N, _, H, W = x.shape
        f = self._total_downsampling
        Hp, Wp = H + get_pad_size(H, f), W + get_pad_size(W, f)
        xp, mp = ops.gan_pad_input(x, mask, Hp, Wp)          # [N, Hp, Wp] each
        xp4, mp4 = xp.view(N, 1, Hp, Wp), mp.view(N, 1, Hp, Wp)
        # encoder: the first input is cat(x_pad, mask_pad) * mask_pad
        srcs = [(xp4, mp), (mp4, mp)]
        Hc, Wc = Hp, Wp
        feats, masks = [], []
        for blk in self.encoder_blocks:
            y, m = blk.run(srcs, Hc, Wc, keep_y=False)
            feats.append(y)
            masks.append(m)
            Hc, Wc = y.shape[2:]
            srcs = [(y, m)]
        d, dm = feats[-1], masks[-1]
        for i, blk in enumerate(self.decoder_blocks):
            j = len(feats) - 2 - i
            Hs, Ws = feats[j].shape[2:]
            if (2 * d.shape[2], 2 * d.shape[3]) != (Hs, Ws):
                raise RuntimeError("decoder/skip size mismatch (cannot happen after padding to "
                                   "the total downsampling factor)")
            cap = PConvUNet.capture
            if cap is not None and i in cap.get("decoder", ()):
                # profiling hook (bench.py's in-step roofline operands): this
                # block's sources as the step launches them
                cap[f"decoder{i}"] = ([(d, dm), (feats[j], masks[j])], Hs, Ws)
            d, dm = blk.run([(d, dm), (feats[j], masks[j])], Hs, Ws, keep_y=False)
        if (2 * d.shape[2], 2 * d.shape[3]) != (Hp, Wp):
            raise RuntimeError(f"Size mismatch before final layer. Dec: {d.shape[2:]}, "
                               f"Skip: {(Hp, Wp)}")
        pc1, pc2 = self.final_decoder_layer[0], self.final_decoder_layer[2]
        if PConvUNet.capture is not None:
            PConvUNet.capture["final"] = ([(d, dm), (xp4, mp)], Hp, Wp)
        y1, m1, _ = pc1.run([(d, dm), (xp4, mp)], Hp, Wp, act=ops.ACT_LEAKY)
        # final PartialConv2d (Cout=1) + Tanh + crop to the input size in one launch
        out, _, _ = pc2.run([(y1, m1)], Hp, Wp, act=ops.ACT_TANH, crop=(H, W))
        return out.view(N, 1, H, W)


def _ld4(P):
    """Pixel rows padded to a multiple of 4 (16-byte GEMM loads)."""
    return P + (-P) % 4


def _pconv_weight_data_grads(pc, gc, srcs, Hin, Win, dsrcs):
    """Weight gradient of a PartialConv2d's conv and the gradients of its
    sources from gc [N, Cout, ldo] = d(conv output) (window ratio applied):
      dW [Cout, Cin*k*k] = sum_n gc_n . im2col(input_n)^T   (MFMA GEMM, split-K)
      dinput = col2im(W^T . gc),  dsrc (+)= mask * block-sum(dinput[channels])
    input = cat(nearest(x0) * m0, x1 * m1) (networks.py:79-82,297-313).
    dsrcs: per source a (tensor to accumulate into, accumulate flag) or None."""
    w = pc.conv.weight
    Cout, Cin, k, _ = w.shape
    s, p = pc.stride, pc.padding
    bf16 = pc.ainp_bf16
    N, _, ldo = gc.shape
    xin = ops.pconv_src_materialize(srcs[0], srcs[1] if len(srcs) > 1 else None, Hin, Win)
    K = Cin * k * k
    col = ops.im2col(xin, k, s, p, ldp=ldo)                       # [N, K, ldo]
    dw = torch.empty(Cout, K, device=gc.device)
    ops.gemm_batched_splitk(Cout, K, ldo, [gc[n] for n in range(N)], ldo, 1,
                            [col[n] for n in range(N)], 1, ldo, dw, bf16=bf16)
    del col
    if any(d is not None for d in dsrcs):
        dcol = torch.empty(N, K, ldo, device=gc.device)
        ops.gemm(K, ldo, Cout, [w], 1, K, [gc], ldo, 1, [dcol], ldo, 1, strideB=Cout * ldo,
                 strideC=K * ldo, nstrided=N, bf16=bf16)
        dxin = ops.col2im(dcol, N, Cin, Hin, Win, k, s, p)
        del dcol
        c_off = 0
        for (x, m), d in zip(srcs, dsrcs):
            if d is not None:
                dst, acc = d
                ops.pconv_src_grad(dxin, c_off, m, dst, acc)
            c_off += x.shape[1]
    return dw.view_as(w)


class _PConvUNetFn(torch.autograd.Function):
    """PConvUNet forward with autograd (the opt-in generator training of
    SURVEY §7, fix_generator_grad): forward = PConvUNet._forward_tape; backward
    in reverse block order -- Tanh + crop, the final PartialConv2d pair with
    their biases, then each decoder / encoder block: LeakyReLU + BatchNorm2d
    backward (batch statistics; SyncBN sums all-reduced under DP) times the
    window ratio, the conv's weight gradient and its sources' gradients (the
    skip's added to the encoder block's output gradient, the upsampled
    decoder input's 2x2-summed into the previous block's).  The input x and
    the mask get no gradient (data)."""

    @staticmethod
    def forward(ctx, x, mask, unet, *params):
        out, tape = unet._forward_tape(x, mask)
        ctx.tape = tape
        ctx.unet = unet
        ctx.params = params
        return out

    @staticmethod
    def backward(ctx, g):
        tape, unet = ctx.tape, ctx.unet
        if tape is None:
            raise RuntimeError("PConvUNet backward ran twice through the same graph: its saved "
                               "activations are released after the first backward "
                               "(retain_graph=True is not supported); run the forward again")
        ctx.tape = None
        grads = {}
        Hp, Wp, H, W = tape["Hp"], tape["Wp"], tape["H"], tape["W"]
        g = g.contiguous()
        N = g.shape[0]
        P = Hp * Wp
        ldo = _ld4(P)
        # ---- final PartialConv2d (Cout = 1) + Tanh + crop (networks.py:331-337)
        t2 = tape["pc2"]
        pc2 = t2["pc"]
        gz, gc = ops.gen_act_bwd(g, t2["a"], ops.ACT_TANH, SLOPE, t2["ratio"], Hp, Wp, ldo)
        grads[pc2.bias] = ops.rowsum_batched(gz.view(N, 1, P))
        y1 = tape["pc1"]["a"]
        dy1 = torch.empty_like(y1)
        grads[pc2.conv.weight] = _pconv_weight_data_grads(pc2, gc, t2["srcs"], Hp, Wp,
                                                          [(dy1, False)])
        # ---- PartialConv2d(64+1 -> 64) + LeakyReLU (networks.py:327-329)
        t1 = tape["pc1"]
        pc1 = t1["pc"]
        C1 = y1.shape[1]
        gz, gc = ops.gen_act_bwd(dy1, y1, ops.ACT_LEAKY, SLOPE, t1["ratio"], Hp, Wp, ldo)
        grads[pc1.bias] = ops.rowsum_batched(gz.view(N, C1, P))
        del gz
        blocks = tape["blocks"]
        n_enc = tape["n_enc"]
        # gradient accumulators of every block output (decoder inputs, skips)
        ga = [None] * len(blocks)
        last = len(blocks) - 1
        ga[last] = torch.empty_like(blocks[last]["a"])
        grads[pc1.conv.weight] = _pconv_weight_data_grads(pc1, gc, t1["srcs"], Hp, Wp,
                                                          [(ga[last], False), None])
        del gc
        # ---- decoder blocks (reverse), then encoder blocks (reverse)
        for bi in range(last, -1, -1):
            rec = blocks[bi]
            blk = rec["blk"]
            y, a = rec["y"], rec["a"]
            Nn, C, Ho, Wo = y.shape
            Pb = Ho * Wo
            ldb = _ld4(Pb)
            gab = ga[bi]
            if isinstance(blk.norm, nn.BatchNorm2d):
                bn = blk.norm
                comm = getattr(bn, "ainp_comm", None)
                if rec["eval"]:
                    sums = ops.bn_act_bwd_reduce(gab, y, rec["sc"], rec["sh"], rec["save"], SLOPE)
                    cnt = -1
                elif comm is not None and comm.world_size > 1:
                    sums = comm.allreduce_sum_(ops.bn_act_bwd_reduce(gab, y, rec["sc"], rec["sh"],
                                                                     rec["save"], SLOPE,
                                                                     count=Nn * Pb))
                    cnt = 0
                else:
                    sums = ops.bn_act_bwd_reduce(gab, y, rec["sc"], rec["sh"], rec["save"], SLOPE)
                    cnt = Nn * Pb
                gc, dgam, dbet = ops.bn_act_bwd_apply(gab, y, rec["sc"], rec["sh"], rec["save"],
                                                      bn.weight, sums, cnt, SLOPE, rec["ratio"],
                                                      ldb)
                if cnt == 0:
                    # SyncBN: dgamma / dbeta came from the all-reduced sums, so every
                    # rank already holds the global sum; the trainer's reducer SUMs
                    # over ranks and divides by world_size, so hand it the per-rank
                    # share (torch SyncBN uses the local sums here; for equal
                    # per-rank batches the two are the same, exactly for 2^k ranks)
                    dgam.div_(comm.world_size)
                    dbet.div_(comm.world_size)
                grads[bn.weight], grads[bn.bias] = dgam, dbet
            else:
                _, gc = ops.gen_act_bwd(gab, a, ops.ACT_LEAKY, SLOPE, rec["ratio"], Ho, Wo, ldb,
                                        want_gz=False)
            srcs = rec["srcs"]
            if bi == 0:
                dsrcs = [None, None]                      # cat(x_pad, mask_pad): data
            elif bi < n_enc:
                if ga[bi - 1] is None:
                    ga[bi - 1] = torch.empty_like(blocks[bi - 1]["a"])
                    dsrcs = [(ga[bi - 1], False)]
                else:
                    dsrcs = [(ga[bi - 1], True)]
            else:
                # decoder block i = bi - n_enc: sources (previous output, skip j)
                i = bi - n_enc
                prev = bi - 1                              # the block whose output is upsampled
                j = n_enc - 2 - i
                dsrcs = []
                for tgt in (prev, j):
                    if ga[tgt] is None:
                        ga[tgt] = torch.empty_like(blocks[tgt]["a"])
                        dsrcs.append((ga[tgt], False))
                    else:
                        dsrcs.append((ga[tgt], True))
            grads[blk.pconv.conv.weight] = _pconv_weight_data_grads(
                blk.pconv, gc, srcs, rec["Hin"], rec["Win"], dsrcs)
            ga[bi] = None
            del gc
        out = []
        for p in ctx.params:
            out.append(grads.get(p))
        return (None, None, None, *out)


# ------------------------------------------------------------ discriminator
class DiscriminatorBlock(nn.Module):
    """networks.py:352-373."""

    def __init__(self, in_channels, out_channels, kernel_size=4, stride=2, padding=1,
                 use_spectral_norm=True, activation=None, use_norm=False):
        super().__init__()
        if use_norm or not use_spectral_norm:
            raise NotImplementedError("the reference Discriminator uses spectral norm, no BN")
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=True)
        conv = spectral_norm(conv)
        self.block = nn.Sequential(conv, nn.Identity(),
                                   activation if activation is not None
                                   else nn.LeakyReLU(SLOPE, inplace=True))

    def forward(self, x):
        raise RuntimeError("use Discriminator.forward (the blocks run fused)")


class _DiscriminatorFn(torch.autograd.Function):
    """The 5 spectral-norm convs (+LeakyReLU on the first 4) forward/backward.
    params per layer: (weight_orig, bias); sn = (inv_sigma [L], u clones, v clones)."""

    @staticmethod
    def forward(ctx, x, cfg, bf16, inv, us, vs, *params):
        h = x.contiguous()
        ins, outs = [], []
        L = len(cfg)
        # bf16: each conv whose successor is a channel-last bf16 conv (Cout > 1)
        # writes that conv's source itself (no separate nchw_to_nhwc16 pass)
        with ops.nhwc16_memo():
            for l, (k, s, p, act) in enumerate(cfg):
                w, b = params[2 * l], params[2 * l + 1]
                nxt16 = bf16 and l + 1 < L and params[2 * (l + 1)].shape[0] > 1
                y, _ = ops.conv_gen((h, None), w, stride=s, pad=p, bias=b, scale=inv[l:l + 1],
                                    act=ops.ACT_LEAKY if act else ops.ACT_NONE, slope=SLOPE,
                                    bf16=bf16, out16=nxt16)
                ins.append(h)
                outs.append(y)
                h = y
            # the channel-last bf16 inputs the convs read: the bf16 backward's
            # weight gradients gather from them (ainp_wgrad16_nhwc)
            keep = bf16 and WGRAD16_NHWC
            ctx.h16 = [ops.nhwc16_memo_get(t) if keep else None for t in ins]
        ctx.cfg = cfg
        ctx.bf16 = bf16
        ctx.nl = len(cfg)
        ctx.save_for_backward(inv, *ins, *outs, *us, *vs, *params)
        return h

    @staticmethod
    def backward(ctx, g):
        L = ctx.nl
        st = ctx.saved_tensors
        inv = st[0]
        ins, outs = st[1:1 + L], st[1 + L:1 + 2 * L]
        us, vs = st[1 + 2 * L:1 + 3 * L], st[1 + 3 * L:1 + 4 * L]
        params = st[1 + 4 * L:]
        if ctx.bf16 and D_BWD16:
            return _d_backward16(ctx, g, inv, ins, outs, us, vs, params)
        grads = [None] * len(params)
        g = g.contiguous()
        gx = None
        for l in range(L - 1, -1, -1):
            k, s, p, act = ctx.cfg[l]
            w = params[2 * l]
            N, Cout, Ho, Wo = g.shape
            P = Ho * Wo
            # pixel rows padded to a multiple of 4 (zeros) for 16-byte GEMM loads
            P4 = P if (P % 4 == 0 or not act) else P + (-P) % 4
            if act:
                g = ops.leaky_bwd(g, outs[l], SLOPE, ldo=P4).view(N, Cout, P4)
            else:
                g = g.view(N, Cout, P)
            h = ins[l]
            Cin, H, W = h.shape[1:]
            K = Cin * k * k
            # [dW | db] = sum_n g_n [Cout, P] . [col_n ; 1]^T, P split into chunks
            col = ops.im2col(h, k, s, p, ones_row=True, ldp=P4)    # [N, K+1, P4]
            Gw = torch.empty(Cout, K + 1, device=g.device)
            ops.gemm_batched_splitk(Cout, K + 1, P4, [g[n] for n in range(N)], P4, 1,
                                    [col[n] for n in range(N)], 1, P4, Gw, bf16=ctx.bf16)
            dw, db = ops.sn_weight_grad(Gw, w, us[l], vs[l], inv[l:l + 1], with_bias=True)
            grads[2 * l], grads[2 * l + 1] = dw.view_as(w), db
            if l > 0 or ctx.needs_input_grad[0]:
                wn = ops.scale_by_scalar(w, inv[l:l + 1])
                dcol = torch.empty(N, K, P4, device=g.device)    # padded columns unused
                ops.gemm(K, P4, Cout, [wn], 1, K, [g], P4, 1, [dcol], P4, 1, strideB=Cout * P4,
                         strideC=K * P4, nstrided=N, bf16=ctx.bf16)
                g = ops.col2im(dcol, N, Cin, H, W, k, s, p)
                if l == 0:
                    gx = g
        return (gx, None, None, None, None, None, *grads)


# Discriminator forward: the spectral-norm u / v snapshots for the backward as
# one multi-tensor copy, none without autograd (AINP_SN_FOREACH=0: per-tensor
# clones in every pass, A/B)
SN_FOREACH = os.environ.get("AINP_SN_FOREACH", "1") != "0"

# bf16 configurations: the D backward on bf16 operands in HBM (csrc/dconv16.hip);
# AINP_D_BWD16=0 keeps the fp32-staged im2col / GEMM / col2im loop
D_BWD16 = os.environ.get("AINP_D_BWD16", "1") != "0"
# AINP_WGRAD16_NHWC=1: weight gradients of layers with a channel-last bf16
# input copy as implicit GEMMs over it (ainp_wgrad16_nhwc, bit-identical).  Off:
# in the C4 step 9.35 -> 9.54 ms/step; standalone it wins only at layer 1 (119
# vs 157 us) and loses at layers 2 / 3 (122 vs 100, 311 vs 184 us): the 128 x
# 128 tiles re-gather the input per Cout tile (profiles/r04p_summary.txt)
WGRAD16_NHWC = os.environ.get("AINP_WGRAD16_NHWC", "0") == "1"
# the data gradient of a layer writes the lower layer's bf16 gradient operands
# itself where it runs unsplit (ainp_dgrad16_prep; 0: dgrad16 + d_prep16, A/B)
D_PREP_FUSED = os.environ.get("AINP_D_PREP_FUSED", "1") != "0"
# the logit conv's weight gradient by ainp_wgrad_cout1 (0: im2col16 + GEMM, A/B)
WGRAD_COUT1 = os.environ.get("AINP_WGRAD_COUT1", "1") != "0"


# AINP_D_WGRAD_SIDE=1: the discriminator's weight gradients (im2col16 + GEMM +
# spectral-norm gradient) on a side stream beside the data-gradient chain of
# the layers below (bit-identical).  Off: C4 9.12-9.15 -> 9.32-9.36 ms/step
# with it, the two chains' kernels slow each other (profiles/r04z4_summary.txt)
D_WGRAD_SIDE = os.environ.get("AINP_D_WGRAD_SIDE", "0") == "1"
_D_SIDE: dict = {}


def _d_side(device):
    """(side stream, its own reduction workspace) of the device."""
    key = str(device)
    ent = _D_SIDE.get(key)
    if ent is None:
        st = torch.cuda.Stream(device=device)
        with torch.cuda.stream(st):
            ws = torch.empty_like(ops._reduce_ws(device))
        ent = _D_SIDE[key] = (st, ws)
    return ent


def _d_backward16(ctx, g, inv, ins, outs, us, vs, params):
    """_DiscriminatorFn.backward with bf16 operands: per layer the gradient is
    cast once into a pixel-contiguous and a channel-last bf16 copy (LeakyReLU
    backward and the split-K slabs of the layer above folded in; written by
    the layer above's data-gradient epilogue where that runs unsplit), the weight
    gradient is one bf16 GEMM over every image's pixels (on a side stream),
    the data gradient a parity-class implicit GEMM (csrc/dconv16.hip)."""
    L = ctx.nl
    grads = [None] * len(params)
    gsrc, nslab = g.contiguous(), 1
    gx = None
    pre = None    # this layer's (gA, gT), written by the layer above's data gradient
    dev = g.device
    side, side_ws = _d_side(dev) if D_WGRAD_SIDE else (None, None)
    main = torch.cuda.current_stream(dev)
    for l in range(L - 1, -1, -1):
        k, s, p, act = ctx.cfg[l]
        w = params[2 * l]
        N, Cout, Ho, Wo = outs[l].shape
        P = Ho * Wo
        ldA = -(-N * P // 64) * 64
        need_dx = l > 0 or ctx.needs_input_grad[0]
        h = ins[l]
        Cin, H, W = h.shape[1:]
        y_act = outs[l] if act else None
        if WGRAD_COUT1 and Cout == 1 and k in (3, 4):
            # the logit conv: a GEMV, straight from h (no materialised columns)
            def wgrad(h=h, gsrc=gsrc, nslab=nslab, y_act=y_act, k=k, s=s, p=p):
                return ops.wgrad_cout1(h, gsrc, nslab, y_act, SLOPE, k, s, p)
            deps = [h, gsrc] + ([y_act] if act else [])
            gT = ops.d_prep16(gsrc, nslab, y_act, SLOPE, N, Cout, P, ldA,
                              want_gT=True)[1] if need_dx else None
        else:
            if pre is not None:
                gA, gT = pre
            else:
                gA, gT = ops.d_prep16(gsrc, nslab, y_act, SLOPE, N, Cout, P, ldA,
                                      want_gT=need_dx)
            h16 = ctx.h16[l] if WGRAD16_NHWC else None
            if h16 is not None and Cin % 8 == 0:
                # implicit GEMM over the forward's channel-last input copy
                def wgrad(gA=gA, h16=h16, k=k, s=s, p=p):
                    return ops.wgrad16_nhwc(gA, h16, k, s, p, max_split=512)
                deps = [gA, h16]
            else:
                def wgrad(gA=gA, h=h, k=k, s=s, p=p, ldA=ldA):
                    col = ops.im2col16(h, k, s, p, ldA)          # [Cin*k*k + 1, ldA]
                    return ops.gemm_bf16nt_splitk(gA, col, ldA, max_split=512)
                deps = [gA, h]
        sn = (w, us[l], vs[l], inv[l:l + 1])
        if side is not None:
            # the operands are complete on the main stream at this point
            ready = torch.cuda.Event()
            ready.record(main)
            with torch.cuda.stream(side):
                side.wait_event(ready)
                dw, db = ops.sn_weight_grad(wgrad(), *sn, with_bias=True, ws=side_ws)
            for t in deps + list(sn):
                t.record_stream(side)     # not reused while the side stream reads it
            for t in (dw, db):
                t.record_stream(main)     # consumed by autograd on the main stream
        else:
            dw, db = ops.sn_weight_grad(wgrad(), *sn, with_bias=True)
        grads[2 * l], grads[2 * l + 1] = dw.view_as(w), db
        pre = None
        if need_dx:
            S = ops.dgrad16_nsplit(N, Cin, H, W, k, s, Cout)
            wd = ops.dgrad16_weight(w, s, p)
            if D_PREP_FUSED and l > 0 and S == 1 and Cin % 4 == 0:
                # the lower layer's gA / gT straight from this data gradient's
                # epilogue (no fp32 dx, no d_prep16 pass)
                act_lo = ctx.cfg[l - 1][3]
                pre = ops.dgrad16_prep(gT.view(N, Ho, Wo, Cout), wd, Cin, H, W, k, s, p,
                                       outs[l - 1] if act_lo else None, SLOPE,
                                       -(-N * H * W // 64) * 64, scale=inv[l:l + 1],
                                       want_gT=l - 1 > 0 or ctx.needs_input_grad[0])
                continue
            gsrc = ops.dgrad16(gT.view(N, Ho, Wo, Cout), wd, Cin, H, W,
                               k, s, p, scale=inv[l:l + 1], nsplit=S)
            nslab = S
            if l == 0:
                gx = gsrc[0] if S == 1 else ops.sum_slabs(gsrc, S).view(N, Cin, H, W)
    if side is not None:
        main.wait_stream(side)            # the weight gradients are complete
    return (gx, None, None, None, None, None, *grads)


def _split_count(n):
    for s in (8, 4, 2, 1):
        if n % s == 0:
            return s
    return 1


class Discriminator(nn.Module):
    """networks.py:375-409."""

    def __init__(self, input_channels=1,
                 layer_cfg=((64, 2, False), (128, 2, False), (256, 2, False), (512, 1, False)),
                 final_out_channels=1, kernel_size=4, padding=1, use_spectral_norm=True,
                 activation=None):
        super().__init__()
        if not use_spectral_norm:
            raise NotImplementedError("the reference Discriminator uses spectral norm")
        act = activation if activation is not None else nn.LeakyReLU(SLOPE, inplace=True)
        layers = []
        in_c = input_channels
        self._cfg = []
        for out_c, stride, use_norm in layer_cfg:
            layers.append(DiscriminatorBlock(in_c, out_c, kernel_size, stride, padding, True, act,
                                             use_norm))
            self._cfg.append((kernel_size, stride, padding, True))
            in_c = out_c
        final = spectral_norm(nn.Conv2d(in_c, final_out_channels, kernel_size, stride=1,
                                        padding=padding, bias=True))
        layers.append(final)
        self._cfg.append((kernel_size, 1, padding, False))
        self.model = nn.Sequential(*layers)
        if final_out_channels != 1:
            raise NotImplementedError("final_out_channels must be 1 (the reference's)")
        self.ainp_bf16 = False   # set_compute_dtype(): bf16 conv / GEMM operands (C4 / C5)

    def _convs(self):
        return [m.block[0] for m in self.model[:-1]] + [self.model[-1]]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _need_cuda(x, "Discriminator")
        convs = self._convs()
        ws = [c.weight_orig for c in convs]
        # torch spectral_norm: a power iteration per forward in train mode,
        # u / v updated in place; the forward uses clones (constants for autograd)
        training = convs[0].training
        inv = ops.sn_power(ws, [c.weight_u for c in convs], [c.weight_v for c in convs],
                           update=training)
        L = len(convs)
        if SN_FOREACH and not (torch.is_grad_enabled() and any(w.requires_grad for w in ws)):
            # no backward (the G step's D pass): nothing keeps u / v
            us, vs = [c.weight_u for c in convs], [c.weight_v for c in convs]
        elif SN_FOREACH:
            # the 2L clones as one multi-tensor launch (x * 1.0 is an exact copy)
            uv = torch._foreach_mul([c.weight_u for c in convs] + [c.weight_v for c in convs], 1.0)
            us, vs = uv[:L], uv[L:]
        else:
            us = [c.weight_u.clone() for c in convs]
            vs = [c.weight_v.clone() for c in convs]
        params = []
        for c in convs:
            params += [c.weight_orig, c.bias]
        return _DiscriminatorFn.apply(x.contiguous().float(), self._cfg, self.ainp_bf16, inv, us,
                                      vs, *params)


# ------------------------------------------------------------ losses
class _BCEConstFn(torch.autograd.Function):
    """nn.BCEWithLogitsLoss()(logits, full_like(logits, target)) (mean)."""

    @staticmethod
    def forward(ctx, logits, target):
        loss, grad = ops.bce_logits(logits.contiguous(), target, want_grad=logits.requires_grad)
        ctx.save_for_backward(grad if grad is not None else logits)
        return loss.to(torch.float32)

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return ops.scale_by_scalar(grad, g), None


def bce_with_logits_const(logits, target: float):
    return _BCEConstFn.apply(logits, float(target))


VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
             512, 512, 512, 512, "M"]


def vgg19_features() -> nn.Sequential:
    """Same module tree / state_dict keys as torchvision vgg19().features."""
    layers, in_c = [], 3
    for v in VGG19_CFG:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            conv = nn.Conv2d(in_c, v, 3, padding=1)
            nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
            nn.init.constant_(conv.bias, 0)
            layers += [conv, nn.ReLU(inplace=True)]
            in_c = v
    return nn.Sequential(*layers)


class VGGLoss(nn.Module):
    """loss.py:6-131.  The pretrained VGG19_Weights.DEFAULT cannot be fetched
    offline: pass `weights` (a torchvision vgg19 features state_dict, or a path
    to one saved with torch.save, loaded with weights_only=True) to use them;
    otherwise the features keep torchvision's own random init."""

    def __init__(self, device, layer_indices_style=(0, 5, 10, 19, 28),
                 layer_indices_perceptual=(2, 7, 12, 21, 30), weights=None):
        super().__init__()
        vgg = vgg19_features()
        if weights is not None:
            sd = torch.load(weights, map_location="cpu", weights_only=True) \
                if isinstance(weights, (str, Path)) else weights
            vgg.load_state_dict(sd)
        vgg = vgg.to(device).eval()
        for p in vgg.parameters():
            p.requires_grad = False
        self.vgg_layers = vgg
        self.layer_indices_style = set(layer_indices_style)
        self.layer_indices_perceptual = set(layer_indices_perceptual)
        idx = list(layer_indices_style) + list(layer_indices_perceptual)
        self.max_layer_idx = max(idx) if idx else -1
        self._tables = {}
        self.ainp_bf16 = False   # set_compute_dtype(): bf16 conv / Gram operands (C4 / C5)

    def _prep_tables(self, H, W, device, S=224, short=256):
        key = (H, W, str(device))
        t = self._tables.get(key)
        if t is None:
            nh, nw = (short, int(short * W / H)) if H <= W else (int(short * H / W), short)
            top, left = int(round((nh - S) / 2.0)), int(round((nw - S) / 2.0))
            ry0, rn, rw = ops.aa_bilinear_weights(H, nh, top, S)
            cx0, cn, cw = ops.aa_bilinear_weights(W, nw, left, S)
            t = tuple(torch.from_numpy(a).to(device) for a in (ry0, rn, rw, cx0, cn, cw))
            self._tables[key] = t
        return t

    def _prepare(self, x, generated):
        if x.dim() == 3:
            x = x.unsqueeze(1)
        if x.shape[1] != 1:
            raise ValueError(f"Input tensor must have 1 channel here, got {x.shape[1]}")
        x = x.contiguous().float()
        tables = self._prep_tables(x.shape[2], x.shape[3], x.device)
        comm = getattr(self, "comm", None)
        if not generated and comm is not None and comm.world_size > 1:
            # loss.py:78 scales by the max over the WHOLE batch: MAX-all-reduce it
            mx = comm.allreduce_max_(ops.vgg_target_max(x))
            return ops.vgg_prep(x, generated, tables, target_max=mx)
        return ops.vgg_prep(x, generated, tables)

    def _extract_features(self, x, tape=None) -> Dict[int, torch.Tensor]:
        """loss.py:41-51 incl. the inplace-ReLU effect: a collected conv output
        is the post-ReLU value unless the loop stops right after it.  tape (the
        generated batch's input gradient, _VGGLossFn): every executed layer as
        (kind, layer, input, output, feature indices of its output)."""
        feats = {}
        want = self.layer_indices_style | self.layer_indices_perceptual
        layers = list(self.vgg_layers)
        i = 0
        with ops.nhwc16_memo() if tape is None else _nullctx():
            while i < len(layers):
                lay = layers[i]
                xin = x
                if isinstance(lay, nn.Conv2d):
                    relu_next = (i < self.max_layer_idx and i + 1 < len(layers)
                                 and isinstance(layers[i + 1], nn.ReLU))
                    # bf16: a conv feeding the next conv directly (no max-pool between)
                    # also writes that conv's channel-last bf16 source
                    j = i + 2 if relu_next else i + 1
                    nxt16 = (self.ainp_bf16 and j <= self.max_layer_idx and j < len(layers)
                             and isinstance(layers[j], nn.Conv2d) and tape is None)
                    x, _ = ops.conv_gen((x, None), lay.weight, stride=1, pad=1, bias=lay.bias,
                                        act=ops.ACT_RELU if relu_next else ops.ACT_NONE,
                                        bf16=self.ainp_bf16, out16=nxt16)
                    idx = [i]
                    if i in want:
                        feats[i] = x
                    if relu_next:
                        i += 1          # the ReLU ran inside the conv epilogue
                        idx.append(i)
                        if i in want:
                            feats[i] = x
                    if tape is not None:
                        tape.append(("conv", lay, xin, x, relu_next, [q for q in idx if q in want]))
                elif isinstance(lay, nn.MaxPool2d):
                    # bf16: the pooled plane's channel-last copy for the next conv
                    nxt16 = (self.ainp_bf16 and tape is None and i + 1 <= self.max_layer_idx
                             and i + 1 < len(layers) and isinstance(layers[i + 1], nn.Conv2d))
                    x = ops.maxpool2(x, out16=nxt16)
                    if i in want:
                        feats[i] = x
                    if tape is not None:
                        tape.append(("pool", lay, xin, x, False, [i] if i in want else []))
                if i >= self.max_layer_idx:
                    break
                i += 1
        return feats

    def _gram(self, x):
        """Gram matrices F F^T / (c h w) (loss.py:53-62), split-K over h*w."""
        b, c, h, w = x.shape
        hw = h * w
        g = torch.empty(b, c, c, device=x.device)
        ops.gemm_batched_splitk(c, c, hw, [x[i] for i in range(b)], hw, 1,
                                [x[i] for i in range(b)], 1, hw, g, alpha=1.0 / (c * hw),
                                per_batch_out=True, bf16=self.ainp_bf16)
        return g

    def forward(self, generated, target):
        """loss.py:89-131 -> (perceptual, style).  With autograd on and a
        generated batch that requires grad (the generator training of
        fix_generator_grad) the losses carry its input gradient through VGG19
        (_VGGLossFn); otherwise no graph is built (the reference's loop)."""
        _need_cuda(generated, "VGGLoss")
        if torch.is_grad_enabled() and generated.requires_grad:
            return _VGGLossFn.apply(generated, target, self)
        with torch.no_grad():
            return self._losses(generated, target)

    def _losses(self, generated, target, keep=None):
        """keep (dict, _VGGLossFn): the generated batch's layer tape, features,
        Gram matrices and prepared input for the backward."""
        xg, xt = self._prepare(generated, True), self._prepare(target, False)
        tape = [] if keep is not None else None
        B = xg.shape[0]
        if xg.shape == xt.shape:
            # one VGG pass over both batches (no normalisation layers in
            # vgg19.features: each image's features are those of its own pass)
            f = self._extract_features(torch.cat([xg, xt]), tape)
            fg = {i: v[:B] for i, v in f.items()}
            ft = {i: v[B:] for i, v in f.items()}
            split = True
        else:
            fg, ft = self._extract_features(xg, tape), self._extract_features(xt)
            split = False
        # each L1 term written into its slot of one float64 vector, summed in
        # order by one reduction per loss (no per-term scalar adds)
        p_idx = [i for i in self.layer_indices_perceptual if i in fg and i in ft]
        s_idx = [i for i in self.layer_indices_style if i in fg and i in ft]
        n_p, n_s = len(p_idx), len(s_idx)
        terms = torch.zeros(max(1, n_p + n_s), device=generated.device, dtype=torch.float64)
        grams = {}
        for k, i in enumerate(p_idx):
            ops.absdiff_mean(fg[i], ft[i], out=terms[k])
        for k, i in enumerate(s_idx):
            gg, gt = self._gram(fg[i]), self._gram(ft[i])
            ops.absdiff_mean(gg, gt, out=terms[n_p + k])
            grams[i] = (gg, gt)
        perc = terms[:n_p].sum() / n_p if n_p else terms.new_zeros(())
        style = terms[n_p:n_p + n_s].sum() / n_s if n_s else terms.new_zeros(())
        if keep is not None:
            keep.update(tape=tape, fg=fg, ft=ft, grams=grams, n_p=n_p, n_s=n_s, B=B, split=split,
                        xg_shape=tuple(generated.shape))
        return perc.to(torch.float32), style.to(torch.float32)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class _VGGLossFn(torch.autograd.Function):
    """VGGLoss.forward with the generated batch's input gradient (loss.py:
    89-131 under autograd; VGG19 frozen, the target needs no gradient):
    perceptual L1 backward sign(fg - ft) / numel, style through the Gram L1
    (sign symmetrised, times F / (c h w): bmm's backward), then back through
    the executed layers -- max-pool (first-maximum rule), ReLU (output > 0),
    conv data gradient as a conv with the flipped transposed weights -- and
    the input preparation (normalisation, repeat, antialiased resize + crop,
    clamp((x+1)/2))."""

    @staticmethod
    def forward(ctx, generated, target, vgg):
        keep = {}
        perc, style = vgg._losses(generated, target, keep)
        ctx.keep, ctx.vgg = keep, vgg
        ctx.gen = generated.detach()
        return perc, style

    @staticmethod
    def backward(ctx, gp, gs):
        keep, vgg = ctx.keep, ctx.vgg
        if keep is None:
            raise RuntimeError("VGGLoss backward ran twice through the same graph: its saved "
                               "features are released after the first backward "
                               "(retain_graph=True is not supported)")
        ctx.keep = None
        B = keep["B"]
        fg, ft = keep["fg"], keep["ft"]
        gp = gp.reshape(1).float().contiguous()
        gs = gs.reshape(1).float().contiguous()
        grams = keep["grams"]

        def feature_grad(q, g):
            """g (+)= d loss / d feature q (g: a tensor this backward owns)."""
            if keep["n_p"] and q in vgg.layer_indices_perceptual and q in fg and q in ft:
                g = ops.absdiff_grad(fg[q], ft[q], gp, 1.0 / (keep["n_p"] * fg[q].numel()),
                                     out=g, accumulate=g is not None)
            if keep["n_s"] and q in grams:
                gg, gt = grams[q]
                b, c, h, w = fg[q].shape
                sg = ops.gram_sign_sym(gg, gt, gs, 1.0 / (keep["n_s"] * gg.numel()))
                beta = 1.0 if g is not None else 0.0
                if g is None:
                    g = torch.empty_like(fg[q])
                # dF_b = (dG + dG^T)_b F_b / (c h w)   (bmm(F, F^T)'s backward)
                ops.gemm(c, h * w, c, [sg], c, 1, [fg[q]], h * w, 1, [g], h * w, 1,
                         alpha=1.0 / (c * h * w), beta=beta, strideA=c * c, strideB=c * h * w,
                         strideC=c * h * w, nstrided=b, bf16=vgg.ainp_bf16)
            return g

        g = None
        for kind, lay, xin, xout, relu, idx in reversed(keep["tape"]):
            for q in idx:
                g = feature_grad(q, g)
            if g is None:
                continue
            if keep["split"]:
                xin, xout = xin[:B], xout[:B]
            if kind == "pool":
                g = ops.maxpool2_bwd(g, xin.contiguous())
            else:
                if relu:                 # ReLU backward: the output's sign
                    g = ops.leaky_bwd(g, xout.contiguous(), 0.0)
                wt = ops.conv_weight_flip_t(lay.weight)
                g, _ = ops.conv_gen((g, None), wt, stride=1, pad=1, bf16=vgg.ainp_bf16)
        gen = ctx.gen
        if g is None:
            return torch.zeros_like(gen), None, None
        x = gen.unsqueeze(1) if gen.dim() == 3 else gen
        tables = vgg._prep_tables(x.shape[2], x.shape[3], x.device)
        gx = ops.vgg_prep_bwd(g, x.contiguous().float(), tables)
        return gx.view_as(gen), None, None


def set_compute_dtype(module: nn.Module, dtype: str = "fp32") -> nn.Module:
    """Select the GAN compute precision (the optional `accel.dtype` config
    key; not in the reference's YAML): "bf16" runs every PartialConv2d, the
    Discriminator's spectral-norm convs (forward and the backward GEMMs) and
    VGGLoss's convs / Gram GEMMs with bf16 operands and fp32 accumulation --
    BASELINE configs C4 / C5; BatchNorm statistics, the 1-channel convs, the
    losses and the weights stay fp32.  Returns the module."""
    if dtype not in ("fp32", "bf16"):
        raise ValueError(f"accel.dtype must be fp32 or bf16, got {dtype!r}")
    for m in module.modules():
        if hasattr(m, "ainp_bf16"):
            m.ainp_bf16 = dtype == "bf16"
    return module


def calculate_losses(cfg, generated_mag, original_mag, mask, d_fake_pred,
                     vgg_loss_calculator: Optional[VGGLoss] = None, comm=None):
    """train.py:33-88 -> dict of 0-dim float32 tensors (g_adv differentiable
    w.r.t. d_fake_pred).  comm (data parallel): the hole / valid L1 normalisers
    and numerators are summed over ranks, so Lv / Lh are the global-batch
    values; the mean-type terms are per-rank means (their rank average is the
    global mean, taken by the trainer for logging)."""
    lc = cfg["training"]
    adv = bce_with_logits_const(d_fake_pred, 1.0)
    mask = mask.view_as(generated_mag) if mask.dim() < generated_mag.dim() else mask
    if generated_mag.shape[1] != 1:
        generated_mag = generated_mag[:, :1]
    if original_mag.shape[1] != 1:
        original_mag = original_mag[:, :1]
    if torch.is_grad_enabled() and generated_mag.requires_grad:
        # generator training (fix_generator_grad): the three terms carry the
        # gradient w.r.t. the generated magnitude (train.py:49-63 under autograd)
        rec = _ReconFn.apply(generated_mag.contiguous().float(), original_mag.contiguous().float(),
                             mask.contiguous().float(), comm)
    elif comm is not None and comm.world_size > 1:
        sums = comm.allreduce_sum_(ops.gan_recon_sums(generated_mag.contiguous().float(),
                                                      original_mag.contiguous().float(),
                                                      mask.contiguous().float()))
        rec = ops.gan_recon_from_sums(sums, generated_mag.numel() * comm.world_size)
    else:
        rec = ops.gan_recon_losses(generated_mag.contiguous().float(),
                                   original_mag.contiguous().float(), mask.contiguous().float())
    rec = rec.to(torch.float32)
    l1v, l1h, lw = rec[0], rec[1], rec[2]
    dev = generated_mag.device
    perc = torch.zeros((), device=dev)
    style = torch.zeros((), device=dev)
    if vgg_loss_calculator is not None and (lc["lambda_vgg_perceptual"] > 0
                                            or lc["lambda_vgg_style"] > 0):
        perc, style = vgg_loss_calculator(generated_mag, original_mag)
    total = (lc["lambda_adv"] * adv + lc["lambda_l1_valid"] * l1v + lc["lambda_l1_hole"] * l1h
             + lc["lambda_mag_weighted"] * lw + lc["lambda_vgg_perceptual"] * perc
             + lc["lambda_vgg_style"] * style)
    return {"g_total": total, "g_adv": adv, "g_l1_valid": l1v, "g_l1_hole": l1h,
            "g_mag_weighted": lw, "g_vgg_perceptual": perc, "g_vgg_style": style}


class _ReconFn(torch.autograd.Function):
    """calculate_losses' (Lv, Lh, Lw) (train.py:49-63) as float32 [3] with the
    gradient w.r.t. the generated magnitude (ainp_gan_recon_bwd).  Under DP the
    normalisers and numerators are the all-reduced global sums."""

    @staticmethod
    def forward(ctx, g, o, m, comm):
        sums = ops.gan_recon_sums(g, o, m)
        ws = 1
        if comm is not None and comm.world_size > 1:
            comm.allreduce_sum_(sums)
            ws = comm.world_size
        n_total = g.numel() * ws
        ctx.save_for_backward(g, o, m, sums)
        ctx.n_total = n_total
        ctx.ws = ws
        return ops.gan_recon_from_sums(sums, n_total).to(torch.float32)

    @staticmethod
    def backward(ctx, gout):
        g, o, m, sums = ctx.saved_tensors
        # Under DP the three terms are global-batch values, so this rank's
        # gradient is already its full share of d(global loss); the trainer's
        # reducer then SUMs over ranks and divides by world_size (the averaging
        # the per-rank-mean terms need).  Pre-scaling by world_size here makes
        # that average return exactly d(global L1 terms)/d(theta).
        gout = gout.float()
        if ctx.ws > 1:
            gout = gout * float(ctx.ws)
        return (ops.gan_recon_bwd(g, o, m, sums, gout.contiguous(), ctx.n_total),
                None, None, None)


def find_latest_checkpoint(checkpoint_dir: Path):
    """train.py:90-129 (file-name logic only)."""
    checkpoint_dir = Path(checkpoint_dir)
    latest_epoch, latest_opt = -1, None
    opt_files = list(checkpoint_dir.glob("*.pth"))
    if not opt_files:
        return None, None, None, -1
    for f in opt_files:
        m = re.search(r"optimizers_epoch_(\d+).pth", f.name)
        if m and int(m.group(1)) > latest_epoch:
            latest_epoch, latest_opt = int(m.group(1)), f
    if latest_epoch == -1:
        return None, None, None, -1
    gen = checkpoint_dir / f"generator_epoch_{latest_epoch:04d}.pth"
    disc = checkpoint_dir / f"discriminator_epoch_{latest_epoch:04d}.pth"
    if gen.exists() and disc.exists() and latest_opt.exists():
        return gen, disc, latest_opt, latest_epoch
    cands = [f for f in opt_files if re.search(r"optimizers_epoch_(\d+).pth", f.name)]
    cands.sort(key=lambda f: int(re.search(r"optimizers_epoch_(\d+).pth", f.name).group(1)),
               reverse=True)
    for f in cands:
        e = int(re.search(r"optimizers_epoch_(\d+).pth", f.name).group(1))
        g_ = checkpoint_dir / f"generator_epoch_{e:04d}.pth"
        d_ = checkpoint_dir / f"discriminator_epoch_{e:04d}.pth"
        if g_.exists() and d_.exists():
            return g_, d_, f, e
    return None, None, None, -1
