"""ctypes binding of libainp.so (the C ABI declared in include/ainp.h).

The library is the product: every call here launches a hand-written gfx950
kernel.  There is no fallback path -- if the shared object is missing or was
not built for this machine, import fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AINP_LIB", os.path.join(_HERE, "libainp.so"))


class AinpError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libainp.so not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` or "
            "`make -C ml-audio-inpainting_amd/csrc`")
    return ctypes.CDLL(LIB_PATH)


lib = _load()

P = c_void_p
PP = POINTER(c_void_p)
_SIGS = {
    "ainp_abi_version": (c_int, []),
    "ainp_build_target": (c_char_p, []),
    "ainp_last_error": (c_char_p, []),
    "ainp_range_push": (c_int, [c_char_p]),
    "ainp_range_pop": (c_int, []),
    "ainp_mark": (None, [c_char_p]),
    "ainp_stft_features": (c_int, [P, c_int64, c_int64, P, P, c_int64, c_int64, c_int64,
                                   P, c_int, c_int, c_int64, c_int, P, P, P, P, P]),
    "ainp_stft": (c_int, [P, c_int, c_int64, c_int64, P, c_int, c_int, c_int, c_int64, P, P]),
    "ainp_gemm_f32": (c_int, [c_int64, c_int64, c_int64, c_float, PP, c_int64, c_int64,
                              c_int64, PP, c_int64, c_int64, c_int64, c_float, PP,
                              c_int64, c_int64, c_int64, PP, PP, c_int, c_int64, c_int, P]),
    "ainp_gemm_f32_workspace": (c_size_t, [c_int64, c_int64, c_int64, c_int, c_int64, c_int]),
    "ainp_gemm_f32_ws": (c_int, [c_int64, c_int64, c_int64, c_float, PP, c_int64, c_int64,
                                 c_int64, PP, c_int64, c_int64, c_int64, c_float, PP,
                                 c_int64, c_int64, c_int64, PP, PP, c_int, c_int64, c_int,
                                 P, c_size_t, P]),
    "ainp_gemm_f32_ex": (c_int, [c_int64, c_int64, c_int64, c_float, PP, c_int64, c_int64,
                                 c_int64, PP, c_int64, c_int64, c_int64, c_float, PP,
                                 c_int64, c_int64, c_int64, PP, PP, c_int, c_int64, c_int,
                                 c_int, P, c_size_t, P]),
    "ainp_conv3x3_fwd_stat_parts": (c_int, [c_int64, c_int64, c_int64]),
    "ainp_conv3x3_fwd_stat_rows": (c_int64, [c_int64, c_int, c_int, c_int64, c_int64]),
    "ainp_conv3x3_fwd_stat_rows_ex": (c_int64, [c_int64, c_int, c_int, c_int64, c_int64, c_int]),
    "ainp_conv3x3_fwd": (c_int, [P, P, P, P, P, P, P, c_int64, c_int, c_int, c_int64,
                                 c_int64, P]),
    "ainp_conv3x3_dgrad": (c_int, [P, P, P, P, c_int64, c_int, c_int, c_int64, c_int64, P]),
    "ainp_conv3x3_wgrad_workspace": (c_size_t, [c_int64, c_int, c_int, c_int64, c_int64]),
    "ainp_conv3x3_wgrad": (c_int, [P, P, P, P, P, P, P, c_int64, c_int, c_int, c_int64,
                                   c_int64, P]),
    "ainp_conv3x3_fwd_ex": (c_int, [P, P, P, P, P, P, P, c_int64, c_int, c_int, c_int64,
                                    c_int64, c_int, P]),
    "ainp_conv3x3_dgrad_bnr_workspace": (c_int64, [c_int64, c_int, c_int, c_int64, c_int64]),
    "ainp_conv3x3_dgrad_bnr": (c_int, [P, P, P, c_int64, c_int, c_int, c_int64, c_int64, c_int,
                                       P, P, P, P, P, P, c_int, P]),
    "ainp_conv3x3_dgrad_ex": (c_int, [P, P, P, P, c_int64, c_int, c_int, c_int64, c_int64, c_int,
                                      P]),
    "ainp_conv3x3_wgrad_ex": (c_int, [P, P, P, P, P, P, P, c_int64, c_int, c_int, c_int64,
                                      c_int64, c_int, P]),
    "ainp_bn_stats_reduce": (c_int, [P, c_int, P, c_int, P]),
    "ainp_bn_reduce_finalize": (c_int, [P, c_int, c_int64, P, P, P, P, c_float, c_float, P, P,
                                        P, c_int, P]),
    "ainp_bn_finalize": (c_int, [P, c_int64, P, P, P, P, c_float, c_float, P, P, P, c_int, P]),
    "ainp_bn_eval_affine": (c_int, [P, P, P, P, c_float, P, P, c_int, P]),
    "ainp_bn_relu_apply": (c_int, [P, P, P, P, c_int64, c_int, c_int64, c_int64, c_int, P]),
    "ainp_bn_relu_bwd_workspace": (c_size_t, [c_int64, c_int, c_int64, c_int64]),
    "ainp_bn_relu_bwd_reduce": (c_int, [P, P, P, P, P, P, P, c_int64, c_int, c_int64,
                                        c_int64, c_int, P]),
    "ainp_bn_relu_bwd_apply": (c_int, [P, P, P, P, P, P, P, c_int64, P, P, P, c_int64, c_int,
                                       c_int64, c_int64, c_int, P]),
    "ainp_bn_relu_bwd_apply_ex": (c_int, [P, P, P, P, P, P, P, c_int64, P, P, P, c_int64, c_int,
                                          c_int64, c_int64, c_int, c_int, P]),
    "ainp_conv3x3_dy16_ok": (c_int, [c_int64, c_int, c_int, c_int64, c_int64]),
    "ainp_conv3x3_io16_ok": (c_int, [c_int64, c_int, c_int, c_int64, c_int64]),
    "ainp_conv3x3_cl_ok": (c_int, [c_int64, c_int, c_int, c_int64, c_int64]),
    "ainp_conv3x3_dgrad_cfnt_ok": (c_int, [c_int64, c_int, c_int, c_int64, c_int64]),
    "ainp_conv3x3_dgrad_bnapply": (c_int, [P, P, P, P, P, P, P, P, c_int64, P, c_int, P, P,
                                           c_int64, c_int, c_int, c_int64, c_int64, P]),
    "ainp_conv3x3_wgrad_bnapply": (c_int, [P, P, P, P, P, P, P, P, P, P, c_int64, P, P, P, P, P,
                                           c_int64, c_int, c_int, c_int64, c_int64, P]),
    "ainp_bn_relu_bwd_reduce_ex": (c_int, [P, P, P, P, P, P, P, c_int64, c_int, c_int64, c_int64,
                                           c_int, c_int, P]),
    "ainp_lstm_rec_fwd": (c_int, [P, PP, P, P, P, c_int64, c_int64, c_int, P]),
    "ainp_lstm_rec_bwd": (c_int, [P, P, P, PP, P, c_int64, c_int64, c_int, P]),
    "ainp_lstm_hprev": (c_int, [P, P, c_int64, c_int64, c_int, P]),
    "ainp_l1_pow10_loss": (c_int, [P, P, P, c_int64, P, P, c_float, P]),
    "ainp_scale_by_dev": (c_int, [P, P, c_int64, P, P]),
    "ainp_sum_slabs": (c_int, [P, c_int64, c_int64, P, P]),
    "ainp_rowsum_batched": (c_int, [P, c_int64, c_int64, c_int64, P, P]),
    "ainp_colsum": (c_int, [P, c_int64, c_int64, c_int64, P, c_int, P]),
    "ainp_colsum_slabs": (c_int, [P, c_int64, c_int64, c_int64, c_int64, P, P]),
    "ainp_adam": (c_int, [PP, PP, PP, PP, POINTER(c_int64), c_int, c_double, c_double,
                          c_double, c_double, c_double, c_int64, P]),
    "ainp_adam_ex": (c_int, [PP, PP, PP, PP, POINTER(c_int64), c_int, c_double, c_double,
                             c_double, c_double, c_double, c_int64, P, P, P]),
    "ainp_conv_gen_stat_parts": (c_int, [c_int64, c_int, c_int, c_int, c_int, c_int64, c_int64]),
    "ainp_conv_weight_kmajor": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "ainp_conv_gen_workspace": (c_size_t, [c_int64, c_int, c_int, c_int, c_int, c_int64, c_int64]),
    "ainp_conv_gen_fwd": (c_int, [P, P, c_int, c_int, c_int, P, P, c_int, c_int, c_int,
                                  P, P, P, P, P, P, P, c_int64, c_int, c_int, c_int, c_int,
                                  c_int, c_int, c_int, c_int, c_float, c_int, c_int, P, P]),
    "ainp_conv_gen_fwd_ex": (c_int, [P, P, c_int, c_int, c_int, P, P, c_int, c_int, c_int,
                                     P, P, P, P, P, P, P, c_int64, c_int, c_int, c_int, c_int,
                                     c_int, c_int, c_int, c_int, c_float, c_int, c_int, c_int, P,
                                     P]),
    "ainp_conv_gen_fwd_out16": (c_int, [P, P, c_int, c_int, c_int, P, P, c_int, c_int, c_int,
                                        P, P, P, P, P, P, P, c_int64, c_int, c_int, c_int, c_int,
                                        c_int, c_int, c_int, c_int, c_float, c_int, c_int, c_int,
                                        P, P, P]),
    "ainp_pconv_mask": (c_int, [P, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int64,
                                c_int, c_int, c_int, c_int, c_int, c_int, c_float, P, P, P]),
    "ainp_gan_pad_input": (c_int, [P, P, c_int64, c_int, c_int, c_int, c_int, P, P, P]),
    "ainp_affine_act": (c_int, [P, P, P, c_int64, c_int, c_int64, c_int, c_float, P]),
    "ainp_affine_act_nhwc16": (c_int, [P, P, P, c_int64, c_int, c_int, c_int, c_int, c_float, P,
                                       P, P]),
    "ainp_affine_act_nhwc16_ex": (c_int, [P, P, P, c_int64, c_int, c_int, c_int, c_int, c_float, P,
                                          P, c_int, P]),
    "ainp_maxpool2": (c_int, [P, P, c_int64, c_int, c_int, P]),
    "ainp_maxpool2_nhwc16": (c_int, [P, P, c_int64, c_int, c_int, c_int, P, P]),
    "ainp_vgg_prep": (c_int, [P, c_int64, c_int, c_int, c_int, P, P, P, P, c_int, P, P, P,
                              c_int, c_int, P, P]),
    "ainp_reduce_workspace": (c_size_t, []),
    "ainp_absdiff_mean": (c_int, [P, P, c_int64, P, P, P]),
    "ainp_bce_logits": (c_int, [P, c_int64, c_float, P, c_float, P, P, P]),
    "ainp_gan_recon_losses": (c_int, [P, P, P, c_int64, P, P, P]),
    "ainp_gan_recon_sums": (c_int, [P, P, P, c_int64, P, P, P]),
    "ainp_vgg_target_max": (c_int, [P, c_int64, P, P]),
    "ainp_flac_info": (c_int, [P, c_size_t, P, P, P, P, P]),
    "ainp_flac_decode": (c_int, [P, c_size_t, P, c_int64, P]),
    "ainp_flac_encode_bound": (c_size_t, [c_int64, c_int, c_int]),
    "ainp_flac_encode": (c_int, [P, c_int64, c_int, c_int, c_int, P, c_size_t, P]),
    "ainp_sn_workspace": (c_size_t, [c_int, c_int]),
    "ainp_sn_power": (c_int, [PP, PP, PP, P, P, c_int, c_float, P, c_int, P, c_int, P]),
    "ainp_sn_weight_grad": (c_int, [P, c_int, P, P, P, P, c_int, c_int, P, P, P, P]),
    "ainp_im2col": (c_int, [P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                            P, P]),
    "ainp_col2im": (c_int, [P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "ainp_leaky_bwd": (c_int, [P, P, c_int64, c_float, P, P]),
    "ainp_im2col_ld": (c_int, [P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_int, c_int64, P, P]),
    "ainp_leaky_bwd_ld": (c_int, [P, P, c_int64, c_int64, c_float, c_int64, P, P]),
    "ainp_col2im_ld": (c_int, [P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_int64, P, P]),
    "ainp_mul": (c_int, [P, P, c_int64, P, P]),
    "ainp_istft_workspace": (c_size_t, [c_int64, c_int64, c_int]),
    "ainp_l1_pow10_loss_slots": (c_int64, [c_int64]),
    "ainp_gemm_x6_multi": (c_int, [P, c_int, P]),
    "ainp_gemm_bf16nt_multi": (c_int, [P, c_int, P]),
    "ainp_gl_stft_update": (c_int, [P, c_int64, c_int64, P, c_int, c_int64, P, P, c_float, c_int,
                                    P]),
    "ainp_istft": (c_int, [P, P, c_int, c_int64, c_int, c_int64, P, c_int, c_int, c_int, P, P,
                           P]),
    "ainp_gl_update": (c_int, [P, P, P, c_int64, c_float, c_int, P]),
    "ainp_channel_sum": (c_int, [P, c_int64, c_int, c_int64, P, P]),
    "ainp_bn_relu_apply_ntcf_bf16": (c_int, [P, P, P, P, P, c_int64, c_int64, c_int, c_int64,
                                             c_int64, P]),
    "ainp_bn_relu_apply_ntcf_bf16_ex": (c_int, [P, P, P, P, P, c_int64, c_int64, c_int, c_int64,
                                                c_int64, c_int, P]),
    "ainp_bn_relu_apply_ntcf_cl": (c_int, [P, P, P, P, P, P, c_int64, c_int64, c_int, c_int64,
                                           c_int64, c_int, P]),
    "ainp_gemm_bf16nt": (c_int, [c_int64, c_int64, c_int64, P, c_int64, P, c_int64, P, c_int64,
                                 P, P, P, P, c_int64, c_int, c_int64, c_int64, P]),
    "ainp_cast_bf16_t": (c_int, [P, c_int64, c_int64, c_int64, P, c_int64, P, c_int64, P]),
    "ainp_transpose_f32": (c_int, [P, c_int64, c_int64, c_int64, P, c_int64, P]),
    "ainp_gemm_x6nt_256": (c_int, [c_int64, c_int64, c_int64, P, c_int64, P, P, c_int64, c_int64,
                                   P, c_int64, P, P, P, P, c_int64, c_int, c_int64, c_int64, P]),
    "ainp_d_prep16": (c_int, [P, c_int, c_int64, P, c_float, c_int64, c_int, c_int64, P, c_int64,
                              P, P]),
    "ainp_wgrad_cout1": (c_int, [P, P, c_int, c_int64, P, c_float, c_int64, c_int, c_int, c_int,
                                 c_int, c_int, c_int, P, P, P]),
    "ainp_wgrad_cout1_workspace": (c_int64, [c_int, c_int]),
    "ainp_im2col16": (c_int, [P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              P, c_int64, P]),
    "ainp_dgrad16_weight": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "ainp_dgrad16": (c_int, [P, c_int64, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, c_int,
                             c_int, P, P, c_int, c_int64, P]),
    "ainp_wgrad16_nhwc": (c_int, [P, c_int64, c_int, P, c_int64, c_int, c_int, c_int, c_int,
                                  c_int, c_int, P, c_int, c_int64, P]),
    "ainp_dgrad16_prep": (c_int, [P, c_int64, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int,
                                  c_int, c_int, P, P, c_float, P, c_int64, P, P]),
    "ainp_nchw_to_nhwc16": (c_int, [P, P, c_int64, c_int, c_int, c_int, P, P]),
    "ainp_conv_weight_nhwc16": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "ainp_im2col_nhwc16": (c_int, [P, P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                   c_int, c_int, P, P]),
    "ainp_conv16_set_variant": (c_int, [c_int]),
    "ainp_conv_gen_fwd_nhwc16": (c_int, [P, c_int, c_int, c_int, P, c_int, c_int, c_int, P, P, P,
                                         P, P, P, c_int64, c_int, c_int, c_int, c_int, c_int,
                                         c_int, c_int, c_int, c_float, P, P]),
    "ainp_conv_gen_fwd_nhwc16_ex": (c_int, [P, c_int, c_int, c_int, P, c_int, c_int, c_int, P, P,
                                            P, P, P, P, c_int64, c_int, c_int, c_int, c_int, c_int,
                                            c_int, c_int, c_int, c_float, P, P, P]),
    # generator backward (csrc/gan_bwd.hip)
    "ainp_affine_leaky_out": (c_int, [P, P, P, c_int64, c_int, c_int64, c_float, P, P]),
    "ainp_pconv_src_materialize": (c_int, [P, P, c_int64, c_int, c_int, c_int, P, P, c_int, c_int,
                                           c_int, P, P]),
    "ainp_pconv_src_grad": (c_int, [P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    P, P, c_int, P]),
    "ainp_gen_act_bwd": (c_int, [P, c_int, c_int, P, c_int, c_float, P, c_int64, c_int, c_int,
                                 c_int, c_int64, P, P, P]),
    "ainp_bn_act_bwd_workspace": (c_size_t, [c_int64, c_int, c_int64]),
    "ainp_bn_act_bwd_reduce": (c_int, [P, P, P, P, P, c_float, c_int64, c_int, c_int64, P, P, P]),
    "ainp_bn_act_bwd_apply": (c_int, [P, P, P, P, P, P, P, c_int64, c_float, P, c_int64, c_int,
                                      c_int64, c_int64, P, P, P, P]),
    "ainp_maxpool2_bwd": (c_int, [P, P, c_int64, c_int, c_int, P, P]),
    "ainp_vgg_prep_bwd_workspace": (c_size_t, [c_int64, c_int, c_int]),
    "ainp_vgg_prep_bwd": (c_int, [P, P, c_int64, c_int, c_int, P, P, P, c_int, P, P, P, c_int,
                                  c_int, P, P, P]),
    "ainp_absdiff_grad": (c_int, [P, P, c_int64, P, c_float, P, c_int, P]),
    "ainp_gram_sign_sym": (c_int, [P, P, c_int64, c_int, P, c_float, P, P]),
    "ainp_gan_recon_bwd": (c_int, [P, P, P, c_int64, P, P, c_double, P, P]),
    "ainp_conv_weight_flip_t": (c_int, [P, c_int, c_int, c_int, P, P]),
}

EXPORTED = tuple(_SIGS)

for _name, (_res, _args) in _SIGS.items():
    _fn = getattr(lib, _name)  # AttributeError here = ABI mismatch: fail loudly
    _fn.restype = _res
    _fn.argtypes = _args


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.ainp_last_error().decode(errors="replace")
        raise AinpError(f"{what} failed ({rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib, name)(*args), name)


def ptr_array(ptrs) -> ctypes.Array:
    arr = (c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def int64_array(vals) -> ctypes.Array:
    arr = (c_int64 * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr
