"""CPU-only checks: the C-ABI library loads and exports every symbol that
include/ainp.h declares (no kernel launches), and host-side glue is sound."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ainp.h")
LIB = os.path.join(ROOT, "ml-audio-inpainting_amd", "ainp", "libainp.so")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ainp_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("ainp_stft_features", "ainp_gemm_f32", "ainp_conv3x3_fwd", "ainp_lstm_rec_fwd",
              "ainp_lstm_rec_bwd", "ainp_adam", "ainp_l1_pow10_loss"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build libainp.so first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (ainp_[a-z0-9_]+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_ctypes_binding_covers_header():
    import ainp
    from ainp import _lib
    assert set(_lib.EXPORTED) == set(declared_symbols())
    assert _lib.lib.ainp_build_target().decode() == "gfx950"
    assert _lib.lib.ainp_abi_version() >= 1


def test_library_contains_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", LIB],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob


def test_size_queries_are_pure_host():
    from ainp import _lib
    assert _lib.lib.ainp_conv3x3_fwd_stat_parts(32, 257, 334) == 32 * 33 * 7
    assert _lib.lib.ainp_conv3x3_wgrad_workspace(32, 32, 64, 257, 334) > 0
    assert _lib.lib.ainp_bn_relu_bwd_workspace(32, 64, 257, 334) > 0


def test_bad_arguments_fail_without_launching():
    """Argument validation happens before any HIP call (no GPU needed)."""
    from ainp import _lib
    rc = _lib.lib.ainp_conv3x3_fwd(None, None, None, None, None, None, None, 1, 1, 1, 1, 1, None)
    assert rc == -1
    assert b"bad argument" in _lib.lib.ainp_last_error()
    rc = _lib.lib.ainp_lstm_rec_fwd(None, None, None, None, None, 1, 1, 128, None)
    assert rc == -1
    # generator backward (csrc/gan_bwd.hip): shapes checked before any launch
    rc = _lib.lib.ainp_pconv_src_grad(None, 1, 4, 8, 8, 0, 2, 3, 3, None, None, 0, None)
    assert rc == -1 and b"pconv_src_grad" in _lib.lib.ainp_last_error()
    rc = _lib.lib.ainp_gen_act_bwd(None, 4, 4, None, 2, 0.2, None, 1, 1, 4, 4, 16, None, None,
                                   None)
    assert rc == -1 and b"gen_act_bwd" in _lib.lib.ainp_last_error()
    assert _lib.lib.ainp_bn_act_bwd_workspace(2, 64, 10000) == 2 * 64 * 3 * 16
    # bf16 dy storage: refused without the bf16 arithmetic flag, before any launch
    rc = _lib.lib.ainp_conv3x3_dgrad_ex(1, 1, 1, None, 1, 16, 32, 8, 8, 4, None)
    assert rc == -1 and b"bad argument" in _lib.lib.ainp_last_error()
    rc = _lib.lib.ainp_bn_relu_bwd_apply_ex(None, None, None, None, None, None, None, 1, None,
                                            None, None, 1, 1, 1, 1, 0, 1, None)
    assert rc == -1
    # fused data gradient + BatchNorm reduce: a channel count the channel-last
    # reduce has no instance for (24) is refused up front, not in the fallback
    for cin in (8, 24, 48):
        rc = _lib.lib.ainp_conv3x3_dgrad_bnr(16, 16, 16, 1, cin, 2 * cin, 8, 8, 64, 16, 16, 16,
                                             16, 16, 16, 0, None)
        assert rc == -1 and b"C in {16, 32, 64}" in _lib.lib.ainp_last_error(), cin


def test_dy16_routing_query():
    """ainp_conv3x3_dy16_ok (host-only): the CNNBLSTM's 16/32/64-channel convs
    take a bf16 dy in both gradients; the 1 <-> 16 channel ones (exact fp32
    kernels) and passes wider than 32 input channels do not."""
    from ainp import _lib
    q = _lib.lib.ainp_conv3x3_dy16_ok
    for cin, cout in ((16, 32), (32, 16), (32, 64)):
        assert q(32, cin, cout, 257, 334) == 1, (cin, cout)
    for cin, cout in ((1, 16), (16, 1), (64, 32), (8, 24)):
        assert q(32, cin, cout, 257, 334) == 0, (cin, cout)
    # bf16 pre-BN storage: forward (act(x) source, y) + the weight gradient's source
    q = _lib.lib.ainp_conv3x3_io16_ok
    for cin, cout in ((16, 32), (32, 16), (32, 64)):
        assert q(32, cin, cout, 257, 334) == 1, (cin, cout)
    for cin, cout in ((1, 16), (16, 1), (64, 32), (8, 24)):
        assert q(32, cin, cout, 257, 334) == 0, (cin, cout)
    rc = _lib.lib.ainp_conv3x3_fwd_ex(1, 1, None, None, None, 1, None, 1, 16, 32, 8, 8, 16, None)
    assert rc == -1          # AINP_CONV_Y16 without the bf16 arithmetic
    # channel-last activations (round 5): every conv of the model, none other
    q = _lib.lib.ainp_conv3x3_cl_ok
    for cin, cout in ((1, 16), (16, 32), (32, 64), (32, 16), (16, 1)):
        assert q(32, cin, cout, 257, 334) == 1, (cin, cout)
    for cin, cout in ((2, 16), (16, 2), (64, 32), (8, 24), (16, 16)):
        assert q(32, cin, cout, 257, 334) == 0, (cin, cout)
    # an unknown flag bit is refused before any launch (256 = AINP_CONV_YCFNT:
    # data gradients only)
    rc = _lib.lib.ainp_conv3x3_fwd_ex(1, 1, None, None, None, 1, None, 1, 16, 32, 8, 8, 256, None)
    assert rc == -1
    # round 6: dx as [C][H][N][W] -- the decoder's 16 -> 32 conv (dy 32, dx 16) only
    q = _lib.lib.ainp_conv3x3_dgrad_cfnt_ok
    assert q(32, 16, 32, 257, 334) == 1
    for cin, cout in ((32, 16), (32, 64), (1, 16), (16, 1), (16, 64)):
        assert q(32, cin, cout, 257, 334) == 0, (cin, cout)
    rc = _lib.lib.ainp_conv3x3_dgrad_ex(1, 1, 1, None, 1, 32, 16, 8, 8, 256, None)
    assert rc == -1 and b"YCFNT" in _lib.lib.ainp_last_error()
    rc = _lib.lib.ainp_conv3x3_dgrad_ex(1, 1, 1, None, 1, 16, 32, 8, 8, 256 | 64, None)
    assert rc == -1 and b"bad argument" in _lib.lib.ainp_last_error()
    # the fused first-conv weight gradient + BatchNorm apply: Conv2d(1, 16) only
    rc = _lib.lib.ainp_conv3x3_wgrad_bnapply(16, None, None, 16, 16, 16, 16, None, 16, 16, 8, 16,
                                             16, 16, 16, 16, 1, 16, 32, 8, 8, None)
    assert rc == -1 and b"wgrad_bnapply" in _lib.lib.ainp_last_error()
    rc = _lib.lib.ainp_conv3x3_dgrad_bnapply(16, 16, 16, 16, 16, None, 16, 16, 8, 16, 0, 16, 16,
                                             1, 32, 1, 8, 8, None)
    assert rc == -1 and b"dgrad_bnapply" in _lib.lib.ainp_last_error()


def test_ops_refuse_cpu_tensors():
    import torch
    from ainp import ops
    with pytest.raises(RuntimeError, match="GPU"):
        ops.conv3x3_fwd(torch.zeros(1, 1, 4, 4), torch.zeros(1, 1, 3, 3))


HOST_ONLY = {"ainp_abi_version", "ainp_build_target", "ainp_last_error", "ainp_reduce_workspace",
             "ainp_flac_info", "ainp_flac_decode", "ainp_flac_encode_bound", "ainp_flac_encode",
             "ainp_l1_pow10_loss_slots", "ainp_range_push", "ainp_range_pop", "ainp_mark",
             "ainp_conv16_set_variant", "ainp_conv3x3_dy16_ok", "ainp_conv3x3_io16_ok",
             "ainp_conv3x3_cl_ok", "ainp_conv3x3_dgrad_cfnt_ok"}


def test_torch_library_registers_every_gpu_entry_point():
    """b2: torch.ops.ainp.* (csrc/torch_ops.cpp) covers every launching entry
    point of include/ainp.h -- the newest form of each (_ex / _ld / _out16 variants);
    the remaining symbols are host-only queries or older forms of the same
    launch."""
    import torch
    from ainp import ops  # noqa: F401  (loads libainp_torch.so)
    names = sorted(n.split("::")[1] for n in torch._C._dispatch_get_all_op_names()
                   if n.startswith("ainp::"))
    declared = set(declared_symbols())
    covered = set()
    for n in names:
        cands = [f"ainp_{n}{suf}" for suf in ("", "_ex", "_f32_ex", "_out16", "_nhwc16")]
        hit = [c for c in cands if c in declared]
        assert hit, n
        covered.update(hit)
    older = {"ainp_gemm_f32", "ainp_gemm_f32_ws", "ainp_conv3x3_fwd", "ainp_conv3x3_dgrad",
             "ainp_conv3x3_wgrad", "ainp_conv_gen_fwd", "ainp_adam", "ainp_im2col",
             "ainp_col2im"}
    rest = {s for s in declared - covered - HOST_ONLY - older
            if not s.endswith(("_workspace", "_stat_parts", "_stat_rows", "_stat_rows_ex"))}
    assert not rest, rest
    # CUDA-key kernels only: CPU tensors stop in the dispatcher, nothing runs
    with pytest.raises(NotImplementedError):
        torch.ops.ainp.mul(torch.zeros(3), torch.zeros(3), torch.zeros(3))
