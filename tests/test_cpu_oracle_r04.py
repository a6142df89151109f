"""Round-4 fixture sanity (CPU): cnnblstm_c2_bf16emu.npz, the reference model
with the bf16 configuration's rounding points emulated
(tests/golden/gen_golden_r04.py).  The GPU gate (tests/test_gpu_model.py::
test_bf16_c2_batch32_forward_backward_tracks_reference) compares the HIP bf16
path with these gradients; here: the fixture covers every parameter, the
emulation's fp32-vs-fp64 floor is far below that gate, and the emulated loss
sits within bf16 distance of the reference's fp32 loss."""
import os

import numpy as np

BN_FED = {"encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "decoder.0.bias",
          "decoder.3.bias"}


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


def test_bf16emu_fixture_covers_c2_and_floor_is_small(golden_dir):
    emu = np.load(os.path.join(golden_dir, "cnnblstm_c2_bf16emu.npz"), allow_pickle=False)
    ref = np.load(os.path.join(golden_dir, "cnnblstm_c2.npz"), allow_pickle=False)
    names = sorted(k[len("gnorm/"):] for k in ref.files if k.startswith("gnorm/"))
    assert len(names) == 48
    for tag in ("emu32", "emu64"):
        for k in names:
            assert np.isfinite(emu[f"{tag}/gsample/{k}"]).all(), (tag, k)
            assert emu[f"{tag}/gsample/{k}"].shape == ref["gsample/" + k].shape, k
    worst = 0.0
    for k in names:
        if k in BN_FED:
            continue
        floor = rel(emu["emu32/gsample/" + k], emu["emu64/gsample/" + k])
        worst = max(worst, floor)
        # bf16 rounding moves the gradients (ill-conditioned model: saturated
        # random-init gates), but not beyond 50 % -- the encoder's, behind
        # three rounded activations (incl. the bf16-stored pre-BN outputs),
        # move most: 0.32-0.45
        assert rel(emu["emu32/gsample/" + k], ref["gsample/" + k]) < 0.5, k
    assert worst < 1e-2, worst
    assert abs(emu["emu32/loss"][0] - ref["loss"][0]) / ref["loss"][0] < 2e-3
    assert abs(emu["emu64/loss"][0] - emu["emu32/loss"][0]) / emu["emu64/loss"][0] < 1e-4


def test_gstep_fixture_fp32_and_fp64_runs_agree(golden_dir):
    """gan_gstep_small.npz (tests/golden/gen_golden_r04.py gstep): the
    reference G-step in fp32 and fp64 agree to 1e-4 on every G gradient (so
    the GPU test's 1e-4 gate against the fp64 run is meaningful), and every
    trainable G parameter of the reduced generator has a gradient."""
    f = np.load(os.path.join(golden_dir, "gan_gstep_small.npz"), allow_pickle=False)
    names = [k[len("r32/g_grad/"):] for k in f.files if k.startswith("r32/g_grad/")]
    assert len(names) == 43   # 7 + 6 blocks x (conv W, BN gamma, beta) + 2 x (W, b)
    for k in names:
        assert rel(f["r32/g_grad/" + k], f["r64/g_grad/" + k]) < 1e-4, k
        assert np.linalg.norm(f["r64/g_grad/" + k]) > 0, k
    assert abs(f["r32/loss/g_total"][0] - f["r64/loss/g_total"][0]) < 1e-5
