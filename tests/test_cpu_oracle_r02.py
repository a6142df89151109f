"""Pin the oracle against the round-2 fixtures made by the reference's own
model.py / networks.py (tests/golden/gen_golden_r02.py): the C2 batch of 32,
the 30-step loss curve, the 8 s / T=1001 GAN shapes and the full-size GAN
step.  CPU only; these make the oracle trustworthy as the checker of the
GPU tests at the same shapes (tests/test_gpu_model.py, test_gpu_gan.py)."""
import os

import numpy as np
import torch

from oracle import cnnblstm_ref as C
from oracle import gan_ref as R


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_oracle_loss_curve_30_steps(golden_dir):
    from ainp.smoke import small_config
    g = np.load(os.path.join(golden_dir, "cnnblstm_curve.npz"), allow_pickle=False)
    cfgv = g["config"]
    n_fft, hop, win, H, L, N, T, steps = [int(v) for v in cfgv]
    p = {k[len("init/"):]: torch.from_numpy(np.array(g[k])).clone() for k in g.files
         if k.startswith("init/")}
    tr = C.Trainer(p, H, L, lr=1e-4)
    data = [tuple(torch.from_numpy(g[f"{n}{b}"]) for n in ("x", "mask", "target"))
            for b in range(4)]
    losses = [float(tr.step(*data[s % 4])[1]) for s in range(steps)]
    assert np.max(np.abs(np.array(losses) - g["losses"]) / g["losses"]) < 1e-5
    for k, v in p.items():
        if not k.endswith("num_batches_tracked"):
            assert rel(v.detach(), g["final/" + k]) < 1e-4, k


def test_oracle_c2_batch32_forward_loss(golden_dir):
    from golden.gen_golden_r02 import c2_config, c2_inputs, checksum
    g = np.load(os.path.join(golden_dir, "cnnblstm_c2.npz"), allow_pickle=False)
    cfg = c2_config()
    x, m, t, starts = c2_inputs()
    np.testing.assert_array_equal(starts, g["starts"])
    assert np.allclose(checksum(x), g["x_check"], rtol=1e-12, atol=0)
    p = C.init_params(cfg, 0)
    for k, v in p.items():
        assert np.allclose(checksum(v.numpy()), g["check/" + k], rtol=1e-9, atol=1e-12), k
    with torch.no_grad():
        y = C.forward(p, torch.from_numpy(x).unsqueeze(1), 128, 3)
        loss = C.loss_fn(y, torch.from_numpy(m), torch.from_numpy(t))
    assert rel(y.numpy().reshape(-1)[::97], g["y_sample"]) < 1e-5
    assert abs(float(loss) - g["loss"][0]) <= 1e-5 * g["loss"][0]


def test_oracle_gan_t1001(golden_dir):
    g = np.load(os.path.join(golden_dir, "gan_t1001.npz"), allow_pickle=False)
    pg = R.init_generator(0)
    pd = R.init_discriminator(1)
    x, m = torch.from_numpy(g["x"]), torch.from_numpy(g["mask"])
    with torch.no_grad():
        y = R.generator(pg, x, m, True)
        logits = R.discriminator(pd, x)
    assert tuple(y.shape) == tuple(int(v) for v in g["y_shape"])
    assert rel(y.numpy().reshape(-1)[::97], g["y_sample"]) < 1e-5
    assert rel(logits, g["d_logits"]) < 1e-5
    for k in g.files:
        if k.startswith("g_after/"):
            assert rel(pg[k[len("g_after/"):]], g[k]) < 1e-5, k
        if k.startswith("d_after/"):
            assert rel(pd[k[len("d_after/"):]], g[k]) < 1e-5, k


def test_oracle_gan_full_step_d_side(golden_dir):
    """The reference-structured D step at B=2, T=626 (the VGG-free part of the
    fixture; its VGG terms were produced by this oracle, so they pin nothing)."""
    from golden.gen_golden_r02 import GSTEP, checksum, gan_step_inputs
    g = np.load(os.path.join(golden_dir, "gan_step_full.npz"), allow_pickle=False)
    orig, imp, mask = gan_step_inputs()
    assert np.allclose(checksum(orig), g["orig_check"], rtol=1e-12, atol=0)
    pg = R.init_generator(GSTEP["g_seed"])
    pd = R.init_discriminator(GSTEP["d_seed"])
    st = R.GanStep(pg, pd, None)
    out = st.step(torch.from_numpy(orig), torch.from_numpy(imp), torch.from_numpy(mask))
    gf = out["generated"].numpy().reshape(-1)
    assert rel(gf[::97], g["gen_sample"]) < 1e-5
    assert abs(float(out["d_loss"]) - g["d_losses"][0]) <= 1e-5 * abs(g["d_losses"][0])
    for k in ("g_adv", "g_l1_valid", "g_l1_hole", "g_mag_weighted"):
        r = float(g["oracle_loss/" + k][0])
        assert abs(float(out[k]) - r) <= 1e-5 * abs(r), k
    for k in g.files:
        if k.startswith("g_after/"):
            assert rel(pg[k[len("g_after/"):]], g[k]) < 1e-5, k
