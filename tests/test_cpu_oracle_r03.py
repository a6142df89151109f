"""Pin the oracle against the round-3 fixtures made by the reference's own
model.py / networks.py (tests/golden/gen_golden_r03.py): the loss curve with
the BN-fed conv biases frozen, and the C5-shape GAN step (B=2, 8 s, T=1001,
0.1 s gaps).  CPU only; the GPU tests at the same shapes use this oracle and
these fixtures as their checker."""
import os

import numpy as np
import torch

from oracle import cnnblstm_ref as C
from oracle import gan_ref as R


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_oracle_loss_curve_frozen_bn_biases(golden_dir):
    g = np.load(os.path.join(golden_dir, "cnnblstm_curve_fixbias.npz"), allow_pickle=False)
    n_fft, hop, win, H, L, N, T, steps = [int(v) for v in g["config"]]
    frozen = [str(k) for k in g["frozen"]]
    p = {k[len("init/"):]: torch.from_numpy(np.array(g[k])).clone() for k in g.files
         if k.startswith("init/")}
    tr = C.Trainer(p, H, L, lr=1e-4, frozen=frozen)
    data = [tuple(torch.from_numpy(g[f"{n}{b}"]) for n in ("x", "mask", "target"))
            for b in range(4)]
    losses = [float(tr.step(*data[s % 4])[1]) for s in range(steps)]
    assert np.max(np.abs(np.array(losses) - g["losses"]) / g["losses"]) < 1e-5
    for k, v in p.items():
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(g["final/" + k])
        elif k in frozen:
            assert torch.equal(v.detach(), torch.from_numpy(g["init/" + k])), k
            assert np.array_equal(g["final/" + k], g["init/" + k]), k
        else:
            # running_mean included: no absolute allowance with the biases frozen
            assert rel(v.detach(), g["final/" + k]) < 1e-4, k


def test_oracle_gan_step_t1001_d_side(golden_dir):
    """The reference-structured D step at the C5 shape (B=2, T=1001, g=1600);
    the VGG-free G-step losses (its VGG terms were produced by this oracle)."""
    from golden.gen_golden_r02 import checksum
    from golden.gen_golden_r03 import GSTEP1001, gan_step1001_inputs
    g = np.load(os.path.join(golden_dir, "gan_step_t1001.npz"), allow_pickle=False)
    orig, imp, mask = gan_step1001_inputs()
    assert orig.shape == (2, 1, 257, 1001)
    assert np.allclose(checksum(orig), g["orig_check"], rtol=1e-12, atol=0)
    assert np.allclose(checksum(mask), g["mask_check"], rtol=1e-12, atol=0)
    # 0.1 s at hop 128: 13-14 hole frames per example
    holes = (mask[:, 0, 0] == 0).sum(-1)
    assert set(holes.tolist()) <= {13, 14}, holes
    pg = R.init_generator(GSTEP1001["g_seed"])
    pd = R.init_discriminator(GSTEP1001["d_seed"])
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
