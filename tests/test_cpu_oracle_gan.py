"""Pin the GAN oracle (oracle/gan_ref.py) against fixtures produced by the
reference's own models/GAN/networks.py (tests/golden/gen_golden_gan.py).
CPU only: these tests make the oracle trustworthy as the checker of the HIP
GAN path (tests/test_gpu_gan.py)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import gan_ref as R


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def small(golden_dir):
    return np.load(os.path.join(golden_dir, "gan_small.npz"), allow_pickle=False)


def _pdict(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.array(g[k])).clone()
            for k in g.files if k.startswith(prefix)}


def test_partial_conv_cases(small):
    for ci in range(4):
        cin, cout, k, s, p, hb = [int(v) for v in small[f"pc{ci}/cfg"]]
        w = torch.from_numpy(small[f"pc{ci}/w"])
        b = torch.from_numpy(small[f"pc{ci}/b"]) if hb else None
        y, um = R.pconv(torch.from_numpy(small[f"pc{ci}/x"]), torch.from_numpy(small[f"pc{ci}/m"]),
                        w, b, s, p)
        assert rel(y, small[f"pc{ci}/y"]) < 1e-6, ci
        np.testing.assert_array_equal(um.numpy(), small[f"pc{ci}/um"])


def test_generator_small_forward_and_bn_stats(small):
    from golden.gen_golden_gan import SMALL_DEC, SMALL_ENC
    p = _pdict(small, "g_init/")
    with torch.no_grad():
        y = R.generator(p, torch.from_numpy(small["g_x"]), torch.from_numpy(small["g_mask"]),
                        True, SMALL_ENC, SMALL_DEC)
    assert rel(y, small["g_y"]) < 1e-5
    after = _pdict(small, "g_after/")
    for k, v in after.items():
        if "running" in k:
            assert rel(p[k], v) < 1e-5, k
        elif k.endswith("num_batches_tracked"):
            assert int(p[k]) == int(v) == 1


def test_discriminator_small_step(small):
    from golden.gen_golden_gan import SMALL_D
    p = _pdict(small, "d_init/")
    keys = R.d_trainable_keys(p)
    for k in keys:
        p[k].requires_grad_(True)
    opt = torch.optim.Adam([p[k] for k in keys], lr=2e-4, betas=(0.5, 0.999))
    dr = R.discriminator(p, torch.from_numpy(small["d_real_in"]), True, SMALL_D)
    after1 = _pdict(small, "d_after_fwd1/")
    for k in after1:
        if k.endswith("weight_u") or k.endswith("weight_v"):
            assert rel(p[k].detach(), after1[k]) < 1e-5, k
    lr_ = F.binary_cross_entropy_with_logits(dr, torch.ones_like(dr))
    df = R.discriminator(p, torch.from_numpy(small["d_fake_in"]), True, SMALL_D)
    lf = F.binary_cross_entropy_with_logits(df, torch.zeros_like(df))
    dl = (lr_ + lf) / 2
    dl.backward()
    assert rel(dr.detach(), small["d_real_logits"]) < 1e-5
    assert rel(df.detach(), small["d_fake_logits"]) < 1e-5
    assert abs(dl.item() - small["d_loss"][0]) < 1e-5 * abs(small["d_loss"][0])
    for k in keys:
        assert rel(p[k].grad, small["d_grad/" + k]) < 1e-4, k
    opt.step()
    after = _pdict(small, "d_after_step/")
    for k, v in after.items():
        assert rel(p[k].detach(), v) < 1e-5, k


def test_full_generator_and_discriminator(golden_dir):
    g = np.load(os.path.join(golden_dir, "gan_full.npz"), allow_pickle=False)
    p = R.init_generator(0)
    for k, v in p.items():
        assert abs(float(v.double().sum()) - g["check/" + k][0]) <= 1e-6 * max(1, abs(g["check/" + k][0])), k
    x, m = torch.from_numpy(g["x"]), torch.from_numpy(g["mask"])
    with torch.no_grad():
        y = R.generator(p, x, m, True)
    yf = y.numpy().reshape(-1)
    assert rel(yf[::97], g["y_sample"]) < 1e-4
    assert abs(np.linalg.norm(yf.astype(np.float64)) - g["y_norm"][0]) < 1e-4 * g["y_norm"][0]
    d = R.init_discriminator(1)
    with torch.no_grad():
        logits = R.discriminator(d, x, True)
    assert rel(logits, g["d_logits"]) < 1e-5


def test_vgg_prepare_geometry():
    """ImageClassification geometry at the C4/C5 shapes: resize
    257 x T -> 256 x int(256*T/257), centre crop offsets (16, 200) / (16, 386)."""
    assert R.resized_size(257, 626) == (256, 623)
    assert R.resized_size(257, 1001) == (256, 997)
    x = torch.rand(2, 1, 257, 626) * 2 - 1
    v = R.vgg_prepare(x, True)
    assert v.shape == (2, 3, 224, 224)
    assert int(round((623 - 224) / 2.0)) == 200 and int(round((997 - 224) / 2.0)) == 386


def test_vgg_feature_relu_semantics():
    """Collected features are post-ReLU (torchvision inplace ReLU), except
    index 30 where loss.py's loop breaks before ReLU 31."""
    p = R.vgg19_init(0)
    x = torch.randn(1, 3, 32, 32)
    f = R.vgg_features(p, x)
    for i in (0, 2, 5, 7, 10, 12, 19, 21, 28):
        assert float(f[i].min()) >= 0.0, i
    assert float(f[30].min()) < 0.0


def test_product_modules_match_reference_init(golden_dir):
    """ainp.gan modules: same state_dict keys and init RNG draws as networks.py."""
    from ainp import gan as G
    g = np.load(os.path.join(golden_dir, "gan_full.npz"), allow_pickle=False)
    torch.manual_seed(0)
    sd = G.PConvUNet().state_dict()
    assert sorted(sd) == sorted(k[6:] for k in g.files if k.startswith("check/"))
    for k, v in sd.items():
        assert abs(float(v.double().sum()) - g["check/" + k][0]) <= 1e-6 * max(1, abs(g["check/" + k][0])), k
    torch.manual_seed(1)
    sd = G.Discriminator().state_dict()
    assert sorted(sd) == sorted(k[7:] for k in g.files if k.startswith("dcheck/"))
    for k, v in sd.items():
        assert abs(float(v.double().sum()) - g["dcheck/" + k][0]) <= 1e-6 * max(1, abs(g["dcheck/" + k][0])), k
    # VGG19 features: torchvision's key layout
    v = G.VGGLoss("cpu")
    assert "vgg_layers.28.weight" in v.state_dict() and "vgg_layers.34.bias" in v.state_dict()
