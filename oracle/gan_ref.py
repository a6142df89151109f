"""torch-CPU restatement of the reference GAN training path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used by tests/ as the
checker (and pinned there against fixtures generated from the reference's own
models/GAN/networks.py); never imported by the product.

Follows, by function:
  pconv            models/GAN/networks.py:63-106   PartialConv2d.forward
  generator        models/GAN/networks.py:247-345  PConvUNet.forward (EncoderBlock /
                   DecoderBlock :139-168 = pconv -> BatchNorm2d -> LeakyReLU(0.2))
  sn_weight        torch.nn.utils.spectral_norm (compute_weight): one power
                   iteration per train-mode forward, u/v updated in place, then
                   W = W_orig / (u . W v) with u, v constants for autograd
  discriminator    models/GAN/networks.py:352-409
  vgg_prepare      models/GAN/loss.py:65-86 + torchvision ImageClassification
                   (resize shorter side 256 bilinear antialias, centre-crop 224,
                   ImageNet normalize; torchvision itself is absent here)
  vgg_losses       models/GAN/loss.py:41-131 (features collected after the in-place
                   ReLU that follows them, except index 30 where the loop stops)
  generator_losses models/GAN/train.py:33-88 (calculate_losses)
  gan_step         models/GAN/train.py:341-378
Parameters live in plain dicts keyed by the reference's state_dict names.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

ENC_CFG = [(64, 7, 2, 3), (128, 5, 2, 2), (256, 5, 2, 2),
           (512, 3, 2, 1), (512, 3, 2, 1), (512, 3, 2, 1), (512, 3, 2, 1)]
DEC_CFG = [(512, 3, 1, 1), (512, 3, 1, 1), (512, 3, 1, 1),
           (256, 3, 1, 1), (128, 3, 1, 1), (64, 3, 1, 1)]
D_CFG = [(64, 2, False), (128, 2, False), (256, 2, False), (512, 1, False)]
VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
             512, 512, 512, 512, "M"]
VGG_STYLE = (0, 5, 10, 19, 28)
VGG_PERCEPTUAL = (2, 7, 12, 21, 30)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ---------------------------------------------------------------- init
FINAL_CFG = {"interim_ch": 64, "out_ch": 1, "kernel": 3, "padding": 1}


def _pconv_init(out, pre, cin, cout, k, bias):
    """PartialConv2d.__init__ (networks.py:26-61) RNG draws: conv (kaiming
    uniform, no bias), mask_conv (drawn, then filled with 1), zero bias."""
    import torch.nn as nn
    conv = nn.Conv2d(cin, cout, k, bias=False)
    mconv = nn.Conv2d(cin, 1, k, bias=False)
    out[pre + ".conv.weight"] = conv.weight.detach().clone()
    out[pre + ".mask_conv.weight"] = torch.ones_like(mconv.weight.detach())
    if bias:
        out[pre + ".bias"] = torch.zeros(cout)


def _bn_init(out, pre, c):
    out[pre + ".weight"] = torch.ones(c)
    out[pre + ".bias"] = torch.zeros(c)
    out[pre + ".running_mean"] = torch.zeros(c)
    out[pre + ".running_var"] = torch.ones(c)
    out[pre + ".num_batches_tracked"] = torch.tensor(0)


def init_generator(seed=None, enc_cfg=ENC_CFG, dec_cfg=DEC_CFG, final_cfg=FINAL_CFG):
    """PConvUNet parameters in construction order (networks.py:194-244)."""
    if seed is not None:
        torch.manual_seed(seed)
    p, cin, chans = {}, 2, []
    for i, (c, k, s, pd) in enumerate(enc_cfg):
        _pconv_init(p, f"encoder_blocks.{i}.pconv", cin, c, k, False)
        _bn_init(p, f"encoder_blocks.{i}.norm", c)
        chans.append(c)
        cin = c
    rev = chans[::-1]
    up = rev[0]
    for i, (c, k, s, pd) in enumerate(dec_cfg):
        _pconv_init(p, f"decoder_blocks.{i}.pconv", up + rev[i + 1], c, k, False)
        _bn_init(p, f"decoder_blocks.{i}.norm", c)
        up = c
    fk = final_cfg["kernel"]
    _pconv_init(p, "final_decoder_layer.0", up + 1, final_cfg["interim_ch"], fk, True)
    _pconv_init(p, "final_decoder_layer.2", final_cfg["interim_ch"], final_cfg["out_ch"], fk, True)
    return p


def init_discriminator(seed=None, cfg=D_CFG, k=4):
    """Discriminator parameters + spectral-norm buffers (networks.py:380-407;
    torch spectral_norm draws u ~ N(0,1)^h, v ~ N(0,1)^w at wrap time)."""
    import torch.nn as nn
    if seed is not None:
        torch.manual_seed(seed)
    p, cin = {}, 1
    layers = [(c, s) for c, s, _ in cfg] + [(1, 1)]
    for i, (c, s) in enumerate(layers):
        pre = f"model.{i}.block.0" if i < len(cfg) else f"model.{i}"
        conv = nn.Conv2d(cin, c, k, s, 1, bias=True)
        w = conv.weight.detach().clone()
        h, wd = w.shape[0], w[0].numel()
        u = F.normalize(torch.empty(h).normal_(0, 1), dim=0, eps=1e-12)
        v = F.normalize(torch.empty(wd).normal_(0, 1), dim=0, eps=1e-12)
        p[pre + ".bias"] = conv.bias.detach().clone()
        p[pre + ".weight_orig"] = w
        p[pre + ".weight_u"] = u
        p[pre + ".weight_v"] = v
        cin = c
    return p


# ----------------------------------------------------------------- generator
def pconv(x, mask, w, bias, stride, padding):
    """PartialConv2d.forward (networks.py:63-106), multi_channel=False."""
    cin, k = w.shape[1], w.shape[2]
    if mask.shape[1] == 1 and cin > 1:
        mask = mask.repeat(1, cin, 1, 1)
    out = F.conv2d(x * mask, w, None, stride, padding)
    with torch.no_grad():
        upd = F.conv2d(mask, torch.ones(1, cin, k, k, dtype=mask.dtype), None, stride, padding)
    ratio = float(cin * k * k) / (upd + 1e-8)
    out = out * ratio
    if bias is not None:
        out = out + bias.view(1, -1, 1, 1)
    upd = torch.clamp(upd, 0.0, 1.0)
    if upd.shape[1] == 1 and w.shape[0] > 1:
        upd = upd.repeat(1, w.shape[0], 1, 1)
    return out, upd


def _bn_lrelu(x, p, pre, training):
    x = F.batch_norm(x, p[pre + ".running_mean"], p[pre + ".running_var"], p[pre + ".weight"],
                     p[pre + ".bias"], training=training, momentum=0.1, eps=1e-5)
    if training:
        p[pre + ".num_batches_tracked"] += 1
    return F.leaky_relu(x, 0.2)


def total_downsampling(enc_cfg=ENC_CFG):
    f = 1
    for _, _, s, _ in enc_cfg:
        if s > 1:
            f *= s
    return f


def pad_size(n, f):
    return 0 if n % f == 0 else f - n % f


def generator(p, x, mask, training=True, enc_cfg=ENC_CFG, dec_cfg=DEC_CFG):
    """PConvUNet.forward (networks.py:247-345); x, mask [B,1,H,W]."""
    _, _, H, W = x.shape
    f = total_downsampling(enc_cfg)
    pad = (0, pad_size(W, f), 0, pad_size(H, f))
    xp = F.pad(x, pad, mode="reflect")
    mp = F.pad(mask, pad, mode="constant", value=1.0)
    feat = torch.cat([xp, mp], dim=1)
    m = mp
    feats, masks = [], []
    for i, (_, k, s, pd) in enumerate(enc_cfg):
        pre = f"encoder_blocks.{i}"
        feat, m = pconv(feat, m, p[pre + ".pconv.conv.weight"], None, s, pd)
        feat = _bn_lrelu(feat, p, pre + ".norm", training)
        feats.append(feat)
        masks.append(m)
    d, dm = feats[-1], masks[-1]
    for i, (_, k, s, pd) in enumerate(dec_cfg):
        d = F.interpolate(d, scale_factor=2, mode="nearest")
        dm = F.interpolate(dm, scale_factor=2, mode="nearest")
        j = len(feats) - 2 - i
        if d.shape[2:] != feats[j].shape[2:]:
            d = F.interpolate(d, size=feats[j].shape[2:], mode="nearest")
            dm = F.interpolate(dm, size=masks[j].shape[2:], mode="nearest")
        pre = f"decoder_blocks.{i}"
        d, dm = pconv(torch.cat([d, feats[j]], 1), torch.cat([dm, masks[j]], 1),
                      p[pre + ".pconv.conv.weight"], None, s, pd)
        d = _bn_lrelu(d, p, pre + ".norm", training)
    d = F.interpolate(d, scale_factor=2, mode="nearest")
    dm = F.interpolate(dm, scale_factor=2, mode="nearest")
    if d.shape[2:] != xp.shape[2:]:
        raise RuntimeError("Size mismatch before final layer")
    d, m1 = pconv(torch.cat([d, xp], 1), torch.cat([dm, mp], 1),
                  p["final_decoder_layer.0.conv.weight"], p["final_decoder_layer.0.bias"], 1, 1)
    d = F.leaky_relu(d, 0.2)
    d, _ = pconv(d, m1, p["final_decoder_layer.2.conv.weight"], p["final_decoder_layer.2.bias"], 1, 1)
    return torch.tanh(d)[:, :, :H, :W]


# ------------------------------------------------------------- discriminator
def sn_weight(p, pre, training=True, eps=1e-12):
    """torch spectral_norm compute_weight (n_power_iterations=1, dim=0)."""
    w = p[pre + ".weight_orig"]
    u, v = p[pre + ".weight_u"], p[pre + ".weight_v"]
    wm = w.reshape(w.shape[0], -1)
    if training:
        with torch.no_grad():
            v.copy_(F.normalize(torch.mv(wm.t(), u), dim=0, eps=eps))
            u.copy_(F.normalize(torch.mv(wm, v), dim=0, eps=eps))
        u, v = u.clone(), v.clone()
    sigma = torch.dot(u, torch.mv(wm, v))
    return w / sigma


def discriminator(p, x, training=True, cfg=D_CFG):
    """Discriminator.forward (networks.py:409): 4 x [SN-conv4x4 + LeakyReLU] + SN-conv."""
    for i, (_, s, _) in enumerate(cfg):
        pre = f"model.{i}.block.0"
        x = F.conv2d(x, sn_weight(p, pre, training), p[pre + ".bias"], s, 1)
        x = F.leaky_relu(x, 0.2)
    pre = f"model.{len(cfg)}"
    return F.conv2d(x, sn_weight(p, pre, training), p[pre + ".bias"], 1, 1)


# ----------------------------------------------------------------------- VGG
def vgg19_feature_keys():
    """state_dict keys of torchvision vgg19().features: index -> (conv?)"""
    layers, i, cin = [], 0, 3
    for v in VGG19_CFG:
        if v == "M":
            layers.append(("pool", i))
            i += 1
        else:
            layers.append(("conv", i, cin, v))
            layers.append(("relu", i + 1))
            i += 2
            cin = v
    return layers


def vgg19_init(seed=0):
    """Seeded stand-in for VGG19_Weights.DEFAULT (pretrained weights cannot be
    downloaded offline): torchvision's own init for vgg19 convs is
    kaiming_normal_(fan_out, relu) weights and zero biases."""
    g = torch.Generator().manual_seed(seed)
    p = {}
    for lay in vgg19_feature_keys():
        if lay[0] == "conv":
            _, i, cin, cout = lay
            std = math.sqrt(2.0 / (cout * 9))
            p[f"{i}.weight"] = torch.randn(cout, cin, 3, 3, generator=g) * std
            p[f"{i}.bias"] = torch.randn(cout, generator=g) * 0.01
    return p


def resized_size(h, w, short=256):
    """torchvision _compute_resized_output_size for size=[short]."""
    if h <= w:
        return short, int(short * w / h)
    return int(short * h / w), short


def vgg_prepare(x, is_generated, crop=224, resize=256):
    """loss.py:65-86 then ImageClassification (resize/crop/normalize)."""
    if x.dim() == 3:
        x = x.unsqueeze(1)
    if is_generated:
        xs = (x + 1.0) / 2.0
    else:
        xc = torch.clamp(x, min=0.0)
        mx = torch.max(xc).item() + 1e-6
        xs = xc / mx if mx > 1e-5 else xc
    xs = torch.clamp(xs, 0.0, 1.0).repeat(1, 3, 1, 1)
    nh, nw = resized_size(xs.shape[2], xs.shape[3], resize)
    xs = F.interpolate(xs, size=(nh, nw), mode="bilinear", align_corners=False, antialias=True)
    top = int(round((nh - crop) / 2.0))
    left = int(round((nw - crop) / 2.0))
    xs = xs[:, :, top:top + crop, left:left + crop]
    mean = torch.tensor(IMAGENET_MEAN, dtype=xs.dtype).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD, dtype=xs.dtype).view(1, 3, 1, 1)
    return (xs - mean) / std


def vgg_features(p, x, want=VGG_STYLE + VGG_PERCEPTUAL):
    """loss.py:41-51 with torchvision's inplace ReLUs: a collected conv output
    is overwritten by the ReLU that follows it, unless the loop stopped first."""
    feats = {}
    last = max(want)
    for lay in vgg19_feature_keys():
        i = lay[1]
        if lay[0] == "conv":
            x = F.conv2d(x, p[f"{i}.weight"], p[f"{i}.bias"], 1, 1)
        elif lay[0] == "relu":
            x = F.relu(x)
            if (i - 1) in feats:
                feats[i - 1] = x
        else:
            x = F.max_pool2d(x, 2, 2)
        if i in want:
            feats[i] = x
        if i >= last:
            break
    return feats


def gram(x):
    b, c, h, w = x.shape
    f = x.reshape(b, c, h * w)
    return torch.bmm(f, f.transpose(1, 2)) / (c * h * w)


def vgg_losses(p, generated, target):
    """VGGLoss.forward (loss.py:89-131) -> (perceptual, style)."""
    fg = vgg_features(p, vgg_prepare(generated, True))
    ft = vgg_features(p, vgg_prepare(target, False))
    perc = sum(torch.mean(torch.abs(fg[i] - ft[i])) for i in VGG_PERCEPTUAL) / len(VGG_PERCEPTUAL)
    style = sum(torch.mean(torch.abs(gram(fg[i]) - gram(ft[i]))) for i in VGG_STYLE) / len(VGG_STYLE)
    return perc, style


# -------------------------------------------------------------------- losses
LAMBDAS = {"lambda_adv": 0.01, "lambda_l1_valid": 1.0, "lambda_l1_hole": 2.0,
           "lambda_vgg_perceptual": 4.0, "lambda_vgg_style": 500.0, "lambda_mag_weighted": 0.2}


def generator_losses(gen, orig, mask, d_fake, vgg_p=None, lam=LAMBDAS):
    """calculate_losses (train.py:33-88)."""
    adv = F.binary_cross_entropy_with_logits(d_fake, torch.ones_like(d_fake))
    mask = mask.view_as(gen) if mask.dim() < gen.dim() else mask
    l1v = torch.sum(torch.abs(gen * mask - orig * mask)) / (torch.sum(mask) + 1e-8)
    hole = 1.0 - mask
    l1h = torch.sum(torch.abs(gen * hole - orig * hole)) / (torch.sum(hole) + 1e-8)
    lw = torch.mean(torch.abs(gen - orig) * torch.abs(orig))
    perc = torch.tensor(0.0)
    style = torch.tensor(0.0)
    if vgg_p is not None and (lam["lambda_vgg_perceptual"] > 0 or lam["lambda_vgg_style"] > 0):
        perc, style = vgg_losses(vgg_p, gen, orig)
    total = (lam["lambda_adv"] * adv + lam["lambda_l1_valid"] * l1v + lam["lambda_l1_hole"] * l1h
             + lam["lambda_mag_weighted"] * lw + lam["lambda_vgg_perceptual"] * perc
             + lam["lambda_vgg_style"] * style)
    return {"g_total": total, "g_adv": adv, "g_l1_valid": l1v, "g_l1_hole": l1h,
            "g_mag_weighted": lw, "g_vgg_perceptual": perc, "g_vgg_style": style}


def d_trainable_keys(pd):
    return [k for k in pd if k.endswith("weight_orig") or k.endswith(".bias")]


class GanStep:
    """One reference GAN iteration (train.py:341-378) on parameter dicts:
    G forward under no_grad (train-mode BN), D step (real + fake, mean of the
    two BCE terms, Adam(d_lr, betas)), then the generator-loss forward
    (third D forward + VGG).  The G-step backward only fills D grads that the
    next d_optimizer.zero_grad() discards; it is run here too so
    the D .grad left behind matches the reference."""

    def __init__(self, pg, pd, pvgg=None, lr=2e-4, betas=(0.5, 0.999), lam=LAMBDAS):
        self.pg, self.pd, self.pvgg, self.lam = pg, pd, pvgg, lam
        self.dkeys = d_trainable_keys(pd)
        for k in self.dkeys:
            pd[k].requires_grad_(True)
        self.opt = torch.optim.Adam([pd[k] for k in self.dkeys], lr=lr, betas=betas)

    def step(self, orig, imp, mask):
        self.opt.zero_grad()
        with torch.no_grad():
            gen = generator(self.pg, imp, mask, training=True)
        d_real = discriminator(self.pd, orig)
        l_real = F.binary_cross_entropy_with_logits(d_real, torch.ones_like(d_real))
        d_fake = discriminator(self.pd, gen.detach())
        l_fake = F.binary_cross_entropy_with_logits(d_fake, torch.zeros_like(d_fake))
        d_loss = (l_real + l_fake) / 2
        d_loss.backward()
        self.opt.step()
        d_fake_g = discriminator(self.pd, gen)
        losses = generator_losses(gen, orig, mask, d_fake_g, self.pvgg, self.lam)
        losses["g_total"].backward()
        out = {k: v.detach() for k, v in losses.items()}
        out.update(d_loss=d_loss.detach(), d_real=l_real.detach(), d_fake=l_fake.detach(),
                   generated=gen)
        return out
