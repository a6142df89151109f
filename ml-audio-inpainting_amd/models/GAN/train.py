"""Drop-in for models/GAN/train.py on the MI355X kernels.

Same loop as the reference (train.py:131-619): config.yaml from the cwd,
SpeechInpaintingDataset train/valid, random Subset of train_limit files,
batch_size with drop_last, PConvUNet + spectral-norm Discriminator + VGGLoss,
Adam(g_lr / d_lr, (b1, b2)), per iteration the D step then the G step
(ainp.gan_train.GanTrainer), loss logging every log_interval steps, validation
every 5 epochs (eval mode: BatchNorm running stats, no power iteration),
checkpoints generator_/discriminator_/optimizers_epoch_{:04d}.pth every
checkpoint_interval epochs, resume from a run directory (find_latest_checkpoint).

Differences (documented): features for a whole batch come from one fused GPU
launch (not 2 librosa STFTs per item in CPU workers); checkpoints are loaded
with weights_only=True; spectrogram figures are not produced (plotting is out
of scope) but the sample audio is (train.py:419-504: combined log-magnitude,
original and impaired, each ISTFT'd with the original phase on the GPU and
written as FLAC + add_audio); the G-step backward that only fills
soon-discarded D grads is skipped (GanTrainer(faithful_g_backward=
True) restores it).  Data parallel: the train_limit subset is drawn on rank 0
and broadcast (the reference's unseeded random.sample would differ per rank),
initial weights are broadcast from rank 0 (GanTrainer), losses are global-batch
means.
"""
from __future__ import annotations

import logging
import os
import random
import sys
import time
from pathlib import Path

import torch
import yaml
from torch.utils.data import DataLoader

HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(os.path.dirname(HERE))
for p in (HERE, _PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# package-qualified: the CNNBLSTM scripts also have a `dataset` module
from models.GAN.dataset import SpeechInpaintingDataset  # noqa: E402
from models.GAN.loss import VGGLoss  # noqa: E402
from models.GAN.networks import Discriminator, PConvUNet  # noqa: E402

from ainp.dist import Comm, init_from_env  # noqa: E402
from ainp.gan import bce_with_logits_const, calculate_losses, find_latest_checkpoint  # noqa: E402
import utils  # noqa: E402
from ainp.gan_train import GanTrainer  # noqa: E402


def load_config(config_path="config.yaml"):
    with open(config_path, "r") as f:
        return yaml.safe_load(f)


class _RawItems(torch.utils.data.Dataset):
    """Host stage only (decode + gap draw); features run batched on the GPU."""

    def __init__(self, ds, indices=None):
        self.ds = ds
        self.indices = list(range(len(ds))) if indices is None else list(indices)

    def __len__(self):
        return len(self.indices)

    def __getitem__(self, i):
        return self.ds.raw(self.indices[i])


def _collate(items):
    import numpy as np
    return np.stack([a for a, _ in items]), [s for _, s in items]


class _NullWriter:
    def add_scalar(self, *a, **k):
        pass

    def add_audio(self, *a, **k):
        pass

    def close(self):
        pass


def _writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=str(log_dir))
    except Exception:
        return _NullWriter()


def train_subset(n, limit, rank=0, world=1):
    """train.py:248-250 random.sample(range(n), k=min(limit, n)); under DP the
    draw is made once on rank 0 and broadcast so every rank shards one subset."""
    idx = random.sample(range(n), k=min(limit, n)) if rank == 0 else None
    if world > 1:
        import torch.distributed as dist
        box = [idx]
        dist.broadcast_object_list(box, src=0)
        idx = box[0]
    return idx


TRAIN_TAGS = (  # train.py:404-413
    ("Loss_Train/Generator_Total", "g_total"), ("Loss_Train/Discriminator", "d_loss"),
    ("Loss_Train/Generator_Adversarial", "g_adv"), ("Loss_Train/Generator_L1_Valid", "g_l1_valid"),
    ("Loss_Train/Generator_L1_Hole", "g_l1_hole"),
    ("Loss_Train/Generator_MagWeighted", "g_mag_weighted"),
    ("Loss_Train/Generator_VGG_Perceptual", "g_vgg_perceptual"),
    ("Loss_Train/Generator_VGG_Style", "g_vgg_style"),
    ("Loss_Train/Discriminator_Real", "d_real"), ("Loss_Train/Discriminator_Fake", "d_fake"))
AVG_TAGS = (  # train.py:521-528 (Loss_Epoch/...) and 592-599 (Loss_Val/...)
    ("Generator_Total_Avg", "g_total"), ("Discriminator_Avg", "d_loss"),
    ("Generator_Adv_Avg", "g_adv"), ("Generator_L1V_Avg", "g_l1_valid"),
    ("Generator_L1H_Avg", "g_l1_hole"), ("Generator_Lw_Avg", "g_mag_weighted"),
    ("Generator_VGG_P_Avg", "g_vgg_perceptual"), ("Generator_VGG_S_Avg", "g_vgg_style"))


def log_train_step(writer, out, trainer, global_step):
    """train.py:403-416: the 10 loss scalars and the 2 learning rates."""
    for tag, k in TRAIN_TAGS:
        writer.add_scalar(tag, float(out[k]), global_step)
    writer.add_scalar("LR/Generator", trainer.g_opt.param_groups[0]["lr"], global_step)
    writer.add_scalar("LR/Discriminator", trainer.d_opt.param_groups[0]["lr"], global_step)


def save_samples(writer, b, generated, spec_cfg, sr, sample_dir, global_step):
    """train.py:419-504 without the figures: item 0 of the batch; the combined
    log1p magnitude (generated in the hole, original elsewhere), the original
    and the impaired log1p magnitudes go through the ISTFT with the original
    phase as magnitudes, as the reference passes them."""
    o, i = b["original_magnitude"][0, 0], b["impaired_magnitude"][0, 0]
    m, ph = b["mask"][0, 0], b["original_phase"][0, 0]
    g = generated[0, 0].float()
    kw = dict(n_fft=spec_cfg["n_fft"], hop_length=spec_cfg["hop_length"],
              win_length=spec_cfg["win_length"], window=spec_cfg.get("window", "hann"))
    combined = (g * (1 - m) + o * m).contiguous()
    rec = utils.spectrogram_to_audio(combined, ph, **kw).cpu().numpy()
    writer.add_audio("Audio/Generated_CombinedLogMag_OrigPhase", rec, global_step, sample_rate=sr)
    utils.save_audio(rec, Path(sample_dir) / f"step_{global_step}_recon_comb_origphase.flac", sr)
    for name, mag in (("original", o), ("impaired", i)):
        a = utils.spectrogram_to_audio(mag.contiguous(), ph, **kw).cpu().numpy()
        utils.save_audio(a, Path(sample_dir) / f"step_{global_step}_{name}.flac", sr)
    return rec


def main(config_path="config.yaml"):
    cfg = load_config(config_path)
    train_cfg, paths_cfg, log_cfg = cfg["training"], cfg["paths"], cfg["logging"]
    data_cfg = cfg["data"]
    rank, world, local = init_from_env()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    comm = Comm() if world > 1 else None

    run_name = f"{log_cfg['run_name']}_vgg_{time.strftime('%Y%m%d_%H%M%S')}"
    resume = train_cfg.get("resume_from_chkpt", False)
    resume_dir = (Path(paths_cfg["checkpoint_dir"]) / train_cfg["resume_run_name"]
                  if resume and train_cfg.get("resume_run_name") else None)
    tb_dir = Path(paths_cfg["tensorboard_dir"]) / run_name
    chkpt_dir = Path(paths_cfg["checkpoint_dir"]) / run_name
    log_dir = Path(paths_cfg["log_dir"])
    sample_dir = Path(paths_cfg["sample_dir"]) / run_name
    if rank == 0:
        for d in (tb_dir, chkpt_dir, sample_dir, log_dir):
            d.mkdir(parents=True, exist_ok=True)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [%(levelname)s] %(message)s",
                        handlers=[logging.StreamHandler()])
    logger = logging.getLogger()
    writer = _writer(tb_dir) if rank == 0 else _NullWriter()

    train_ds = SpeechInpaintingDataset(cfg, "train", device=device)
    valid_ds = SpeechInpaintingDataset(cfg, "valid", device=device)
    idx = train_subset(len(train_ds), data_cfg["train_limit"], rank, world)
    sampler = None
    train_items = _RawItems(train_ds, idx)
    if world > 1:
        from torch.utils.data.distributed import DistributedSampler
        sampler = DistributedSampler(train_items, num_replicas=world, rank=rank, shuffle=True)
    train_loader = DataLoader(train_items, batch_size=train_cfg["batch_size"],
                              shuffle=sampler is None, sampler=sampler, drop_last=True,
                              num_workers=log_cfg.get("num_workers", 0), collate_fn=_collate)
    valid_loader = DataLoader(_RawItems(valid_ds), batch_size=train_cfg["batch_size"],
                              shuffle=False, num_workers=log_cfg.get("num_workers", 0),
                              collate_fn=_collate)

    gcfg = cfg["model"]["generator"]
    generator = PConvUNet(input_channels=gcfg["input_channels"], mask_channels=gcfg["mask_channels"],
                          output_channels=gcfg["output_channels"],
                          **({"enc_layer_cfg": gcfg["enc_layer_cfg"]} if "enc_layer_cfg" in gcfg
                             else {})).to(device)
    dcfg = cfg["model"]["discriminator"]
    discriminator = Discriminator(input_channels=dcfg["input_channels"],
                                  **({"layer_cfg": dcfg["layer_cfg"]} if "layer_cfg" in dcfg
                                     else {}),
                                  use_spectral_norm=dcfg["use_spectral_norm"]).to(device)
    use_vgg = train_cfg["lambda_vgg_perceptual"] > 0 or train_cfg["lambda_vgg_style"] > 0
    vgg = VGGLoss(device=device, weights=train_cfg.get("vgg_weights")) if use_vgg else None
    trainer = GanTrainer(cfg, generator, discriminator, vgg, comm=comm, fail_fast=True)

    start_epoch, global_step = 0, 0
    if resume_dir is not None and resume_dir.exists():
        e = train_cfg.get("resume_epoch")
        if e is not None:
            g_p = resume_dir / f"generator_epoch_{e:04d}.pth"
            d_p = resume_dir / f"discriminator_epoch_{e:04d}.pth"
            o_p = resume_dir / f"optimizers_epoch_{e:04d}.pth"
            if not (g_p.exists() and d_p.exists() and o_p.exists()):
                g_p = d_p = o_p = None
        else:
            g_p, d_p, o_p, e = find_latest_checkpoint(resume_dir)
        if g_p is not None:
            generator.load_state_dict(torch.load(g_p, map_location=device, weights_only=True))
            discriminator.load_state_dict(torch.load(d_p, map_location=device, weights_only=True))
            ck = torch.load(o_p, map_location=device, weights_only=True)
            if "g_optimizer_state_dict" in ck:
                trainer.g_opt.load_state_dict(ck["g_optimizer_state_dict"])
            if "d_optimizer_state_dict" in ck:
                trainer.d_opt.load_state_dict(ck["d_optimizer_state_dict"])
            start_epoch = ck.get("epoch", -1) + 1
            global_step = ck.get("global_step", 0)
            logger.info(f"Resumed from epoch {start_epoch}, global step {global_step}")

    for epoch in range(start_epoch, train_cfg["epochs"]):
        if sampler is not None:
            sampler.set_epoch(epoch)
        sums, count = {}, 0
        for audio, starts in train_loader:
            b = train_ds.features(audio, starts)
            out = trainer.step(b["original_magnitude"], b["impaired_magnitude"], b["mask"])
            for _, k in AVG_TAGS:
                sums[k] = sums.get(k, 0.0) + float(out[k])
            count += 1
            global_step += 1
            if global_step % log_cfg["log_interval"] == 0:
                log_train_step(writer, out, trainer, global_step)
            if rank == 0 and global_step % log_cfg["sample_interval"] == 0:
                save_samples(writer, b, out["generated"], data_cfg["spectrogram"],
                             data_cfg["sample_rate"], sample_dir, global_step)
        if rank == 0 and count:
            avg = {k: v / count for k, v in sums.items()}
            logger.info(f"Epoch {epoch + 1} Summary: Avg G Loss: {avg['g_total']:.4f}, "
                        f"Avg D Loss: {avg['d_loss']:.4f}")
            logger.info(f"  Avg G Losses -> Adv: {avg['g_adv']:.4f}, L1V: {avg['g_l1_valid']:.4f}, "
                        f"L1H: {avg['g_l1_hole']:.4f}, Lw: {avg['g_mag_weighted']:.4f}, "
                        f"VGG_P: {avg['g_vgg_perceptual']:.4f}, VGG_S: {avg['g_vgg_style']:.4f}")
            for tag, k in AVG_TAGS:
                writer.add_scalar(f"Loss_Epoch/{tag}", avg[k], epoch + 1)
        if (epoch + 1) % log_cfg.get("validation_interval", 5) == 0:
            generator.eval()
            discriminator.eval()
            vsums, vcount = {}, 0
            logger.info(f"Running validation for epoch {epoch + 1}...")
            with torch.no_grad():
                for audio, starts in valid_loader:
                    b = valid_ds.features(audio, starts)
                    gen = generator(b["impaired_magnitude"], b["mask"])
                    d_real = discriminator(b["original_magnitude"])
                    d_fake = discriminator(gen)
                    losses = calculate_losses(cfg, gen, b["original_magnitude"], b["mask"],
                                              d_fake, vgg)
                    losses["d_loss"] = (bce_with_logits_const(d_real, 1.0)
                                        + bce_with_logits_const(d_fake, 0.0)) / 2
                    for _, k in AVG_TAGS:
                        vsums[k] = vsums.get(k, 0.0) + float(losses[k])
                    vcount += 1
            if rank == 0 and vcount:
                va = {k: v / vcount for k, v in vsums.items()}
                logger.info(f"Epoch {epoch + 1} Validation: Avg G Loss: {va['g_total']:.4f}, "
                            f"Avg D Loss: {va['d_loss']:.4f}")
                for tag, k in AVG_TAGS:
                    writer.add_scalar(f"Loss_Val/{tag}", va[k], global_step)
            generator.train()
            discriminator.train()
        if rank == 0 and ((epoch + 1) % log_cfg["checkpoint_interval"] == 0
                          or epoch == train_cfg["epochs"] - 1):
            torch.save(generator.state_dict(), chkpt_dir / f"generator_epoch_{epoch + 1:04d}.pth")
            torch.save(discriminator.state_dict(),
                       chkpt_dir / f"discriminator_epoch_{epoch + 1:04d}.pth")
            torch.save({"g_optimizer_state_dict": trainer.g_opt.state_dict(),
                        "d_optimizer_state_dict": trainer.d_opt.state_dict(),
                        "epoch": epoch, "global_step": global_step},
                       chkpt_dir / f"optimizers_epoch_{epoch + 1:04d}.pth")
    writer.close()
    if rank == 0:
        logger.info("Training finished.")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "config.yaml")
