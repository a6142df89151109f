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
with weights_only=True; spectrogram figures and Griffin-Lim audio samples are
not produced (plotting is out of scope, ISTFT/GL is SURVEY §8 f1); the G-step
backward that only fills soon-discarded D grads is skipped (SURVEY Q1,
GanTrainer(faithful_g_backward=True) restores it).
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
from ainp.gan import calculate_losses, find_latest_checkpoint  # noqa: E402
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

    def close(self):
        pass


def _writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=str(log_dir))
    except Exception:
        return _NullWriter()


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
    if rank == 0:
        for d in (tb_dir, chkpt_dir, Path(paths_cfg["sample_dir"]) / run_name, log_dir):
            d.mkdir(parents=True, exist_ok=True)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [%(levelname)s] %(message)s",
                        handlers=[logging.StreamHandler()])
    logger = logging.getLogger()
    writer = _writer(tb_dir) if rank == 0 else _NullWriter()

    train_ds = SpeechInpaintingDataset(cfg, "train", device=device)
    valid_ds = SpeechInpaintingDataset(cfg, "valid", device=device)
    idx = random.sample(range(len(train_ds)), k=min(data_cfg["train_limit"], len(train_ds)))
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
    trainer = GanTrainer(cfg, generator, discriminator, vgg, comm=comm)

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
            for k in ("g_total", "d_loss", "g_adv", "g_l1_valid", "g_l1_hole", "g_mag_weighted",
                      "g_vgg_perceptual", "g_vgg_style"):
                sums[k] = sums.get(k, 0.0) + float(out[k])
            count += 1
            global_step += 1
            if global_step % log_cfg["log_interval"] == 0:
                writer.add_scalar("Loss_Train/Generator_Total", float(out["g_total"]), global_step)
                writer.add_scalar("Loss_Train/Discriminator", float(out["d_loss"]), global_step)
        if rank == 0 and count:
            logger.info(f"Epoch {epoch + 1} Summary: Avg G Loss: {sums['g_total'] / count:.4f}, "
                        f"Avg D Loss: {sums['d_loss'] / count:.4f}")
        if (epoch + 1) % log_cfg.get("validation_interval", 5) == 0:
            generator.eval()
            discriminator.eval()
            vsum, vcount = 0.0, 0
            with torch.no_grad():
                for audio, starts in valid_loader:
                    b = valid_ds.features(audio, starts)
                    gen = generator(b["impaired_magnitude"], b["mask"])
                    d_fake = discriminator(gen)
                    losses = calculate_losses(cfg, gen, b["original_magnitude"], b["mask"],
                                              d_fake, vgg)
                    vsum += float(losses["g_total"])
                    vcount += 1
            if rank == 0 and vcount:
                logger.info(f"Epoch {epoch + 1} Validation: Avg G Loss: {vsum / vcount:.4f}")
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
