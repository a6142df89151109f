"""Drop-in for models/CNNBLSTM/train.py on the MI355X kernels.

Same loop as the reference (train.py:26-199): YAML config from the cwd,
StackedBLSTMCNN, LibriSpeechDataset + DataLoader(batch_size, shuffle=True),
L1(sum) on 10**y inside the gap, Adam(starter_learning_rate), per-epoch test
loss, 'Train_Loss' every metric_interval steps / 'Test_Loss' per epoch to
TensorBoard (when installed), state_dict checkpoints named
blstm_cnn_epoch_{n}.pt every checkpoint_interval epochs.

Differences (documented): the batch reshape uses the actual batch size (the
reference crashes on a partial last batch); resume loads with
weights_only=True; spectrogram figures are not produced (plotting is out of
scope); the audio samples are (train.py:178-189, every audio_interval steps on
the GPU ISTFT / Griffin-Lim, with the reference's default hop of 512 -- the
call passes only n_fft).
Data parallel: launched under torchrun (WORLD_SIZE > 1) each rank trains on a
DistributedSampler shard with SUM-all-reduced gradients and SyncBN; rank 0's
initial weights are broadcast; the layer-0 input-weight gradient is
all-reduced chunk by chunk as the BLSTM backward produces it (model.grad_reducer).
"""
from __future__ import annotations

import os
import sys
from datetime import datetime
from pathlib import Path

import torch
import yaml
from torch.utils.data import DataLoader

HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(os.path.dirname(HERE))
for p in (HERE, _PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# package-qualified: the GAN scripts also have a `dataset` module
from models.CNNBLSTM.dataset import LibriSpeechDataset  # noqa: E402
from models.CNNBLSTM.model import StackedBLSTMCNN  # noqa: E402

from ainp.cnnblstm import l1_pow10_loss  # noqa: E402
from ainp.failfast import check_finite  # noqa: E402
from ainp.trace import phase  # noqa: E402
from ainp.dist import Comm, GradAllReducer, init_from_env  # noqa: E402
from ainp.optim import Adam  # noqa: E402


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


def _flatten(batch):
    lg, gi, gm, tg = batch
    n = lg.shape[0] * lg.shape[1]  # actual batch, not BATCH_SIZE (Q2)
    return (lg.reshape(n, lg.shape[2], lg.shape[3]), gi.reshape(n, 2),
            gm.reshape(n, gm.shape[2], gm.shape[3]), tg.reshape(n, tg.shape[2], tg.shape[3]))


def save_audio_samples(writer, model, config, x, mask, target, sample_dir, global_step):
    """train.py:178-189 on the first item of the last test batch: the clean
    complex spectrogram and the gapped one (target * (1 - mask)) through the
    ISTFT, the reconstruction 10**reconstruct_spectrogram through Griffin-Lim
    (n_iter 64); spectrogram_to_audio gets only n_fft, so hop_length is its
    default 512 (reference quirk kept)."""
    import utils
    n_fft, sr = config["data"]["spectrogram"]["n_fft"], config["data"]["sample_rate"]
    with torch.no_grad():
        rec = (10 ** model.reconstruct_spectrogram(x, mask))[0].float().contiguous()
    orig = target[0].contiguous()
    gap = (target[0] * (1 - mask[0])).contiguous()
    audio = {
        "orig": utils.spectrogram_to_audio(orig, phase_info=True, n_fft=n_fft),
        "gap": utils.spectrogram_to_audio(gap, phase_info=True, n_fft=n_fft),
        "reconstructed": utils.spectrogram_to_audio(rec, phase_info=False, n_fft=n_fft),
    }
    audio = {k: v.cpu().numpy() for k, v in audio.items()}
    for k, v in audio.items():
        utils.save_audio(v, Path(sample_dir) / f"{k}_audio_{global_step}.flac")
    for tag, k in (("Audio/Original", "orig"), ("Audio/Impaired", "gap"),
                   ("Audio/Generated", "reconstructed")):
        writer.add_audio(tag, audio[k], global_step, sample_rate=sr)
    return audio


def main(config_path="cnn_blstm.yaml"):
    with open(config_path, "r") as f:
        config = yaml.safe_load(f)
    rank, world, local = init_from_env()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    model = StackedBLSTMCNN(config_path)
    if config["paths"].get("resume_mdl_path") is not None:
        model.load_state_dict(torch.load(config["paths"]["resume_mdl_path"], weights_only=True))
    if rank == 0:
        print(model)
    model.to(device)
    comm = Comm() if world > 1 else None
    model.comm = comm
    if comm is not None:
        comm.broadcast_module_(model)

    BATCH_SIZE = config["training"]["batch_size"]
    train_dataset = LibriSpeechDataset(config_path, dataset_type="train", device=device)
    test_dataset = LibriSpeechDataset(config_path, dataset_type="test", device=device)
    sampler = None
    if world > 1:
        from torch.utils.data.distributed import DistributedSampler
        sampler = DistributedSampler(train_dataset, num_replicas=world, rank=rank, shuffle=True)
    train_loader = DataLoader(train_dataset, batch_size=BATCH_SIZE, shuffle=sampler is None,
                              sampler=sampler)
    test_loader = DataLoader(test_dataset, batch_size=BATCH_SIZE, shuffle=True)

    paths_cfg = config["paths"]
    run_name = datetime.today().strftime("%Y_%m_%d_%H%M")
    tb_dir = Path(paths_cfg["tensorboard_dir"]) / run_name
    chkpt_dir = Path(paths_cfg["checkpoint_dir"]) / run_name
    sample_dir = Path(paths_cfg["sample_dir"]) / run_name
    if rank == 0:
        for d in (tb_dir, chkpt_dir, sample_dir, Path(paths_cfg["log_dir"])):
            d.mkdir(parents=True, exist_ok=True)
    writer = _writer(tb_dir) if rank == 0 else _NullWriter()

    if config["training"]["optimizer_type"] == "adam":
        optimizer = Adam(model.parameters(), lr=config["training"]["starter_learning_rate"])
    else:
        raise ValueError("only optimizer_type: adam is used by the reference")
    reducer = GradAllReducer(model.parameters(), comm) if comm is not None else None
    model.grad_reducer = reducer

    num_epochs = config["training"]["max_n_epochs"]
    global_step = 0
    for epoch in range(num_epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)
        model.train()
        running_loss = 0.0
        for batch_idx, batch in enumerate(train_loader):
            with phase("data"):
                x, _, mask, target = _flatten(batch)
            optimizer.zero_grad()
            with phase("fwd"):
                y = model(x.unsqueeze(1))
                loss = l1_pow10_loss(y, mask, target)
            with phase("bwd"):
                loss.backward()
            if reducer is not None:
                with phase("allreduce"):
                    reducer.allreduce()
            # the reference's per-step loss.item() (train.py:111), read before
            # the optimizer step: a NaN/inf loss stops training (all DP ranks)
            lv = check_finite(loss, "Train_Loss", global_step, comm)
            with phase("optimizer"):
                optimizer.step()
            running_loss += lv
            if global_step % config["logging"]["metric_interval"] == 0:
                writer.add_scalar("Train_Loss", lv, global_step)
            global_step += 1
        if rank == 0:
            print(f"Epoch [{epoch + 1}/{num_epochs}], Average Loss: "
                  f"{running_loss / max(1, len(train_loader)):.4f}", flush=True)

        model.eval()
        running_test_loss = 0.0
        last = None
        with torch.no_grad():
            for batch in test_loader:
                x, _, mask, target = _flatten(batch)
                y = model(x.unsqueeze(1))
                running_test_loss += l1_pow10_loss(y, mask, target).item()
                last = (x, mask, target)
        if rank == 0 and last is not None and \
                global_step % config["logging"]["audio_interval"] == 0:
            save_audio_samples(writer, model, config, *last, sample_dir, global_step)
        writer.add_scalar("Test_Loss", running_test_loss / max(1, len(test_loader)), epoch + 1)

        if rank == 0 and (epoch + 1) % config["logging"]["checkpoint_interval"] == 0:
            torch.save(model.state_dict(), chkpt_dir / f"blstm_cnn_epoch_{epoch + 1}.pt")
    writer.close()
    if rank == 0:
        print("Training Complete!")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "cnn_blstm.yaml")
