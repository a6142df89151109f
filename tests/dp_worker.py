"""Data-parallel step on the MI355X kernels, shared by tests/test_gpu_dist.py.

run_cnnblstm / run_gan execute ONE training step of the global batch's slice
that belongs to `rank` (comm=None, rank 0, world 1: the whole batch in one
process) and return the state the reference would hold afterwards.  Run as a
script, it is one rank of a gloo process group on the box's single GPU:

  RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python dp_worker.py <mode> <out>
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "ml-audio-inpainting_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

CNNBLSTM_CFG = {
    "data": {"sample_rate": 16000, "spectrogram": {"n_fft": 64, "hop_length": 16,
                                                   "win_length": 64}},
    "model": {"in_channels": 1, "num_lstm_layers": 2, "lstm_hidden_dim": 32,
              "enc_filters": [16, 32], "dec_filters": [16, 32]},
}
GAN_CFG = {"training": {"g_lr": 2e-4, "d_lr": 2e-4, "b1": 0.5, "b2": 0.999, "lambda_adv": 0.01,
                        "lambda_l1_valid": 1.0, "lambda_l1_hole": 2.0,
                        "lambda_vgg_perceptual": 4.0, "lambda_vgg_style": 500.0,
                        "lambda_mag_weighted": 0.2}}


def _cnnblstm_batch(n=4, F=33, T=24):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, 1, F, T, generator=g) - 2.0
    mask = torch.zeros(n, F, T)
    for i in range(n):
        s = 3 + 4 * i
        mask[i, :, s:s + 5] = 1.0
    tgt = torch.complex(torch.rand(n, F, T, generator=g), torch.rand(n, F, T, generator=g))
    return x, mask, tgt


def run_cnnblstm(comm=None, rank=0, world=1):
    from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
    from ainp.dist import GradAllReducer
    from ainp.optim import Adam
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = StackedBLSTMCNN(config=CNNBLSTM_CFG).to(dev).train()
    model.comm = comm
    opt = Adam(model.parameters(), lr=1e-3)
    red = GradAllReducer(model.parameters(), comm) if comm is not None else None
    x, mask, tgt = _cnnblstm_batch()
    per = x.shape[0] // world
    sl = slice(rank * per, (rank + 1) * per)
    x, mask, tgt = x[sl].to(dev), mask[sl].to(dev), tgt[sl].to(dev)
    opt.zero_grad()
    loss = l1_pow10_loss(model(x), mask, tgt)
    loss.backward()
    if red is not None:
        red.allreduce()
    opt.step()
    loss = loss.detach().double().reshape(1)
    if comm is not None:
        comm.allreduce_sum_(loss)            # the reference loss is a batch SUM
    torch.cuda.synchronize()
    state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    return {"loss": loss.cpu(), "state": state}


def _gan_batch(n=2, F=257, T=100):
    g = torch.Generator().manual_seed(11)
    orig = torch.rand(n, 1, F, T, generator=g) * 2.0
    mask = torch.ones(n, 1, F, T)
    for i in range(n):
        mask[i, :, :, 10 + 7 * i:22 + 7 * i] = 0.0
    imp = orig * mask
    return orig, imp, mask


def run_gan(comm=None, rank=0, world=1):
    from ainp import gan as G
    from ainp.gan_train import GanTrainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    gen = G.PConvUNet().to(dev)
    disc = G.Discriminator().to(dev)
    vgg = G.VGGLoss(dev)
    tr = GanTrainer(GAN_CFG, gen, disc, vgg, comm=comm)
    orig, imp, mask = _gan_batch()
    per = orig.shape[0] // world
    sl = slice(rank * per, (rank + 1) * per)
    out = tr.step(orig[sl].to(dev), imp[sl].to(dev), mask[sl].to(dev))
    torch.cuda.synchronize()
    losses = {k: v.detach().double().cpu() for k, v in out.items() if k != "generated"}
    dstate = {k: v.detach().cpu().clone() for k, v in disc.state_dict().items()}
    gbn = {k: v.detach().cpu().clone() for k, v in gen.state_dict().items()
           if "running" in k}
    return {"losses": losses, "disc": dstate, "gen_bn": gbn}


def main():
    mode, out = sys.argv[1], sys.argv[2]
    import torch.distributed as dist
    from ainp.dist import Comm
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm()
    res = (run_cnnblstm if mode == "cnnblstm" else run_gan)(comm, rank, world)
    torch.save(res, f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
