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


# H = 64: 4H = 256 gate rows per direction, so the fp32 layer-0 backward runs
# as the fused gemm_x6r pair (ops.l0_bwd_x6r_eligible: NT >= 256 per rank)
CNNBLSTM_PAIR_CFG = {
    "data": CNNBLSTM_CFG["data"],
    "model": dict(CNNBLSTM_CFG["model"], lstm_hidden_dim=64),
}


def _cnnblstm_batch(n=4, F=33, T=24):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, 1, F, T, generator=g) - 2.0
    mask = torch.zeros(n, F, T)
    for i in range(n):
        s = 3 + 4 * i
        mask[i, :, s:s + 5] = 1.0
    tgt = torch.complex(torch.rand(n, F, T, generator=g), torch.rand(n, F, T, generator=g))
    return x, mask, tgt


def run_cnnblstm(comm=None, rank=0, world=1, uneven=False, steps=1, defer=True, pair=False):
    """uneven: rank 0 takes 3 of the 4 examples, rank 1 one (SyncBN must use
    the global element count).  The ranks start from different seeds and get
    rank 0's weights by broadcast; the layer-0 input weights' gradients go to
    the reducer chunk by chunk (model.grad_reducer).  pair: H = 64 and T = 128,
    where the fp32 layer-0 backward is the fused gemm_x6r pair launch, whose
    weight gradients are handed to the reducer right behind it."""
    from ainp.cnnblstm import StackedBLSTMCNN, l1_pow10_loss
    from ainp.dist import GradAllReducer
    from ainp.optim import Adam
    dev = torch.device("cuda", 0)
    torch.manual_seed(0 if comm is None else 100 * rank)
    model = StackedBLSTMCNN(config=CNNBLSTM_PAIR_CFG if pair else CNNBLSTM_CFG).to(dev).train()
    # side-stream weight gradients (on by default; under DP they are
    # all-reduced from the side stream as they are written)
    model.defer_wgrad = model.defer_wgrad_encoder = defer
    if comm is not None:
        comm.broadcast_module_(model)
    model.comm = comm
    opt = Adam(model.parameters(), lr=1e-3)
    red = GradAllReducer(model.parameters(), comm) if comm is not None else None
    model.grad_reducer = red
    x, mask, tgt = _cnnblstm_batch(T=128 if pair else 24)
    if uneven and world == 2:
        sl = slice(0, 3) if rank == 0 else slice(3, 4)
    else:
        per = x.shape[0] // world
        sl = slice(rank * per, (rank + 1) * per)
    x, mask, tgt = x[sl].to(dev), mask[sl].to(dev), tgt[sl].to(dev)
    early = side = npair = 0
    bad_storage = []
    for _ in range(steps):
        opt.zero_grad()
        loss = l1_pow10_loss(model(x), mask, tgt)
        loss.backward()
        if red is not None:
            early, side, npair = red.early_chunks, red.side_reductions, red.pair_reductions
            # every buffer a hand-off reduced is the storage of p.grad (the
            # tensor the optimizer reads), not a copy autograd made of it
            byid = {id(p): n for n, p in model.named_parameters()}
            for n, p in model.named_parameters():
                ptrs = red.reduced_storage.get(id(p))
                if ptrs is not None and (p.grad is None or
                                         ptrs != {p.grad.untyped_storage().data_ptr()}):
                    bad_storage.append(n)
            assert set(red.reduced_storage) <= set(byid)
            red.allreduce()
        opt.step()
    loss = loss.detach().double().reshape(1)
    if comm is not None:
        comm.allreduce_sum_(loss)            # the reference loss is a batch SUM
    torch.cuda.synchronize()
    state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    return {"loss": loss.cpu(), "state": state, "early_chunks": early, "side_reductions": side,
            "pair_reductions": npair, "bad_storage": bad_storage}


def _gan_batch(n=2, F=257, T=100):
    g = torch.Generator().manual_seed(11)
    orig = torch.rand(n, 1, F, T, generator=g) * 2.0
    mask = torch.ones(n, 1, F, T)
    for i in range(n):
        mask[i, :, :, 10 + 7 * i:22 + 7 * i] = 0.0
    imp = orig * mask
    return orig, imp, mask


def run_gan(comm=None, rank=0, world=1, faithful=False, steps=1, g_nan_rank=None, fix_g=False):
    """faithful: GanTrainer(faithful_g_backward=True), whose G-step backward
    fills D grads that must not reach the gradient reducer.  g_nan_rank: that
    rank's G-step total loss is made NaN (fail_fast on): every rank must stop
    before g_optimizer.step(); returns the error text instead of the state."""
    from ainp import gan as G
    from ainp.failfast import NonFiniteLossError
    from ainp.gan_train import GanTrainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    gen = G.PConvUNet().to(dev)
    disc = G.Discriminator().to(dev)
    vgg = G.VGGLoss(dev)
    tr = GanTrainer(GAN_CFG, gen, disc, vgg, comm=comm, faithful_g_backward=faithful,
                    fail_fast=g_nan_rank is not None, fix_generator_grad=fix_g)
    if g_nan_rank == rank:
        calc = G.calculate_losses

        def nan_losses(*a, **k):
            out = calc(*a, **k)
            out["g_total"] = out["g_total"] * float("nan")
            return out
        G.calculate_losses = nan_losses
    orig, imp, mask = _gan_batch()
    per = orig.shape[0] // world
    sl = slice(rank * per, (rank + 1) * per)
    for _ in range(steps):
        try:
            out = tr.step(orig[sl].to(dev), imp[sl].to(dev), mask[sl].to(dev))
        except NonFiniteLossError as e:
            if g_nan_rank is None:
                raise
            return {"error": str(e)}
    torch.cuda.synchronize()
    losses = {k: v.detach().double().cpu() for k, v in out.items() if k != "generated"}
    dstate = {k: v.detach().cpu().clone() for k, v in disc.state_dict().items()}
    gbn = {k: v.detach().cpu().clone() for k, v in gen.state_dict().items()
           if "running" in k}
    res = {"losses": losses, "disc": dstate, "gen_bn": gbn}
    if fix_g:
        # G's gradients as g_optimizer.step() consumed them (after the
        # reducer's exchange; Adam's update itself is nearly scale-free, so
        # the gradients are what pins the DP scaling)
        res["gen_grad"] = {n: p.grad.detach().cpu().clone() for n, p in gen.named_parameters()
                           if p.grad is not None}
        res["gen"] = {k: v.detach().cpu().clone() for k, v in gen.state_dict().items()}
    return res


def main():
    mode, out = sys.argv[1], sys.argv[2]
    import torch.distributed as dist
    from ainp.dist import Comm
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # "<mode>:dev": device tensors go to gloo's async CUDA collectives (no
    # host staging): the Work objects hold the reduced gradients until wait(),
    # as RCCL's do
    mode, _, flavour = mode.partition(":")
    comm = Comm(host_staging=False if flavour == "dev" else None)
    assert comm.grad_group is not comm.group     # SyncBN and gradients: two communicators
    if mode == "cnnblstm":
        res = run_cnnblstm(comm, rank, world)
    elif mode == "cnnblstm_nodefer":
        res = run_cnnblstm(comm, rank, world, defer=False)
    elif mode == "cnnblstm_pair":
        res = run_cnnblstm(comm, rank, world, pair=True)
    elif mode == "cnnblstm_pair_nodefer":
        res = run_cnnblstm(comm, rank, world, defer=False, pair=True)
    elif mode == "cnnblstm_uneven":
        res = run_cnnblstm(comm, rank, world, uneven=True, steps=2)
    elif mode == "gan_gnan":
        res = run_gan(comm, rank, world, faithful=True, g_nan_rank=1)
    elif mode == "gan_fixg":
        res = run_gan(comm, rank, world, fix_g=True)
    elif mode == "gan_faithful":
        res = run_gan(comm, rank, world, faithful=True, steps=2)
    else:
        res = run_gan(comm, rank, world)
    torch.save(res, f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
