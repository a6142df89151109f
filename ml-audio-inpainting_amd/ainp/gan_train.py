"""One GAN training iteration on the MI355X kernels (models/GAN/train.py:341-378).

  D step   generated = G(impaired, mask) under no_grad (train-mode BatchNorm:
           running statistics update), BCE(D(original), 1) and BCE(D(generated), 0)
           averaged, backward through D, Adam(d_lr, (b1, b2)).
  G step   D(generated) a third time (one more spectral-norm power iteration),
           calculate_losses (adversarial, L1 valid / hole, magnitude-weighted,
           VGG perceptual / style), g_optimizer.step().

SURVEY Q1: `generated` carries no graph, so g_loss.backward() only fills D's
.grad, which the next d_optimizer.zero_grad() discards, and g_optimizer.step()
is a no-op (G never gets a gradient).  Parameters, buffers and every loss
value are therefore the same with or without that backward; it is skipped
unless faithful_g_backward=True (then D's .grad after the step also matches).

fix_generator_grad=True (or `training.fix_generator_grad: true` in the config;
SURVEY §7's opt-in deviation) trains G: the generator forward runs with
autograd (the reference loop without its torch.no_grad(), train.py:349-350),
the D step still sees generated.detach(), and the G step back-propagates the
total generator loss through D, VGG19 and the L1 terms into G
(ainp.gan._PConvUNetFn) before g_optimizer.step().
"""
from __future__ import annotations

import torch

from . import gan as G
from .optim import Adam
from .trace import phase


class GanTrainer:
    def __init__(self, cfg, generator, discriminator, vgg=None, faithful_g_backward=False,
                 comm=None, fail_fast=False, fix_generator_grad=None):
        """fail_fast: read the D loss on the host before d_optimizer.step()
        and raise ainp.failfast.NonFiniteLossError if it is NaN/inf on any
        rank (models/GAN/train.py reads the losses every step anyway; off for
        the bench, which must not add a mid-step sync)."""
        tc = cfg["training"]
        self.fail_fast = fail_fast
        self.nstep = 0
        self.cfg = cfg
        self.G, self.D, self.vgg = generator, discriminator, vgg
        betas = (tc.get("b1", 0.5), tc.get("b2", 0.999))
        # accel.capturable: device-side Adam step counters, so the whole step
        # can be captured in a HIP graph and replayed (tools/gan_graph.py)
        cap = bool((cfg.get("accel") or {}).get("capturable", False))
        self.g_opt = Adam(generator.parameters(), lr=tc.get("g_lr", 2e-4), betas=betas,
                          capturable=cap)
        self.d_opt = Adam(discriminator.parameters(), lr=tc.get("d_lr", 2e-4), betas=betas,
                          capturable=cap)
        self.faithful = faithful_g_backward
        if fix_generator_grad is None:
            fix_generator_grad = bool(tc.get("fix_generator_grad", False))
        self.fix_g = bool(fix_generator_grad)
        self.comm = comm
        dtype = (cfg.get("accel") or {}).get("dtype", "fp32")
        for m in (generator, discriminator, vgg):
            if m is not None:
                G.set_compute_dtype(m, dtype)
        self.reducer = None
        self.g_reducer = None
        if comm is not None and comm.world_size > 1:
            from .dist import GradAllReducer
            # identical starting weights on every rank (as DDP broadcasts at wrap time)
            for m in (generator, discriminator, vgg):
                if m is not None:
                    comm.broadcast_module_(m)
            self.reducer = GradAllReducer(discriminator.parameters(), comm)
            # fix_generator_grad: G's gradients are exchanged like D's (averaged)
            self.g_reducer = (GradAllReducer(generator.parameters(), comm) if self.fix_g
                              else None)
            # SyncBN for G's BatchNorms and the global VGG target max: the
            # N-rank step then equals the 1-process step on the whole batch
            for m in generator.modules():
                if isinstance(m, torch.nn.BatchNorm2d):
                    m.ainp_comm = comm
            if vgg is not None:
                vgg.comm = comm

    def step(self, original_mag, impaired_mag, mask):
        self.G.train()
        self.D.train()
        # ---- discriminator step (train.py:348-363)
        self.d_opt.zero_grad()
        with phase("fwd_G"):
            if self.fix_g:
                generated = self.G(impaired_mag, mask)       # with autograd: G trains
            else:
                with torch.no_grad():
                    generated = self.G(impaired_mag, mask)
        with phase("fwd_D"):
            d_real = self.D(original_mag)
            l_real = G.bce_with_logits_const(d_real, 1.0)
            d_fake = self.D(generated.detach())
            l_fake = G.bce_with_logits_const(d_fake, 0.0)
            d_loss = (l_real + l_fake) / 2
        with phase("bwd_D"):
            d_loss.backward()
        if self.reducer is not None:
            with phase("allreduce"):
                # the reference loss is a per-rank mean: DP averages D's gradients
                self.reducer.allreduce()
                for p in self.D.parameters():
                    if p.grad is not None:
                        p.grad.div_(self.comm.world_size)
        if self.fail_fast:
            from .failfast import check_finite
            check_finite(d_loss, "D loss", self.nstep, self.comm)
        self.nstep += 1
        with phase("optimizer"):
            self.d_opt.step()
        # ---- generator step (train.py:366-378)
        self.g_opt.zero_grad()
        if self.fix_g:
            with phase("g_losses"):
                d_fake_g = self.D(generated)
                losses = G.calculate_losses(self.cfg, generated, original_mag, mask, d_fake_g,
                                            self.vgg, comm=self.comm)
            # D's gradients from this backward are discarded by the next
            # zero_grad (as in the reference): not exchanged
            if self.reducer is not None:
                self.reducer.paused = True
            try:
                with phase("bwd_G"):
                    losses["g_total"].backward()
            finally:
                if self.reducer is not None:
                    self.reducer.paused = False
            if self.g_reducer is not None:
                with phase("allreduce"):
                    self.g_reducer.allreduce()
                    for p in self.G.parameters():
                        if p.grad is not None:
                            p.grad.div_(self.comm.world_size)
        elif self.faithful:
            d_fake_g = self.D(generated)
            losses = G.calculate_losses(self.cfg, generated, original_mag, mask, d_fake_g, self.vgg,
                                        comm=self.comm)
            # this backward only fills D grads that the next zero_grad discards
            # (SURVEY Q1): they are not exchanged, so the reducer ignores them
            if self.reducer is not None:
                self.reducer.paused = True
            try:
                losses["g_total"].backward()
            finally:
                if self.reducer is not None:
                    self.reducer.paused = False
        else:
            with torch.no_grad(), phase("g_losses"):
                d_fake_g = self.D(generated)
                losses = G.calculate_losses(self.cfg, generated, original_mag, mask, d_fake_g,
                                            self.vgg, comm=self.comm)
        if self.fail_fast:
            # the reference reads both losses every step: a non-finite G loss
            # stops every rank before g_optimizer.step() too
            from .failfast import check_finite
            check_finite(losses["g_total"], "G loss", self.nstep - 1, self.comm)
        self.g_opt.step()   # no-op unless fix_generator_grad: G has no gradients (Q1)
        out = {k: v.detach() for k, v in losses.items()}
        out.update(d_loss=d_loss.detach(), d_real=l_real.detach(), d_fake=l_fake.detach())
        if self.comm is not None and self.comm.world_size > 1:
            # per-rank batch means -> global-batch means (equal per-rank batches)
            keys = sorted(out)
            vec = torch.stack([out[k].to(torch.float64).reshape(()) for k in keys])
            self.comm.allreduce_sum_(vec)
            vec /= self.comm.world_size
            out = {k: vec[i].to(torch.float32) for i, k in enumerate(keys)}
        out["generated"] = generated.detach()
        return out
