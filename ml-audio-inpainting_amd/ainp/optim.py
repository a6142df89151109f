"""torch.optim.Adam drop-in whose step is the multi-tensor libainp kernel.

Replaces optim.Adam(model.parameters(), lr=...) of models/CNNBLSTM/train.py:
71-72 (step at :108).  Subclasses torch.optim.Optimizer, so param_groups,
zero_grad(), state_dict()/load_state_dict() behave as torch's (state per
parameter: 'step' as a float32 CPU tensor, 'exp_avg', 'exp_avg_sq').
"""
from __future__ import annotations

import torch

from . import ops


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, *, maximize=False):
        if amsgrad or maximize:
            raise NotImplementedError("ainp.optim.Adam: amsgrad/maximize are not used "
                                      "by the reference training loop")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                        amsgrad=False, maximize=False, foreach=None, capturable=False,
                        differentiable=False, fused=None)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            by_step: dict = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                s = int(st["step"].item())
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                by_step.setdefault(s, ([], [], [], []))
                lst = by_step[s]
                lst[0].append(p); lst[1].append(g)
                lst[2].append(st["exp_avg"]); lst[3].append(st["exp_avg_sq"])
            for s, (ps, gs, ms, vs) in by_step.items():
                ops.adam_step(ps, gs, ms, vs, group["lr"], beta1, beta2, group["eps"],
                              group["weight_decay"], s)
                # the kernel wrote the parameters in place through raw pointers:
                # record it like any in-place op (autograd checks, weight caches)
                for p in ps:
                    torch.autograd.graph.increment_version(p)
        return loss
