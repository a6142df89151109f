"""torch.optim.Adam drop-in whose step is the multi-tensor libainp kernel.

Replaces optim.Adam(model.parameters(), lr=...) of models/CNNBLSTM/train.py:
71-72 (step at :108).  Subclasses torch.optim.Optimizer, so param_groups,
zero_grad(), state_dict()/load_state_dict() behave as torch's (state per
parameter: 'step', 'exp_avg', 'exp_avg_sq').

capturable=False (default): 'step' is a float32 CPU tensor, as torch's, and
the bias corrections are formed on the host.  capturable=True (torch's
contract of the same name): 'step' lives on the device -- one tensor shared by
the parameters of a group -- and the kernel advances it and forms the bias
corrections on the device (ainp_adam_ex), so a training step containing
opt.step() can be captured in a HIP graph and replayed.  Both forms give the
same arithmetic (double bias corrections, one rounding to f32).
"""
from __future__ import annotations

import torch

from . import ops


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, *, maximize=False, capturable=False):
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
                        amsgrad=False, maximize=False, foreach=None, capturable=capturable,
                        differentiable=False, fused=None)
        super().__init__(params, defaults)
        self._dev_step: dict = {}     # group index -> (shared step [()], scalars [2])

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev_step.clear()

    def _group_step(self, gi, group, ps):
        """The group's shared device step tensor (created, or unified from the
        loaded per-parameter steps, outside any capture: it reads them once)."""
        ent = self._dev_step.get(gi)
        if ent is not None:
            return ent
        steps = [self.state[p]["step"] for p in ps if "step" in self.state[p]]
        vals = {float(s) for s in steps}
        if len(vals) > 1 or (vals and len(steps) != len(ps)):
            raise RuntimeError("ainp Adam(capturable=True): the parameters of a group must "
                               "share one step count")
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("ainp Adam(capturable=True): run one step before capturing "
                               "(state initialisation reads the step counts)")
        dev = ps[0].device
        step = torch.full((), vals.pop() if vals else 0.0, dtype=torch.float32, device=dev)
        for p in ps:
            self.state[p]["step"] = step
        ent = (step, torch.empty(2, dtype=torch.float32, device=dev))
        self._dev_step[gi] = ent
        return ent

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            ps = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients")
                ps.append(p)
            if not ps:
                continue
            for p in ps:
                st = self.state[p]
                if "exp_avg" not in st:
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if group["capturable"]:
                step_dev, scalars = self._group_step(gi, group, ps)
                batches = {None: ps}
            else:
                batches = {}
                for p in ps:
                    st = self.state[p]
                    if "step" not in st:
                        st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["step"] += 1
                    batches.setdefault(int(st["step"].item()), []).append(p)
            for s, bp in batches.items():
                gs = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in bp]
                ms = [self.state[p]["exp_avg"] for p in bp]
                vs = [self.state[p]["exp_avg_sq"] for p in bp]
                if s is None:
                    ops.adam_step(bp, gs, ms, vs, group["lr"], beta1, beta2, group["eps"],
                                  group["weight_decay"], 0, step_dev=step_dev, scalars_dev=scalars)
                else:
                    ops.adam_step(bp, gs, ms, vs, group["lr"], beta1, beta2, group["eps"],
                                  group["weight_decay"], s)
                # the kernel wrote the parameters in place through raw pointers:
                # record it like any in-place op (autograd checks, weight caches)
                for p in bp:
                    torch.autograd.graph.increment_version(p)
        return loss
