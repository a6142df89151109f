"""Fail-fast guards for the training loops (SURVEY §5 "failure detection":
fail fast on a NaN loss and on collective errors).

The reference reads the loss on the host every step (models/CNNBLSTM/train.py
:111, models/GAN/train.py:381-388) and lets a NaN flow into Adam.  Here the
loop reads it once per step *before* the optimizer step (the same one sync,
moved ahead of the Adam launch), so a non-finite loss stops training with the
weights of the last finite step intact.  Under data parallelism every rank
takes the same decision: the non-finite flag is MAX-all-reduced, so no rank
is left waiting in the next collective while another one raises.
"""
from __future__ import annotations

import math

import torch


class NonFiniteLossError(FloatingPointError):
    """Raised by check_finite when a training loss is NaN or infinite."""


def check_finite(loss: torch.Tensor, what: str, step: int, comm=None) -> float:
    """Host value of a scalar loss; raises NonFiniteLossError if it (on any
    DP rank) is not finite.  comm: ainp.dist.Comm or None."""
    if comm is not None and comm.world_size > 1:
        flag = (~torch.isfinite(loss.detach().reshape(-1)[:1])).to(torch.float32)
        comm.allreduce_max_(flag)
        bad_any = bool(flag.item())
    else:
        bad_any = False
    v = float(loss.detach().reshape(-1)[0].item())
    if bad_any or not math.isfinite(v):
        where = "on this rank" if not math.isfinite(v) else "on another DP rank"
        raise NonFiniteLossError(
            f"{what} is not finite at step {step} ({v!r} {where}); stopping before the "
            f"optimizer step (parameters hold the last finite step)")
    return v
