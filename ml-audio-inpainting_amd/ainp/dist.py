"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL.

The reference has no distributed code; this is the build's DP
layer for the CNNBLSTM step:
  * each rank trains on its own examples (weak scaling, no data-path traffic);
  * gradients are all-reduced with SUM -- the reference loss is a sum
    (models/CNNBLSTM/train.py:70), so the N-rank gradient equals the
    single-process gradient of the concatenated batch (DDP's mean would scale
    it by 1/N);
  * BatchNorm batch statistics (forward sums, backward sums) are all-reduced
    so every rank normalises with the global-batch statistics (SyncBN): the
    model's `comm` hook (ainp.cnnblstm._ConvStackFn) calls allreduce_sum_.
Everything here works with the gloo backend on CPU tensors too, which is how
the N>1 logic is tested without GPUs (tests/test_cpu_dist.py).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class Comm:
    """All-reduce helper bound to a process group."""

    def __init__(self, group=None):
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t


class GradAllReducer:
    """Bucketed SUM all-reduce of parameter gradients.

    Gradients are packed into flat buckets of at most `bucket_bytes` (fewer,
    larger collectives suit xGMI's point-to-point links), reduced, and
    unpacked.  Parameters larger than a bucket are reduced in place.
    """

    def __init__(self, params, comm: Comm, bucket_bytes: int = 64 << 20):
        self.params = [p for p in params if p.requires_grad]
        self.comm = comm
        self.bucket_bytes = bucket_bytes

    def _buckets(self):
        cur, size = [], 0
        for p in self.params:
            if p.grad is None:
                continue
            nb = p.grad.numel() * p.grad.element_size()
            if nb >= self.bucket_bytes:
                yield [p]
                continue
            if size + nb > self.bucket_bytes and cur:
                yield cur
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            yield cur

    @torch.no_grad()
    def allreduce(self):
        if self.comm.world_size == 1:
            return
        for bucket in self._buckets():
            if len(bucket) == 1:
                self.comm.allreduce_sum_(bucket[0].grad)
                continue
            flat = torch.cat([p.grad.reshape(-1) for p in bucket])
            self.comm.allreduce_sum_(flat)
            off = 0
            for p in bucket:
                n = p.grad.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n


def init_from_env(backend: str | None = None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun).
    Returns (rank, world_size, local_rank); single-process when unset."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=rank, world_size=ws)
    return rank, ws, local
