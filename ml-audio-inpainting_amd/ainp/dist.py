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

import datetime
import os

import torch
import torch.distributed as dist


class Comm:
    """All-reduce helper bound to two process groups over the same ranks:

    group       the synchronous, latency-bound exchanges the model makes
                mid-step (SyncBN sums, the VGG target max, loss normalisers);
    grad_group  the gradient buckets (GradAllReducer).

    On RCCL a process group is one communicator whose collectives run in FIFO
    order on its own stream.  Sharing one would queue the encoder's SyncBN
    backward exchange behind the 34 MB W_ih_l0 gradient buckets, and the
    compute stream waits on SyncBN.  With separate communicators the gradient
    all-reduce overlaps the rest of the backward."""

    def __init__(self, group=None, grad_group="new", host_staging=None):
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # gloo with GPU tensors (the multi-rank tests on a one-GPU box): stage
        # through host memory; RCCL ("nccl") reduces device tensors directly.
        # host_staging=False (or AINP_GLOO_DEVICE=1) hands device tensors to
        # gloo's own async CUDA path instead: the collective then runs behind
        # the issuing stream and its Work holds the reduced tensors until
        # wait(), the RCCL semantics the side-stream hand-offs must survive
        if host_staging is None:
            host_staging = (dist.get_backend(group) == "gloo"
                            and os.environ.get("AINP_GLOO_DEVICE", "0") != "1")
        self.host_staging = bool(host_staging)
        if grad_group == "new":
            # collective call: every rank constructs its Comm at the same point
            ranks = dist.get_process_group_ranks(group) if group is not None else \
                list(range(self.world_size))
            grad_group = dist.new_group(ranks=ranks) if self.world_size > 1 else group
        self.grad_group = grad_group

    def _allreduce(self, t: torch.Tensor, op, group="sync") -> torch.Tensor:
        g = self.group if group == "sync" else group
        if self.world_size > 1:
            if self.host_staging and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, op=op, group=g)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=op, group=g)
        return t

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        return self._allreduce(t, dist.ReduceOp.SUM)

    def allreduce_max_(self, t: torch.Tensor) -> torch.Tensor:
        return self._allreduce(t, dist.ReduceOp.MAX)

    def broadcast_module_(self, module: torch.nn.Module, src: int = 0) -> torch.nn.Module:
        """Every parameter and buffer from rank `src` (as DDP does at wrap
        time): identical starting weights no matter how each rank's RNG was
        consumed, and after a resume."""
        if self.world_size > 1:
            with torch.no_grad():
                for t in list(module.parameters()) + list(module.buffers()):
                    if self.host_staging and t.is_cuda:
                        h = t.detach().cpu()
                        dist.broadcast(h, src, group=self.group)
                        t.copy_(h)
                    else:
                        dist.broadcast(t.data, src, group=self.group)
                    # the write went through storage (t.data / a host copy) that
                    # does not bump t._version: bump it, so every weight cache
                    # keyed on (data_ptr, _version) -- the k-major / bf16 weight
                    # copies of ainp.ops -- rebuilds from the broadcast values
                    torch.autograd.graph.increment_version(t)
        return module


class _Done:
    """Completed-work stand-in for a synchronous (host-staged) reduction."""

    def wait(self):
        return True


class GradAllReducer:
    """Bucketed SUM all-reduce of parameter gradients, overlapped with backward.

    With overlap=True (default) a post-accumulate-grad hook on every parameter
    appends its gradient to the open bucket in the order gradients become
    ready.  That order is the same on every rank (same graph), so the
    collectives match.  A bucket that reaches `bucket_bytes` is launched at
    once as an async all-reduce.  On RCCL it runs on the communicator's own
    stream, which waits only for the work already enqueued.  So the reduction
    of the decoder/projection/LSTM gradients overlaps the encoder's backward
    kernels.  `allreduce()` (called after loss.backward()) flushes the last
    partial bucket, waits for all of them and unpacks.  A gradient larger
    than a bucket is reduced in place; smaller ones are packed into one flat
    buffer (fewer, larger collectives suit xGMI's point-to-point links).
    overlap=False keeps the plain post-backward bucketed reduce.
    """

    def __init__(self, params, comm: Comm, bucket_bytes: int = 32 << 20, overlap: bool = True):
        self.params = [p for p in params if p.requires_grad]
        self.comm = comm
        self.group = getattr(comm, "grad_group", comm.group)
        self.bucket_bytes = bucket_bytes
        self.overlap = overlap and comm.world_size > 1
        self._open, self._open_bytes = [], 0
        self._inflight = []          # (work, params, flat or None)
        self._seen = set()           # params queued since the last allreduce()
        self._chunked = set()        # params reduced chunk by chunk since then
        self.reduced_storage = {}    # id(p) -> storage pointers reduce_chunk reduced
        self._hooks = []
        self.paused = False          # hooks ignore gradients (e.g. a discarded backward)
        if self.overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._ready))

    # -- chunked early reduction ------------------------------------------------
    @property
    def early_ok(self):
        """The model may hand gradient chunks over as they are computed."""
        return self.overlap and not self.paused

    def defer(self, p):
        """p's gradient will be handed over later through reduce_chunk (a
        side-stream weight gradient): its accumulate hook must not launch a
        collective on the buffer before the side stream has written it."""
        self._seen.add(id(p))
        self._chunked.add(id(p))

    @torch.no_grad()
    def reduce_chunk(self, p, chunk: torch.Tensor, kind="early"):
        """All-reduce (SUM) one finished chunk of p's gradient now, from the
        caller's current stream: the collective waits for exactly the work
        queued on that stream (e.g. a side-stream weight-gradient GEMM) rather
        than for everything on the compute stream.  The caller owns p.grad
        (it sets it to the full buffer); allreduce() waits for the chunk."""
        self._seen.add(id(p))
        self._chunked.add(id(p))
        # storage each hand-off reduced (checked against p.grad by the DP tests:
        # the reduced buffer must be the one the optimizer reads)
        self.reduced_storage.setdefault(id(p), set()).add(chunk.untyped_storage().data_ptr())
        if self.comm.host_staging and chunk.is_cuda:
            self.comm._allreduce(chunk, dist.ReduceOp.SUM, group=self.group)
            work = _Done()
        else:
            work = dist.all_reduce(chunk, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._inflight.append((work, [], None))
        if kind == "early":
            self.early_chunks += 1
        elif kind == "pair":
            self.pair_reductions += 1
        else:
            self.side_reductions += 1

    early_chunks = 0        # layer-0 input-weight gradient chunks (reduce_chunk)
    pair_reductions = 0     # layer-0 input-weight gradients from the fused pair launch
    side_reductions = 0     # side-stream weight gradients (kind="side")

    # -- overlapped path ------------------------------------------------------
    def _ready(self, p):
        # the accumulate hook may still fire for a parameter whose .grad the
        # model set itself and handed over chunk by chunk (reduce_chunk)
        if self.paused or id(p) in self._chunked:
            return
        if id(p) in self._seen:
            raise RuntimeError("GradAllReducer: a gradient became ready twice before "
                               "allreduce() (one backward per allreduce())")
        self._seen.add(id(p))
        nb = p.grad.numel() * p.grad.element_size()
        if nb >= self.bucket_bytes:
            self._launch([p])
            return
        self._open.append(p)
        self._open_bytes += nb
        if self._open_bytes >= self.bucket_bytes:
            self._flush()

    def _flush(self):
        if self._open:
            self._launch(self._open)
        self._open, self._open_bytes = [], 0

    @torch.no_grad()
    def _launch(self, bucket):
        if len(bucket) == 1:
            flat = None
            t = bucket[0].grad
        else:
            flat = torch.cat([p.grad.reshape(-1) for p in bucket])
            t = flat
        if self.comm.host_staging and t.is_cuda:
            self.comm._allreduce(t, dist.ReduceOp.SUM, group=self.group)
            work = _Done()
        else:
            work = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._inflight.append((work, bucket, flat))

    @torch.no_grad()
    def _finish(self):
        self._flush()
        for work, bucket, flat in self._inflight:
            work.wait()
            if flat is not None:
                off = 0
                for p in bucket:
                    n = p.grad.numel()
                    p.grad.copy_(flat[off:off + n].view_as(p.grad))
                    off += n
        self._inflight = []

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.overlap = False

    # -- post-backward path ---------------------------------------------------
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
        """Call after loss.backward(): completes the SUM all-reduce of every
        parameter gradient (waits for the overlapped buckets)."""
        if self.comm.world_size == 1:
            return
        if self.overlap:
            # gradients that did not arrive through a hook (set by hand, or a
            # parameter outside this backward's graph) are reduced here
            for p in self.params:
                if p.grad is not None and id(p) not in self._seen:
                    self._ready(p)
            self._finish()
            self._seen.clear()
            self._chunked.clear()
            self.reduced_storage = {}
            return
        for bucket in self._buckets():
            self._launch(bucket)
        self._finish()


def init_from_env(backend: str | None = None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun).
    Returns (rank, world_size, local_rank); single-process when unset."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:
        # AINP_DIST_BACKEND=gloo: rehearse several ranks on one GPU (RCCL needs
        # one GPU per rank); default RCCL ("nccl") when GPUs are present
        backend = os.environ.get("AINP_DIST_BACKEND") or \
            ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl" or torch.cuda.is_available():
        torch.cuda.set_device(local if backend == "nccl" else local % max(1, torch.cuda.device_count()))
    if backend == "nccl":
        # collective failures raise instead of hanging (RCCL async error
        # handling: a failed/timed-out collective aborts the communicator)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if not dist.is_initialized():
        # AINP_DIST_TIMEOUT_S bounds every collective (default 600 s)
        timeout = datetime.timedelta(seconds=float(os.environ.get("AINP_DIST_TIMEOUT_S", "600")))
        dist.init_process_group(backend=backend, rank=rank, world_size=ws, timeout=timeout)
    return rank, ws, local
