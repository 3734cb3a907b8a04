"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL.

The env step shards naturally (envs never interact), so the only exchange is
in the PPO update: the flattened gradient (one bucket, ~566 KB
for the 256x256 MLPs) is all-reduced per mini-batch, the KL mean is averaged
so the adaptive learning rate stays identical on every rank, advantage
statistics are global, and rank 0's initial parameters are broadcast.  On a
single process every helper is a no-op.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
    """torchrun contract (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*); returns (rank, local_rank, world)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    r = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(lr)
        dist.init_process_group(backend=backend, rank=r, world_size=ws)
    return r, lr, ws


def broadcast_params(module: torch.nn.Module, src: int = 0):
    if not is_dist():
        return
    for p in module.parameters():
        dist.broadcast(p.data, src=src)
    for b in module.buffers():
        dist.broadcast(b, src=src)


class FlatGrads:
    """One persistent flat gradient buffer; every parameter's `.grad` is a view of it.

    The PPO update zeroes the gradients in place (`zero_grad(set_to_none=False)`, 0 + g == g exactly), so
    autograd accumulates into the views and the data-parallel exchange is a single in-place all-reduce of
    `flat` (~566 KB for the 256x256 MLPs: latency-bound on xGMI, one message), with no concatenation or
    scatter-back.  The graph-captured update writes its gradients into the same views."""

    def __init__(self, params, extra: int = 1):
        self.params = list(params)
        p0 = self.params[0]
        n = sum(p.numel() for p in self.params)
        # `extra` trailing slots ride along in the same message: the graph-captured update's KL mean (ppo.py)
        self.flat = torch.zeros(n + extra, device=p0.device, dtype=p0.dtype)
        self.extra = self.flat[n:]
        self.views, off = [], 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        self.bind()

    def bind(self):
        for p, v in zip(self.params, self.views):
            p.grad = v

    def bound(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(self.params, self.views))

    # measurement hook (bench.py): when a list, every exchange appends a (start, end) pair of events recorded on the
    # current stream around the collective and the division, i.e. the time the update's stream waits for the exchange
    timings: list | None = None

    def allreduce_(self):
        """Average over ranks in place (the views see the result)."""
        if is_dist():
            ev = None
            if FlatGrads.timings is not None and self.flat.is_cuda:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
            self.flat.div_(world_size())
            if ev is not None:
                ev[1].record()
                FlatGrads.timings.append(ev)


def allreduce_grads(params, flat: FlatGrads | None = None) -> None:
    """Average gradients over ranks in ONE flat bucket (latency-bound message on xGMI): in place when the
    gradients are the views of `flat`, else through a concatenated copy."""
    if not is_dist():
        return
    if flat is not None and flat.bound():
        flat.allreduce_()
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat.div_(world_size())
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


def allreduce_max_int(v: int, device) -> int:
    """Max of an integer over ranks (the host value is exchanged in a one-element tensor on the backend's device:
    CUDA for RCCL, CPU for gloo)."""
    if not is_dist():
        return int(v)
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def allreduce_mean(t: torch.Tensor) -> torch.Tensor:
    if not is_dist():
        return t
    t = t.clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t / world_size()


def global_mean_std(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Mean / unbiased std of x over all ranks (== torch.mean/std of the concatenation)."""
    if not is_dist():
        return x.mean(), x.std()
    n = torch.tensor(float(x.numel()), device=x.device, dtype=torch.float64)
    s = x.sum().double()
    stats = torch.stack([n, s])
    dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    mean = stats[1] / stats[0]
    sq = ((x.double() - mean) ** 2).sum()
    dist.all_reduce(sq, op=dist.ReduceOp.SUM)
    std = torch.sqrt(sq / (stats[0] - 1))
    return mean.float(), std.float()
