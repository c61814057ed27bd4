"""Data-parallel process group helpers (PAR-01..PAR-04, C-01/C-02).

One process per GPU; ``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm, over xGMI
inside a node) for device tensors, ``gloo`` for CPU-only runs/tests. Collectives used by the
engine are all *sums/max of statistics* (histograms, docFreq, gradients, root totals) whose
results are bitwise identical on every rank, so every rank takes the same split decisions and no
model broadcast is needed during training.

Launch: ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...`` or
``launch.spawn(fn, world_size)`` for tests.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def forced() -> bool:
    """``FDX_FORCE_COLLECTIVES=1`` with an initialised group of any size (including 1): run every
    collective through the backend instead of short-circuiting, so a one-GPU box exercises the
    RCCL reduce-scatter / all-gather path of the trainers."""
    return (os.environ.get("FDX_FORCE_COLLECTIVES") == "1" and dist.is_available() and dist.is_initialized())


def _comm() -> bool:
    return is_dist() or forced()


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", rank()))


def init_from_env(backend: Optional[str] = None, timeout_s: float = 600.0) -> bool:
    """Initialise from torchrun's env (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT). Returns True if a
    multi-process group is active. A world-size-1 group is only created in forced-collectives
    mode (``FDX_FORCE_COLLECTIVES=1``)."""
    if dist.is_initialized():
        return dist.get_world_size() > 1
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 and os.environ.get("FDX_FORCE_COLLECTIVES") != "1":
        return False
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", str(ws))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local_rank() % max(1, torch.cuda.device_count()))
    if "MASTER_PORT" not in os.environ:
        from .launch import free_port

        os.environ["MASTER_PORT"] = str(free_port())
    dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    return ws > 1


def backend() -> str:
    return dist.get_backend() if dist.is_initialized() else "none"


def _on_comm_device(t: torch.Tensor):
    """gloo needs host tensors; nccl device tensors."""
    if backend() == "gloo" and t.is_cuda:
        return t.cpu(), True
    return t, False


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if not _comm():
        return t
    x, moved = _on_comm_device(t.contiguous())
    BYTES["all_reduce"] += x.numel() * x.element_size()
    CALLS["all_reduce"] += 1
    dist.all_reduce(x, op=op)
    return x.to(t.device) if moved else x


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    return all_reduce(t, dist.ReduceOp.SUM)


def all_reduce_max(t: torch.Tensor) -> torch.Tensor:
    return all_reduce(t, dist.ReduceOp.MAX)


def all_gather_var(*tensors: torch.Tensor) -> tuple:
    """All-gather 1-D tensors of different lengths per rank; returns the concatenation. The
    lengths travel in one all-gather and are read back with ONE host sync."""
    if not _comm():
        return tensors
    dev = tensors[0].device
    n = torch.tensor([tensors[0].numel()], dtype=torch.int64, device=dev)
    sizes = all_gather(n).view(-1).tolist()
    m = max(sizes)
    out = []
    for t in tensors:
        pad = torch.zeros(m, dtype=t.dtype, device=t.device)
        pad[: t.numel()] = t
        p, moved = _on_comm_device(pad)
        bufs = [torch.empty_like(p) for _ in range(world_size())]
        CALLS["all_gather"] += 1
        dist.all_gather(bufs, p)
        cat = torch.cat([b[:s] for b, s in zip(bufs, sizes)])
        out.append(cat.to(t.device) if moved else cat)
    return tuple(out)


def broadcast_object(obj, src: int = 0):
    if not is_dist():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def barrier() -> None:
    if is_dist():
        if backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def shard_range(n: int, r: Optional[int] = None, w: Optional[int] = None) -> tuple:
    """Contiguous row shard [lo, hi) of ``n`` rows for rank ``r`` of ``w``."""
    r = rank() if r is None else r
    w = world_size() if w is None else w
    base, extra = divmod(n, w)
    lo = r * base + min(r, extra)
    return lo, lo + base + (1 if r < extra else 0)


# bytes this process handed to each collective (payload sizes, for the per-level DP accounting)
# and the number of collective calls issued (every backend call, per kind)
BYTES = {"reduce_scatter": 0, "all_gather": 0, "all_reduce": 0}
CALLS = {"reduce_scatter": 0, "all_gather": 0, "all_reduce": 0}


def reset_bytes() -> None:
    for k in BYTES:
        BYTES[k] = 0
        CALLS[k] = 0


def total_calls() -> int:
    return int(sum(CALLS.values()))


def reduce_scatter(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum ``x`` [world, ...] over ranks and return this rank's slice [...] with
    ``reduce_scatter_tensor``: each rank sends (N-1)/N of the buffer instead of an all-reduce's
    2(N-1)/N. The same call runs on RCCL (device tensors) and on gloo (host copies), so the CPU
    multi-process tests exercise the code path the GPUs take. ``out`` (contiguous, x[0]'s size):
    the collective writes there (a prefix of a larger level buffer, no copy on RCCL)."""
    if not _comm():
        if out is None:
            return x[0]
        return out.view(x.shape[1:]).copy_(x[0])
    x = x.contiguous()
    BYTES["reduce_scatter"] += x.numel() * x.element_size()
    CALLS["reduce_scatter"] += 1
    xc, moved = _on_comm_device(x)
    # flat buffers (gloo wants the concatenated form; RCCL takes either)
    n = xc.numel() // xc.shape[0]
    if out is not None and not moved:
        assert out.is_contiguous() and out.numel() == n and out.dtype == xc.dtype
        dist.reduce_scatter_tensor(out.view(-1), xc.view(-1))
        return out.view(xc.shape[1:])
    res = torch.empty(n, dtype=xc.dtype, device=xc.device)
    dist.reduce_scatter_tensor(res, xc.view(-1))
    res = res.view(xc.shape[1:])
    if out is not None:
        return out.view(xc.shape[1:]).copy_(res)
    return res.to(x.device) if moved else res


def all_gather(x: torch.Tensor) -> torch.Tensor:
    """[...] on every rank -> [world, ...] (same shape on every rank), ``all_gather_into_tensor``
    on RCCL and gloo alike."""
    if not _comm():
        return x.unsqueeze(0)
    x = x.contiguous()
    BYTES["all_gather"] += x.numel() * x.element_size()
    CALLS["all_gather"] += 1
    xc, moved = _on_comm_device(x)
    out = torch.empty(world_size() * xc.numel(), dtype=xc.dtype, device=xc.device)
    dist.all_gather_into_tensor(out, xc.view(-1))
    out = out.view((world_size(),) + tuple(xc.shape))
    return out.to(x.device) if moved else out


class Collectives:
    """Bundle of the collectives the trainers need (no-ops when not distributed)."""

    def __init__(self):
        self.force = forced()
        self.active = is_dist() or self.force
        self.world = world_size()
        self.rank = rank()

    def reduce_scatter(self, x, out=None):
        if self.active:
            return reduce_scatter(x, out)
        return x[0] if out is None else out.view(x.shape[1:]).copy_(x[0])

    def all_gather(self, x):
        return all_gather(x) if self.active else x.unsqueeze(0)

    def sum(self, t):
        return all_reduce_sum(t) if self.active else t

    def max(self, t):
        return all_reduce_max(t) if self.active else t

    def min(self, t):
        return all_reduce(t, dist.ReduceOp.MIN) if self.active else t

    def gather_keys(self, keys, counts):
        return all_gather_var(keys, counts) if self.active else (keys, counts)
