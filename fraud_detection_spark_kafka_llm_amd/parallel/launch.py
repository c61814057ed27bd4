"""Single-node multi-process launcher (one rank per GPU, or CPU ranks over gloo for tests).

``spawn(fn, world_size, *args)`` starts ``world_size`` processes with RANK/LOCAL_RANK/WORLD_SIZE/
MASTER_ADDR=127.0.0.1/MASTER_PORT set, initialises the process group (``nccl`` = RCCL when GPUs
are visible, else ``gloo``), runs ``fn(rank, world_size, *args)`` and returns the per-rank results
(pickled back through a queue). For production jobs use ``torchrun --nproc-per-node N
--master-addr 127.0.0.1`` with ``dist.init_from_env()``.
"""
from __future__ import annotations

import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, backend, fn, args, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    try:
        from . import dist

        dist.init_from_env(backend)
        out = fn(rank, world, *args)
        q.put((rank, "ok", out))
    except Exception:   # report instead of hanging the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as td

        if td.is_initialized():
            td.destroy_process_group()


def spawn(fn, world_size: int, *args, backend: str = "gloo", timeout: float = 600.0) -> list:
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world_size, port, backend, fn, args, q)) for r in range(world_size)]
    for p in procs:
        p.start()
    results: dict = {}
    errors = []
    try:
        for _ in range(world_size):
            rank, status, payload = q.get(timeout=timeout)
            if status == "ok":
                results[rank] = payload
            else:
                errors.append(f"rank {rank}:\n{payload}")
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errors:
        raise RuntimeError("distributed run failed:\n" + "\n".join(errors))
    return [results[r] for r in range(world_size)]
