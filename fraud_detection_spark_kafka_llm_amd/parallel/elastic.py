"""Elastic multi-process launcher with a parent watchdog (failure detection,
checkpoint/resume).

``run_elastic(fn, world_size, *args)`` starts one process per rank (``spawn`` start method: the
children are fresh interpreters, never an exec of a GPU-initialised process), each with
RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT and ``FDX_ATTEMPT`` set, initialises the
process group and runs ``fn(rank, world, *args)``. The parent watches the ranks: a rank that
raises, exits abnormally or is killed (e.g. a lost GPU) makes the parent terminate the survivors
(they would otherwise block in the next collective) and relaunch the job with one rank fewer, down
to ``min_world``. The trainers checkpoint every few trees and resume with any world size (the
histogram sums do not depend on the row sharding), so the relaunched job continues from the last
checkpoint (``fn`` reads ``attempt() > 0`` to resume) and ends with the same model.

The reference has no failure handling at all: a Spark executor loss restarts the whole job.
"""
from __future__ import annotations

import os
import queue as _queue
import time
import traceback
from dataclasses import dataclass, field

import torch.multiprocessing as mp

from ..utils.logging import get_logger
from .launch import free_port

log = get_logger("elastic")


def attempt() -> int:
    """Relaunch counter of the current job (0 = first launch)."""
    return int(os.environ.get("FDX_ATTEMPT", "0"))


@dataclass
class ElasticReport:
    results: list
    world_size: int
    attempts: int
    failures: list = field(default_factory=list)     # (attempt, world, rank, reason)


def _entry(rank, world, port, backend, fn, args, q, att):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "FDX_ATTEMPT": str(att)})
    try:
        from . import dist

        dist.init_from_env(backend)
        out = fn(rank, world, *args)
        q.put((rank, "ok", out))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as td

        if td.is_initialized():
            td.destroy_process_group()


def run_elastic(fn, world_size: int, *args, backend: str = "gloo", min_world: int = 1, max_restarts: int = 3,
                timeout: float = 3600.0, poll_s: float = 0.1) -> ElasticReport:
    ctx = mp.get_context("spawn")
    world = int(world_size)
    failures = []
    for att in range(max_restarts + 1):
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=_entry, args=(r, world, port, backend, fn, args, q, att), daemon=False)
                 for r in range(world)]
        for p in procs:
            p.start()
        results: dict = {}
        failed = None
        deadline = time.time() + timeout
        while len(results) < world and failed is None:
            try:
                rank, status, payload = q.get(timeout=poll_s)
                if status == "ok":
                    results[rank] = payload
                else:
                    failed = (rank, payload.strip().splitlines()[-1] if payload else "error")
                continue
            except _queue.Empty:
                pass
            for r, p in enumerate(procs):
                if p.exitcode not in (None, 0) and r not in results:
                    failed = (r, f"process exited with code {p.exitcode}")
                    break
            if failed is None and time.time() > deadline:
                failed = (-1, f"timeout after {timeout:.0f}s")
        if failed is None:
            for p in procs:
                p.join(timeout=60)
            return ElasticReport([results[r] for r in range(world)], world, att + 1, failures)
        # survivors report collective errors (connection reset) as soon as a peer dies: blame
        # a rank that died without reporting, if one shows up within a short grace period
        grace = time.time() + 2.0
        while time.time() < grace:
            dead = [r for r, p in enumerate(procs) if p.exitcode not in (None, 0) and r not in results]
            if dead:
                failed = (dead[0], f"process exited with code {procs[dead[0]].exitcode}")
                break
            time.sleep(0.05)
        # a rank is gone: the survivors would block in their next collective -> stop them all
        for p in procs:
            if p.is_alive():
                p.kill()
        for p in procs:
            p.join(timeout=30)
        failures.append((att, world, failed[0], failed[1]))
        log.warning("attempt %d (world %d): rank %s failed: %s", att, world, failed[0], failed[1])
        if world - 1 < min_world:
            break
        world -= 1
    raise RuntimeError(f"elastic job failed after {len(failures)} attempt(s): {failures}")
