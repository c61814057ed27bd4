"""Data-parallel level machinery of the tree grower (models/grower.py): the level counters and
collective timing, the CollStep protocol of the Python device loop and the LevelBatcher that serves
a batch of trees' reduce-scatter / all-gather with one collective each, the feature shards of a
data-parallel level (FeatureShards), and the native runners' collective callbacks and direct RCCL
communicator (_DpCollectives, _rccl_comm). Reference: /root/reference/fraud_detection_spark.py:67-83
(Spark's tree aggregation over executors, SURVEY PAR-05)."""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch

from ..utils import tracing
from ..utils.streams import StreamSwitch
from .quantize import Quantized

# device level loop counters (bench/gbdt_train.py reports the histogram payload per level: what a
# data-parallel level reduce-scatters, before the 1/S shard split)
LEVEL_STATS = {"levels": 0, "built_nodes": 0, "hist_bytes": 0, "coll_calls": 0, "coll_ms": 0.0,
               # preselected RF passes (a wave per active item): items active vs waves launched
               "listed_passes": 0, "listed_active_items": 0, "listed_grid_waves": 0}
# (begin, end) timing events of the data-parallel levels' collectives, resolved lazily by
# level_collective_ms() so that timing never adds a host wait to the level loop
_COLL_EVENTS: list = []


def reset_level_stats() -> None:
    for r in _DP_RUNNERS:                   # (their counters restart too)
        r.dp_coll_stats()
    _COLL_EVENTS.clear()
    for k in LEVEL_STATS:
        LEVEL_STATS[k] = 0


def level_collective_ms() -> float:
    dp_runner_stats()
    return _level_collective_ms()


def _level_collective_ms() -> float:
    """Milliseconds the level loops' streams spent in their reduce-scatter + all-gather (device
    event pairs around every LEVEL_TIMING-th collective, scaled by LEVEL_TIMING; as the issuing
    stream sees them: a lane whose collective queues behind another lane's on the
    communicator's stream counts that wait too)."""
    while _COLL_EVENTS:
        b, e = _COLL_EVENTS.pop(0)
        e.synchronize()
        LEVEL_STATS["coll_ms"] += b.elapsed_time(e) * max(LEVEL_TIMING, 1)
    return float(LEVEL_STATS["coll_ms"])


# Timing events around the level collectives: every LEVEL_TIMING-th collective is timed and the
# total scaled by LEVEL_TIMING (event records cost the host thread that drives the RF lanes a few
# microseconds each: timing every call added ~5 % to a forest); 1: every call, 0: none
LEVEL_TIMING = 8


class _CollTimer:
    """Times one level's collectives on the current stream (device events; host clock on the CPU)."""

    def __init__(self, dev: torch.device):
        self.cuda = dev.type == "cuda"
        self.on = LEVEL_TIMING > 0 and LEVEL_STATS["coll_calls"] % LEVEL_TIMING == 0

    def __enter__(self):
        if not self.on:
            return self
        if self.cuda:
            self.b = torch.cuda.Event(enable_timing=True)
            self.b.record()
        else:
            self.b = time.perf_counter()
        return self

    def __exit__(self, *exc):
        LEVEL_STATS["coll_calls"] += 1
        if not self.on:
            return False
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _COLL_EVENTS.append((self.b, e))
            if len(_COLL_EVENTS) > 8192:        # bounded: resolve the oldest half (long finished)
                for b, e in _COLL_EVENTS[:4096]:
                    e.synchronize()
                    LEVEL_STATS["coll_ms"] += b.elapsed_time(e) * LEVEL_TIMING
                del _COLL_EVENTS[:4096]
        else:
            LEVEL_STATS["coll_ms"] += (time.perf_counter() - self.b) * 1e3 * LEVEL_TIMING
        return False
class CollStep:
    """What a data-parallel level asks of its driver (``device_tree_steps`` yields these when it
    has ``shards``), in this order per level:
      ``alloc``  this level's histogram rows (``rows`` built nodes of width ``Bs`` bins, ``sub_rows``
                 rows for the subtracted siblings, ``n_open`` best-split tuples, the root's local
                 ``totals`` to sum) -> a :class:`LaneBufs` view into the batch's buffers;
      ``rs``     the histograms are queued: reduce-scatter them;
      ``ag``     the best-split tuples are queued: all-gather them -> [S, n_open, 5].
    A :class:`LevelBatcher` serves the same step of every tree in flight with ONE collective, so
    a forest's collective count is per batch-level, not per tree-level (SURVEY PAR-05: Spark
    aggregates the nodes of many trees in one pass)."""

    __slots__ = ("kind", "rows", "Bs", "n_open", "totals", "sub_rows")

    def __init__(self, kind: str, rows: int = 0, Bs: int = 0, n_open: int = 0, totals=None, sub_rows: int = 0):
        self.kind, self.rows, self.Bs, self.n_open, self.totals, self.sub_rows = kind, rows, Bs, n_open, totals, sub_rows


class LaneBufs:
    """One tree's share of a batched data-parallel level (LevelBatcher.serve). The send buffer is
    shard-major ``target`` [S, R, Bs, 2]: the tree's built rows are rows [row0, row0 + rows) of
    every shard chunk, so its histogram passes write with row stride Bs and shard stride R * Bs;
    the root's local (g, h) totals ride in bin ``tot_bin`` of every chunk (the reduce-scatter then
    sums them too: no separate all-reduce per tree). The reduced rows land in ``out`` [R + subs,
    Bs, 2] (the collective writes rows [0, R)); rows [sub_base, sub_base + rows) take the tree's
    subtracted siblings, so no histogram row is copied. ``ag_in`` [n_open, 5]: where the split
    search writes the tree's best-split tuples for the batched all-gather."""

    __slots__ = ("target", "row0", "rows", "R", "Bs", "tot_bin", "ag_in", "out", "sub_base")

    def __init__(self, target, row0, rows, R, Bs, tot_bin, ag_in, out, sub_base):
        self.target, self.row0, self.rows, self.R, self.Bs = target, row0, rows, R, Bs
        self.tot_bin, self.ag_in, self.out, self.sub_base = tot_bin, ag_in, out, sub_base

    @property
    def shard_bins(self) -> int:
        return self.R * self.Bs

    def prepare(self, totals=None) -> torch.Tensor:
        """Place the root totals (the batch zeroed the buffer); returns the [*, Bs, 2] view the
        histogram passes write through (row 0 = this tree's first row of shard 0)."""
        if totals is not None:
            self.target.view(self.target.shape[0], -1, 2)[:, self.tot_bin] = totals
        return self.target.view(-1, self.Bs, 2)[self.row0:]

    def mine(self) -> torch.Tensor:
        return self.out[self.row0:self.row0 + self.rows]

    def reduced_totals(self) -> torch.Tensor:
        return self.out.view(-1, 2)[self.tot_bin]


class _Lane:
    """A tree in flight: its step generator, the step / event it is parked at, its stream (and
    that stream's reusable switch and join event)."""

    __slots__ = ("gen", "item", "stream", "tid", "switch", "event")

    def __init__(self, gen, item, stream, tid=None, switch=None, event=None):
        self.gen, self.item, self.stream, self.tid = gen, item, stream, tid
        self.switch = switch if switch is not None else StreamSwitch(stream)
        self.event = event

    def send(self, value) -> None:
        with self.switch:
            self.item = self.gen.send(value)


class LevelBatcher:
    """Serves the data-parallel collectives of a batch of trees in flight (each parked at an
    ``alloc`` CollStep) with one reduce-scatter and one all-gather for the whole batch. Buffers
    are allocated on the coordinator stream; each tree's kernels run on its own stream, joined to
    the coordinator by events around the two collectives. The batch's buffers are held until
    ``release()`` -- called by the driver once it has waited for every tree's next event, which
    follows all of the tree's reads of them (so the caching allocator never hands them out early).
    Every rank serves the same batches in the same order (the drivers' orders are functions of the
    tree shapes, identical on every rank), so the collective sequences match."""

    def __init__(self, coll, S: int, dev: torch.device, coord=None):
        self.coll, self.S, self.dev = coll, int(S), dev
        self.coord = coord if coord is not None else (torch.cuda.current_stream(dev) if dev.type == "cuda" else None)
        self.switch = StreamSwitch(self.coord)
        self.coord_event = torch.cuda.Event() if self.coord is not None else None
        self.hold = None
        self.batches = 0

    def release(self) -> None:
        self.hold = None

    def _ctx(self):
        return self.switch

    def _join_in(self, lanes) -> None:
        """The coordinator stream waits for every lane's queued work (reusable per-lane events)."""
        if self.coord is None:
            return
        for ln in lanes:
            if ln.stream is not None and ln.stream != self.coord:
                if ln.event is None:
                    ln.event = torch.cuda.Event()
                ln.event.record(ln.stream)
                self.coord.wait_event(ln.event)

    def _join_out(self, lanes) -> None:
        if self.coord is None:
            return
        recorded = False
        for ln in lanes:
            if ln.stream is not None and ln.stream != self.coord:
                if not recorded:
                    self.coord_event.record(self.coord)
                    recorded = True
                ln.stream.wait_event(self.coord_event)

    def serve(self, lanes: list) -> None:
        reqs = [ln.item for ln in lanes]
        assert all(isinstance(r, CollStep) and r.kind == "alloc" for r in reqs), [getattr(r, "kind", r) for r in reqs]
        S = self.S
        Bs = max(max(r.Bs for r in reqs), 1)
        nrows = sum(r.rows for r in reqs)
        ntot = sum(1 for r in reqs if r.totals is not None)
        R = nrows + (-(-ntot // Bs) if ntot else 0)
        subs = sum(r.sub_rows for r in reqs)
        nl = sum(r.n_open for r in reqs)
        with self._ctx():
            # one zero fill for the whole batch, on the coordinator stream; every tree's stream
            # waits for it before its histogram passes add into the buffer
            target = torch.zeros((S, R, Bs, 2), dtype=torch.int64, device=self.dev)
            out = torch.empty((R + subs, Bs, 2), dtype=torch.int64, device=self.dev)
            ag_in = torch.empty((nl, 5), dtype=torch.int64, device=self.dev)
        self._join_out(lanes)
        row0 = sub0 = l0 = t = 0
        slots = []
        for ln, r in zip(lanes, reqs):
            tb = -1
            if r.totals is not None:
                tb = nrows * Bs + t
                t += 1
            bufs = LaneBufs(target, row0, r.rows, R, Bs, tb, ag_in[l0:l0 + r.n_open], out, R + sub0)
            slots.append((l0, r.n_open))
            row0 += r.rows
            sub0 += r.sub_rows
            l0 += r.n_open
            ln.send(bufs)
        assert all(isinstance(ln.item, CollStep) and ln.item.kind == "rs" for ln in lanes)
        self._join_in(lanes)
        with self._ctx(), tracing.span("tree.reduce_scatter", trees=len(lanes)), _CollTimer(self.dev):
            self.coll.reduce_scatter(target, out=out[:R])
        self._join_out(lanes)
        for ln in lanes:
            ln.send(None)
        assert all(isinstance(ln.item, CollStep) and ln.item.kind == "ag" for ln in lanes)
        self._join_in(lanes)
        with self._ctx(), tracing.span("tree.all_gather", trees=len(lanes)), _CollTimer(self.dev):
            allt = self.coll.all_gather(ag_in)                           # [S, sum n_open, 5]
        self._join_out(lanes)
        for ln, (a, n) in zip(lanes, slots):
            ln.send(allt[:, a:a + n])
        self.hold = (target, out, ag_in, allt)
        self.batches += 1


class FeatureShards:
    """Split-find ownership for data-parallel training: rank r owns the contiguous feature range
    [fs[r], fs[r+1]) (balanced by bin count). The histogram passes of a DP level write straight
    into a SHARD-MAJOR buffer [S, n_build, Bs, 2] (``boff_packed``: per-feature bin offsets that
    fold in the feature's shard), so the level's ONE reduce-scatter sends that buffer as it
    stands, with no repacking copy; the shard's own boff/nbins/zbin/fid_orig drive the split
    kernel on the reduced slice."""

    def __init__(self, Q: Quantized, S: int, rank: int):
        boff = np.asarray(Q.boff_host, dtype=np.int64)
        TB, Fa = int(boff[-1]), Q.Fa
        cuts = np.searchsorted(boff, [TB * s / S for s in range(1, S)], side="left")
        fs = np.concatenate([[0], np.clip(cuts, 0, Fa), [Fa]]).astype(np.int64)
        fs = np.maximum.accumulate(fs)
        lo, hi = boff[fs[:-1]], boff[fs[1:]]
        self.S, self.fs = S, fs
        self.max_shard_features = int((fs[1:] - fs[:-1]).max()) if S else 0
        self.Bs = max(1, int((hi - lo).max()))
        dev = Q.device
        shard_of = np.searchsorted(fs[1:], np.arange(Fa + 1), side="right").clip(0, S - 1).astype(np.int64)
        local = boff - lo[shard_of]
        local[Fa] = 0
        shard_of[Fa] = S                      # boff[Fa] -> the end of the buffer
        self._shard_of = torch.from_numpy(shard_of).to(dev)
        self._local = torch.from_numpy(local).to(dev)
        self._boffp: dict = {}
        f0, f1 = int(fs[rank]), int(fs[rank + 1])
        self.bin_lo = torch.from_numpy(np.append(lo, boff[-1]).astype(np.int64)).to(dev)   # [S + 1] shard bin starts
        self.f0, self.Fa, self.bins = f0, f1 - f0, int(hi[rank] - lo[rank])
        self.boff = (Q.boff[f0: f1 + 1] - Q.boff[f0]).contiguous()
        self.nbins = Q.nbins[f0:f1].contiguous()
        # compact RF levels (compact()): per-level layout buffers of this workspace
        self._nbins_all = Q.nbins
        self._fs_dev = torch.from_numpy(fs).to(dev)
        self.max_nb = int(Q.nbins.max()) if Fa else 1
        # two sets (level parity): level d + 1's layout is computed while level d is in flight
        self._local_c = [torch.zeros(Fa + 1, dtype=torch.int64, device=dev) for _ in range(2)]
        self._sizes = [torch.zeros(S, dtype=torch.int64, device=dev) for _ in range(2)]
        self.sizes_host = [torch.zeros(S, dtype=torch.int64) for _ in range(2)]
        if dev.type == "cuda":
            self.sizes_host = [t.pin_memory() for t in self.sizes_host]
        self._thr = [None, None]
        self._mask = [torch.empty(Fa, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.zbin = Q.zbin[f0:f1].contiguous()
        self.fid_orig = Q.fid_orig[f0:f1].contiguous()

    def boff_packed(self, nb: int) -> torch.Tensor:
        """[Fa+1] bin offsets into the shard-major [S * nb, Bs] histogram rows: bin b of feature f
        (shard s) of node slot n lands in row s * nb + n at column local(f) + b, i.e. at offset
        n * Bs + (s * nb * Bs + local(f)) + b with the kernels' hist_stride = Bs. Cached per nb."""
        t = self._boffp.get(nb)
        if t is None:
            t = self._boffp[nb] = (self._shard_of * (nb * self.Bs) + self._local).contiguous()
        return t

    def target(self, nb: int, dev) -> torch.Tensor:
        """Zeroed shard-major partial histograms [S, nb, Bs, 2] of a DP level."""
        return torch.zeros((self.S, nb, self.Bs, 2), dtype=torch.int64, device=dev)

    def boff_batched(self, shard_bins: int, local: Optional[torch.Tensor] = None) -> torch.Tensor:
        """[Fa+1] bin offsets into a batched level's send buffer (LaneBufs): feature f of shard s
        at s * shard_bins + local(f) (+ the row's slot * Bs in the kernels). ``local``: a compact
        level's per-level offsets (not cached); None: the full layout's (cached per stride)."""
        if local is not None:
            return torch.add(local, self._shard_of, alpha=int(shard_bins))
        key = ("b", int(shard_bins))
        t = self._boffp.get(key)
        if t is None:
            t = self._boffp[key] = (self._shard_of * int(shard_bins) + self._local).contiguous()
        return t

    def sample_compact(self, C, p: int, seed: int, tree: int, nodes: torch.Tensor, F: int, k: int,
                       fid_orig: torch.Tensor) -> None:
        """Feature sample of the open nodes ``nodes`` (-1 padding allowed) into parity-``p``
        buffers, then the level's compact layout (csrc/tree.h RfCompactArgs): the features of the
        union sample mask packed per shard, the rest aimed at a per-shard trash range. Queues the
        copy of the shard sizes to ``sizes_host[p]``: read it after the next event the caller
        records on this stream."""
        n = int(nodes.numel())
        thr = self._thr[p]
        if thr is None or thr.numel() < n:
            thr = self._thr[p] = torch.empty(max(n, 2), dtype=torch.float64, device=nodes.device)
        C.tree_rf_sample(seed, tree, nodes, F, k, fid_orig, thr[:n], self._mask[p], None)
        C.tree_rf_compact(self._mask[p], self._nbins_all, self._fs_dev, self._local_c[p], self._sizes[p],
                          self.max_shard_features)
        self.sizes_host[p].copy_(self._sizes[p], non_blocking=nodes.is_cuda)

    def compact_thr(self, p: int, n: int) -> torch.Tensor:
        """The parity-``p`` per-node sampling thresholds, at least ``n`` long (sample_compact's)."""
        thr = self._thr[p]
        if thr is None or thr.numel() < n:
            thr = self._thr[p] = torch.empty(max(n, 2), dtype=torch.float64, device=self._mask[p].device)
        return thr

    def compact_mask(self, p: int) -> torch.Tensor:
        """The parity-``p`` level's union feature mask (sample_compact)."""
        return self._mask[p]

    def compact_level(self, p: int, n_open: int):
        """(feat_thr [n_open], feat_mask, local offsets [Fa + 1], stride) of the parity-``p`` layout
        (its sizes must have reached the host): stride = the largest shard's sampled bins plus
        the trash range."""
        return (self._thr[p][:n_open], self._mask[p], self._local_c[p],
                int(self.sizes_host[p].max()) + self.max_nb)


def drive(steps, batcher: Optional[LevelBatcher] = None):
    """Run a step generator to its end, synchronising every event it yields and serving its
    data-parallel CollSteps with ``batcher`` (a batch of one tree); returns its value."""
    try:
        lane = _Lane(steps, next(steps), None)
        while True:
            if isinstance(lane.item, CollStep):
                batcher.serve([lane])
            else:
                lane.item.synchronize()
                batcher is not None and batcher.release()
                lane.item = steps.send(None)
    except StopIteration as stop:
        return stop.value


class _DpCollectives:
    """The level collectives the runner's data-parallel GBDT loop calls back into
    (csrc/bindings_level.cpp gbdt_dp_level): the level's reduce-scatter into the runner's buffer,
    the all-gather of the best-split tuples, the quantisation max (in place)."""

    def __init__(self, coll, dev: torch.device):
        self.coll, self.dev = coll, dev

    def rs(self, send: torch.Tensor, out: torch.Tensor) -> None:
        with tracing.span("tree.reduce_scatter"), _CollTimer(self.dev):
            self.coll.reduce_scatter(send, out=out)

    def ag(self, x: torch.Tensor) -> torch.Tensor:
        with tracing.span("tree.all_gather"), _CollTimer(self.dev):
            return self.coll.all_gather(x).contiguous()

    def mx(self, t: torch.Tensor) -> None:
        r = self.coll.max(t)
        if r is not t:
            t.copy_(r)


# data-parallel GBDT runners that issue RCCL themselves (their collective counts / timings are
# pulled into parallel.dist.CALLS and LEVEL_STATS by dp_runner_stats)
_DP_RUNNERS: list = []


def _rccl_comm(dev: torch.device) -> tuple:
    """(ncclComm_t as int, path of torch's librccl.so) of the default process group on ``dev``, or
    (None, None) when the backend is not RCCL (gloo) or the communicator is not reachable."""
    import torch.distributed as dist

    try:
        from . import grower as G            # (the switch lives there; tests flip it)
        if not G.DP_DIRECT_RCCL or dev.type != "cuda" or dist.get_backend() != "nccl":
            return None, None
        pg = dist.distributed_c10d._get_default_group()
        ptr = int(pg._get_backend(dev)._comm_ptr())
    except Exception:                                       # noqa: BLE001 (the callbacks then)
        return None, None
    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return (ptr, lib) if ptr and os.path.exists(lib) else (None, None)


def dp_runner_stats() -> None:
    """Adds the direct-RCCL runners' collective calls and timed milliseconds to
    parallel.dist.CALLS and LEVEL_STATS (resolves their timing events: a sync point)."""
    from ..parallel import dist as D

    for r in _DP_RUNNERS:
        rs, ag, ar, ms = r.dp_coll_stats()
        D.CALLS["reduce_scatter"] += int(rs)
        D.CALLS["all_gather"] += int(ag)
        D.CALLS["all_reduce"] += int(ar)
        LEVEL_STATS["coll_calls"] += int(rs + ag)
        LEVEL_STATS["coll_ms"] += ms
