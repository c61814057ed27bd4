"""Random-forest trees in flight together (PAR-05).

Spark's RandomForest grows nodes of many trees per pass over the data (node groups sized by
``maxMemoryInMB``; /root/reference/fraud_detection_spark.py:67-74 trains 100 trees). A forest
level with ⌈√F⌉ features sampled per node is a small GPU job on MI355X: at 10M rows the root
pass of one tree activates ~2K CSC work items (a few waves per CU of 256) and a level of 16 nodes
~33K, so one tree at a time leaves most of the chip idle while its level waits on its own
dependent kernels (sample -> histogram -> split -> plan -> partition).

Here up to ``TREES_IN_FLIGHT`` trees run the device level loop (grower.device_tree_steps) at once,
each on its own HIP stream with its own workspace (digit words, row -> node map, level state:
~0.2 GB per lane at 10M rows). One host thread drives them: whenever a tree reaches a point where
it needs a device result (the next level's 16-byte counts, its finished node table) the driver
moves on to another tree, so the kernels of different trees overlap on the device. Every tree
depends only on (seed, tree index) and its own buffers, so the forest is bitwise the forest of
one-at-a-time growth (tested on the host and the GPU).

Data parallelism (BASELINE config 3, RF at DP=8): the lanes are split into ``LANE_GROUPS`` groups
that take turns. A group's turn advances every one of its trees by one level: the host waits for
each tree's counts (refilling lanes whose tree finished), then ONE batched reduce-scatter and ONE
all-gather (grower.LevelBatcher) carry the level histograms and best splits of all the group's
trees -- 2 collectives per group-level instead of 2 per tree-level (500 trees x 5 levels: 5,000
-> ~625 with 2 groups of 8), and a tree's root totals ride in its first reduce-scatter. While one
group's collectives are in flight the other group's kernels keep the GPU busy. Turn order,
lane order and refill order are functions of the tree shapes only, which every rank computes
identically from the same reduced histograms, so every rank issues the same collective sequence.
(Alone, the driver advances "the first lane whose event completed", an order that depends on
timing and needs no agreement.)

The shared read-only state the lanes read (the CSC work items and their wave order, the shard
tables) is built on the caller's stream BEFORE the lanes fork from it, never lazily by whichever
lane touches it first (that would leave the other lanes' streams unordered with the build).

(An earlier design grew 8 trees in lockstep through one multi-tree histogram kernel with 24 bytes
of per-row records; it lost to per-tree passes, profiles/r2_rf_batch_ab.txt, and was replaced.)
"""
from __future__ import annotations

import time
import os
from collections import deque
from typing import Optional

import torch

import numpy as np

from ..ops import native
from ..utils import tracing
from ..utils.streams import StreamSwitch
from . import grower as G
from .grower import CollStep, GrowParams, LevelBatcher, Workspace, _Lane, device_tree_steps
from .quantize import Quantized

# 500 trees x depth 5 on 10M rows (profiles/r4/rf500_sweep_*.json): 4 lanes with 4 histogram
# streams each 1.02 s, 8 x 1 0.97 s, 12 x 1 0.95 s, 16 x 1 0.92 s (+0.27 GB of workspace per lane)
TREES_IN_FLIGHT = int(os.environ.get("FDX_RF_INFLIGHT", "16"))
# histogram side streams per lane (grower.Workspace.run_concurrent): the lanes already overlap
# whole trees, and every extra stream is another HW-queue mapping and cross-stream event per level
LANE_HIST_STREAMS = 1
# data parallelism: groups of lanes whose levels share one reduce-scatter + all-gather
LANE_GROUPS = int(os.environ.get("FDX_RF_GROUPS", "2"))
# sampled RF trees grow in lockstep batches on the native runner (csrc/bindings_level.cpp RfBatch):
# every stage of a level is ONE lane-batched launch for all the trees in flight and the level loop
# runs in C++ (0: the per-tree lanes driven from Python)
BATCH = os.environ.get("FDX_RF_BATCH", "1") == "1"
# ... in this many batches that take turns on the stream (1: the host-side level work is ~0.15 ms
# per batch-level, RfBatch.host_times; 2 batches of 8 measured 0.26 vs 0.22 s on the DP=8 shard,
# profiles/r6/rf_batches_sweep.txt): while the host waits for one batch's
# level counts and queues its next level, the GPU runs the other batch's level
BATCHES = int(os.environ.get("FDX_RF_BATCHES", "1"))


class ForestLanes:
    """Per-lane workspaces and streams (lane 0 reuses the caller's workspace)."""

    def __init__(self, Q: Quantized, lanes: int, ws0: Optional[Workspace] = None):
        self.ws = [ws0 if (i == 0 and ws0 is not None) else Workspace(Q) for i in range(lanes)]
        for w in self.ws:
            w.hist_streams = LANE_HIST_STREAMS
        cuda = Q.device.type == "cuda"
        self.streams = [torch.cuda.Stream(Q.device) for _ in range(lanes)] if cuda else [None] * lanes
        self.switches = [StreamSwitch(s) for s in self.streams]
        self.events = [torch.cuda.Event() if cuda else None for _ in range(lanes)]
        self.dev = Q.device

    def stream_ctx(self, i: int):
        return self.switches[i]


def batch_ok(Q: Quantized, params: GrowParams, weight) -> bool:
    """The lockstep batch covers the default sampled-RF configuration on the device (the lean
    runner level loop with fused packed row state and the LDS-atomic count passes)."""
    return (BATCH and Q.device.type == "cuda" and G.NATIVE_LEVELS and G.SAMPLED and G.FUSED_PACK and
            G.RF_LDS and params.feat_k > 0 and G._choose_np(params, weight) == 1 and params.max_depth >= 1 and
            G.device_levels_ok(params, weight))


class ForestBatch:
    """The lanes' workspaces, level states and runners handed to one native RfBatch (built once
    per ForestLanes and tree parameters): per lane the level buffers of the runner's level loop
    plus two pinned node-table copies (the host builds one batch's trees while the next grows)."""

    def __init__(self, Q: Quantized, wss: list, params: GrowParams, coll=None, shards: list = None):
        dev = Q.device
        presel = G.PRESELECT and Q.n_rows >= G.PRESELECT_MIN_ROWS
        item_groups = Q.groups + Q.hot_groups
        sel_ids = [gi for gi, grp in enumerate(item_groups) if grp.num_items] if presel else []
        dp = shards is not None and shards[0] is not None
        compact = dp and 0 < params.feat_k < Q.num_features and \
            (G.RF_COMPACT == "1" or (G.RF_COMPACT == "auto" and shards[0].S > 1))
        D = int(params.max_depth)
        self.Q, self.params, self.dp, self.compact = Q, params, dp, bool(compact)
        self.views, lane_cfg = [], []
        self.n_lanes = len(wss)
        self.parity = 0
        for i, ws in enumerate(wss):
            st = getattr(ws, "_levels", None)
            if st is None or st.max_depth != D or st.n_sel != len(sel_ids):
                st = ws._levels = G.LevelState(Q, D, len(sel_ids))
            runner = G._level_runner(Q, ws, st, params, item_groups, True)
            if st.rf_thr is None:
                st.rf_thr = [torch.empty(st.cap, dtype=torch.float64, device=dev) for _ in range(2)]
                st.rf_mask = [torch.empty(Q.Fa, dtype=torch.uint8, device=dev) for _ in range(2)]
            hosts = [st.arena_host, torch.zeros_like(st.arena_host).pin_memory()]
            self.views.append([{k: v.numpy() for k, v in st.host_views(h).items()} for h in hosts])
            lc = dict(runner=runner, open0=st.open[0], open1=st.open[1], totals0=st.totals[0], totals1=st.totals[1],
                      arena=st.arena, arena_init=st.arena_init_dev, arena_host0=hosts[0], arena_host1=hosts[1],
                      tot_scratch=ws.totals, rowpack=ws.rowpack(),
                      sel=[ws.item_list(gi, grp)[0] if gi in sel_ids else None for gi, grp in enumerate(item_groups)],
                      listed=[ws.item_list(gi, grp) if grp.num_items else (None, None)
                              for gi, grp in enumerate(item_groups)])
            if compact:
                sh = shards[i]
                for p in (0, 1):
                    lc[f"thr{p}"] = sh.compact_thr(p, st.cap)
                    lc[f"mask{p}"] = sh.compact_mask(p)
                    lc[f"sh_local{p}"] = sh._local_c[p]
                    lc[f"sh_sizes{p}"] = sh._sizes[p]
                    lc[f"sh_sizes_host{p}"] = sh.sizes_host[p]
            else:
                for p in (0, 1):
                    lc[f"thr{p}"] = st.rf_thr[p]
                    lc[f"mask{p}"] = st.rf_mask[p]
            if not dp:
                # the level's histograms: every open node built, the deepest level opens 2^(D-1)
                lc["hist"] = torch.empty((max(1, 1 << (D - 1)), Q.TB, 2), dtype=torch.int64, device=dev)
                lc["packed"] = torch.empty((st.cap, 5), dtype=torch.int64, device=dev)
            lane_cfg.append(lc)
        st0 = wss[0]._levels
        cfg = dict(lanes=lane_cfg, max_depth=D, boff=Q.boff, listed_max_nodes=G.LISTED_MAX_NODES, presel=bool(sel_ids),
                   one=st0.one, zero1=st0.zero1, iota=wss[0].iota(64), dp=dp)
        if dp:
            sh = shards[0]
            cfg.update(S=int(sh.S), Bs=int(sh.Bs), max_nb=int(sh.max_nb), compact=bool(compact), shard_of=sh._shard_of,
                       sh_local=sh._local, sh_boff=sh.boff, sh_nbins=sh.nbins, sh_zbin=sh.zbin, sh_fid=sh.fid_orig,
                       sh_fs=sh._fs_dev, nbins_all=Q.nbins, f0=int(sh.f0), Fa_s=int(sh.Fa),
                       max_shard_features=int(sh.max_shard_features),
                       wide=G._wide_features(sh.nbins, sh.Fa) if G.SPLIT_WIDE else None)
        else:
            cfg["wide"] = G._wide_features(Q.nbins, Q.Fa) if G.SPLIT_WIDE else None
        self.cfg = cfg
        self.native = None

    def bind(self, coll) -> None:
        """Creates the native batch (with the collectives of ``coll`` under data parallelism)."""
        if self.native is not None:
            return
        cfg = dict(self.cfg)
        if self.dp:
            cb = G._DpCollectives(coll, self.Q.device)
            comm, lib = G._rccl_comm(self.Q.device)
            cfg.update(rs=cb.rs, ag=cb.ag, comm=comm, rccl_lib=lib)
        self.native = native.lib().RfBatch(cfg)


def grow_forest_batched(Q: Quantized, lanes: ForestLanes, params: GrowParams, tree_ids: list, label: torch.Tensor,
                        weight: Optional[torch.Tensor], bootstrap: bool, coll=None) -> list:
    """Grows ``tree_ids`` in lockstep batches (RfBatch); returns them in order. The lanes are split
    into BATCHES batches that take turns on the one stream: each turn waits for one batch's level
    counts and queues its next level, so the GPU runs the other batch's level meanwhile; a batch
    whose trees finished queues its node tables and starts the next trees at once, and the host
    builds the finished trees while that batch's new root level runs. The turn order depends on
    the tree shapes only, so under data parallelism every rank issues the same collectives."""
    use_coll = coll is not None and coll.active
    shards = build_shared_state(Q, lanes, coll if use_coll else None)
    nl = len(lanes.ws)
    nb = max(1, min(BATCHES, nl))
    key = (params.max_depth, params.mode, params.min_gain, params.min_child, params.seed, params.feat_k,
           shards[0] is not None, nb)
    cached = getattr(lanes, "_batch", None)
    if cached is None or cached[0] != key:
        parts = [range(g * nl // nb, (g + 1) * nl // nb) for g in range(nb)]
        cached = lanes._batch = (key, [ForestBatch(Q, [lanes.ws[i] for i in r], params, coll if use_coll else None,
                                                   [shards[i] for i in r]) for r in parts])
    fbs = cached[1]
    for fb in fbs:
        fb.bind(coll if use_coll else None)
    from ..parallel import dist as D

    todo = deque(tree_ids)
    out: dict = {}
    running: list = [None] * nb

    def launch(i: int) -> None:
        running[i] = None
        if not todo:
            return
        fb = fbs[i]
        ids = [todo.popleft() for _ in range(min(fb.n_lanes, len(todo)))]
        fb.parity ^= 1
        t0 = time.perf_counter()
        with tracing.span("forest.batch", trees=len(ids)):
            fb.native.start(ids, label, weight, bool(bootstrap), int(Q.row0))
        HOST_TIMES["start_s"] += time.perf_counter() - t0
        running[i] = ids

    def account(fb, stat) -> None:
        G.LEVEL_STATS["levels"] += stat[0]
        G.LEVEL_STATS["built_nodes"] += stat[1]
        G.LEVEL_STATS["hist_bytes"] += stat[1] * Q.TB * 16
        G.LEVEL_STATS["listed_passes"] += stat[2]
        G.LEVEL_STATS["listed_active_items"] += stat[3]
        G.LEVEL_STATS["listed_grid_waves"] += stat[4]
        if fb.dp and fb.native.direct():    # (RCCL called by the batch itself; the callbacks count their own)
            G.LEVEL_STATS["coll_calls"] += stat[5] + stat[6]
            D.CALLS["reduce_scatter"] += stat[5]
            D.CALLS["all_gather"] += stat[6]

    if EVENT_PROBE:
        p0 = torch.cuda.Event(enable_timing=True)
        p0.record()
    for i in range(nb):
        launch(i)
    while any(r is not None for r in running):
        for i in range(nb):
            ids = running[i]
            ts = time.perf_counter()
            if ids is None or fbs[i].native.step():
                continue
            fb = fbs[i]
            par = fb.parity
            t0 = time.perf_counter()
            HOST_TIMES["last_step_s"] += t0 - ts
            account(fb, fb.native.finish(par))
            t1 = time.perf_counter()
            if EVENT_PROBE:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
            launch(i)                     # the slot's next trees, queued before the host builds these
            if EVENT_PROBE and running[i] is not None:
                e2 = torch.cuda.Event(enable_timing=True)
                e2.record()
                _probe.append((e1, e2))
            HOST_TIMES["turn_s"] += time.perf_counter() - ts
            if running[i] is not None and fb.compact:
                # (a compact DP batch queues its root level once the root's shard sizes are back:
                # that wait is short, and the GPU then runs the level while the host builds trees)
                fb.native.step()
            t2 = time.perf_counter()
            fb.native.wait()              # (its event: the node tables just queued, not re-recorded yet)
            t3 = time.perf_counter()
            for lane, t in enumerate(ids):
                out[t] = G.tree_from_host(Q, params, fb.views[lane][par])
            HOST_TIMES["finish_s"] += t1 - t0
            HOST_TIMES["tables_wait_s"] += t3 - t2
            HOST_TIMES["build_s"] += time.perf_counter() - t3
    if EVENT_PROBE:
        p1 = torch.cuda.Event(enable_timing=True)
        p1.record()
        torch.cuda.synchronize()
        HOST_TIMES["gpu_phase_ms"] += p0.elapsed_time(p1)
    if EVENT_PROBE and _probe:
        torch.cuda.synchronize()
        HOST_TIMES["gpu_turn_ms"] += sum(a.elapsed_time(b) for a, b in _probe)
        _probe.clear()
    for fb in fbs:
        if fb.dp and fb.native.direct():
            G.LEVEL_STATS["coll_ms"] += fb.native.coll_ms()
        lv, fl, wt = fb.native.host_times()
        HOST_TIMES["levels_s"] += lv
        HOST_TIMES["flush_s"] += fl
        HOST_TIMES["wait_s"] += wt
    return [out[t] for t in tree_ids]


# host seconds of the lockstep batches (RfBatch.host_times): queuing levels, of which flushes, waits
HOST_TIMES = {"levels_s": 0.0, "flush_s": 0.0, "wait_s": 0.0, "start_s": 0.0, "finish_s": 0.0, "tables_wait_s": 0.0,
              "build_s": 0.0, "last_step_s": 0.0, "turn_s": 0.0, "gpu_turn_ms": 0.0,
              "gpu_phase_ms": 0.0}
EVENT_PROBE = os.environ.get("FDX_RF_EVENT_PROBE") == "1"
_probe: list = []


def build_shared_state(Q: Quantized, lanes: ForestLanes, coll=None) -> list:
    """Build every lazily created structure more than one lane reads, on the current stream:
    the CSC histogram items (Q.groups, Q.hot_groups, Q.h_row/h_key) and each group's wave order;
    under data parallelism each lane's feature-shard tables. Returns the per-lane shards (or
    Nones)."""
    for grp in Q.groups + Q.hot_groups:
        if grp.num_items:
            grp.wave_order()
    Q.h_row, Q.h_key                                           # noqa: B018 (built by the access)
    if coll is not None and coll.active and (coll.world > 1 or getattr(coll, "force", False)):
        return [ws.shards(coll) for ws in lanes.ws]
    return [None] * len(lanes.ws)


def grow_forest_concurrent(Q: Quantized, lanes: ForestLanes, params: GrowParams, tree_ids: list,
                           label: torch.Tensor, weight: Optional[torch.Tensor], bootstrap: bool,
                           coll=None) -> list:
    """Grow the trees ``tree_ids`` with up to ``len(lanes.ws)`` in flight; returns them in order.
    ``coll`` (parallel.dist.Collectives, active): data-parallel levels, lanes advanced in FIFO
    order so that every rank issues the same collective sequence."""
    cuda = lanes.dev.type == "cuda"
    use_coll = coll is not None and coll.active
    if batch_ok(Q, params, weight):
        return grow_forest_batched(Q, lanes, params, tree_ids, label, weight, bootstrap, coll)
    shards = build_shared_state(Q, lanes, coll if use_coll else None)
    if cuda:                                   # the lanes see everything queued before (Q, label, shared state)
        main = torch.cuda.current_stream(lanes.dev)
        start = main.record_event()
        for s in lanes.streams:
            s.wait_event(start)
    if use_coll and any(sh is not None for sh in shards):
        out = _grow_batched(Q, lanes, params, tree_ids, label, weight, bootstrap, coll, shards,
                            main if cuda else None)
        if cuda:
            for s in lanes.streams:
                main.wait_stream(s)
        return out
    todo = deque(tree_ids)
    out: dict = {}
    live: dict = {}                            # lane -> [tree id, steps, event]
    order: deque = deque()                     # lanes in the order their events were recorded

    def advance(i: int) -> None:
        rec = live[i]
        with lanes.stream_ctx(i):
            try:
                rec[2] = next(rec[1])
                order.append(i)
                return
            except StopIteration as stop:
                out[rec[0]] = stop.value
        del live[i]
        launch(i)

    def launch(i: int) -> None:
        if not todo:
            return
        t = todo.popleft()
        with tracing.span("forest.tree", tree=t, lane=i):
            live[i] = [t, device_tree_steps(Q, lanes.ws[i], params, t, None, None, weight,
                                            coll if use_coll else None, shards[i], label=label,
                                            bootstrap=bootstrap), None]
        advance(i)

    for i in range(len(lanes.ws)):
        launch(i)
    while order:
        if use_coll:
            # rank-deterministic: always the oldest pending event (the collective order follows)
            ready = order[0]
            live[ready][2].synchronize()
        else:
            # the first lane whose event completed, else wait for the oldest one
            ready = next((i for i in order if live[i][2].query()), None)
            if ready is None:
                ready = order[0]
                live[ready][2].synchronize()
        order.remove(ready)
        advance(ready)
    if cuda:
        for s in lanes.streams:
            main.wait_stream(s)
    return [out[t] for t in tree_ids]


def _grow_batched(Q: Quantized, lanes: ForestLanes, params: GrowParams, tree_ids: list, label: torch.Tensor,
                  weight: Optional[torch.Tensor], bootstrap: bool, coll, shards: list, coord) -> list:
    """The data-parallel driver (module docstring): lane groups take turns; a turn waits for the
    group's trees, refills finished lanes, and serves one batched level of collectives."""
    nl = len(lanes.ws)
    ng = max(1, min(LANE_GROUPS, nl))
    groups = [list(range(g * nl // ng, (g + 1) * nl // ng)) for g in range(ng)]
    # a coordinator stream per group: a group's batch fill and collectives never queue behind the
    # other group's (RCCL still runs them on its own stream in issue order)
    coords = [None] * ng
    if coord is not None:
        start = coord.record_event()
        coords = [torch.cuda.Stream(lanes.dev) for _ in range(ng)]
        for c in coords:
            c.wait_event(start)
    batchers = [LevelBatcher(coll, shards[0].S, lanes.dev, c) for c in coords]
    todo = deque(tree_ids)
    out: dict = {}
    state: list = [None] * nl                  # lane -> _Lane (tid = tree id) or None

    def start(i: int) -> None:
        state[i] = None
        if not todo:
            return
        t = todo.popleft()
        with tracing.span("forest.tree", tree=t, lane=i), lanes.stream_ctx(i):
            gen = device_tree_steps(Q, lanes.ws[i], params, t, None, None, weight, coll, shards[i], label=label,
                                    bootstrap=bootstrap)
            state[i] = _Lane(gen, next(gen), lanes.streams[i], t, lanes.switches[i], lanes.events[i])

    def resume(i: int) -> None:
        ln = state[i]
        ln.item.synchronize()
        try:
            ln.send(None)
        except StopIteration as stop:
            out[ln.tid] = stop.value
            start(i)

    for i in range(nl):
        start(i)
    turns = deque(range(ng))
    while turns:
        g = turns.popleft()
        while True:          # every tree of the group up to its next collective step (or done)
            waiting = [i for i in groups[g] if state[i] is not None and not isinstance(state[i].item, CollStep)]
            if not waiting:
                break
            for i in waiting:
                resume(i)
        batchers[g].release()
        live = [state[i] for i in groups[g] if state[i] is not None]
        if live:
            batchers[g].serve(live)
            turns.append(g)
    if coord is not None:
        for c in coords:
            coord.wait_stream(c)
    return [out[t] for t in tree_ids]
