"""Level-wise histogram tree grower shared by DecisionTree, RandomForest and GBDT (X-09, X-10, X-13).

Per tree, ``tree_quant`` quantises the two row statistics (GBDT g*w, h*w; classification
w*[y==0], w*[y==1]) to integers q = rint(v * 2^k) (csrc/tree.h); the exponent k comes from the
global max |v| (all-reduced under data parallelism). Every histogram is then an exact int64 sum,
so trees are bitwise identical on the host, on the device and at any world size. A level (all its
nodes batched into every launch):
  1. histograms of the built nodes -- GBDT: the row-group engine (csrc/row_kernels.hip: row lists
     of the built rows, LDS int64 tables per bin group, the smaller sibling only); RF / DT: the CSC
     work items of the sampled features (csrc/tree_kernels.hip hist_lds_kernel, LDS atomics);
  2. data parallel: ONE reduce-scatter of the level's partials by feature shard (RCCL);
  3. split search over this rank's features (the larger sibling subtracted inside it), best
     split per node; data parallel: ONE all-gather of the per-shard best tuples;
  4. ``level_plan`` on the device: applies the splits to the device node table and plans the
     next level (open list, builds, subtraction rows; RF: the next level's feature sample and its
     active work items);
  5. partition of the rows to the children (zeroing the next level's histograms on the way).
The host reads a 16-byte count row per level and the node table once per tree. Drivers, fastest
first: the native runner's C++ level loops (csrc/bindings_level.cpp: RfLevels.gbdt_levels /
gbdt_dp_levels for GBDT, RfBatch for RF trees in lockstep batches, models/forest_batch.py), the
Python device loop ``device_tree_steps`` (the test oracle of the native loops, and the CPU path
through the kernels' host twins), and the host loop ``grow_tree`` (deep trees). The data-parallel
machinery (level counters, LevelBatcher, feature shards, the runners' collectives) is in
models/dp_batch.py, the host-side trees (GrowParams, TreeTable, tree_from_host) in
models/tree_table.py; both are re-exported here.
"""
from __future__ import annotations

import functools
import os
from typing import Optional

import numpy as np
import torch

from ..ml.tree_model import Tree
from ..ops import native
from ..utils import tracing
from . import quantize as qmod
from .dp_batch import (LEVEL_STATS, LEVEL_TIMING, CollStep, FeatureShards, LaneBufs, LevelBatcher,  # noqa: F401
                       _CollTimer, _DP_RUNNERS, _DpCollectives, _Lane, _level_collective_ms, _rccl_comm, drive,
                       dp_runner_stats, level_collective_ms, reset_level_stats)
from .quantize import Quantized
from .tree_table import GrowParams, PendingTree, TreeTable, _impurity, leaf_values_device, tree_from_host  # noqa: F401

NEG_INF = float("-inf")
MAX_CT = 8                      # column tiles per pass (csrc/tree_kernels.hip launch_hist)
DENSE_RANGE_ROWS = 32768        # max rows per wave of the dense hot-feature histogram kernel


def dense_range_rows(n_rows: int, ngroups: int) -> int:
    """Rows per wave of the dense hot-feature kernel (fixed: shorter ranges for launches with few
    feature groups measured no better, profiles/r2_gbdt_knob_sweep.txt)."""
    return DENSE_RANGE_ROWS
# levels 0..DENSE_MAX_DEPTH build the hot features' histograms with the dense kernel (every row
# streamed, slot-masked); deeper levels use their CSC items (only live entries multiplied)
DENSE_MAX_DEPTH = 2
# histogram launches of one pass (CSC groups, dense groups) run concurrently on this many HIP
# streams: they add into disjoint feature ranges with integer atomics, so the order is free and
# the kernels fill each other's tails
HIST_STREAMS = 4


# row-group histogram engine (models/quantize.RowGroups, csrc/row_kernels.hip): every level's
# histograms from the row-group CSR of the built rows, in place of the CSC / dense passes
ROWHIST = True
RG_DBG = 0   # diagnostics only (csrc/tree.h RgHistArgs::dbg)
# RF passes over sampled features: packed row state (slot + class counts in one word per row) and
# a device-compacted list of the active work items (tree_hist_sampled)
SAMPLED = True
LISTED_MAX_NODES = 2
# RF levels >= 1 launch one wave per active work item from lists compacted with the previous
# level's plan (0: the r4 passes, a wave per item slot or a fixed listed grid)
PRESELECT = True
# ... on shards of at least this many rows. Once the packed items skip their unsampled features
# and the selects of a level are one launch, the listed passes win at 1.25M rows too (DP=8 shard,
# forced collectives: 0.456 -> 0.446 s a forest, profiles/r5/rf_lean_presel_ab_1M.jsonl; before,
# 143 -> 207 us a pass the other way); at 10M rows they win (0.768 -> 0.747 s)
PRESELECT_MIN_ROWS = 0
# RF levels >= 1 read the packed row state (slot | class-count digits) written by the previous
# level's partition instead of a row pass of their own (slot pack / masked digits: ~87 us per level
# at 10M rows, 173 ms of a 500-tree forest's kernel time, profiles/r5/NOTES.md)
FUSED_PACK = True
# RF device levels issue their kernels through the native per-level runner (csrc/bindings_level.cpp
# RfLevels: hist / split / plan / partition, one host call each) instead of ~20 Python-level calls
NATIVE_LEVELS = True
# single-process runner levels subtract the larger siblings inside the split search
SPLIT_SUBTRACT = True
# the partition's row pass writes the next level's row-list counts (runner levels, <= 4M rows)
PARTITION_COUNTS = True
# single-slot row-group passes reduce per-workgroup partial tables (0: every workgroup's atomics)
RG_PARTIALS = True
# ... and so do the listed passes over several slots (a workgroup whose chunk straddles a slot
# boundary still flushes with atomics)
RG_PARTIALS_MULTI = True
# single-process GBDT trees on the row-group engine: the level loop runs in the runner (C++,
# RfLevels.gbdt_levels; 0: the generic Python loop)
GBDT_CXX_LEVELS = True
# ... which builds the sibling with fewer rows (not the smaller hessian sum) where the row lists
# count their own rows (above 4M rows, or FDX_PARTITION_COUNTS=0): same trees, shorter lists;
# the partition's rows per node, kept per 512-row wave, also stand in for the lists' counting pass
GBDT_CHOOSE_ROWS = True
LIST_NODE_COUNTS = True
# RF / DT count passes: the LDS-atomic kernel (one ds_add_u64 per entry) instead of i8 MFMA
RF_LDS = True
# split search: a wave per (node, feature) for the features with > 16 bins
SPLIT_WIDE = True
# partition splits on dense-block features in the row pass (FDX_PARTITION_DENSE=0: CSC column pass)
PARTITION_DENSE = True
# RF levels under data parallelism reduce-scatter only the bins of the level's sampled features
# (FeatureShards.sample_compact). "auto": when the reduce-scatter crosses ranks (world > 1; at
# world 1 it is a local copy and the layout pass only costs); "1" always (the world-1 RCCL
# rehearsal of the path); "0" never
RF_COMPACT = os.environ.get("FDX_RF_COMPACT", "auto")


# GBDT trees grow with the device-resident level loop (grow_tree_device): split application and
# next-level planning run on the GPU, the host reads 16 bytes per level and the node table once
# per tree (FDX_DEVICE_LEVELS=0: host loop)
DEVICE_LEVELS = True
PARTITION_WPS = 256  # blocks per column split (device partition)
# debug: check on the host that every open node of a data-parallel level is built or subtracted
# (its histogram row is then written before the split search reads it)
LEVEL_CHECKS = os.environ.get("FDX_LEVEL_CHECKS", "0") == "1"


class Workspace:
    """Per-engine device buffers reused across trees (digits, slot table, row -> node map)."""

    def __init__(self, Q: Quantized, max_nodes_per_level: int = 0):
        dev = Q.device
        self.rowdig = torch.empty((Q.n_rows, 2), dtype=torch.int32, device=dev)
        self.kexp = torch.zeros(2, dtype=torch.int32, device=dev)
        self.totals = torch.zeros(2, dtype=torch.int64, device=dev)
        self.maxabs = torch.zeros(2, dtype=torch.float64, device=dev)
        # padded to a multiple of 64 rows for the dense kernel (pad bytes stay 0xff = no slot)
        self.slot8_pad = torch.full((Q.n_pad,), 0xFF, dtype=torch.uint8, device=dev)
        self.slot8 = self.slot8_pad[:Q.n_rows]
        self.digp = torch.zeros((8, Q.n_pad), dtype=torch.uint8, device=dev) if Q.dense is not None else None
        self._dense_groups: dict = {}
        self.dense_waves = int(native.lib().tree_dense_waves())
        self.row_node = torch.zeros(Q.n_rows, dtype=torch.int32, device=dev)
        self.Fa = Q.Fa
        self.dev = dev
        self.Q = Q
        self._shards = None
        self.staging = Staging(dev)
        self._streams = None
        self.split_cache: dict = {}          # _best_splits scratch per level shape

    def rowgroups(self):
        """The row-group CSR when the row-group engine is on and covers every feature (else None),
        plus the level's row-list buffers."""
        if not ROWHIST:
            return None
        rg = self.Q.rowgroups()
        if not rg.complete:
            return None
        if getattr(self, "rg_list", None) is None:
            self.rg_list = torch.empty(self.Q.n_rows, dtype=torch.int32, device=self.dev)
            self.rg_start = torch.zeros(66, dtype=torch.int32, device=self.dev)
            nw = -(-self.Q.n_rows // native.lib().tree_rg_list_rows(self.Q.n_rows))   # waves of the list kernels
            self.rg_work = torch.zeros(64 * (2 + nw), dtype=torch.int32, device=self.dev)
            self.rg_listdig = torch.empty((self.Q.n_rows, 2), dtype=torch.int32, device=self.dev)
        return rg

    def rg_emdig(self) -> torch.Tensor:
        """[N, 2] digit words zeroed outside the one built node (entry-major listed pass)."""
        if getattr(self, "_rg_emdig", None) is None:
            self._rg_emdig = torch.empty((self.Q.n_rows, 2), dtype=torch.int32, device=self.dev)
        return self._rg_emdig

    def rg_part(self, rg, other_work=None) -> torch.Tensor:
        """[n_wg, gbins, 2] int64 scratch of a row-group pass's partial tables (sized for the
        larger of rg.work() and ``other_work``)."""
        n_wg = max(int(rg.work().shape[1]), int(other_work.shape[1]) if other_work is not None else 0)
        need = n_wg * int(rg.gbin.shape[1]) * 2
        t = getattr(self, "_rg_part", None)
        if t is None or t.numel() < need:
            t = self._rg_part = torch.empty(need, dtype=torch.int64, device=self.dev)
        return t

    def dig16(self) -> torch.Tensor:
        """[N] int16: the rows' two class-count digits (RF), written by the runner's quantisation
        for the fused partition's packed row state (2 bytes a row instead of the 8-byte word)."""
        if getattr(self, "_dig16", None) is None:
            self._dig16 = torch.empty(self.Q.n_rows + 8, dtype=torch.int16, device=self.dev)
        return self._dig16

    def rowpack(self) -> torch.Tensor:
        """[N] int32 packed row state of the sampled (RF) passes: slot | class-count digits << 8."""
        if getattr(self, "_rowpack", None) is None:
            self._rowpack = torch.empty(self.Q.n_rows, dtype=torch.int32, device=self.dev)
        return self._rowpack

    def item_list(self, gi: int, grp) -> tuple:
        """(list, count) device scratch of a listed pass over item group ``gi`` (one per group: the
        groups' passes run on concurrent streams)."""
        lists = getattr(self, "_item_lists", None)
        if lists is None:
            lists = self._item_lists = {}
        slots = grp.wave_order().numel()
        need = 8 * ((-(-slots // 4) + 7) // 8 * 4)          # per-XCD lists (tree_kernels.hip hist_select)
        cur = lists.get(gi)
        if cur is None or cur[0].numel() < need:
            cur = lists[gi] = (torch.empty(need, dtype=torch.int32, device=self.dev),
                               torch.zeros(8, dtype=torch.int32, device=self.dev))
        return cur

    def run_concurrent(self, launches: list) -> None:
        """Run the launches on HIST_STREAMS side streams joined back into the current stream
        (serially on the current stream on the host or with one stream). The first launch (the
        long cold-feature CSC pass) runs on the current stream and the others share the
        HIST_STREAMS - 1 side streams, so none queues behind it (a short launch behind it added
        0.15-0.25 ms to every level)."""
        nstreams = getattr(self, "hist_streams", HIST_STREAMS)
        if self.dev.type != "cuda" or nstreams <= 1 or len(launches) <= 1:
            for fn in launches:
                fn()
            return
        if self._streams is None:
            self._streams = [torch.cuda.Stream(self.dev) for _ in range(nstreams - 1)]
        main = torch.cuda.current_stream(self.dev)
        start = main.record_event()
        ns = len(self._streams)
        # the long first launch stays on the current stream and is issued first: it starts right
        # behind the slot pass and the next level's kernels follow it in stream order, with no
        # cross-stream event wait on the critical path (~15 + ~35 us per level measured on the
        # side-stream variant); the side streams wait for ``start``, recorded before it
        launches[0]()
        for i, fn in enumerate(launches[1:]):
            s = self._streams[i % ns]
            s.wait_event(start)
            with torch.cuda.stream(s):
                fn()
        for s in self._streams[:min(len(launches) - 1, ns)]:
            main.wait_stream(s)

    def dense_groups(self, bt: int, fg: int, keep: Optional[np.ndarray] = None):
        """(gfid, gdense) device arrays [ngroups * fg] of the hot features with ``bt`` row tiles
        (optionally only those with ``keep[d]``), -1 padded; cached when ``keep`` is None."""
        key = (bt, fg)
        if keep is None and key in self._dense_groups:
            return self._dense_groups[key]
        Q = self.Q
        d = np.nonzero((Q.hot_bt == bt) & (keep if keep is not None else True))[0]
        per_wg = fg * self.dense_waves
        ng = (d.size + per_wg - 1) // per_wg * self.dense_waves
        gfid = np.full(ng * fg, -1, dtype=np.int32)
        gden = np.zeros(ng * fg, dtype=np.int32)
        gfid[:d.size] = Q.hot[d]
        gden[:d.size] = d
        out = (torch.from_numpy(gfid).to(self.dev), torch.from_numpy(gden).to(self.dev))
        if keep is None:
            self._dense_groups[key] = out
        return out

    def gh(self) -> tuple:
        """[N] float32 g, h buffers of the GBDT rounds (computed on the device per round)."""
        if getattr(self, "_gh", None) is None:
            self._gh = (torch.empty(self.Q.n_rows, dtype=torch.float32, device=self.dev),
                        torch.empty(self.Q.n_rows, dtype=torch.float32, device=self.dev))
        return self._gh

    def iota(self, n: int) -> torch.Tensor:
        """[0, 1, ..., n - 1] int32 on the device (cached: one allocation per workspace)."""
        t = getattr(self, "_iota", None)
        if t is None or t.numel() < n:
            t = self._iota = torch.arange(max(n, 64), dtype=torch.int32, device=self.dev)
        return t[:n]

    def shards(self, coll) -> "FeatureShards":
        if getattr(self, "_shards", None) is None or self._shards.S != coll.world:
            self._shards = FeatureShards(self.Q, coll.world, coll.rank)
        return self._shards


class Staging:
    """Per-level small host arrays (slot maps, subtraction triples, node totals, partition lists)
    gathered into one pinned buffer and sent with ONE async H2D copy, instead of a synchronous
    pageable copy per array (~15 per level, the bulk of the grower's host overhead). Two pinned
    buffers alternate; an event guards reuse. Tensors returned by ``upload`` are views into a
    device buffer that the next upload overwrites in stream order, so callers consume them before
    uploading again (the grower uploads at level start and after the split decisions)."""

    def __init__(self, dev: torch.device, cap: int = 1 << 16):
        self.dev = dev
        self.cuda = dev.type == "cuda"
        self._cap = 0
        self._host, self._events, self._flip = [None, None], [None, None], 0
        self._reserve(cap)
        self._items: list = []
        self._off = 0

    def _reserve(self, cap: int) -> None:
        if cap <= self._cap:
            return
        if self.cuda:
            torch.cuda.synchronize(self.dev)
        self._cap = cap
        mk = (lambda: torch.empty(cap, dtype=torch.uint8).pin_memory()) if self.cuda else \
            (lambda: torch.empty(cap, dtype=torch.uint8))
        self._host = [mk(), mk()]
        self._events = [None, None]
        self._dev = torch.empty(cap, dtype=torch.uint8, device=self.dev)

    def add(self, arr) -> int:
        a = np.ascontiguousarray(arr)
        self._items.append(a)
        return len(self._items) - 1

    def upload(self) -> list:
        offs, total = [], 0
        for a in self._items:
            total = (total + 7) & ~7
            offs.append(total)
            total += a.nbytes
        if total > self._cap:
            self._reserve(max(total, 2 * self._cap))
        k = self._flip
        self._flip ^= 1
        if self._events[k] is not None:
            self._events[k].synchronize()
        host = self._host[k].numpy()
        for a, o in zip(self._items, offs):
            host[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
        if self.cuda:
            self._dev[:total].copy_(self._host[k][:total], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[k] = ev
            src = self._dev
        else:
            src = self._host[k].clone()
        out = []
        for a, o in zip(self._items, offs):
            t = src[o:o + a.nbytes].view(_TORCH_DTYPE[a.dtype.str[1:]]).view(a.shape)
            out.append(t)
        self._items = []
        return out


_TORCH_DTYPE = {"i4": torch.int32, "i8": torch.int64, "f8": torch.float64, "f4": torch.float32}


def slots_per_tile(np_: int) -> int:
    """Node slots per 16-column MFMA tile: 2 statistics x ``np_`` digit planes per slot."""
    return 16 // (2 * np_)


def pass_ct(np_: int, cnt: int) -> int:
    """Column tiles (power of two) for ``cnt`` node slots."""
    per = slots_per_tile(np_)
    ct = 1
    while ct * per < cnt:
        ct *= 2
    return ct


def _best_splits(C, hist, totals, boff, nbins, zbin, fid_orig, node_ids, kexp, params, feat_thr, tree_index, Fa,
                 f0, node_tree=None, cache: Optional[dict] = None, out: Optional[torch.Tensor] = None,
                 row_of: Optional[torch.Tensor] = None):
    """Per node: (gain float64, feature (+f0) int64, bin int64, left sums int64 [2]) of the best
    split over Fa features of ``hist`` [nodes, boff[Fa], 2]; gain -inf without a valid candidate.
    Returned as one int64 tensor [nodes, 5] (gain bit-cast) for a single device->host copy.
    ``cache`` (a workspace dict): the per-(node, feature) scratch is allocated once per level
    shape and reused (stream order: the previous level's split kernels are done with it).
    ``out``: write the tuples there (a tree's rows of a batched all-gather). ``row_of``: the
    histogram row of each node (data-parallel levels; default row = node index). (The kernels
    take the row stride from hist.size(1), never from boff[Fa]: a compact RF level's boff[Fa]
    is the next shard's first offset, not this shard's end.)"""
    dev = hist.device
    nl = int(node_ids.numel())
    if Fa == 0:
        if out is None:
            out = torch.empty((nl, 5), dtype=torch.int64, device=dev)
        out.zero_()
        out[:, 0] = torch.tensor(NEG_INF, dtype=torch.float64).view(torch.int64)
        out[:, 1:3] = -1
        return out
    bufs = cache.get((nl, Fa)) if cache is not None else None
    if bufs is None:
        bufs = (torch.empty((nl, Fa), dtype=torch.float64, device=dev), torch.empty((nl, Fa), dtype=torch.int32, device=dev),
                torch.empty((nl, Fa, 2), dtype=torch.int64, device=dev))
        if cache is not None:
            cache[(nl, Fa)] = bufs
    out_gain, out_bin, out_left = bufs
    # features with > 16 bins get a wave each (tree_kernels.hip split_wide_kernel): listed once per
    # nbins tensor (kept on the tensor itself, shared by every forest lane; one read of the counts)
    wide = None
    if dev.type == "cuda" and SPLIT_WIDE:
        memo = getattr(nbins, "_fdx_wide", None)
        if memo is None or memo[0] != Fa:
            idx = np.nonzero(nbins[:Fa].cpu().numpy() > 16)[0].astype(np.int32)
            memo = (Fa, torch.from_numpy(idx).to(dev))
            nbins._fdx_wide = memo
        wide = memo[1]
    C.tree_split_find(hist, totals, boff, nbins, zbin, fid_orig, node_ids, kexp, int(params.mode),
                      float(params.lambda_), float(params.min_child), feat_thr, int(params.seed), int(tree_index),
                      out_gain, out_bin, out_left, node_tree, wide, row_of)
    # best gain per node, ties to the lowest feature index (deterministic whatever the batch shape):
    # one native reduction instead of ~9 small torch launches per level
    if out is None:
        out = torch.empty((nl, 5), dtype=torch.int64, device=dev)
    if nl:
        C.tree_split_best(out_gain, out_bin, out_left, int(f0), out)
    return out


def _choose_np(params: GrowParams, weight) -> int:
    """Digit planes per statistic: integer class counts (Poisson(1) <= 32, no instance weights)
    fit one signed byte; everything else uses 4 planes (30-bit fixed point)."""
    return 1 if (params.mode != 0 and weight is None) else 4


def grow_tree(Q: Quantized, ws: Workspace, params: GrowParams, tree_index: int,
              g: Optional[torch.Tensor] = None, h: Optional[torch.Tensor] = None,
              label: Optional[torch.Tensor] = None, weight: Optional[torch.Tensor] = None,
              bootstrap: bool = False, coll=None, deferred: bool = False, on_first_wait=None,
              margin: Optional[torch.Tensor] = None):
    """``coll`` (parallel.dist.Collectives): data-parallel level with feature-sharded split
    finding when world > 1 -- partial histograms are reduce-scattered by feature shard, every
    rank searches splits of its own shard, and the per-node best tuples are all-gathered
    (SURVEY PAR-02). ``coll.force`` runs the same collective path at world size 1 (RCCL check)."""
    C = native.lib()
    use_coll = coll is not None and coll.active
    shards = ws.shards(coll) if use_coll and (coll.world > 1 or getattr(coll, "force", False)) else None
    if device_levels_ok(params, weight):
        return grow_tree_device(Q, ws, params, tree_index, g, h, weight, coll if use_coll else None, shards,
                                label=label, bootstrap=bootstrap, deferred=deferred, on_first_wait=on_first_wait,
                                margin=margin)
    if margin is not None and g is None:           # (GBDT: this round's gradients)
        g, h = ws.gh()
        C.tree_logistic_grad(margin, label, weight, g, h)
    if on_first_wait is not None:
        on_first_wait()
    dev = Q.device
    mode_rs = 0 if params.mode == 0 else 1
    np_ = _choose_np(params, weight)
    spt = slots_per_tile(np_)
    pass_slots = spt * MAX_CT
    max_nodes = 2 ** (params.max_depth + 1)
    # host node table

    ws.row_node.zero_()
    with tracing.span("tree.quant"):
        seed = int(params.seed)
        if np_ == 4:
            C.tree_quant_max(g, h, label, weight, seed, int(tree_index), bool(bootstrap), mode_rs, Q.n_rows,
                             ws.maxabs, Q.row0)
            mx = coll.max(ws.maxabs) if use_coll else ws.maxabs
            C.tree_quant(g, h, label, weight, seed, int(tree_index), bool(bootstrap), mode_rs, 4, mx, ws.rowdig,
                         ws.kexp, ws.totals, ws.digp, Q.row0)
        else:
            C.tree_quant(g, h, label, weight, seed, int(tree_index), bool(bootstrap), mode_rs, 1, None, ws.rowdig,
                         ws.kexp, ws.totals, ws.digp, Q.row0)
    tot = coll.sum(ws.totals) if use_coll else ws.totals
    head = torch.cat([tot, ws.kexp.to(torch.int64)]).cpu().numpy()
    tab = TreeTable(head[:2].astype(np.int64))
    parent, left, right, stats, is_leaf = tab.parent, tab.left, tab.right, tab.stats, tab.is_leaf
    kexp = head[2:4].astype(np.int64)
    scale = np.ldexp(1.0, -kexp)                    # value of one quantisation step per statistic
    level = [0]
    prev_hist = None
    prev_index: dict = {}
    TB = Q.TB
    feat_thr_all = None

    for d in range(params.max_depth + 1):
        open_nodes = [n for n in level if not is_leaf[n]]
        if d == params.max_depth or not open_nodes:
            for n in open_nodes:
                is_leaf[n] = True
            break
        # --- decide which nodes to build (smaller sibling) and which to subtract
        build, subtract = [], []
        if d == 0 or params.feat_k:
            # RF: a feature sampled at this level may not have been built for the parent, so
            # sibling subtraction would read a missing parent histogram: build every open node
            build = list(open_nodes)
        else:
            seen = set()
            for n in open_nodes:
                p = parent[n]
                if p in seen:
                    continue
                seen.add(p)
                a, b = left[p], right[p]
                a_open, b_open = not is_leaf[a], not is_leaf[b]
                if a_open and b_open:
                    wa = _weight(stats[a], params.mode)
                    wb = _weight(stats[b], params.mode)
                    small, large = (a, b) if wa <= wb else (b, a)
                    build.append(small)
                    subtract.append((large, p, small))
                elif a_open:
                    build.append(a)
                elif b_open:
                    build.append(b)
        local = {n: i for i, n in enumerate(open_nodes)}
        nl = len(open_nodes)
        nb = len(build)
        if shards is None:
            cur_hist = torch.zeros((nl, TB, 2), dtype=torch.int64, device=dev)
            hist_target, target_of, h_boff, h_stride = cur_hist, local, Q.boff, TB
        else:
            # local partials of the built nodes, shard-major (reduce-scattered as they stand)
            rs_buf = shards.target(nb, dev)
            hist_target = rs_buf.view(shards.S * nb, shards.Bs, 2)
            target_of = {n: k for k, n in enumerate(build)}
            h_boff, h_stride = shards.boff_packed(nb), shards.Bs
        # --- small per-level arrays, one staged upload
        stg = ws.staging
        h_ns = None
        if d > 0:
            ns = np.full(max_nodes, -1, dtype=np.int32)
            ns[np.asarray(build, dtype=np.int64)] = np.arange(nb, dtype=np.int32)
            h_ns = stg.add(ns)
        passes = []
        for s0 in range(0, nb, pass_slots):
            cnt = min(pass_slots, nb - s0)
            s2n = np.array([target_of[build[s0 + k]] for k in range(cnt)], dtype=np.int32)
            passes.append((s0, cnt, stg.add(s2n)))
        h_sub = None
        if subtract:
            h_sub = (stg.add(np.array([local[a] for a, _, _ in subtract], dtype=np.int32)),
                     stg.add(np.array([prev_index[p] for _, p, _ in subtract], dtype=np.int32)),
                     stg.add(np.array([local[s] for _, _, s in subtract], dtype=np.int32)))
        h_tot = stg.add(np.stack([stats[n] for n in open_nodes]).astype(np.int64))
        h_ids = stg.add(np.array(open_nodes, dtype=np.int32))
        h_bidx = stg.add(np.array([local[n] for n in build], dtype=np.int64))
        up = stg.upload()
        node_slot = up[h_ns] if h_ns is not None else None
        # RF: exact k-of-F feature sample per open node (k-th smallest priority, on device) and
        # the level's union mask; histogram items without a sampled feature are skipped
        feat_thr = feat_mask = None
        if params.feat_k:
            feat_thr = torch.empty(nl, dtype=torch.float64, device=dev)
            feat_mask = torch.empty(Q.Fa, dtype=torch.uint8, device=dev)
            C.tree_rf_sample(int(params.seed), int(tree_index), up[h_ids], int(Q.num_features), int(params.feat_k),
                             Q.fid_orig, feat_thr, feat_mask, None)
        # --- histograms, up to `pass_slots` node slots per pass
        with tracing.span("tree.hist"):
            # RF levels read only the sampled features' CSC items (the dense block would stream
            # every hot feature for a handful of sampled ones)
            use_dense = Q.dense is not None and d <= DENSE_MAX_DEPTH and not params.feat_k
            sel_groups = Q.groups if use_dense else Q.groups + Q.hot_groups
            hot_keep = None
            for s0, cnt, h_s2n in passes:
                slot8 = None
                if d > 0:
                    C.tree_slot8(ws.row_node, node_slot, s0, cnt, ws.slot8, None, None)
                    slot8 = ws.slot8
                ct = pass_ct(np_, cnt)
                s2n = up[h_s2n]
                launches = []
                for grp in sel_groups:
                    if grp.num_items == 0:
                        continue
                    launches.append(functools.partial(
                        C.tree_hist_build, grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(),
                        Q.h_row, Q.h_key, slot8, ws.rowdig, h_boff, Q.nbins, s2n, hist_target, h_stride, grp.bt, ct,
                        np_, feat_mask))
                if use_dense:
                    for bt in (1, 2, 4):
                        fg = C.tree_dense_fg(bt, ct if d > 0 else 1)
                        gfid, gden = ws.dense_groups(bt, fg, hot_keep)
                        if gfid.numel():
                            rr = dense_range_rows(Q.n_rows, gfid.numel() // fg)
                            launches.append(functools.partial(
                                C.tree_hist_dense, Q.dense, ws.digp, ws.rowdig, None if d == 0 else ws.slot8_pad,
                                gfid, gden, h_boff, Q.nbins, s2n, hist_target, h_stride, Q.n_rows, rr, bt, ct, np_))
                ws.run_concurrent(launches)
        totals, node_ids = up[h_tot], up[h_ids]
        sub_t = tuple(up[h] for h in h_sub) if h_sub is not None else None
        if shards is None:
            if sub_t is not None:
                C.tree_hist_subtract(prev_hist, cur_hist, *sub_t, TB)
            with tracing.span("tree.split"):
                packed = _best_splits(C, cur_hist, totals, Q.boff, Q.nbins, Q.zbin, Q.fid_orig, node_ids, ws.kexp,
                                      params, feat_thr, tree_index, Q.Fa, 0)
                packed = packed.cpu().numpy()
        else:
            with tracing.span("tree.reduce_scatter"), _CollTimer(dev):
                # rows keep the shard-major stride Bs (>= this shard's bins): the split search
                # reads them in place; every open node is built or subtracted, so no zero fill
                mine = coll.reduce_scatter(rs_buf) if nb else None            # [nb, Bs, 2]
                # (cur_hist below is left uninitialised: every open node must be built or subtracted)
                assert nb + len(subtract) == nl, (d, nb, len(subtract), nl)
                if nb == nl and build == open_nodes:
                    cur_hist = mine
                else:
                    cur_hist = torch.empty((nl, shards.Bs, 2), dtype=torch.int64, device=dev)
                    if nb:
                        cur_hist.index_copy_(0, up[h_bidx], mine)
            if sub_t is not None:
                C.tree_hist_subtract(prev_hist, cur_hist, *sub_t, shards.Bs)
            with tracing.span("tree.split"):
                mine = _best_splits(C, cur_hist, totals, shards.boff, shards.nbins, shards.zbin, shards.fid_orig,
                                    node_ids, ws.kexp, params, feat_thr, tree_index, shards.Fa, shards.f0)
                with _CollTimer(dev):
                    allt = coll.all_gather(mine)                              # [S, nl, 5]
                gains = allt[:, :, 0].contiguous().view(torch.float64)
                best_s = torch.argmax(gains, dim=0)                           # ties -> lowest shard = lowest feature
                packed = allt[best_s, torch.arange(nl, device=dev)].cpu().numpy()
        # --- create children
        next_level, default_child, splits = tab.apply_splits(open_nodes, packed, d, Q, params, scale, max_nodes)
        if splits:
            with tracing.span("tree.partition"):
                _partition(C, Q, ws, default_child, splits)
        prev_hist = cur_hist
        prev_index = local
        level = next_level

    return tab.build(Q, params, scale)


def device_levels_ok(params: GrowParams, weight, device_levels: Optional[bool] = None) -> bool:
    """The device level loop covers every tree whose deepest level builds <= one pass of node
    slots: GBDT to depth 6, class-count trees to depth 7 (RF with per-node feature sampling,
    which builds every open node, to depth 7; weighted ones to depth 5)."""
    on = DEVICE_LEVELS if device_levels is None else device_levels
    deepest = 2 ** max(params.max_depth - (1 if params.feat_k else 2), 0)
    return on and deepest <= slots_per_tile(_choose_np(params, weight)) * MAX_CT


class LevelState:
    """Device buffers of the level loop (node table, ping-pong open lists, partition and plan
    tables), allocated once per workspace and depth."""

    def record_event(self, stream=None):
        """An event recorded on ``stream`` (default: the current stream; a reused event on the
        device, _Done on the host). Passing the stream saves a torch.cuda.current_stream() lookup
        (~10 us of host time per call)."""
        if self._events is None:
            return _Done()
        ev = self._events[self._ev_i]
        self._ev_i = (self._ev_i + 1) % len(self._events)
        ev.record(stream)
        return ev

    def host_views(self, buf: torch.Tensor) -> dict:
        """Named views of a host copy of the arena (node table fields + exponents)."""
        return {name: buf[o:o + n].view(dt).view(shape) for name, dt, shape, o, n in self._layout}

    def __init__(self, Q: Quantized, max_depth: int, n_sel: int = 0):
        dev = Q.device
        M = 2 ** (max_depth + 1)
        cap = 2 ** max_depth
        # RF levels with preselected item lists (PRESELECT): per level the 4 plan counts, then
        # 8 per-XCD active-item counts per sampled item group, read by the host in one copy
        self.n_sel = n_sel
        self.rf_thr = [torch.empty(cap, dtype=torch.float64, device=dev) for _ in range(2)] if n_sel else None
        self.rf_mask = [torch.empty(Q.Fa, dtype=torch.uint8, device=dev) for _ in range(2)] if n_sel else None
        i32 = lambda n: torch.full((n,), -1, dtype=torch.int32, device=dev)   # noqa: E731
        self.M, self.cap, self.max_depth = M, cap, max_depth
        # the node table (+ the tree's quantisation exponents) lives in ONE device arena, mirrored by
        # one pinned host arena: the host reads a finished tree with a single D2H copy (eleven
        # separate small copies cost ~0.4 ms per tree at ~25-30 us each)
        layout = [("stats", torch.int64, (M, 2)), ("gain", torch.float64, (M,)), ("n_nodes", torch.int32, (1,)),
                  ("kexp", torch.int32, (2,)), ("parent", torch.int32, (M,)), ("feat", torch.int32, (M,)),
                  ("bin", torch.int32, (M,)), ("left", torch.int32, (M,)), ("right", torch.int32, (M,)),
                  ("leaf", torch.uint8, (M,))]
        offs, nbytes = [], 0
        for _, dt, shape in layout:
            isz = torch.empty(0, dtype=dt).element_size()
            nbytes = (nbytes + 7) // 8 * 8
            offs.append(nbytes)
            nbytes += isz * int(np.prod(shape))
        nbytes = (nbytes + 7) // 8 * 8         # (copied in 8-byte words by the GBDT prologue)
        self.arena = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        self.arena_host = torch.zeros(nbytes, dtype=torch.uint8)
        if dev.type == "cuda":
            self.arena_host = self.arena_host.pin_memory()
        self._layout = []
        for (name, dt, shape), o in zip(layout, offs):
            n = torch.empty(0, dtype=dt).element_size() * int(np.prod(shape))
            setattr(self, name if name != "kexp" else "kexp_slot", self.arena[o:o + n].view(dt).view(shape))
            self._layout.append((name, dt, shape, o, n))
        self.host = self.host_views(self.arena_host)
        self.n_nodes.fill_(1)
        for t_ in (self.parent, self.left, self.right, self.feat, self.bin):
            t_.fill_(-1)
        self.gain.fill_(-1.0)
        # the root state of every tree (node 0 only, stats filled per tree): one H2D copy of this
        # image replaces ~9 fill launches at the start of each tree
        self.arena_init = self.arena.to("cpu", copy=True)       # (a copy also when dev is the CPU)
        if dev.type == "cuda":
            self.arena_init = self.arena_init.pin_memory()
        self.arena_init_dev = self.arena.clone()       # (the fused GBDT prologue copies it in on the device)
        self.zero1 = torch.zeros(1, dtype=torch.int32, device=dev)      # the root level's slot -> row table
        self.open = [i32(cap), i32(cap)]
        self.totals = [torch.zeros((cap, 2), dtype=torch.int64, device=dev) for _ in range(2)]
        self.counts = torch.zeros((max_depth + 1, 4 + 8 * n_sel), dtype=torch.int32, device=dev)
        self.counts_host = torch.zeros((max_depth + 1, 4 + 8 * n_sel), dtype=torch.int32)
        if dev.type == "cuda":
            self.counts_host = self.counts_host.pin_memory()
        self.one = torch.ones(1, dtype=torch.int32, device=dev)
        # events the level loop records for the host (re-recorded round robin: each one is waited on
        # before the loop records four more)
        self._events = [torch.cuda.Event() for _ in range(4)] if dev.type == "cuda" else None
        self._ev_i = 0
        self.default_child, self.node_slot = i32(M), i32(M)
        self.cs = [i32(cap) for _ in range(5)]          # feat, default, other, bin, left_default
        self.s2n, self.sub_dst, self.sub_par, self.sub_sib = i32(cap), i32(cap), i32(cap), i32(cap)
        self.sub_of = i32(cap)          # (runner levels) open index -> subtraction slot (-1)
        # data-parallel levels (tree.h LevelRowsArgs): histogram row per open node (level parity)
        # and the subtraction triples as rows
        self.row_of = [i32(cap), i32(cap)]
        self.dst_row, self.par_row, self.sib_row = i32(cap), i32(cap), i32(cap)
        self.node_dense = self.hot_row = None
        if Q.dense is not None and PARTITION_DENSE:
            hot_row = np.full(Q.Fa, -1, dtype=np.int32)
            hot_row[Q.hot] = np.arange(len(Q.hot), dtype=np.int32)
            self.hot_row = torch.from_numpy(hot_row).to(dev)
            self.node_dense = i32(4 * M)


def grow_tree_device(Q: Quantized, ws: Workspace, params: GrowParams, tree_index: int, g: torch.Tensor,
                     h: torch.Tensor, weight: Optional[torch.Tensor] = None, coll=None,
                     shards: Optional["FeatureShards"] = None, label: Optional[torch.Tensor] = None,
                     bootstrap: bool = False, deferred: bool = False, on_first_wait=None,
                     margin: Optional[torch.Tensor] = None):
    """One tree through :func:`device_tree_steps`, waiting on each event it yields."""
    batcher = LevelBatcher(coll, shards.S, Q.device) if shards is not None else None
    return drive(device_tree_steps(Q, ws, params, tree_index, g, h, weight, coll, shards, label, bootstrap,
                                   deferred, on_first_wait, margin), batcher)


def _wide_features(nbins: torch.Tensor, Fa: int) -> torch.Tensor:
    """Indices of the features with > 16 bins (split_wide_kernel), memoised on the nbins tensor."""
    memo = getattr(nbins, "_fdx_wide", None)
    if memo is None or memo[0] != Fa:
        idx = np.nonzero(nbins[:Fa].cpu().numpy() > 16)[0].astype(np.int32)
        memo = (Fa, torch.from_numpy(idx).to(nbins.device))
        nbins._fdx_wide = memo
    return memo[1]


def _level_runner(Q: Quantized, ws: Workspace, st: "LevelState", params: GrowParams, item_groups: list,
                  sampled: bool):
    """The lane's native level runner (csrc/bindings_level.cpp RfLevels), built once per workspace,
    level state and tree parameters. RF (``sampled``): every kernel of a level; GBDT: the tree
    prologue, the fused split + plan and the partition (the row-group passes stay in Python)."""
    key = (params.mode, params.max_depth, params.min_gain, params.min_child, params.seed, params.feat_k,
           params.lambda_, sampled)
    cached = getattr(ws, "_rf_runner", None)
    if cached is not None and cached[0] is st and cached[1] == key:
        return cached[2]
    cfg = dict(groups=[(g.item_start, g.item_end, g.item_f0, g.item_meta, g.wave_order(), int(g.bt))
                       for g in item_groups],
               h_row=Q.h_row if sampled else None, h_key=Q.h_key if sampled else None, csc_row=Q.csc_row,
               csc_bin=Q.csc_bin, colptr=Q.colptr, nbins=Q.nbins,
               zbin=Q.zbin, fid_orig=Q.fid_orig, dense=Q.dense if st.node_dense is not None else None,
               hot_row=st.hot_row, rowdig=ws.rowdig, rowpack=ws.rowpack() if sampled else None, row_node=ws.row_node,
               kexp=ws.kexp, build_all=bool(params.feat_k), arena_stats=st.stats[0], open0=st.open[0],
               totals0=st.totals[0], kexp_slot=st.kexp_slot,
               stats=st.stats, parent=st.parent, left=st.left, right=st.right, feat=st.feat, bin=st.bin, leaf=st.leaf,
               gain=st.gain, n_nodes=st.n_nodes, counts=st.counts, counts_host=st.counts_host,
               default_child=st.default_child, cs_feat=st.cs[0], cs_default=st.cs[1], cs_other=st.cs[2],
               cs_bin=st.cs[3], cs_left_default=st.cs[4], node_slot=st.node_slot, s2n=st.s2n, sub_dst=st.sub_dst,
               sub_par=st.sub_par, sub_sib=st.sub_sib, sub_of=st.sub_of, node_dense=st.node_dense, mode=int(params.mode),
               max_depth=int(params.max_depth), min_gain=float(params.min_gain), lambda_=float(params.lambda_),
               mcw=float(params.min_child), seed=int(params.seed), F=int(Q.num_features), k=int(params.feat_k),
               lds=bool(RF_LDS), wps=int(PARTITION_WPS), arena=st.arena, dig16=ws.dig16() if sampled else None,
               fmix=_feature_mix(Q) if (params.feat_k and FEATURE_MIX) else None)
    runner = native.lib().RfLevels(cfg)
    ws._rf_runner = (st, key, runner)
    return runner


# the sampler and split search look mix64(feature) up in a table instead of recomputing it: off,
# the table reads cost more than the hash (rf_window_threshold 24.6 -> 27.2 ms a forest,
# profiles/r6/rf_dp_busy_fmix_REJECTED.txt); kept for the record, host twins ignore it
FEATURE_MIX = False


def _feature_mix(Q: Quantized) -> torch.Tensor:
    """mix64(f) over the F features on the device (the RF priorities' per-feature hash, looked up
    by the sampler and the split search instead of recomputed per node), once per Q."""
    t = getattr(Q, "_fmix", None)
    if t is None:
        t = Q._fmix = native.lib().tree_feature_mix(int(Q.num_features), Q.nbins)
    return t


def _gbdt_levels_setup(Q, ws, st, params, runner, rg):
    """Hands the runner the row-group tables and fixed level buffers of its C++ GBDT level loop
    (RfLevels.gbdt_setup), once per runner; returns the two level-histogram tensors (the root's
    is row 0 of the first, zeroed by the prologue)."""
    key = (RG_DBG, GBDT_CHOOSE_ROWS, LIST_NODE_COUNTS, PARTITION_COUNTS, RG_PARTIALS, RG_PARTIALS_MULTI, SPLIT_WIDE,
           qmod.RG_LIST_WGS, qmod.RG_ALPHA, qmod.RG_EM_MIN_FRAC)
    cached = getattr(ws, "_gbdt_levels", None)
    if cached is not None and cached[0] is runner and cached[2] == key:     # (in-process A/Bs flip these)
        return cached[1]
    dev, TB, D = Q.device, Q.TB, int(params.max_depth)
    # level d opens at most 2^d nodes; even and odd levels alternate between the two tensors
    rows = [max([1] + [1 << d for d in range(k, D, 2)]) for k in (0, 1)]
    hists = [torch.empty((r, TB, 2), dtype=torch.int64, device=dev) for r in rows]
    em = rg.erow is not None and qmod.RG_EM_MIN_FRAC <= 1.0
    part = ws.rg_part(rg, rg.list_work()) if RG_PARTIALS else None
    runner.gbdt_setup(dict(
        rg_wg_list=rg.list_work(), rg_wg_first_list=rg.list_work_first() if RG_PARTIALS else None,
        rg_ptr=rg.ptr, rg_ent=rg.ent, rg_gbase=rg.gbase, rg_gbin=rg.gbin, rg_gmode=rg.gmode, rg_wg=rg.work(),
        rg_erow=rg.erow, rg_ebase=int(rg.ebase) if rg.erow is not None else 0,
        emdig=ws.rg_emdig() if em else None, em_min_rows=max(1, int(qmod.RG_EM_MIN_FRAC * Q.n_rows)),
        rg_part=part, rg_wg_first=rg.work_first() if RG_PARTIALS else None,
        list_work=ws.rg_work, rg_start=ws.rg_start, rg_list=ws.rg_list, rg_listdig=ws.rg_listdig,
        hist_a=hists[0], hist_b=hists[1], packed=torch.empty((1 << (D - 1), 5), dtype=torch.int64, device=dev),
        one=st.one, zero1=st.zero1, open1=st.open[1], totals1=st.totals[1], boff=Q.boff,
        wide=_wide_features(Q.nbins, Q.Fa) if SPLIT_WIDE else None, counted=PARTITION_COUNTS, dbg=RG_DBG,
        part_multi=RG_PARTIALS_MULTI, choose_rows=GBDT_CHOOSE_ROWS, node_counts=LIST_NODE_COUNTS))
    ws._gbdt_levels = (runner, hists, key)
    return hists
# the DP runner calls RCCL directly on the process group's communicator (0: through Python)
DP_DIRECT_RCCL = os.environ.get("FDX_DP_DIRECT_RCCL", "1") == "1"


def _gbdt_dp_setup(Q, ws, st, params, runner, rg, shards, coll) -> torch.Tensor:
    """Hands the runner its data-parallel GBDT level loop (RfLevels.gbdt_dp_setup): the row-group
    tables, the shard-major send buffer, the two reduced-level buffers, the feature shard's split
    tables and the collective callbacks; once per runner. Returns the root level's send region
    (zeroed by the prologue)."""
    cached = getattr(ws, "_gbdt_dp", None)
    if cached is not None and cached[0] is runner:
        return cached[1]
    dev, D, S, Bs = Q.device, int(params.max_depth), int(shards.S), int(shards.Bs)
    widest = max(1 << max(D - 1, 1), 2)
    send = torch.empty(S * widest * Bs * 2, dtype=torch.int64, device=dev)
    outs = [torch.empty((widest, Bs, 2), dtype=torch.int64, device=dev) for _ in range(2)]
    em = rg.erow is not None and qmod.RG_EM_MIN_FRAC <= 1.0
    cb = _DpCollectives(coll, dev)
    comm, lib = _rccl_comm(dev)
    runner.gbdt_dp_setup(dict(
        comm=comm, rccl_lib=lib,
        rg_wg_list=rg.list_work(), rg_wg_first_list=rg.list_work_first() if RG_PARTIALS else None,
        rg_ptr=rg.ptr, rg_ent=rg.ent, rg_gbase=rg.gbase, rg_gbin=rg.gbin, rg_gmode=rg.gmode, rg_wg=rg.work(),
        rg_erow=rg.erow, rg_ebase=int(rg.ebase) if rg.erow is not None else 0,
        emdig=ws.rg_emdig() if em else None, em_min_rows=max(1, int(qmod.RG_EM_MIN_FRAC * Q.n_rows)),
        rg_part=ws.rg_part(rg, rg.list_work()) if RG_PARTIALS else None,
        rg_wg_first=rg.work_first() if RG_PARTIALS else None,
        list_work=ws.rg_work, rg_start=ws.rg_start, rg_list=ws.rg_list, rg_listdig=ws.rg_listdig,
        one=st.one, zero1=st.zero1, open1=st.open[1], totals1=st.totals[1], boff=Q.boff, wide=None,
        counted=PARTITION_COUNTS, node_counts=LIST_NODE_COUNTS, dbg=RG_DBG, part_multi=RG_PARTIALS_MULTI,
        rs=cb.rs, ag=cb.ag, mx=cb.mx, S=S, Bs=Bs, bin_lo=shards.bin_lo, send=send, out_a=outs[0], out_b=outs[1],
        row_of0=st.row_of[0], row_of1=st.row_of[1], ag_in=torch.empty((widest, 5), dtype=torch.int64, device=dev),
        sboff=shards.boff, snbins=shards.nbins, szbin=shards.zbin, sfid=shards.fid_orig, f0=int(shards.f0),
        swide=_wide_features(shards.nbins, shards.Fa) if SPLIT_WIDE else None, dst_row=st.dst_row,
        par_row=st.par_row, sib_row=st.sib_row, iota=ws.iota(64)))
    root = send[:S * 2 * Bs * 2]
    ws._gbdt_dp = (runner, root)
    if runner.dp_direct():
        _DP_RUNNERS.append(runner)
    return root


def _gbdt_runner_levels(Q, runner, tree_index, on_first_wait):
    """The level loop of a single-process GBDT tree in the runner (C++): level 0 is queued, the
    previous tree's host table is built while it runs (on_first_wait), then levels 1.. run with
    the host waits inside the runner. Same launches and trees as the generic loop."""
    runner.gbdt_root(tree_index)
    if on_first_wait is not None:
        on_first_wait()
    shape = runner.gbdt_levels(tree_index)
    for j in range(0, len(shape), 2):
        LEVEL_STATS["levels"] += 1
        LEVEL_STATS["built_nodes"] += shape[j + 1]
        LEVEL_STATS["hist_bytes"] += shape[j + 1] * Q.TB * 16


def device_tree_steps(Q: Quantized, ws: Workspace, params: GrowParams, tree_index: int, g: torch.Tensor,
                      h: torch.Tensor, weight: Optional[torch.Tensor] = None, coll=None,
                      shards: Optional["FeatureShards"] = None, label: Optional[torch.Tensor] = None,
                      bootstrap: bool = False, deferred: bool = False, on_first_wait=None,
                      margin: Optional[torch.Tensor] = None):
    """A generator: yields an event wherever the host must wait for the device (the next level's
    counts, the finished node table) and returns the Tree (or PendingTree). :func:`drive` runs
    one tree; the forest driver (models/forest_batch.py) interleaves several on their own streams.

    GBDT tree with the level loop on the device (same trees as grow_tree's host loop, bit for
    bit). Per level: histogram passes -> sibling subtraction -> split search -> best split per
    node -> ``tree_level_plan`` (one thread: apply the splits to the device node table, this
    level's partition tables, the next level's open list / builds / subtraction triples) ->
    partition. The host waits only for the plan's 16-byte counts (copied while the partition
    runs) to size the next level's launches, and reads the node table once at the end.
    Data parallel (``shards``): the built nodes' partial histograms are reduce-scattered by
    feature shard and the per-shard best splits all-gathered, all stream-ordered on the device;
    every rank plans the identical next level from the identical gathered splits.
    ``deferred`` (GBDT): return a :class:`PendingTree` whose leaf values were computed on the
    device; the host table is built later (``on_first_wait`` of the next tree runs it while that
    tree's root level is on the GPU), so the GPU never idles on the host's tree build.
    ``margin`` (GBDT, with ``label`` and g = h = None): the round's gradients are computed here,
    fused into the tree's prologue when the native runner drives the levels."""
    C = native.lib()
    dev = Q.device
    np_ = _choose_np(params, weight)
    mode_rs = 0 if params.mode == 0 else 1
    build_all = bool(params.feat_k)
    sampled = SAMPLED and build_all and np_ == 1
    # RF levels >= 1: the next level's feature sample and its active-item lists are queued right
    # after the plan, so the per-XCD item counts reach the host with the level's counts and each
    # histogram pass launches one wave per active item (no grid of ~300K mostly idle wave slots)
    presel = PRESELECT and sampled and dev.type == "cuda" and Q.n_rows >= PRESELECT_MIN_ROWS
    item_groups = (Q.groups + Q.hot_groups) if sampled else []
    sel_ids = [gi for gi, grp in enumerate(item_groups) if grp.num_items] if presel else []
    sel_args = None
    st = getattr(ws, "_levels", None)
    if st is None or st.max_depth != params.max_depth or st.n_sel != len(sel_ids):
        st = ws._levels = LevelState(Q, params.max_depth, len(sel_ids))
    # the native runner: RF levels and GBDT levels (any world size). A single process also fuses
    # the GBDT prologue and the split + plan; under data parallelism the quantisation max is an
    # all-reduce and the levels split around the reduce-scatter / all-gather
    gbdt_native = NATIVE_LEVELS and dev.type == "cuda" and params.mode == 0 and weight is None and not build_all
    # (the runner's level 0 completes the root's sums: at least one level)
    runner = _level_runner(Q, ws, st, params, item_groups, sampled) \
        if (NATIVE_LEVELS and dev.type == "cuda" and (sampled or gbdt_native) and params.max_depth >= 1) else None
    # every step of this generator runs on the stream current now (the forest driver advances a
    # lane inside that lane's stream context)
    cur_stream = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    seed = int(params.seed)
    native_prologue = runner is not None and shards is None and coll is None
    TB = Q.TB
    # the next level's zeroed histograms (at most 2 open nodes per open node) are queued before
    # the host waits for its counts, so the fill runs while the host sizes that level
    pre_hist = None
    # single-process GBDT rounds on the row-group engine: the level loop runs in the runner
    rg_cxx = ws.rowgroups() if (native_prologue and gbdt_native and GBDT_CXX_LEVELS and SPLIT_SUBTRACT and
                                np_ == 4 and margin is not None and g is None) else None
    # data-parallel GBDT rounds on the row-group engine: the same runner loop around the level
    # collectives (RfLevels.gbdt_dp_levels; the collectives are Python callbacks)
    rg_dp = ws.rowgroups() if (runner is not None and shards is not None and gbdt_native and GBDT_CXX_LEVELS and
                               SPLIT_SUBTRACT and np_ == 4 and margin is not None and g is None) else None
    if rg_dp is not None:
        with tracing.span("tree.quant"):
            root_zero = _gbdt_dp_setup(Q, ws, st, params, runner, rg_dp, shards, coll)
            g, h = ws.gh()
            # gradients + max slots (all-reduced by the runner's callback) + arena image + the root's
            # send region zeroed, then the quantisation
            runner.prologue(margin, g, h, label, None, int(tree_index), False, 4, None, ws.totals, None, Q.row0,
                            root_zero, st.arena_init_dev)
    elif native_prologue:
        # the root histogram is zeroed by the prologue's first launch
        if rg_cxx is not None:
            pre_hist = _gbdt_levels_setup(Q, ws, st, params, runner, rg_cxx)[0][:1]
        else:
            pre_hist = torch.empty((1, TB, 2), dtype=torch.int64, device=dev)
        with tracing.span("tree.quant"):
            # (the dense-block digit planes only feed the MFMA dense path, off with the row groups)
            digp = ws.digp if (ws.digp is not None and not build_all and ws.rowgroups() is None) else None
            if np_ == 4 and margin is not None and g is None:
                # gradients + max |g|, |h| + arena image + root histogram zero, then quant: 2 launches
                g, h = ws.gh()
                runner.prologue(margin, g, h, label, None, int(tree_index), False, 4, None, ws.totals, digp,
                                Q.row0, pre_hist, st.arena_init_dev)
            else:
                # arena image first: the quantisation adds the root totals into it
                st.arena.copy_(st.arena_init, non_blocking=True)
                if np_ == 4:
                    C.tree_quant_max(g, h, label, weight, seed, int(tree_index), bool(bootstrap), mode_rs, Q.n_rows,
                                     ws.maxabs, Q.row0)
                    runner.prologue(None, g, h, label, weight, int(tree_index), bool(bootstrap), 4, ws.maxabs,
                                    ws.totals, digp, Q.row0, pre_hist, None)
                else:
                    runner.prologue(None, g, h, label, weight, int(tree_index), bool(bootstrap), 1, None, ws.totals,
                                    digp, Q.row0, pre_hist, None)
    else:
        if margin is not None and g is None:
            g, h = ws.gh()
            C.tree_logistic_grad(margin, label, weight, g, h)
        ws.row_node.zero_()
    with tracing.span("tree.quant"):
        if native_prologue or rg_dp is not None:
            pass
        elif np_ == 4:
            C.tree_quant_max(g, h, label, weight, seed, int(tree_index), bool(bootstrap), mode_rs, Q.n_rows,
                             ws.maxabs, Q.row0)
            mx = coll.max(ws.maxabs) if coll is not None else ws.maxabs
            C.tree_quant(g, h, label, weight, seed, int(tree_index), bool(bootstrap), mode_rs, 4, mx, ws.rowdig,
                         ws.kexp, ws.totals, ws.digp, Q.row0)
        else:
            C.tree_quant(g, h, label, weight, seed, int(tree_index), bool(bootstrap), mode_rs, 1, None, ws.rowdig,
                         ws.kexp, ws.totals, ws.digp, Q.row0)
    # root: node 0, open list [0] with the exact totals (no host round trip); under data
    # parallelism the totals are summed by the root level's reduce-scatter (LaneBufs.tot_bin)
    if not native_prologue and rg_dp is None:
        st.arena.copy_(st.arena_init, non_blocking=True)
        st.open[0][:1].zero_()
    if shards is None and not native_prologue:
        tot = coll.sum(ws.totals) if coll is not None else ws.totals
        st.stats[0].copy_(tot)
        st.totals[0][:1].copy_(tot[None])
    n_open, n_build = 1, 1
    prev_hist = prev_row_of = None
    ev = None
    rg_counted = False
    # RF under data parallelism: each level reduce-scatters only its sampled features' bins; level
    # d + 1's sample and layout are computed right after level d's plan, so their shard sizes reach
    # the host with the level's counts (one wait per level; the root's before the loop)
    compact = shards is not None and build_all and 0 < params.feat_k < Q.num_features and \
        (RF_COMPACT == "1" or (RF_COMPACT == "auto" and shards.S > 1))
    if compact:
        shards.sample_compact(C, 0, seed, int(tree_index), st.open[0][:1], int(Q.num_features), int(params.feat_k),
                              Q.fid_orig)
        yield st.record_event(cur_stream)
    generic_depth = params.max_depth
    if rg_cxx is not None:
        _gbdt_runner_levels(Q, runner, int(tree_index), on_first_wait)
        on_first_wait = None
        generic_depth = 0
    elif rg_dp is not None:
        runner.gbdt_dp_root(int(tree_index))
        if on_first_wait is not None:
            on_first_wait()
            on_first_wait = None
        shape = runner.gbdt_dp_levels(int(tree_index))
        for j in range(0, len(shape), 2):
            LEVEL_STATS["levels"] += 1
            LEVEL_STATS["built_nodes"] += shape[j + 1]
            LEVEL_STATS["hist_bytes"] += shape[j + 1] * TB * 16
        generic_depth = 0
    for d in range(generic_depth):
        cur = d % 2
        if d > 0:
            if on_first_wait is not None:
                on_first_wait()
                on_first_wait = None
            yield ev
            cnt = st.counts_host[d - 1].tolist()
            n_open, n_build = int(cnt[1]), int(cnt[2])
            if n_open == 0:
                break
            if sel_ids:       # largest per-XCD active-item count of each sampled group
                per_xcd = {gi: max(cnt[4 + 8 * j: 12 + 8 * j]) for j, gi in enumerate(sel_ids)}
                for j, gi in enumerate(sel_ids):
                    if per_xcd[gi]:           # (launch_hist: (npx + 3) / 4 x 8 workgroups of 4 waves)
                        LEVEL_STATS["listed_passes"] += 1
                        LEVEL_STATS["listed_active_items"] += sum(cnt[4 + 8 * j: 12 + 8 * j])
                        LEVEL_STATS["listed_grid_waves"] += (per_xcd[gi] + 3) // 4 * 8 * 4
        LEVEL_STATS["levels"] += 1
        LEVEL_STATS["built_nodes"] += n_build
        LEVEL_STATS["hist_bytes"] += n_build * TB * 16          # (g, h) int64 partials of the built nodes
        open_d, totals_d = st.open[cur][:n_open], st.totals[cur][:n_open]
        if d == 0 and native_prologue:
            totals_d = st.stats[:1]             # (unread: the runner sums the prologue's root slots)
        n_open_ptr = st.one if d == 0 else st.counts[d - 1, 1:2]
        # RF: exact k-of-F feature sample per open node and the level's union mask (device)
        feat_thr = feat_mask = None
        if compact:
            feat_thr, feat_mask, local_c, Bs_c = shards.compact_level(cur, n_open)
        elif build_all and sel_ids and d > 0:
            feat_thr, feat_mask = st.rf_thr[cur][:n_open], st.rf_mask[cur]      # (queued with the plan)
        elif build_all:
            feat_thr = torch.empty(n_open, dtype=torch.float64, device=dev)
            feat_mask = torch.empty(Q.Fa, dtype=torch.uint8, device=dev)
            C.tree_rf_sample(seed, int(tree_index), open_d, int(Q.num_features), int(params.feat_k), Q.fid_orig,
                             feat_thr, feat_mask, None)
        split_boff = shards.boff if shards is not None else None
        bufs = None
        if shards is None:
            if pre_hist is not None and pre_hist.shape[0] >= n_open:
                cur_hist = hist_target = pre_hist[:n_open]
            else:
                cur_hist = hist_target = torch.zeros((n_open, TB, 2), dtype=torch.int64, device=dev)
            pre_hist = None
            h_boff, h_stride = Q.boff, TB
        else:
            # the built nodes' local partials go straight into this tree's rows of the batch's
            # shard-major send buffer (LaneBufs); compact levels send only the sampled features'
            # bins (FeatureShards.sample_compact)
            subs = 0 if (build_all or d == 0) else n_build
            bufs = yield CollStep("alloc", rows=n_build, Bs=Bs_c if compact else shards.Bs, n_open=n_open,
                                  totals=ws.totals if d == 0 else None, sub_rows=subs)
            hist_target = bufs.prepare(ws.totals if d == 0 else None)
            if runner is not None:      # (the runner's kernels add the shard offsets themselves)
                h_boff = local_c if compact else shards._local
            else:
                h_boff = shards.boff_batched(bufs.shard_bins, local_c if compact else None)
            h_stride = bufs.Bs
            if compact:
                split_boff = local_c[shards.f0: shards.f0 + shards.Fa + 1]
        with tracing.span("tree.hist"):
            use_dense = Q.dense is not None and d <= DENSE_MAX_DEPTH and not build_all
            slot8 = None
            csc_slot8, csc_dig = None, ws.rowdig
            rg = ws.rowgroups() if (not build_all and np_ == 4) else None
            if d > 0:
                # a single built node: the CSC passes run the root kernel on digit words zeroed
                # outside it (no per-entry slot gather, no compaction; zero rows add nothing).
                # Sampled RF levels with FUSED_PACK read the packed row state the previous level's
                # partition wrote (no row pass here at all)
                single = n_build == 1 and rg is None and not (sampled and FUSED_PACK)
                if single and getattr(ws, "rowdig_masked", None) is None:
                    ws.rowdig_masked = torch.empty_like(ws.rowdig)
                if sampled and FUSED_PACK:
                    pass
                elif rg is None and sampled and not single:
                    C.tree_slot_pack(ws.row_node, st.node_slot, n_build, ws.rowdig, ws.rowpack())
                elif rg is None:        # (the row-group engine lists the built rows from row_node itself)
                    C.tree_slot8(ws.row_node, st.node_slot, 0, n_build, ws.slot8, ws.rowdig if single else None,
                                 ws.rowdig_masked if single else None)
                slot8 = ws.slot8
                csc_slot8, csc_dig = (None, ws.rowdig_masked) if single else (slot8, ws.rowdig)
                s2n = st.s2n[:n_build]
            else:
                s2n = st.zero1
            if shards is not None:      # slot k -> partial row k
                s2n = ws.iota(n_build)
            ct = pass_ct(np_, n_build)
            launches = []
            # (the CSC items are built on first use: the row-group engine never touches them)
            sel_groups = None
            if rg is not None:
                shard_args = (shards.bin_lo, bufs.shard_bins) if shards is not None else (None, 0)
                # single-slot passes: per-workgroup partial tables summed by one reduction instead
                # of every workgroup's atomics on the same bins (RgHistArgs part)
                # (the listed levels have their own, smaller work table: RowGroups.list_work)
                wtab = rg.work() if d == 0 else rg.list_work()
                part = dict(part=ws.rg_part(rg, rg.list_work()), wg_first=rg.work_first() if d == 0 else
                            rg.list_work_first()) \
                    if (RG_PARTIALS and (n_build == 1 or RG_PARTIALS_MULTI) and dev.type == "cuda") else {}
                if d == 0:
                    C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, ws.rowdig, np_, None, None, None, 1, rg.gmode,
                                   wtab, s2n, hist_target, h_stride, *shard_args, RG_DBG, **rg.em_args(), **part)
                else:
                    # one built node: every row's digit words zeroed outside it, for the
                    # entry-major pass of the sparse groups (taken when the node is large)
                    emdig = ws.rg_emdig() if (n_build == 1 and rg.erow is not None and qmod.RG_EM_MIN_FRAC <= 1.0) \
                        else None
                    C.tree_rg_list(ws.row_node, st.node_slot, None, Q.n_rows, n_build, ws.rg_work, ws.rg_start,
                                   ws.rg_list, ws.rowdig, ws.rg_listdig, emdig, counted=rg_counted)
                    C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, ws.rowdig, np_, ws.rg_list, ws.rg_start,
                                   ws.rg_listdig, n_build, rg.gmode, wtab, s2n, hist_target, h_stride,
                                   *shard_args, RG_DBG, **(rg.em_args(emdig) if emdig is not None else {}), **part)
                sel_groups, use_dense = [], False
            if sel_groups is None:
                sel_groups = Q.groups if use_dense else Q.groups + Q.hot_groups
            if runner is not None and sampled:
                pack = ws.rowpack() if (d > 0 and not single) else None
                lists, cnts, npxs = [], [], []
                for gi, grp in enumerate(sel_groups):
                    lst = cnt = None
                    npx = -1
                    if grp.num_items and sel_ids and d > 0:
                        j = sel_ids.index(gi)
                        lst = ws.item_list(gi, grp)[0]
                        cnt = st.counts[d - 1, 4 + 8 * j: 12 + 8 * j]
                        npx = per_xcd[gi]
                    elif grp.num_items and n_open <= LISTED_MAX_NODES:
                        lst, cnt = ws.item_list(gi, grp)
                    lists.append(lst)
                    cnts.append(cnt)
                    npxs.append(npx)
                runner.hist(n_build, hist_target, h_boff, feat_mask, s2n, pack, lists, cnts, npxs,
                            shards._shard_of if shards is not None else None,
                            bufs.shard_bins if shards is not None else 0)
                sel_groups = []
            for gi, grp in enumerate(sel_groups):
                if grp.num_items == 0:
                    continue
                if sampled:
                    pack = ws.rowpack() if (d > 0 and not single) else None
                    if sel_ids and d > 0:
                        # preselected: exactly one wave per active item (the lists were built with
                        # the previous level's plan)
                        j = sel_ids.index(gi)
                        lst = ws.item_list(gi, grp)[0]
                        cnt = st.counts[d - 1, 4 + 8 * j: 12 + 8 * j]
                        npx = per_xcd[gi]
                    else:
                        # the listed pass wins while few items are active (<= 2 open nodes: ~0.16
                        # vs 0.19 ms at the root); with more, its fixed grid balances worse than a
                        # wave per slot (profiles/r3s3/rf_probe_chunks.txt)
                        lst, cnt = ws.item_list(gi, grp) if n_open <= LISTED_MAX_NODES else (None, None)
                        npx = -1
                    launches.append(functools.partial(
                        C.tree_hist_sampled, grp.item_start, grp.item_end, grp.item_f0, grp.item_meta,
                        grp.wave_order(), Q.h_row, Q.h_key, pack, csc_dig, h_boff, Q.nbins, s2n, hist_target, h_stride,
                        grp.bt, ct, feat_mask, lst, cnt, RF_LDS, npx))
                    continue
                launches.append(functools.partial(
                    C.tree_hist_build, grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(),
                    Q.h_row, Q.h_key, csc_slot8, csc_dig, h_boff, Q.nbins, s2n, hist_target, h_stride, grp.bt, ct,
                    np_, feat_mask))
            if use_dense:
                for bt in (1, 2, 4):
                    fg = C.tree_dense_fg(bt, ct if d > 0 else 1)
                    gfid, gden = ws.dense_groups(bt, fg)
                    if gfid.numel():
                        rr = dense_range_rows(Q.n_rows, gfid.numel() // fg)
                        launches.append(functools.partial(
                            C.tree_hist_dense, Q.dense, ws.digp, ws.rowdig, None if d == 0 else ws.slot8_pad,
                            gfid, gden, h_boff, Q.nbins, s2n, hist_target, h_stride, Q.n_rows, rr, bt, ct, np_))
            ws.run_concurrent(launches)
        row_of = None
        if shards is not None:
            yield CollStep("rs")                  # (the batch's reduce-scatter, LevelBatcher.serve)
            if d == 0:
                tot = bufs.reduced_totals()
                st.stats[0].copy_(tot)
                totals_d.copy_(tot[None])
            if build_all or d == 0:
                # every open node built, slot k = open node k (tree.h level_plan): the reduced
                # rows ARE the level's histograms (stride Bs, read in place by the split search)
                cur_hist = bufs.mine()
            else:
                # the built rows stay where the collective wrote them and the subtraction fills
                # rows after them: per open node its row (tree.h LevelRowsArgs), no copy
                row_of = st.row_of[cur][:n_open]
                C.tree_level_rows(st.s2n, st.sub_dst, st.sub_par, prev_row_of, n_build, bufs.row0, bufs.sub_base,
                                  st.row_of[cur], st.dst_row, st.par_row, st.sib_row)
                if LEVEL_CHECKS:
                    n_sub = int((st.sub_dst[:n_build] >= 0).sum())
                    assert n_build + n_sub == n_open, (d, n_build, n_sub, n_open)
                cur_hist = bufs.out
        # (single-process runner levels subtract inside the split search: split_plan prev_hist)
        fused_sub = runner is not None and shards is None and d > 0 and not build_all and SPLIT_SUBTRACT
        if d > 0 and not build_all and not fused_sub:
            if shards is None:
                C.tree_hist_subtract(prev_hist, cur_hist, st.sub_dst[:n_build], st.sub_par[:n_build],
                                     st.sub_sib[:n_build], TB)
            else:
                C.tree_hist_subtract(prev_hist, cur_hist, st.dst_row[:n_build], st.par_row[:n_build],
                                     st.sib_row[:n_build], bufs.Bs)
        with tracing.span("tree.split"):
            if runner is not None and shards is None:
                packed = ws.split_cache.get(("out", n_open))
                if packed is None:
                    packed = ws.split_cache[("out", n_open)] = torch.empty((n_open, 5), dtype=torch.int64, device=dev)
                # (split search, best split and level plan: 2 launches, below)
            elif runner is not None:
                runner.split(cur_hist, totals_d, split_boff, shards.nbins, shards.zbin, shards.fid_orig, open_d,
                             feat_thr, int(tree_index), shards.f0, bufs.ag_in, row_of,
                             _wide_features(shards.nbins, shards.Fa) if SPLIT_WIDE else None)
                packed = yield CollStep("ag")
            elif shards is None:
                packed = _best_splits(C, cur_hist, totals_d, Q.boff, Q.nbins, Q.zbin, Q.fid_orig, open_d, ws.kexp,
                                      params, feat_thr, tree_index, Q.Fa, 0, cache=ws.split_cache)
            else:
                _best_splits(C, cur_hist, totals_d, split_boff, shards.nbins, shards.zbin, shards.fid_orig,
                             open_d, ws.kexp, params, feat_thr, tree_index, shards.Fa, shards.f0,
                             cache=ws.split_cache, out=bufs.ag_in, row_of=row_of)
                # [S, n_open, 5] (the batch's all-gather): tree_level_plan takes the best over
                # shards per node (ties to the lowest shard = the lowest feature)
                packed = yield CollStep("ag")
        nxt = 1 - cur
        if runner is not None:
            more = d + 1 < params.max_depth
            sample_next = more and (compact or bool(sel_ids))
            if sample_next and compact:
                thr_n, mask_n = shards.compact_thr(nxt, 2 * n_open), shards.compact_mask(nxt)
                lay = (shards._fs_dev, Q.nbins, shards._local_c[nxt], shards._sizes[nxt], shards.sizes_host[nxt],
                       shards.max_shard_features)
            elif sample_next:
                thr_n, mask_n, lay = st.rf_thr[nxt], st.rf_mask[nxt], (None,) * 5 + (0,)
            else:
                thr_n = mask_n = None
                lay = (None,) * 5 + (0,)
            if sel_ids and more:
                if sel_args is None:
                    sel_args = [ws.item_list(gi, grp)[0] if gi in sel_ids else None
                                for gi, grp in enumerate(item_groups)]
                sel = sel_args
            else:
                sel = []
            if shards is None:
                runner.split_plan(d, n_open, cur_hist, totals_d, Q.boff, feat_thr, int(tree_index), packed,
                                  _wide_features(Q.nbins, Q.Fa) if SPLIT_WIDE else None, open_d, n_open_ptr,
                                  st.open[nxt], st.totals[nxt], sample_next, thr_n, mask_n, sel,
                                  prev_hist if fused_sub else None)
            else:
                runner.plan(d, n_open, packed, open_d, n_open_ptr, st.open[nxt], st.totals[nxt], int(tree_index),
                            sample_next, thr_n, mask_n, *lay, sel)
            ev = st.record_event(cur_stream)
            zero = None
            if shards is None and more and not build_all:
                # the next level's histograms, zeroed by the partition kernel on the way
                pre_hist = zero = torch.empty((2 * n_open, TB, 2), dtype=torch.int64, device=dev)
            # the next level's row-list counts written by the partition's row pass (one pass less)
            rg_counted = bool(more and rg is not None and PARTITION_COUNTS and C.tree_partition_counts_ok(Q.n_rows))
            with tracing.span("tree.partition"):
                runner.partition(d, n_open, bool(sampled and FUSED_PACK and more), zero, native_prologue and sampled,
                                 ws.rg_work if rg_counted else None)
            prev_hist = cur_hist
            prev_row_of = row_of
            continue
        C.tree_level_plan(packed, n_open, d, params.max_depth, int(params.mode), build_all, ws.kexp,
                          float(params.min_gain), Q.zbin, st.hot_row,
                          st.n_nodes, st.stats, st.parent, st.left, st.right, st.feat, st.bin, st.leaf, st.gain,
                          open_d, n_open_ptr, st.default_child, st.node_dense, *st.cs, st.counts[d],
                          st.open[nxt], st.totals[nxt], st.node_slot, st.s2n, st.sub_dst, st.sub_par, st.sub_sib)
        if compact and d + 1 < params.max_depth:
            # level d + 1's open list is at most 2 n_open long, -1 padded (tree.h level_plan_reset)
            shards.sample_compact(C, nxt, seed, int(tree_index), st.open[nxt][:2 * n_open], int(Q.num_features),
                                  int(params.feat_k), Q.fid_orig)
        if sel_ids and d + 1 < params.max_depth:
            nxt_open = st.open[nxt][:2 * n_open]
            if compact:
                mask_n = shards.compact_mask(nxt)
            else:
                mask_n = st.rf_mask[nxt]
                C.tree_rf_sample(seed, int(tree_index), nxt_open, int(Q.num_features), int(params.feat_k),
                                 Q.fid_orig, st.rf_thr[nxt][:2 * n_open], mask_n, None)
            if sel_args is None:
                sel_args = ([[item_groups[gi].item_start, item_groups[gi].item_f0, item_groups[gi].item_meta,
                              item_groups[gi].wave_order()] for gi in sel_ids],
                            [ws.item_list(gi, item_groups[gi])[0] for gi in sel_ids])
            C.tree_hist_select_groups(sel_args[0], Q.nbins, mask_n, sel_args[1],
                                      st.counts[d, 4:].view(len(sel_ids), 8))
        st.counts_host[d].copy_(st.counts[d], non_blocking=dev.type == "cuda")
        ev = st.record_event(cur_stream)
        with tracing.span("tree.partition"):
            # (sampled RF levels: the next level's packed row state is written on the way)
            fuse = sampled and FUSED_PACK and d + 1 < params.max_depth
            C.tree_partition_cols(ws.row_node, st.default_child, *st.cs, st.counts[d], Q.colptr, Q.csc_row, Q.csc_bin,
                                  st.node_dense, Q.dense if st.node_dense is not None else None, n_open, PARTITION_WPS,
                                  *((st.node_slot, ws.rowdig, ws.rowpack()) if fuse else (None, None, None)))
        if shards is None and d + 1 < params.max_depth:
            pre_hist = torch.zeros((2 * n_open, TB, 2), dtype=torch.int64, device=dev)
        prev_hist = cur_hist
        prev_row_of = row_of
    if on_first_wait is not None:          # (a one-level tree) the previous table first
        on_first_wait()
    # one read of the node table per tree: the arena (table + exponents) in one D2H copy, one wait
    if not native_prologue and rg_dp is None:      # (the prologue's quantisation wrote them)
        st.kexp_slot.copy_(ws.kexp)
    node_value = None
    if deferred and params.mode == 0:
        # the margin update reads the device node table (one launch with the runner)
        node_value = (runner, params) if runner is not None else leaf_values_device(st.stats, ws.kexp, params)
    st.arena_host.copy_(st.arena, non_blocking=True)
    done = torch.cuda.Event() if dev.type == "cuda" else _Done()
    if dev.type == "cuda":
        done.record(cur_stream)

    def finish() -> Tree:
        done.synchronize()
        return tree_from_host(Q, params, st.host)

    if node_value is not None:
        return PendingTree(node_value, finish)
    yield done
    return finish()


class _Done:
    def synchronize(self):
        pass

    def query(self) -> bool:
        return True


def _weight(st, mode) -> int:
    return int(st[1]) if mode == 0 else int(st[0] + st[1])


def _partition(C, Q: Quantized, ws: Workspace, default_child: np.ndarray, splits: list, chunk: int = 1 << 16,
               row_node: Optional[torch.Tensor] = None):
    """Rows -> children (K-13): every row of a split node moves to the default child, then one pass
    over the split columns moves the rows present in them whose bin falls on the other side."""
    hs = _partition_stage(Q, ws.staging, default_child, splits, chunk)
    up = ws.staging.upload()
    _partition_launch(C, Q, up, hs, ws.row_node if row_node is None else row_node)


def _partition_stage(Q: Quantized, stg, default_child: np.ndarray, splits: list, chunk: int = 1 << 16) -> tuple:
    """Host arrays of one tree's level partition, added to ``stg`` (upload separately)."""
    colptr = Q.colptr.cpu().numpy() if not hasattr(Q, "_colptr_host") else Q._colptr_host
    Q._colptr_host = colptr
    # splits on hot features: the row pass reads the node's bin from the dense block (1 byte per
    # row, coalesced) instead of scattering the column's millions of CSC entries
    node_dense = None
    col_splits = splits
    if Q.dense is not None and PARTITION_DENSE:
        if getattr(Q, "_hot_row", None) is None:
            Q._hot_row = np.full(Q.Fa, -1, dtype=np.int32)
            Q._hot_row[Q.hot] = np.arange(len(Q.hot), dtype=np.int32)
        node_dense = np.full((len(default_child), 4), -1, dtype=np.int32)
        col_splits = []
        for sp in splits:
            fid, dflt, other, b, left_default, n = sp
            hr = int(Q._hot_row[fid])
            if hr >= 0:
                node_dense[n] = (hr, b, dflt if left_default else other, other if left_default else dflt)
            else:
                col_splits.append(sp)
    splits = col_splits
    starts, ends, item_split = [], [], []
    for si, sp in enumerate(splits):
        a, b = int(colptr[sp[0]]), int(colptr[sp[0] + 1])
        for s in range(a, b, chunk):
            starts.append(s)
            ends.append(min(b, s + chunk))
            item_split.append(si)
    hs = [stg.add(default_child), stg.add(np.array(starts, dtype=np.int64)), stg.add(np.array(ends, dtype=np.int64)),
          stg.add(np.array(item_split, dtype=np.int32))]
    hs += [stg.add(np.array([sp[k] for sp in splits], dtype=np.int32)) for k in (1, 2, 3, 4)]
    h_nd = stg.add(node_dense) if node_dense is not None else None
    return hs, h_nd


def _partition_launch(C, Q: Quantized, up: list, staged: tuple, row_node: torch.Tensor) -> None:
    hs, h_nd = staged
    C.tree_partition(row_node, *(up[h] for h in hs), Q.csc_row, Q.csc_bin,
                     up[h_nd] if h_nd is not None else None, Q.dense if h_nd is not None else None)