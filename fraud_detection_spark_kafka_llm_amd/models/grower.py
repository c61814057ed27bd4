"""Level-wise histogram tree grower shared by DecisionTree, RandomForest and GBDT (X-09, X-10, X-13).

Per level (all nodes of the level batched into every launch):
  1. ``tree_slot8``        1-byte slot of the node being built per row (0xff: not built)
  2. ``tree_hist_build``   MFMA histograms of the smaller child of each sibling pair (+ reduce),
                           streaming the per-tree entry-order statistics (``tree_entry_stats``)
  3. all-reduce            histograms of the built nodes across data-parallel ranks (RCCL)
  4. ``tree_hist_subtract`` larger sibling = parent - built sibling
  5. ``tree_split_find``   best (feature, bin) per (node, feature); argmax per node on device
  6. host: create children (tiny D2H of one best split per node)
  7. ``tree_partition``    rows -> children (default side for rows absent from the split column)
Every rank makes identical decisions from identical reduced histograms, so no split broadcast is
needed. Node statistics of children come from the parent's split (as in Spark and XGBoost).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np
import torch

from ..ml.tree_model import Tree
from ..ops import native
from ..utils import tracing
from .quantize import CSC_PAD, Quantized

NEG_INF = float("-inf")


@dataclass
class GrowParams:
    max_depth: int = 5
    mode: int = 1                 # 0 xgboost newton, 1 gini, 2 entropy
    lambda_: float = 1.0          # gbdt L2
    min_child: float = 1.0        # gbdt: min_child_weight (hessian); cls: minInstancesPerNode
    min_gain: float = 0.0         # cls: minInfoGain ; gbdt: gamma (min_split_loss)
    feat_prob: float = 1.0        # RF per-node feature sampling probability
    seed: int = 0
    eta: float = 0.3              # gbdt learning rate (applied to leaf values)
    max_delta_step: float = 0.0


class Workspace:
    """Per-engine device buffers reused across trees (slab, row/entry statistics, slot table)."""

    def __init__(self, Q: Quantized, max_nodes_per_level: int):
        dev = Q.device
        self.rowstats = torch.empty((Q.n_rows, 2), dtype=torch.int32, device=dev)
        nnz = Q.csc_row.numel()
        self.est = torch.zeros((nnz + CSC_PAD, 2), dtype=torch.int32, device=dev)[:nnz]
        self.slot8 = torch.empty(Q.n_rows, dtype=torch.uint8, device=dev)
        self.row_node = torch.zeros(Q.n_rows, dtype=torch.int32, device=dev)
        self.max_items = max((g.num_items for g in Q.groups), default=0)
        self.slab = torch.empty(0, dtype=torch.float32, device=dev)
        self.Fa = Q.Fa
        self.dev = dev

    def slab_for(self, items: int, bt: int, ct: int) -> torch.Tensor:
        need = items * 8 * ct * 32 * bt * 2
        if self.slab.numel() < need:
            self.slab = torch.empty(need, dtype=torch.float32, device=self.dev)
        return self.slab


def _unpack_bf16_pair(col: torch.Tensor) -> torch.Tensor:
    hi = ((col & 0xFFFF) << 16).to(torch.int32).view(torch.float32).to(torch.float64)
    lo = (((col >> 16) & 0xFFFF) << 16).to(torch.int32).view(torch.float32).to(torch.float64)
    return hi + lo


def root_totals(ws: Workspace) -> torch.Tensor:
    st = ws.rowstats.to(torch.int64)
    return torch.stack([_unpack_bf16_pair(st[:, 0]).sum(), _unpack_bf16_pair(st[:, 1]).sum()])


def grow_tree(Q: Quantized, ws: Workspace, params: GrowParams, tree_index: int,
              g: Optional[torch.Tensor] = None, h: Optional[torch.Tensor] = None,
              label: Optional[torch.Tensor] = None, weight: Optional[torch.Tensor] = None,
              bootstrap: bool = False, all_reduce: Optional[Callable] = None) -> Tree:
    C = native.lib()
    dev = Q.device
    mode_rs = 0 if params.mode == 0 else 1
    max_nodes = 2 ** (params.max_depth + 1)
    # host node table
    parent = [-1]
    depth = [0]
    feature = [-1]
    binv = [-1]
    thr = [0.0]
    left = [-1]
    right = [-1]
    gain = [-1.0]
    stats = [None]
    is_leaf = [False]

    ws.row_node.zero_()
    with tracing.span("tree.rowstats"):
        C.tree_rowstats(g, h, label, weight, int(params.seed), int(tree_index), bool(bootstrap), mode_rs,
                        ws.rowstats)
        C.tree_entry_stats(Q.csc_row, ws.rowstats, ws.est)
    tot = root_totals(ws)
    if all_reduce is not None:
        tot = all_reduce(tot)
    stats[0] = tot.cpu().numpy().astype(np.float64)
    level = [0]
    prev_hist = None
    prev_index: dict = {}
    TB = Q.TB
    feat_groups = Q.groups

    for d in range(params.max_depth + 1):
        open_nodes = [n for n in level if not is_leaf[n]]
        if d == params.max_depth or not open_nodes:
            for n in open_nodes:
                is_leaf[n] = True
            break
        # --- decide which nodes to build (smaller sibling) and which to subtract
        build, subtract = [], []
        if d == 0:
            build = open_nodes
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
        cur_hist = torch.zeros((nl, TB, 2), dtype=torch.float64, device=dev)
        # --- node -> slot of the built nodes (slot = position in `build`); the root pass needs none
        if d > 0:
            ns = torch.full((max_nodes,), -1, dtype=torch.int32)
            for s, n in enumerate(build):
                ns[n] = s
            node_slot = ns.to(dev)
        # --- histograms, 8*ct slots per pass
        nb = len(build)
        with tracing.span("tree.hist"):
            for s0 in range(0, nb, 32):
                cnt = min(32, nb - s0)
                ct = 1 if cnt <= 8 else (2 if cnt <= 16 else 4)
                s2n = torch.full((8 * ct,), -1, dtype=torch.int32)
                for k in range(cnt):
                    s2n[k] = local[build[s0 + k]]
                s2n = s2n.to(dev)
                slot8 = None
                if d > 0:
                    C.tree_slot8(ws.row_node, node_slot, s0, cnt, ws.slot8)
                    slot8 = ws.slot8
                for grp in feat_groups:
                    gsel = grp if params.feat_prob >= 1.0 else _rf_subset(grp, Q, params, tree_index,
                                                                          [build[s0 + k] for k in range(cnt)])
                    if gsel.num_items == 0:
                        continue
                    slab = ws.slab_for(gsel.num_items, grp.bt, ct)
                    C.tree_hist_build(gsel.item_start, gsel.item_end, Q.csc_row, Q.csc_bin, slot8, ws.est,
                                      grp.bt, ct, slab, gsel.feat, gsel.feat_item0, gsel.feat_nitems, Q.boff,
                                      Q.nbins, s2n, cur_hist, TB)
        if all_reduce is not None:
            with tracing.span("tree.allreduce"):
                idx = torch.tensor([local[n] for n in build], device=dev)
                part = cur_hist.index_select(0, idx)
                part = all_reduce(part)
                cur_hist.index_copy_(0, idx, part)
        if subtract:
            dst = torch.tensor([local[a] for a, _, _ in subtract], dtype=torch.int32, device=dev)
            par = torch.tensor([prev_index[p] for _, p, _ in subtract], dtype=torch.int32, device=dev)
            sib = torch.tensor([local[s] for _, _, s in subtract], dtype=torch.int32, device=dev)
            C.tree_hist_subtract(prev_hist, cur_hist, dst, par, sib, TB)
        # --- split search
        totals = torch.tensor(np.stack([stats[n] for n in open_nodes]), dtype=torch.float64, device=dev)
        node_ids = torch.tensor(open_nodes, dtype=torch.int32, device=dev)
        out_gain = torch.empty((nl, Q.Fa), dtype=torch.float64, device=dev)
        out_bin = torch.empty((nl, Q.Fa), dtype=torch.int32, device=dev)
        out_left = torch.empty((nl, Q.Fa, 2), dtype=torch.float64, device=dev)
        with tracing.span("tree.split"):
            C.tree_split_find(cur_hist, totals, Q.boff, Q.nbins, Q.zbin, Q.fid_orig, node_ids, int(params.mode),
                              float(params.lambda_), float(params.min_child), float(params.feat_prob),
                              int(params.seed), int(tree_index), out_gain, out_bin, out_left)
            best_gain, best_f = torch.max(out_gain, dim=1)
            ar = torch.arange(nl, device=dev)
            best_bin = out_bin[ar, best_f]
            best_left = out_left[ar, best_f]
            packed = torch.cat([best_gain[:, None], best_f[:, None].double(), best_bin[:, None].double(), best_left], 1)
            packed = packed.cpu().numpy()
        # --- create children
        next_level = []
        default_child = torch.full((max_nodes,), -1, dtype=torch.int32)
        splits = []
        for i, n in enumerate(open_nodes):
            gval, fid, b, l0, l1 = packed[i]
            fid, b = int(fid), int(b)
            ok = b >= 0 and math.isfinite(gval)
            if params.mode == 0:
                ok = ok and gval > max(params.min_gain, 1e-6)
            else:
                ok = ok and gval > 0.0 and gval >= params.min_gain
            if not ok:
                is_leaf[n] = True
                continue
            tl = np.array([l0, l1])
            tr = stats[n] - tl
            li, ri = len(parent), len(parent) + 1
            for child, st in ((li, tl), (ri, tr)):
                parent.append(n)
                depth.append(d + 1)
                feature.append(-1)
                binv.append(-1)
                thr.append(0.0)
                left.append(-1)
                right.append(-1)
                gain.append(-1.0)
                stats.append(st)
                leafy = (d + 1 >= params.max_depth)
                if params.mode != 0:
                    leafy = leafy or _impurity(st, params.mode) == 0.0
                is_leaf.append(leafy)
            feature[n], binv[n], thr[n], left[n], right[n], gain[n] = fid, b, Q.threshold(fid, b), li, ri, gval
            left_default = int(Q.zbin_host[fid]) <= b
            dflt, other = (li, ri) if left_default else (ri, li)
            default_child[n] = dflt
            splits.append((fid, dflt, other, b, int(left_default)))
            next_level += [li, ri]
        if splits:
            with tracing.span("tree.partition"):
                _partition(C, Q, ws, default_child.to(dev), splits)
        prev_hist = cur_hist
        prev_index = local
        level = next_level

    n = len(parent)
    K = 2
    st = np.zeros((n, K))
    for i in range(n):
        st[i] = stats[i]
    feat_orig = np.array([int(Q.fid_host[f]) if f >= 0 and not is_leaf[i] else -1 for i, f in enumerate(feature)],
                         dtype=np.int32)
    left_a = np.array([l if not is_leaf[i] else -1 for i, l in enumerate(left)], dtype=np.int32)
    right_a = np.array([r if not is_leaf[i] else -1 for i, r in enumerate(right)], dtype=np.int32)
    thr_a = np.array(thr, dtype=np.float64)
    gain_a = np.array([gv if not is_leaf[i] else -1.0 for i, gv in enumerate(gain)], dtype=np.float64)
    if params.mode == 0:
        G, H = st[:, 0], st[:, 1]
        w = -G / (H + params.lambda_)
        if params.max_delta_step > 0:
            w = np.clip(w, -params.max_delta_step, params.max_delta_step)
        value = params.eta * w
        imp = np.zeros(n)
        pred = value
        stats_out = np.stack([value, H], 1)
        raw_count = np.zeros(n, dtype=np.int64)
    else:
        imp = np.array([_impurity(s, params.mode) for s in st])
        pred = np.argmax(st, axis=1).astype(np.float64)
        stats_out = st
        raw_count = np.rint(st.sum(1)).astype(np.int64)
    return Tree(feat_orig, thr_a, left_a, right_a, stats_out, imp, gain_a, raw_count, pred, 0)


def _weight(st, mode) -> float:
    return float(st[1]) if mode == 0 else float(st[0] + st[1])


def _impurity(st, mode) -> float:
    c0, c1 = float(st[0]), float(st[1])
    n = c0 + c1
    if n <= 0:
        return 0.0
    p0, p1 = c0 / n, c1 / n
    if mode == 2:
        return -sum(p * math.log2(p) for p in (p0, p1) if p > 0)
    return 1.0 - p0 * p0 - p1 * p1


def _partition(C, Q: Quantized, ws: Workspace, default_child: torch.Tensor, splits: list, chunk: int = 1 << 16):
    colptr = Q.colptr.cpu().numpy() if not hasattr(Q, "_colptr_host") else Q._colptr_host
    Q._colptr_host = colptr
    starts, ends, item_split = [], [], []
    for si, (fid, _, _, _, _) in enumerate(splits):
        a, b = int(colptr[fid]), int(colptr[fid + 1])
        for s in range(a, b, chunk):
            starts.append(s)
            ends.append(min(b, s + chunk))
            item_split.append(si)
    dev = Q.device
    t = lambda v, dt: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    C.tree_partition(ws.row_node, default_child, t(starts, torch.int64), t(ends, torch.int64),
                     t(item_split, torch.int32), t([s[1] for s in splits], torch.int32),
                     t([s[2] for s in splits], torch.int32), t([s[3] for s in splits], torch.int32),
                     t([s[4] for s in splits], torch.int32), Q.csc_row, Q.csc_bin)


def _rf_subset(grp, Q: Quantized, params: GrowParams, tree_index: int, nodes: list):
    """Features sampled by at least one node of this pass (same hash as the split kernel)."""
    from .rf_sampling import node_feature_mask

    mask = node_feature_mask(Q, params, tree_index, nodes)
    return grp.subset(mask)
