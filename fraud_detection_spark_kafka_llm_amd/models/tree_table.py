"""Trees of the grower as the host sees them (models/grower.py): the grow parameters, the host node
table shared by the host loop and the batched drivers (TreeTable), the host build of a tree from
the device node table (tree_from_host), the deferred GBDT tree (PendingTree) and the node
impurity. Reference: /root/reference/fraud_detection_spark.py:57-83 (the Spark DT / RF / XGBoost
estimators whose trees these are)."""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from ..ml.tree_model import Tree
from ..ops import native
from .quantize import Quantized

@dataclass
class GrowParams:
    max_depth: int = 5
    mode: int = 1                 # 0 xgboost newton, 1 gini, 2 entropy
    lambda_: float = 1.0          # gbdt L2
    min_child: float = 1.0        # gbdt: min_child_weight (hessian); cls: minInstancesPerNode
    min_gain: float = 0.0         # cls: minInfoGain ; gbdt: gamma (min_split_loss)
    feat_k: int = 0               # RF: features sampled per node (0 = all)
    seed: int = 0
    eta: float = 0.3              # gbdt learning rate (applied to leaf values)
    max_delta_step: float = 0.0


class TreeTable:
    """Host node table of one tree under construction (shared by grow_tree and the multi-tree RF
    batches, so both create exactly the same nodes from the same best-split tuples)."""

    def __init__(self, root_stats: np.ndarray):
        self.parent, self.depth, self.feature, self.binv, self.thr = [-1], [0], [-1], [-1], [0.0]
        self.left, self.right, self.gain, self.stats, self.is_leaf = [-1], [-1], [-1.0], [root_stats], [False]

    @classmethod
    def from_arrays(cls, Q: Quantized, parent, feat, binv, left, right, gain, stats, leaf) -> "TreeTable":
        """The node table the device level loop built (tree.h level_plan), same numbering."""
        t = cls(stats[0])
        n = len(parent)
        t.parent = [int(v) for v in parent]
        t.depth = [0] * n
        t.feature = [int(v) for v in feat]
        t.binv = [int(v) for v in binv]
        t.thr = [Q.threshold(int(f), int(b)) if f >= 0 else 0.0 for f, b in zip(feat, binv)]
        t.left = [int(v) for v in left]
        t.right = [int(v) for v in right]
        t.gain = [float(v) for v in gain]
        t.stats = [np.asarray(st, dtype=np.int64) for st in stats]
        t.is_leaf = [bool(v) for v in leaf]
        return t

    def apply_splits(self, open_nodes: list, packed: np.ndarray, d: int, Q: Quantized, params: GrowParams,
                     scale: np.ndarray, max_nodes: int) -> tuple:
        """Best-split tuples [len(open_nodes), 5] -> children; returns (next level, default child
        table [max_nodes], partition splits)."""
        next_level = []
        default_child = np.full(max_nodes, -1, dtype=np.int32)
        splits = []
        gains_host = packed[:, 0].copy().view(np.float64)
        for i, n in enumerate(open_nodes):
            gval = float(gains_host[i])
            fid, b = int(packed[i, 1]), int(packed[i, 2])
            ok = b >= 0 and math.isfinite(gval)
            if params.mode == 0:
                ok = ok and gval > max(params.min_gain, 1e-6)
            else:
                ok = ok and gval > 0.0 and gval >= params.min_gain
            if not ok:
                self.is_leaf[n] = True
                continue
            tl = packed[i, 3:5].astype(np.int64)
            tr = self.stats[n] - tl
            li, ri = len(self.parent), len(self.parent) + 1
            for st in (tl, tr):
                self.parent.append(n)
                self.depth.append(d + 1)
                self.feature.append(-1)
                self.binv.append(-1)
                self.thr.append(0.0)
                self.left.append(-1)
                self.right.append(-1)
                self.gain.append(-1.0)
                self.stats.append(st)
                leafy = (d + 1 >= params.max_depth)
                if params.mode != 0:
                    leafy = leafy or _impurity(st * scale, params.mode) == 0.0
                self.is_leaf.append(leafy)
            self.feature[n], self.binv[n], self.thr[n] = fid, b, Q.threshold(fid, b)
            self.left[n], self.right[n], self.gain[n] = li, ri, gval
            left_default = int(Q.zbin_host[fid]) <= b
            dflt, other = (li, ri) if left_default else (ri, li)
            default_child[n] = dflt
            splits.append((fid, dflt, other, b, int(left_default), n))
            next_level += [li, ri]
        return next_level, default_child, splits

    def build(self, Q: Quantized, params: GrowParams, scale: np.ndarray) -> Tree:
        is_leaf = self.is_leaf
        n = len(self.parent)
        st = np.zeros((n, 2), dtype=np.float64)
        for i in range(n):
            st[i] = self.stats[i].astype(np.float64) * scale
        feat_orig = np.array([int(Q.fid_host[f]) if f >= 0 and not is_leaf[i] else -1
                              for i, f in enumerate(self.feature)], dtype=np.int32)
        left_a = np.array([lc if not is_leaf[i] else -1 for i, lc in enumerate(self.left)], dtype=np.int32)
        right_a = np.array([rc if not is_leaf[i] else -1 for i, rc in enumerate(self.right)], dtype=np.int32)
        thr_a = np.array(self.thr, dtype=np.float64)
        gain_a = np.array([gv if not is_leaf[i] else -1.0 for i, gv in enumerate(self.gain)], dtype=np.float64)
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


def tree_from_host(Q: Quantized, params: GrowParams, hv: dict) -> Tree:
    """The Tree of a device node table copied to the host (LevelState.host views of the arena):
    TreeTable.from_arrays(...).build(...) in numpy array operations, the same IEEE operations per
    node (so the same bits; ~10x less host time: a forest builds 500 of these)."""
    if isinstance(hv["n_nodes"], torch.Tensor):      # (numpy views of the same pinned memory)
        hv = {k: v.numpy() for k, v in hv.items()}
    nn = int(hv["n_nodes"][0])
    feat = hv["feat"][:nn].astype(np.int64)
    binv = hv["bin"][:nn].astype(np.int64)
    leaf = hv["leaf"][:nn].astype(bool)
    inner = ~leaf
    kexp = hv["kexp"].astype(np.int64)
    st = hv["stats"][:nn].astype(np.float64) * np.ldexp(1.0, -kexp)
    thr_np = getattr(Q, "_thresholds_np", None)
    if thr_np is None:
        t = Q.thresholds
        thr_np = Q._thresholds_np = (t.cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)).astype(np.float64)
    boff = np.asarray(Q.boff_host, dtype=np.int64)
    has_f = feat >= 0
    fsafe = np.where(has_f, feat, 0)
    thr_a = np.where(has_f, thr_np[boff[fsafe] + np.where(has_f, binv, 0)], 0.0)
    feat_orig = np.where(has_f & inner, np.asarray(Q.fid_host)[fsafe], -1).astype(np.int32)
    left_a = np.where(inner, hv["left"][:nn], -1).astype(np.int32)
    right_a = np.where(inner, hv["right"][:nn], -1).astype(np.int32)
    gain_a = np.where(inner, hv["gain"][:nn].astype(np.float64), -1.0)
    if params.mode == 0:
        G, H = st[:, 0], st[:, 1]
        w = -G / (H + params.lambda_)
        if params.max_delta_step > 0:
            w = np.clip(w, -params.max_delta_step, params.max_delta_step)
        value = params.eta * w
        return Tree(feat_orig, thr_a, left_a, right_a, np.stack([value, H], 1), np.zeros(nn), gain_a,
                    np.zeros(nn, dtype=np.int64), value, 0)
    if params.mode == 1:                       # gini, vectorised (1 - p0 p0 - p1 p1, 0 for empty nodes)
        c0, c1 = st[:, 0], st[:, 1]
        n = c0 + c1
        pos = n > 0
        ns = np.where(pos, n, 1.0)
        p0, p1 = c0 / ns, c1 / ns
        imp = np.where(pos, 1.0 - p0 * p0 - p1 * p1, 0.0)
    else:                                      # (entropy: math.log2 per node, as _impurity)
        imp = np.array([_impurity(s, params.mode) for s in st])
    return Tree(feat_orig, thr_a, left_a, right_a, st, imp, gain_a, np.rint(st.sum(1)).astype(np.int64),
                np.argmax(st, axis=1).astype(np.float64), 0)


def leaf_values_device(stats: torch.Tensor, kexp: torch.Tensor, params: GrowParams) -> torch.Tensor:
    """GBDT leaf values of the device node table, the same fp64 operations as TreeTable.build
    (so bitwise the host's values): G, H = stats * 2^-k (exact), eta * clip(-G / (H + lambda)).
    One native launch over the table (csrc/tree.h leaf_value) instead of ~10 elementwise ops."""
    out = torch.empty(stats.shape[0], dtype=torch.float64, device=stats.device)
    native.lib().tree_leaf_values(stats, kexp, float(params.eta), float(params.lambda_),
                                  float(params.max_delta_step), out)
    return out


class PendingTree:
    """A grown GBDT tree whose host table is not built yet: ``node_value`` (device, per node id)
    is ready in stream order for the margin update -- or (runner, params): the native runner
    updates the margins from the device node table itself; ``result()`` builds the Tree once."""

    def __init__(self, node_value, finish):
        self.node_value = node_value
        self._finish = finish
        self._tree = None

    def update_margin(self, margin: torch.Tensor, row_node: torch.Tensor) -> None:
        """margin[r] += the leaf value of row r's node (queued on the current stream)."""
        if isinstance(self.node_value, tuple):
            runner, p = self.node_value
            runner.leaf_update(margin, float(p.eta), float(p.lambda_), float(p.max_delta_step))
        else:
            native.lib().tree_leaf_update(margin, row_node, self.node_value)

    def finish(self) -> None:
        if self._tree is None:
            self._tree = self._finish()

    def result(self) -> Tree:
        self.finish()
        return self._tree


def _impurity(st, mode) -> float:
    c0, c1 = float(st[0]), float(st[1])
    n = c0 + c1
    if n <= 0:
        return 0.0
    p0, p1 = c0 / n, c1 / n
    if mode == 2:
        return -sum(p * math.log2(p) for p in (p0, p1) if p > 0)
    return 1.0 - p0 * p0 - p1 * p1
