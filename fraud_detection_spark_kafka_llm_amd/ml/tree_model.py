"""Host representation of decision trees + Spark ``NodeData`` persistence.

A ``Tree`` holds per-node numpy arrays (any node order, ``root`` index). Spark stores nodes in
pre-order with ids 0..n-1 (``DecisionTreeModelReadWrite.NodeData.build``): internal nodes carry
``split{featureIndex, leftCategoriesOrThreshold=[threshold], numCategories=-1}``, leaves carry
``leftChild = rightChild = -1``, ``gain = -1`` and ``split{-1, [], -1}`` [Spark-3.5 spec].
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..io import spark_format as sf
from ..ops.text import TreeArrays


@dataclass
class Tree:
    feature: np.ndarray        # int32, -1 for leaves
    threshold: np.ndarray      # float64 (value-space threshold)
    left: np.ndarray           # int32, -1 for leaves
    right: np.ndarray          # int32
    stats: np.ndarray          # float64 [n, K] impurity stats (class counts) or [n, 1] leaf value
    impurity: np.ndarray       # float64
    gain: np.ndarray           # float64 (-1 for leaves)
    raw_count: np.ndarray      # int64
    prediction: np.ndarray     # float64
    root: int = 0

    @property
    def num_nodes(self) -> int:
        return int(self.feature.size)

    def is_leaf(self, i: int) -> bool:
        return self.feature[i] < 0

    def depth(self) -> int:
        def d(i):
            return 0 if self.feature[i] < 0 else 1 + max(d(self.left[i]), d(self.right[i]))
        return d(self.root)

    def preorder(self) -> list:
        out, stack = [], [self.root]
        while stack:
            i = stack.pop()
            out.append(i)
            if self.feature[i] >= 0:
                stack.append(int(self.right[i]))
                stack.append(int(self.left[i]))
        return out

    def compacted(self) -> "Tree":
        """Re-index nodes in pre-order (root = 0), dropping unreachable nodes."""
        order = self.preorder()
        remap = np.full(self.num_nodes, -1, dtype=np.int64)
        remap[np.asarray(order, dtype=np.int64)] = np.arange(len(order))
        o = np.asarray(order, dtype=np.int64)

        def child(a):
            c = a[o]
            return np.where(c >= 0, remap[np.maximum(c, 0)], -1).astype(np.int32)

        return Tree(self.feature[o].astype(np.int32), self.threshold[o], child(self.left), child(self.right),
                    self.stats[o], self.impurity[o], self.gain[o], self.raw_count[o], self.prediction[o], 0)

    # -------------------------------------------------------------- inference (host oracle)
    def leaf_of(self, x: dict, cmp_less: bool = False) -> int:
        i = self.root
        while self.feature[i] >= 0:
            v = x.get(int(self.feature[i]), 0.0)
            go_left = v < self.threshold[i] if cmp_less else v <= self.threshold[i]
            i = int(self.left[i] if go_left else self.right[i])
        return i

    # -------------------------------------------------------------- spark NodeData
    def to_node_rows(self) -> list:
        t = self.compacted()
        rows = []
        for i in range(t.num_nodes):
            leaf = t.feature[i] < 0
            rows.append({
                "id": i,
                "prediction": float(t.prediction[i]),
                "impurity": float(t.impurity[i]),
                "impurityStats": [float(v) for v in t.stats[i]],
                "rawCount": int(t.raw_count[i]),
                "gain": -1.0 if leaf else float(t.gain[i]),
                "leftChild": -1 if leaf else int(t.left[i]),
                "rightChild": -1 if leaf else int(t.right[i]),
                "split": {"featureIndex": -1 if leaf else int(t.feature[i]),
                          "leftCategoriesOrThreshold": [] if leaf else [float(t.threshold[i])],
                          "numCategories": -1},
            })
        return rows

    @classmethod
    def from_node_rows(cls, rows: list) -> "Tree":
        rows = sorted(rows, key=lambda r: r["id"])
        n = len(rows)
        K = max((len(r["impurityStats"] or []) for r in rows), default=1) or 1
        feat = np.full(n, -1, np.int32)
        thr = np.zeros(n)
        left = np.full(n, -1, np.int32)
        right = np.full(n, -1, np.int32)
        stats = np.zeros((n, K))
        for r in rows:
            i = r["id"]
            s = r["split"]
            if r["leftChild"] >= 0:
                if s["numCategories"] not in (-1, None):
                    raise NotImplementedError("categorical splits are not supported")
                feat[i] = s["featureIndex"]
                thr[i] = s["leftCategoriesOrThreshold"][0]
                left[i], right[i] = r["leftChild"], r["rightChild"]
            st = r["impurityStats"] or []
            stats[i, :len(st)] = st
        return cls(feat, thr, left, right, stats,
                   np.asarray([r["impurity"] for r in rows], dtype=np.float64),
                   np.asarray([r["gain"] for r in rows], dtype=np.float64),
                   np.asarray([r.get("rawCount", 0) or 0 for r in rows], dtype=np.int64),
                   np.asarray([r["prediction"] for r in rows], dtype=np.float64), 0)


SPLIT_FIELD = sf.Field.struct("split", [
    sf.Field.simple("featureIndex", "integer"),
    sf.Field.array("leftCategoriesOrThreshold", "double"),
    sf.Field.simple("numCategories", "integer")])
NODE_FIELDS = [
    sf.Field.simple("id", "integer"), sf.Field.simple("prediction", "double"),
    sf.Field.simple("impurity", "double"), sf.Field.array("impurityStats", "double"),
    sf.Field.simple("rawCount", "long"), sf.Field.simple("gain", "double"),
    sf.Field.simple("leftChild", "integer"), sf.Field.simple("rightChild", "integer"), SPLIT_FIELD]


def ensemble_arrays(trees: list, leaf_payload: str, weights: Optional[np.ndarray] = None,
                    cmp_less: bool = False) -> TreeArrays:
    """Concatenate trees into the flat arrays the native scorer traverses.

    ``leaf_payload``: ``"counts"`` (DT rawPrediction = class counts), ``"normalized"`` (RF:
    per-tree normalized class distribution), ``"value"`` (GBDT: scalar leaf value, K=1).
    """
    feats, thrs, lefts, rights, leaves, roots = [], [], [], [], [], []
    off = 0
    K = 1 if leaf_payload == "value" else trees[0].stats.shape[1] if trees else 2
    for t in trees:
        n = t.num_nodes
        feats.append(t.feature.astype(np.int32))
        thrs.append(t.threshold.astype(np.float64))
        lefts.append(np.where(t.left >= 0, t.left + off, -1).astype(np.int32))
        rights.append(np.where(t.right >= 0, t.right + off, -1).astype(np.int32))
        st = t.stats.astype(np.float64)
        if leaf_payload == "normalized":
            s = st.sum(1, keepdims=True)
            st = np.divide(st, s, out=np.zeros_like(st), where=s != 0)
        elif leaf_payload == "value":
            st = st[:, :1]
        leaves.append(st.reshape(n, -1)[:, :K])
        roots.append(t.root + off)
        off += n
    if not trees:
        return TreeArrays(np.full(1, -1), np.zeros(1), np.full(1, -1), np.full(1, -1), np.zeros(K), np.zeros(0, np.int32),
                          np.zeros(0), K, cmp_less)
    w = np.ones(len(trees)) if weights is None else np.asarray(weights, dtype=np.float64)
    return TreeArrays(np.concatenate(feats), np.concatenate(thrs), np.concatenate(lefts), np.concatenate(rights),
                      np.concatenate(leaves), np.asarray(roots, np.int32), w, K, cmp_less)


def feature_importances(trees: list, num_features: int, tree_weights: Optional[np.ndarray] = None) -> np.ndarray:
    """Spark ``TreeEnsembleModel.featureImportances``: per tree Σ gain·count (count = sum of the
    node's impurity stats), normalized per tree, summed, normalized (X-12)."""
    total = np.zeros(num_features)
    for t in trees:
        imp = np.zeros(num_features)
        for i in range(t.num_nodes):
            if t.feature[i] >= 0 and t.left[i] >= 0:
                imp[t.feature[i]] += t.gain[i] * float(t.stats[i].sum())
        s = imp.sum()
        if s > 0:
            imp /= s
        total += imp
    s = total.sum()
    return total / s if s > 0 else total
