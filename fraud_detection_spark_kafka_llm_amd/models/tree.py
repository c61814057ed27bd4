"""DecisionTree / RandomForest training on the histogram engine (X-09, X-10, X-12).

Spark semantics reproduced: gini (or entropy) impurity, maxBins=32 candidate
thresholds, minInstancesPerNode / minInfoGain, a node splits only if its best gain > 0, children
with zero impurity become leaves, and ``toNode(prune=true)`` merges sibling leaves with the same
prediction. RandomForest adds Poisson(1) bootstrap row weights (counter-based, regenerated per
tree, never stored) and per-node sampling of exactly k features without replacement
(``featureSubsetStrategy="auto"`` = ceil(sqrt(F)), models/rf_sampling.py).
Reference configs: /root/reference/fraud_detection_spark.py:59-74.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..ml.linalg import VectorColumn
from ..ml.tree_model import Tree
from ..parallel.dist import Collectives
from ..utils.config import default_device
from ..utils import tracing
from . import forest_batch
from .forest_batch import ForestLanes, grow_forest_concurrent
from .grower import GrowParams, Workspace, device_levels_ok, grow_tree
from .quantize import quantize
from .rf_sampling import features_per_node


@dataclass
class ForestResult:
    trees: list
    num_features: int
    lanes: int = 1                 # trees grown in flight together (PAR-05)


def prepare(features, labels, device=None, max_bins: int = 32, coll: Collectives = None, chunk: int = None):
    dev = torch.device(device) if device is not None else default_device()
    vc = features if isinstance(features, VectorColumn) else VectorColumn.from_rows(list(features))
    vc = vc.to(dev)
    y = labels
    if not isinstance(y, torch.Tensor):
        y = torch.as_tensor(np.asarray([float(v) for v in y], dtype=np.float32))
    y = y.to(device=dev, dtype=torch.float32).contiguous()
    if y.numel() != len(vc):
        raise ValueError("labels and features have different row counts")
    coll = coll or Collectives()
    counts, scale = (vc.tf_counts, vc.tf_scale) if getattr(vc, "count_bins", False) else (None, None)
    with tracing.span("tree.quantize"):
        Q = quantize(vc, max_bins=max_bins, counts=counts, scale=scale,
                     all_reduce_max=coll.max if coll.active else None,
                     all_gather=coll.gather_keys if coll.active else None,
                     **({"chunk": chunk} if chunk else {}))
    # global index of this shard's first row (contiguous rank-ordered shards): bootstrap draws
    # are keyed by global row, so a sharded forest equals the single-process one
    Q.row0 = 0
    if coll.active:
        sizes = coll.all_gather(torch.tensor([len(vc)], dtype=torch.int64, device=dev)).view(-1).cpu()
        Q.row0 = int(sizes[: coll.rank].sum())
    return Q, y, vc.size, vc


def prune_same_prediction(t: Tree) -> Tree:
    """Spark ``LearningNode.toNode(prune = true)``: collapse internal nodes whose two children
    are leaves with the same prediction (bottom-up)."""
    feat, left, right = t.feature.copy(), t.left.copy(), t.right.copy()
    gain = t.gain.copy()

    def rec(i):
        if feat[i] < 0:
            return True
        lleaf, rleaf = rec(left[i]), rec(right[i])
        if lleaf and rleaf and t.prediction[left[i]] == t.prediction[right[i]]:
            feat[i], left[i], right[i], gain[i] = -1, -1, -1, -1.0
            return True
        return False

    rec(t.root)
    return Tree(feat, t.threshold, left, right, t.stats, t.impurity, gain, t.raw_count, t.prediction, t.root).compacted()


def _local_lane_cap(Q) -> int:
    """Trees this rank can keep in flight: FDX_RF_INFLIGHT, and on the device no more lanes than
    half the free HBM holds (each lane holds a workspace of ~27 B per row, utils/memory.py)."""
    inflight = max(1, forest_batch.TREES_IN_FLIGHT)
    if Q.device.type == "cuda" and inflight > 1:
        from ..utils.memory import rf_lanes_that_fit

        inflight = rf_lanes_that_fit(Q.n_rows, inflight, torch.cuda.mem_get_info(Q.device)[0])
    return inflight


def fit_forest(features, labels, num_trees: int = 1, max_depth: int = 5, max_bins: int = 32, min_instances: int = 1,
               min_info_gain: float = 0.0, bootstrap: bool = False, feature_subset: str = "all", seed: int = 0,
               impurity: str = "gini", subsampling_rate: float = 1.0, device=None, weights=None,
               prune: bool = True, checkpoint_dir: Optional[str] = None, checkpoint_every: int = 50,
               resume: bool = False) -> ForestResult:
    """``checkpoint_dir``: the forest so far is written every ``checkpoint_every`` trees (a usable
    RandomForestClassificationModel + ``_resume.json``); ``resume=True`` continues from it. Tree
    t depends only on (seed, t) — bootstrap weights and feature samples are counter-based — so a
    resumed forest equals an uninterrupted one at any world size."""
    from ..parallel.checkpoint import EnsembleCheckpointer, data_fingerprint, maybe_fail

    if subsampling_rate != 1.0:
        raise NotImplementedError("subsamplingRate != 1.0 is not supported (Poisson(1) bootstrap only)")
    coll = Collectives()
    with tracing.span("forest.prepare"):
        Q, y, F, vc = prepare(features, labels, device, max_bins, coll)
    ckpt = None
    if checkpoint_dir:
        shape = dict(num_trees=num_trees, max_depth=max_depth, max_bins=max_bins, min_instances=min_instances,
                     min_info_gain=min_info_gain, bootstrap=bool(bootstrap), feature_subset=str(feature_subset),
                     seed=int(seed), impurity=impurity, weighted=weights is not None)
        ckpt = EnsembleCheckpointer(checkpoint_dir, checkpoint_every, "rf", data_fingerprint(vc, y, coll), shape)
    w = None
    if weights is not None:
        w = torch.as_tensor(np.asarray(weights, dtype=np.float32)).to(Q.device)
    strategy = feature_subset
    if str(strategy).lower() == "auto":
        strategy = "all" if num_trees == 1 else "sqrt"
    k = features_per_node(strategy, F)
    params = GrowParams(max_depth=max_depth, mode=2 if impurity == "entropy" else 1, min_child=float(min_instances),
                        min_gain=float(min_info_gain), feat_k=0 if k >= F else int(k),
                        seed=int(seed) & 0x7FFFFFFFFFFFFFFF)
    with tracing.span("forest.workspace"):
        ws = Workspace(Q)
    trees = ckpt.load_trees() if (ckpt is not None and resume) else []
    # PAR-05: several trees in flight, each on its own stream (models/forest_batch.py); under data
    # parallelism the lanes advance in FIFO order, so every rank issues one collective sequence
    inflight = _local_lane_cap(Q)
    if coll.active:
        # every rank must take the same path with the same lane count (ForestLanes, the lane groups
        # and their batched collective sizes, or the per-tree grow_tree fallback issue different
        # collective sequences): the smallest rank's cap wins
        inflight = int(coll.min(torch.tensor([inflight], dtype=torch.int64, device=Q.device)).item())
    lanes = None
    left = num_trees - len(trees)
    # (on the device every sampled forest, a single tree too, grows on the lockstep batch)
    if left > 0 and device_levels_ok(params, w) and (forest_batch.batch_ok(Q, params, w) or (inflight > 1 and left > 1)):
        with tracing.span("forest.lanes"):
            lanes = ForestLanes(Q, max(1, min(inflight, left)), ws)
    chunk = max(ckpt.every if ckpt is not None else 64, 1)
    t = len(trees)
    while t < num_trees:
        if lanes is not None:
            ids = list(range(t, min(num_trees, t + chunk)))
            grown = grow_forest_concurrent(Q, lanes, params, ids, y, w, bootstrap, coll=coll)
        else:
            ids = [t]
            with tracing.span("forest.tree", tree=t):
                grown = [grow_tree(Q, ws, params, t, label=y, weight=w, bootstrap=bootstrap, coll=coll)]
        for tid, tr in zip(ids, grown):
            before = len(trees)
            trees.append(prune_same_prediction(tr) if prune else tr.compacted())
            if ckpt is not None:
                crossed = (len(trees) // ckpt.every) > (before // ckpt.every)
                ckpt.maybe_save(len(trees), trees, 0.0, F, None, force=crossed or len(trees) == num_trees)
            maybe_fail(tid, model="rf")
        t += len(ids)
    return ForestResult(trees, F, len(lanes.ws) if lanes is not None else 1)
