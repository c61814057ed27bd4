"""Gradient-boosted trees, XGBoost-compatible (``binary:logistic``, hist) — X-13.

Per round: ``tree_logistic_grad`` (g = p - y, h = p(1-p)) -> level-wise histogram tree with
Newton gain ``GL^2/(HL+l) + GR^2/(HR+l) - G^2/(H+l)`` and ``min_child_weight`` on the hessian ->
leaf weights ``-eta * G / (H + l)`` -> ``tree_leaf_update`` (margin += leaf of each row, read from
the final row->node map; training rows are never re-scored). ``GBDTParams`` defaults are
XGBoost's own (max_depth 6, eta 0.3, lambda 1, gamma 0, min_child_weight 1, max_bin 256, the
BASELINE config's depth 6); the reference's ``SparkXGBClassifier(max_depth=5, n_estimators=100)``
(/root/reference/fraud_detection_spark.py:76-83) sets its own through the ML API.
``base_score=None`` estimates the intercept from the label mean like XGBoost >= 2.0.

Precision: g and h are the fp32 values of the logistic loss; histograms are exact int64 sums of
rint(v * 2^k) with k from the round's max |v| (|q| <= 2^30), so a bin sum differs from the fp64
sum of the fp32 g * w by at most count * 2^-(k+1) -- well inside fp32 accumulation error --
and is bitwise identical on host, device and every data-parallel world size.

Data parallel: rows are sharded across ranks, histograms and root totals are all-reduced
(RCCL over xGMI), every rank grows the identical tree.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from ..ml.tree_model import Tree
from ..ops import native
from ..parallel.dist import Collectives
from ..utils import tracing
from .grower import GrowParams, PendingTree, Workspace, grow_tree
from .tree import prepare


@dataclass
class GBDTParams:
    n_estimators: int = 100
    max_depth: int = 6
    learning_rate: float = 0.3
    reg_lambda: float = 1.0
    gamma: float = 0.0
    min_child_weight: float = 1.0
    max_bin: int = 256
    max_delta_step: float = 0.0
    base_score: Optional[float] = None
    seed: int = 0
    # Accepted for API compatibility: training is always bitwise reproducible for any world size
    # and work split (exact int64 histograms of quantised g, h; see models/grower.py).
    deterministic: bool = True


@dataclass
class GBDTResult:
    trees: list
    num_features: int
    base_margin: float
    params: GBDTParams
    history: list = field(default_factory=list)
    train_seconds: float = 0.0
    shape: dict = field(default_factory=dict)     # Fa, TB, nnz of this rank's quantized features


def _logit(p: float) -> float:
    p = min(max(p, 1e-7), 1 - 1e-7)
    return math.log(p / (1 - p))


def fit_gbdt(features, labels, params: GBDTParams = GBDTParams(), device=None, weights=None,
             eval_fn=None, checkpoint=None, start_trees: Optional[list] = None,
             checkpoint_dir: Optional[str] = None, checkpoint_every: int = 10, resume: bool = False) -> GBDTResult:
    """``checkpoint_dir``: write the partial ensemble every ``checkpoint_every`` trees; with
    ``resume=True`` continue from the last checkpoint there (any world size)."""
    from dataclasses import asdict

    from ..parallel.checkpoint import EnsembleCheckpointer, data_fingerprint, maybe_fail

    C = native.lib()
    coll = Collectives()
    t0 = time.perf_counter()
    with tracing.span("gbdt.prepare"):
        Q, y, F, vc = prepare(features, labels, device, params.max_bin, coll)
    ckpt = None
    if checkpoint_dir:
        ckpt = EnsembleCheckpointer(checkpoint_dir, checkpoint_every, "gbdt", data_fingerprint(vc, y, coll),
                                    asdict(params))
    resume_state = ckpt.load() if (ckpt is not None and resume) else None
    if resume_state is not None:
        start_trees = ckpt.load_trees()
        params = GBDTParams(**{**params.__dict__, "base_score": None})
        forced_base = float(resume_state["base_margin"])
    else:
        forced_base = None
    dev = Q.device
    w = None if weights is None else torch.as_tensor(np.asarray(weights, dtype=np.float32)).to(dev)
    N = Q.n_rows
    if forced_base is not None:
        base = forced_base
    elif params.base_score is None:
        s = coll.sum(torch.stack([(y * (w if w is not None else 1.0)).sum().double(),
                                  (w.sum() if w is not None else torch.tensor(float(N), device=dev)).double()]))
        base = _logit(float(s[0] / max(float(s[1]), 1e-12)))
    else:
        base = _logit(float(params.base_score))
    margin = torch.full((N,), base, dtype=torch.float64, device=dev)
    gp = GrowParams(max_depth=params.max_depth, mode=0, lambda_=params.reg_lambda, min_child=params.min_child_weight,
                    min_gain=params.gamma, seed=params.seed, eta=params.learning_rate,
                    max_delta_step=params.max_delta_step)
    with tracing.span("gbdt.workspace"):
        ws = Workspace(Q)
    trees = list(start_trees or [])
    if trees:   # resume: replay the checkpointed trees on this rank's training rows
        from ..ml.tree_model import ensemble_arrays
        from ..ops.sparse import score_csr

        # one tree at a time, in training order: each adds its fp64 leaf value to the margin
        # exactly like tree_leaf_update did ((base + v0) + v1) + ..., so a resumed run is bitwise
        # the uninterrupted one (one summed ensemble score would round in another order)
        for tr in trees:
            margin += score_csr(vc, ensemble_arrays([tr], "value", cmp_less=False))[:, 0]
    history = []
    # without per-round hooks, tree t's host table is built while tree t + 1's root level runs on
    # the GPU (its leaf values come from the device node table, bitwise the host's)
    defer = eval_fn is None and checkpoint is None and ckpt is None
    pending = None
    for t in range(len(trees), params.n_estimators):
        with tracing.span("gbdt.round", round=t):
            # the round's gradients: computed inside the tree's prologue (fused with the max |g|,
            # |h| pass on the device loop's native runner) from the margins and labels
            res = grow_tree(Q, ws, gp, t, label=y, weight=w, coll=coll, deferred=defer, margin=margin,
                            on_first_wait=pending.finish if pending is not None else None)
            if isinstance(res, PendingTree):
                # queued first: the host-side compaction below overlaps the margin update
                res.update_margin(margin, ws.row_node)
            if pending is not None:
                trees.append(pending.result().compacted())
                pending = None
            if isinstance(res, PendingTree):
                pending = res
                maybe_fail(t, model="gbdt")
                continue
            tree = res
            node_value = torch.from_numpy(np.ascontiguousarray(tree.stats[:, 0])).to(dev)
            C.tree_leaf_update(margin, ws.row_node, node_value)
        trees.append(tree.compacted())
        if eval_fn is not None:
            history.append(eval_fn(t, trees, margin))
        if checkpoint is not None:
            checkpoint(t, trees, base)
        if ckpt is not None:
            ckpt.maybe_save(len(trees), trees, base, F, params, force=len(trees) == params.n_estimators)
        maybe_fail(t, model="gbdt")
    if pending is not None:
        trees.append(pending.result().compacted())
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
        from .grower import dp_runner_stats

        dp_runner_stats()             # (the runner's own RCCL calls into parallel.dist.CALLS)
    return GBDTResult(trees, F, base, params, history, time.perf_counter() - t0,
                      {"Fa": Q.Fa, "TB": Q.TB, "nnz": int(Q.csc_row.numel()),
                       "hot": int(Q.hot.size) if Q.hot is not None else 0,
                       "groups": int(Q._rowgroups.G) if getattr(Q, "_rowgroups", None) is not None else 0,
                       "sparse_frac": _sparse_frac(getattr(Q, "_rowgroups", None))})


def _sparse_frac(rg) -> float:
    """Fraction of the row-group entries that carry an entry-major row (utils/memory.py)."""
    if rg is None or rg.erow is None or not rg.entries:
        return 0.0
    return float(rg.group_entries[rg.em_g0:].sum()) / float(rg.entries)


def train_margin_logloss(margin: torch.Tensor, y: torch.Tensor) -> float:
    p = torch.sigmoid(margin)
    eps = 1e-15
    return float(-(y * torch.log(p + eps) + (1 - y) * torch.log(1 - p + eps)).mean())


def smoke_round(res, labels, device) -> None:
    """One boosting round on a featurized batch (used by ``__graft_entry__.smoke``)."""
    from ..ml.linalg import VectorColumn

    indptr, idx, val = res.csr()
    vc = VectorColumn(res.dim, indptr, idx, val.to(torch.float64))
    out = fit_gbdt(vc, labels, GBDTParams(n_estimators=1, max_depth=3), device=device)
    assert len(out.trees) == 1 and out.trees[0].num_nodes >= 1
