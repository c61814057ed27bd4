"""``xgboost.spark.SparkXGBClassifier``-compatible estimator on the gfx950 GBDT engine (R-06, X-13).

Same constructor surface the reference uses (``features_col, label_col, num_workers, max_depth,
n_estimators, eval_metric``; /root/reference/fraud_detection_spark.py:76-83) plus the usual XGBoost
knobs. ``num_workers`` maps to data-parallel ranks: inside a ``torch.distributed`` job each rank
trains on its row shard and histograms are reduce-scattered over RCCL (the reference's Rabit
ring); from a single process ``num_workers > 1`` launches that many rank processes
(parallel/estimator_dp.py) and returns rank 0's model (identical on every rank).

Outputs follow xgboost.spark: ``rawPrediction = [-margin, margin]``, ``probability = [1-p, p]``,
``prediction = p > 0.5``. Models persist in the Spark ML layout (metadata + ``data/`` trees) and
export XGBoost JSON (``save_xgboost_json``; loadable by ``xgboost.Booster.load_model``).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from ..io import spark_format as sf
from ..ops.text import TreeArrays
from .base import Estimator, Param, register
from .classification import ClassificationModelBase
from .frame import Frame
from .tree_model import NODE_FIELDS, Tree, ensemble_arrays


class _XGBParams:
    _params = [Param("features_col", "features column", "features", str),
               Param("label_col", "label column", "label", str),
               Param("prediction_col", "prediction column", "prediction", str),
               Param("probability_col", "probability column", "probability", str),
               Param("raw_prediction_col", "raw prediction column", "rawPrediction", str),
               Param("weight_col", "weight column", None, str, has_default=False),
               Param("num_workers", "data-parallel workers", 1, int),
               Param("max_depth", "max tree depth", 6, int),
               Param("n_estimators", "boosting rounds", 100, int),
               Param("learning_rate", "eta", 0.3, float),
               Param("reg_lambda", "L2 regularisation", 1.0, float),
               Param("gamma", "min split loss", 0.0, float),
               Param("min_child_weight", "min hessian per child", 1.0, float),
               Param("max_bin", "histogram bins per feature", 256, int),
               Param("max_delta_step", "max leaf step", 0.0, float),
               Param("base_score", "initial prediction (None = estimated)", None, float, has_default=False),
               Param("eval_metric", "evaluation metric", "auc", str),
               Param("objective", "objective", "binary:logistic", str),
               Param("tree_method", "tree method", "hist", str),
               Param("seed", "random seed", 0, int),
               Param("deterministic", "accepted for compatibility: training is always bitwise reproducible", True,
                     bool)]

    # ClassificationModelBase reads Spark-style column getters
    def getFeaturesCol(self):  # noqa: N802
        return self.getOrDefault("features_col")

    def getLabelCol(self):  # noqa: N802
        return self.getOrDefault("label_col")

    def getPredictionCol(self):  # noqa: N802
        return self.getOrDefault("prediction_col")

    def getProbabilityCol(self):  # noqa: N802
        return self.getOrDefault("probability_col")

    def getRawPredictionCol(self):  # noqa: N802
        return self.getOrDefault("raw_prediction_col")


@register("xgboost.spark.core.SparkXGBClassifier")
class SparkXGBClassifier(_XGBParams, Estimator):
    _uid_prefix = "SparkXGBClassifier"

    def __init__(self, **kw):
        kw = {("learning_rate" if k == "eta" else k): v for k, v in kw.items()}
        super().__init__(**kw)

    def _fit(self, frame: Frame) -> "SparkXGBClassifierModel":
        from ..models.gbdt import GBDTParams, fit_gbdt

        if self.getOrDefault("objective") != "binary:logistic":
            raise NotImplementedError("only objective='binary:logistic' is supported")
        p = GBDTParams(n_estimators=self.getOrDefault("n_estimators"), max_depth=self.getOrDefault("max_depth"),
                       learning_rate=self.getOrDefault("learning_rate"), reg_lambda=self.getOrDefault("reg_lambda"),
                       gamma=self.getOrDefault("gamma"), min_child_weight=self.getOrDefault("min_child_weight"),
                       max_bin=self.getOrDefault("max_bin"), max_delta_step=self.getOrDefault("max_delta_step"),
                       base_score=self._paramMap.get("base_score"), seed=self.getOrDefault("seed"),
                       deterministic=bool(self.getOrDefault("deterministic")))
        w = frame.column(self.getOrDefault("weight_col")) if self.isSet("weight_col") else None
        X, y = frame.column(self.getFeaturesCol()), frame.column(self.getLabelCol())
        from ..parallel import dist as D
        from ..parallel.estimator_dp import effective_workers

        from ..utils.config import default_device

        dev = default_device()
        nw = effective_workers(self.getOrDefault("num_workers"), len(X), dev, nnz=X.nnz)
        if nw > 1 and not D.is_dist():
            # N rank processes (one per GPU over RCCL, else gloo CPU ranks) behind the watchdog
            from dataclasses import asdict

            from ..parallel.estimator_dp import fit_data_parallel

            (trees, nf, base, secs), self.last_dp_report = fit_data_parallel("gbdt", X, y, w, asdict(p), nw, device=dev)
        else:          # one process, or already one rank of a torchrun job
            res = fit_gbdt(X, y, p, weights=w, device=dev)
            trees, nf, base, secs = res.trees, res.num_features, res.base_margin, res.train_seconds
        m = SparkXGBClassifierModel(trees, nf, base, uid=self.uid)
        m._paramMap.update(self._paramMap)
        m.training_seconds = secs
        return m


@register("xgboost.spark.core.SparkXGBClassifierModel")
class SparkXGBClassifierModel(_XGBParams, ClassificationModelBase):
    _uid_prefix = "SparkXGBClassifierModel"

    def __init__(self, trees=None, num_features: int = 0, base_margin: float = 0.0, **kw):
        super().__init__(**kw)
        self._trees = list(trees or [])
        self._num_features = int(num_features)
        self.base_margin = float(base_margin)
        self._arrays: Optional[TreeArrays] = None
        self.training_seconds = 0.0

    @property
    def numFeatures(self) -> int:  # noqa: N802
        return self._num_features

    @property
    def trees(self) -> list:
        return self._trees

    def scorer(self) -> TreeArrays:
        if self._arrays is None:
            # thresholds are midpoints between bin values: "<" and "<=" agree on all seen values;
            # keep XGBoost's "x < split_condition" semantics
            self._arrays = ensemble_arrays(self._trees, "value", None, cmp_less=True)
        return self._arrays

    def postprocess(self, raw: torch.Tensor):
        m = raw[:, 0] + self.base_margin
        rp = torch.stack([-m, m], dim=1)
        p = torch.sigmoid(m)
        prob = torch.stack([1.0 - p, p], dim=1)
        return rp, prob, (p > 0.5).to(torch.float64)

    def postprocess_numpy(self, raw: np.ndarray):
        m = raw[:, 0] + self.base_margin
        p = np.exp(-m)
        np.add(p, 1.0, out=p)
        np.reciprocal(p, out=p)
        return (m > 0.0).astype(np.float64), p

    def get_booster(self):
        return self

    @property
    def featureImportances(self):  # noqa: N802
        """XGBoost ``total_gain`` importance, normalised (used by word-association analysis)."""
        from .linalg import SparseVector

        imp = np.zeros(self._num_features)
        for t in self._trees:
            for i in range(t.num_nodes):
                if t.feature[i] >= 0:
                    imp[t.feature[i]] += t.gain[i]
        s = imp.sum()
        if s > 0:
            imp /= s
        nz = np.nonzero(imp)[0]
        return SparseVector(self._num_features, nz, imp[nz])

    # ------------------------------------------------------------ persistence
    def _metadata_extra(self):
        return {"numFeatures": self._num_features, "numClasses": 2, "numTrees": len(self._trees),
                "baseMargin": self.base_margin}

    def _save_data(self, path) -> None:
        """xgboost.spark's writer layout: ``metadata/`` (Spark DefaultParamsWriter JSON, written by
        the base class) and ``model/part-00000`` — the booster JSON as a one-line text part, what
        ``SparkXGBModelWriter`` writes with ``saveAsTextFile``. The fp64 split thresholds and node
        statistics of this engine ride in ``learner.attributes["fdx_trees"]`` (XGBoost keeps
        string attributes and ignores unknown ones) so a reload scores bitwise identically."""
        d = Path(path) / "model"
        d.mkdir(parents=True, exist_ok=True)
        booster = self.to_xgboost_json()
        booster["learner"]["attributes"]["fdx_trees"] = json.dumps([t.to_node_rows() for t in self._trees])
        booster["learner"]["attributes"]["fdx_base_margin"] = repr(self.base_margin)
        (d / "part-00000").write_text(json.dumps(booster) + "\n")
        (d / "_SUCCESS").write_text("")

    def _load_data(self, path, md) -> None:
        """Reads the xgboost.spark layout (``model/`` text part), and the earlier layout of this
        package (``data/`` parquet node rows)."""
        part = Path(path) / "model" / "part-00000"
        if part.exists():
            booster = json.loads(part.read_text().splitlines()[0])
            attrs = booster["learner"].get("attributes", {})
            if "fdx_trees" in attrs:
                self._trees = [Tree.from_node_rows(rows) for rows in json.loads(attrs["fdx_trees"])]
                self.base_margin = float(attrs["fdx_base_margin"])
                self._num_features = int(booster["learner"]["learner_model_param"]["num_feature"])
            else:                                   # a booster written by xgboost itself
                other = SparkXGBClassifierModel.from_xgboost_json(booster)
                self._trees, self._num_features, self.base_margin = other._trees, other._num_features, \
                    other.base_margin
        else:
            rows = sf.read_data_parquet(path).to_pylist()
            by_tree: dict = {}
            for r in rows:
                by_tree.setdefault(r["treeID"], []).append(r["nodeData"])
            self._trees = [Tree.from_node_rows(by_tree[k]) for k in sorted(by_tree)]
            self._num_features = int(md.get("numFeatures", 0))
            self.base_margin = float(md.get("baseMargin", 0.0))
        self._arrays = None
        self.training_seconds = 0.0

    def _save_data_legacy(self, path) -> None:
        """The round-1 layout (``data/`` parquet node rows + ``xgboost_model.json``), kept for tests
        of the backward-compatible reader."""
        rows = [{"treeID": t, "nodeData": r} for t, tree in enumerate(self._trees) for r in tree.to_node_rows()]
        sf.write_data_parquet(path, [sf.Field.simple("treeID", "integer"), sf.Field.struct("nodeData", NODE_FIELDS)],
                              rows)
        self.save_xgboost_json(Path(path) / "xgboost_model.json")

    def to_xgboost_json(self) -> dict:
        """XGBoost >= 1.6 JSON model (gbtree, binary:logistic). Split conditions are float32 in
        XGBoost; ours are fp64 midpoints, rounded here (exact for integer-count features)."""
        trees = []
        for tid, t in enumerate(self._trees):
            t = t.compacted()
            n = t.num_nodes
            leaf = t.feature < 0
            parents = np.full(n, 2147483647, dtype=np.int64)
            for i in range(n):
                if not leaf[i]:
                    parents[t.left[i]] = i
                    parents[t.right[i]] = i
            trees.append({
                "base_weights": [float(v) for v in np.where(leaf, t.stats[:, 0], 0.0)],
                "categories": [], "categories_nodes": [], "categories_segments": [], "categories_sizes": [],
                # rows absent from a sparse input carry value 0: route them like a stored 0
                "default_left": [int(leaf[i] or 0.0 < float(np.float32(t.threshold[i]))) for i in range(n)],
                "id": tid,
                "left_children": [int(v) for v in np.where(leaf, -1, t.left)],
                "right_children": [int(v) for v in np.where(leaf, -1, t.right)],
                "loss_changes": [float(v) if not leaf[i] else 0.0 for i, v in enumerate(t.gain)],
                "parents": [int(v) for v in parents],
                "split_conditions": [float(np.float32(t.threshold[i])) if not leaf[i] else float(t.stats[i, 0])
                                     for i in range(n)],
                "split_indices": [int(v) if v >= 0 else 0 for v in t.feature],
                "split_type": [0] * n,
                "sum_hessian": [float(v) for v in t.stats[:, 1]],
                "tree_param": {"num_deleted": "0", "num_feature": str(self._num_features), "num_nodes": str(n),
                               "size_leaf_vector": "1"},
            })
        base_p = 1.0 / (1.0 + np.exp(-self.base_margin))
        return {
            "learner": {
                "attributes": {},
                "feature_names": [], "feature_types": [],
                "gradient_booster": {"model": {"gbtree_model_param": {"num_parallel_tree": "1",
                                                                      "num_trees": str(len(trees))},
                                               "iteration_indptr": list(range(len(trees) + 1)),
                                               "tree_info": [0] * len(trees), "trees": trees},
                                     "name": "gbtree"},
                "learner_model_param": {"base_score": f"{base_p:.9E}", "boost_from_average": "1",
                                        "num_class": "0", "num_feature": str(self._num_features),
                                        "num_target": "1"},
                "objective": {"name": "binary:logistic", "reg_loss_param": {"scale_pos_weight": "1"}},
            },
            "version": [2, 0, 3],
        }

    def save_xgboost_json(self, path) -> None:
        Path(path).write_text(json.dumps(self.to_xgboost_json()))

    @classmethod
    def from_xgboost_json(cls, path_or_dict) -> "SparkXGBClassifierModel":
        d = path_or_dict if isinstance(path_or_dict, dict) else json.loads(Path(path_or_dict).read_text())
        L = d["learner"]
        nf = int(L["learner_model_param"]["num_feature"])
        bp = float(L["learner_model_param"]["base_score"])
        base = float(np.log(bp / (1 - bp)))
        trees = []
        for tj in L["gradient_booster"]["model"]["trees"]:
            lc = np.asarray(tj["left_children"])
            rc = np.asarray(tj["right_children"])
            leaf = lc < 0
            n = lc.size
            cond = np.asarray(tj["split_conditions"], dtype=np.float64)
            feat = np.where(leaf, -1, np.asarray(tj["split_indices"])).astype(np.int32)
            val = np.where(leaf, cond, 0.0)
            hess = np.asarray(tj.get("sum_hessian", [0.0] * n), dtype=np.float64)
            trees.append(Tree(feat, np.where(leaf, 0.0, cond), np.where(leaf, -1, lc).astype(np.int32),
                              np.where(leaf, -1, rc).astype(np.int32), np.stack([val, hess], 1), np.zeros(n),
                              np.asarray(tj["loss_changes"], dtype=np.float64), np.zeros(n, np.int64), val, 0))
        return cls(trees, nf, base)
