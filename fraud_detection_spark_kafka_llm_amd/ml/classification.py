"""Classifiers: LogisticRegression, DecisionTreeClassifier, RandomForestClassifier (+ models).

Models score through the native engine: either fused with the text featurizer
(``ml.fused``; one gfx950 launch from raw bytes to scores) or over an existing feature column
(``ops.sparse.score_csr``). Output columns follow Spark's ProbabilisticClassificationModel:
``rawPrediction`` [N,2], ``probability`` [N,2], ``prediction`` [N] (float64).

Reference: classifiers built at /root/reference/fraud_detection_spark.py:59-83; the shipped
LogisticRegressionModel stage (dialogue_classification_model/stages/4_LogisticRegression_*).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..io import spark_format as sf
from ..ops.text import LinearScorer, TreeArrays
from .base import Estimator, Model, Param, register
from .frame import Frame
from .linalg import DenseVector, VectorColumn
from .tree_model import NODE_FIELDS, Tree, ensemble_arrays, feature_importances


class _PredictorParams:
    _params = [Param("featuresCol", "features column name", "features", str),
               Param("labelCol", "label column name", "label", str),
               Param("predictionCol", "prediction column name", "prediction", str),
               Param("rawPredictionCol", "raw prediction column name", "rawPrediction", str),
               Param("probabilityCol", "probability column name", "probability", str)]


class ClassificationModelBase(_PredictorParams, Model):
    """Common scoring glue. Subclasses provide ``scorer()`` and ``postprocess(raw)``."""

    numClasses = 2

    def scorer(self):
        raise NotImplementedError

    @property
    def numFeatures(self) -> int:  # noqa: N802
        raise NotImplementedError

    def postprocess(self, raw: torch.Tensor):
        """raw kernel output [N, K] fp64 -> (rawPrediction [N,2], probability [N,2], prediction [N])."""
        raise NotImplementedError

    def postprocess_numpy(self, raw: np.ndarray):
        """Streaming hot path: raw [N, K] fp64 numpy -> (prediction [N], P(class 1) [N])."""
        _, prob, pred = self.postprocess(torch.from_numpy(raw))
        return pred.numpy(), prob[:, 1].numpy()

    def _transform(self, frame: Frame) -> Frame:
        from ..ops.sparse import score_csr

        vc = frame.column(self.getFeaturesCol())
        if not isinstance(vc, VectorColumn):
            vc = VectorColumn.from_rows(list(vc))
        if vc.size < self.numFeatures:
            raise ValueError(f"features have size {vc.size}, model expects {self.numFeatures}")
        raw = score_csr(vc, self.scorer())
        return self.attach_outputs(frame, raw)

    def attach_outputs(self, frame: Frame, raw: torch.Tensor) -> Frame:
        rp, prob, pred = self.postprocess(raw)
        if self.getRawPredictionCol():
            frame = frame.withColumn(self.getRawPredictionCol(), rp)
        if self.getProbabilityCol():
            frame = frame.withColumn(self.getProbabilityCol(), prob)
        return frame.withColumn(self.getPredictionCol(), pred)

    def predict(self, features) -> float:
        vc = VectorColumn.from_rows([features], size=self.numFeatures)
        from ..ops.sparse import score_csr

        return float(self.postprocess(score_csr(vc, self.scorer()))[2][0])

    def predictProbability(self, features) -> DenseVector:  # noqa: N802
        vc = VectorColumn.from_rows([features], size=self.numFeatures)
        from ..ops.sparse import score_csr

        return DenseVector(self.postprocess(score_csr(vc, self.scorer()))[1][0].cpu().numpy())


def _argmax_prediction(prob: torch.Tensor) -> torch.Tensor:
    return torch.argmax(prob, dim=1).to(torch.float64)   # first max index on ties (Vector.argmax)


def _normalize(raw: torch.Tensor) -> torch.Tensor:
    s = raw.sum(1, keepdim=True)
    return torch.where(s != 0, raw / torch.where(s != 0, s, torch.ones_like(s)), raw)


# ============================================================================ logistic regression
class _LRParams(_PredictorParams):
    _params = [Param("family", "binomial|multinomial|auto", "auto", str),
               Param("fitIntercept", "fit an intercept", True, bool),
               Param("tol", "convergence tolerance", 1e-6, float),
               Param("standardization", "standardize features", True, bool),
               Param("maxIter", "max iterations", 100, int),
               Param("maxBlockSizeInMB", "block size", 0.0, float),
               Param("aggregationDepth", "treeAggregate depth", 2, int),
               Param("elasticNetParam", "L1 ratio", 0.0, float),
               Param("threshold", "binary threshold", 0.5, float),
               Param("regParam", "regularization", 0.0, float),
               Param("weightCol", "weight column", None, str, has_default=False)]

    _DEFAULT_ORDER = ("family", "predictionCol", "fitIntercept", "tol", "featuresCol", "standardization",
                      "maxIter", "maxBlockSizeInMB", "rawPredictionCol", "labelCol", "probabilityCol",
                      "aggregationDepth", "elasticNetParam", "threshold", "regParam")

    def _default_hook(self) -> None:
        d = self._defaultParamMap
        self._defaultParamMap = {k: d[k] for k in self._DEFAULT_ORDER if k in d}


@register("org.apache.spark.ml.classification.LogisticRegression")
class LogisticRegression(_LRParams, Estimator):
    _uid_prefix = "LogisticRegression"

    def _fit(self, frame: Frame) -> "LogisticRegressionModel":
        from ..models.lr import train_logistic_regression

        vc = frame.column(self.getFeaturesCol())
        y = frame.column(self.getLabelCol())
        w = frame.column(self.getWeightCol()) if self.isSet("weightCol") else None
        coef, intercept, history = train_logistic_regression(
            vc, y, weights=w, max_iter=self.getMaxIter(), tol=self.getTol(), reg_param=self.getRegParam(),
            elastic_net=self.getElasticNetParam(), fit_intercept=self.getFitIntercept(),
            standardization=self.getStandardization())
        m = LogisticRegressionModel(coef, intercept, uid=self.uid)
        m._paramMap.update(self._paramMap)
        m.objectiveHistory = history
        return m


@register("org.apache.spark.ml.classification.LogisticRegressionModel")
class LogisticRegressionModel(_LRParams, ClassificationModelBase):
    _uid_prefix = "LogisticRegression"

    def __init__(self, coefficients=None, intercept: float = 0.0, **kw):
        super().__init__(**kw)
        self.coefficients = np.asarray(coefficients if coefficients is not None else [], dtype=np.float64)
        self.intercept = float(intercept)
        self.objectiveHistory: list = []
        self._scorer = None

    @property
    def numFeatures(self) -> int:  # noqa: N802
        return int(self.coefficients.size)

    def scorer(self) -> LinearScorer:
        if self._scorer is None:
            self._scorer = LinearScorer(self.coefficients, self.intercept)
        return self._scorer

    def postprocess(self, raw: torch.Tensor):
        m = raw[:, 0]
        rp = torch.stack([-m, m], dim=1)
        prob = 1.0 / (1.0 + torch.exp(-rp))           # Spark raw2probability on [-m, m]
        pred = (prob[:, 1] > self.getThreshold()).to(torch.float64)
        return rp, prob, pred

    def postprocess_numpy(self, raw: np.ndarray):
        p = np.exp(-raw[:, 0])
        np.add(p, 1.0, out=p)
        np.reciprocal(p, out=p)
        return (p > self.getThreshold()).astype(np.float64), p

    def _metadata_extra(self):
        return None

    def _save_data(self, path) -> None:
        sf.write_data_parquet(path, [
            sf.Field.simple("numClasses", "integer"), sf.Field.simple("numFeatures", "integer"),
            sf.Field.vector("interceptVector"), sf.Field.matrix("coefficientMatrix"),
            sf.Field.simple("isMultinomial", "boolean")],
            [{"numClasses": 2, "numFeatures": self.numFeatures, "interceptVector": sf.dense_vector([self.intercept]),
              "coefficientMatrix": sf.sparse_matrix_row_major(self.coefficients[None, :]), "isMultinomial": False}])

    def _load_data(self, path, md) -> None:
        row = sf.read_data_parquet(path).to_pylist()[0]
        if row.get("isMultinomial"):
            raise NotImplementedError("multinomial logistic regression models are not supported")
        coef = sf.decode_matrix(row["coefficientMatrix"])
        self.coefficients = coef[0].astype(np.float64)
        self.intercept = float(sf.decode_vector(row["interceptVector"])[0])
        self.objectiveHistory = []
        self._scorer = None


# ============================================================================ trees
class _TreeParams(_PredictorParams):
    _params = [Param("maxDepth", "max tree depth", 5, int),
               Param("maxBins", "max bins for continuous features", 32, int),
               Param("minInstancesPerNode", "min rows per child", 1, int),
               Param("minWeightFractionPerNode", "min weight fraction per child", 0.0, float),
               Param("minInfoGain", "min info gain to split", 0.0, float),
               Param("maxMemoryInMB", "histogram memory budget", 256, int),
               Param("cacheNodeIds", "cache node ids", False, bool),
               Param("checkpointInterval", "checkpoint interval", 10, int),
               Param("impurity", "gini|entropy", "gini", str),
               Param("seed", "random seed", None, int, has_default=False),
               Param("leafCol", "leaf index column", "", str),
               Param("weightCol", "weight column", None, str, has_default=False)]

    def _default_hook(self) -> None:
        # Spark: seed default = hash of the class name
        self._defaultParamMap.setdefault("seed", _java_string_hash(type(self).__name__.replace("Model", "")))


def _java_string_hash(s: str) -> int:
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


class TreeClassificationModelBase(ClassificationModelBase):
    leaf_payload = "counts"

    def __init__(self, trees=None, num_features: int = 0, tree_weights=None, **kw):
        super().__init__(**kw)
        self._trees = list(trees or [])
        self._num_features = int(num_features)
        self._tree_weights = np.asarray(tree_weights if tree_weights is not None else np.ones(len(self._trees)))
        self._arrays: Optional[TreeArrays] = None

    @property
    def numFeatures(self) -> int:  # noqa: N802
        return self._num_features

    @property
    def trees(self) -> list:
        return self._trees

    def scorer(self) -> TreeArrays:
        if self._arrays is None:
            self._arrays = ensemble_arrays(self._trees, self.leaf_payload, None, cmp_less=False)
        return self._arrays

    def postprocess(self, raw: torch.Tensor):
        prob = _normalize(raw)
        return raw, prob, _argmax_prediction(prob)

    @property
    def featureImportances(self):  # noqa: N802
        from .linalg import SparseVector

        imp = feature_importances(self._trees, self._num_features)
        nz = np.nonzero(imp)[0]
        return SparseVector(self._num_features, nz, imp[nz])

    def _metadata_extra(self):
        return {"numFeatures": self._num_features, "numClasses": 2}


@register("org.apache.spark.ml.classification.DecisionTreeClassifier")
class DecisionTreeClassifier(_TreeParams, Estimator):
    _uid_prefix = "DecisionTreeClassifier"

    def _fit(self, frame: Frame):
        from ..models.tree import fit_forest

        res = fit_forest(frame.column(self.getFeaturesCol()), frame.column(self.getLabelCol()),
                         num_trees=1, max_depth=self.getMaxDepth(), max_bins=self.getMaxBins(),
                         min_instances=self.getMinInstancesPerNode(), min_info_gain=self.getMinInfoGain(),
                         bootstrap=False, feature_subset="all", seed=self.getSeed(), impurity=self.getImpurity())
        m = DecisionTreeClassificationModel(res.trees, res.num_features, uid=self.uid)
        m._paramMap.update(self._paramMap)
        return m


@register("org.apache.spark.ml.classification.DecisionTreeClassificationModel")
class DecisionTreeClassificationModel(_TreeParams, TreeClassificationModelBase):
    _uid_prefix = "DecisionTreeClassifier"
    leaf_payload = "counts"

    @property
    def depth(self) -> int:
        return self._trees[0].depth() if self._trees else 0

    @property
    def numNodes(self) -> int:  # noqa: N802
        return self._trees[0].compacted().num_nodes if self._trees else 0

    def _save_data(self, path) -> None:
        sf.write_data_parquet(path, NODE_FIELDS, self._trees[0].to_node_rows())

    def _load_data(self, path, md) -> None:
        rows = sf.read_data_parquet(path).to_pylist()
        self._trees = [Tree.from_node_rows(rows)]
        self._num_features = int(md.get("numFeatures", 0))
        self._tree_weights = np.ones(1)
        self._arrays = None


class _RFParams(_TreeParams):
    _params = [Param("numTrees", "number of trees", 20, int),
               Param("featureSubsetStrategy", "features per node", "auto", str),
               Param("subsamplingRate", "row subsampling rate", 1.0, float),
               Param("bootstrap", "bootstrap rows", True, bool)]


@register("org.apache.spark.ml.classification.RandomForestClassifier")
class RandomForestClassifier(_RFParams, Estimator):
    """``numWorkers`` (extension, not a Spark param): data-parallel rank processes for ``fit``
    (parallel/estimator_dp.py); never persisted, so saved stages stay loadable by Spark."""
    _uid_prefix = "RandomForestClassifier"
    _params = [Param("numWorkers", "data-parallel rank processes (extension)", 1, int)]
    _persist_defaults_only = ("numWorkers",)

    def _fit(self, frame: Frame):
        from ..models.tree import fit_forest
        from ..parallel import dist as D

        n = self.getNumTrees()
        kw = dict(num_trees=n, max_depth=self.getMaxDepth(), max_bins=self.getMaxBins(),
                  min_instances=self.getMinInstancesPerNode(), min_info_gain=self.getMinInfoGain(),
                  bootstrap=bool(self.getBootstrap()) and n > 1, feature_subset=self.getFeatureSubsetStrategy(),
                  seed=self.getSeed(), impurity=self.getImpurity(), subsampling_rate=self.getSubsamplingRate())
        X, y = frame.column(self.getFeaturesCol()), frame.column(self.getLabelCol())
        from ..parallel.estimator_dp import effective_workers

        from ..utils.config import default_device

        dev = default_device()
        nw = effective_workers(self.getOrDefault("numWorkers"), len(X), dev, nnz=X.nnz, kind="rf")
        if nw > 1 and not D.is_dist():
            from ..parallel.estimator_dp import fit_data_parallel

            (trees, nf), self.last_dp_report = fit_data_parallel("rf", X, y, None, kw, nw, device=dev)
        else:
            res = fit_forest(X, y, device=dev, **kw)
            trees, nf = res.trees, res.num_features
        m = RandomForestClassificationModel(trees, nf, uid=self.uid)
        m._paramMap.update({k: v for k, v in self._paramMap.items() if k != "numWorkers"})
        return m


@register("org.apache.spark.ml.classification.RandomForestClassificationModel")
class RandomForestClassificationModel(_RFParams, TreeClassificationModelBase):
    _uid_prefix = "RandomForestClassifier"
    leaf_payload = "normalized"

    @property
    def treeWeights(self) -> list:  # noqa: N802
        return [float(w) for w in self._tree_weights]

    def _metadata_extra(self):
        return {"numFeatures": self._num_features, "numClasses": 2, "numTrees": len(self._trees)}

    def _save_data(self, path) -> None:
        rows = []
        for t, tree in enumerate(self._trees):
            for r in tree.to_node_rows():
                rows.append({"treeID": t, "nodeData": r})
        sf.write_data_parquet(path, [sf.Field.simple("treeID", "integer"),
                                     sf.Field.struct("nodeData", NODE_FIELDS)], rows)
        params_json = sf.spark_json_dumps({"class": "org.apache.spark.ml.classification.DecisionTreeClassificationModel"})
        meta_rows = [{"treeID": t, "metadata": params_json, "weights": float(w)}
                     for t, w in enumerate(self._tree_weights)]
        sf.write_data_parquet(path, [sf.Field.simple("treeID", "integer"), sf.Field.simple("metadata", "string", True),
                                     sf.Field.simple("weights", "double")], meta_rows, subdir="treesMetadata")

    def _load_data(self, path, md) -> None:
        rows = sf.read_data_parquet(path).to_pylist()
        by_tree: dict = {}
        for r in rows:
            by_tree.setdefault(r["treeID"], []).append(r["nodeData"])
        self._trees = [Tree.from_node_rows(by_tree[k]) for k in sorted(by_tree)]
        try:
            meta = sf.read_data_parquet(path, "treesMetadata").to_pylist()
            w = {r["treeID"]: r["weights"] for r in meta}
            self._tree_weights = np.asarray([w.get(k, 1.0) for k in sorted(by_tree)])
        except FileNotFoundError:
            self._tree_weights = np.ones(len(self._trees))
        self._num_features = int(md.get("numFeatures", 0))
        self._arrays = None
