"""Evaluators: BinaryClassificationEvaluator, MulticlassClassificationEvaluator (X-14, X-15, K-18).

Semantics follow Spark 3.5 ``BinaryClassificationMetrics`` / ``MulticlassMetrics`` as called at
/root/reference/fraud_detection_spark.py:93-123:

* areaUnderROC — scores = rawPrediction[1]; distinct scores sorted descending with (pos, neg)
  weights; when #distinct / numBins >= 2 consecutive distinct scores are merged in groups of
  ``#distinct // numBins`` (default numBins = 1000, single partition); ROC = (0,0) + points + (1,1),
  trapezoidal area. areaUnderPR: PR curve starting at (0, precision of the first point).
* accuracy / weightedPrecision / weightedRecall / f1 (= weightedFMeasure, beta 1): per-label
  precision/recall weighted by true-label frequency; a label never predicted has precision 0.

Counting runs on the column's device (bincount = atomics for the confusion matrix, a device sort
for the ROC); only the tiny per-score table reaches the host.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .base import Param, Params
from .frame import Frame
from .linalg import VectorColumn


def _vec_col_to_tensor(col, which: Optional[int] = None) -> torch.Tensor:
    if isinstance(col, torch.Tensor):
        t = col
    elif isinstance(col, np.ndarray):
        t = torch.from_numpy(col)
    elif isinstance(col, VectorColumn):
        t = col.dense if col.dense is not None else torch.stack([torch.as_tensor(v.toArray()) for v in col.to_list()])
    else:
        vals = list(col)
        if vals and hasattr(vals[0], "toArray"):
            t = torch.as_tensor(np.stack([v.toArray() for v in vals]))
        else:
            t = torch.as_tensor(np.asarray([float(v) for v in vals]))
    t = t.to(torch.float64)
    if which is not None and t.dim() == 2:
        t = t[:, which]
    return t


def _labels(col) -> torch.Tensor:
    if isinstance(col, torch.Tensor):
        return col.to(torch.float64)
    if isinstance(col, np.ndarray):
        return torch.from_numpy(col.astype(np.float64))
    return torch.as_tensor([float(v) for v in col], dtype=torch.float64)


def binary_curve_points(scores: torch.Tensor, labels: torch.Tensor, weights: Optional[torch.Tensor] = None,
                        num_bins: int = 1000):
    """Cumulative (tp, fp) at each (binned) distinct score, descending."""
    dev = scores.device
    w = torch.ones_like(scores) if weights is None else weights.to(scores)
    uniq, inv = torch.unique(scores, sorted=True, return_inverse=True)
    pos = torch.zeros(uniq.numel(), dtype=torch.float64, device=dev).index_add_(0, inv, w * (labels > 0.5))
    neg = torch.zeros(uniq.numel(), dtype=torch.float64, device=dev).index_add_(0, inv, w * (labels <= 0.5))
    pos, neg = pos.flip(0), neg.flip(0)      # descending score
    n = uniq.numel()
    if num_bins > 0:
        grouping = n // num_bins
        if grouping >= 2:
            g = torch.arange(n, device=dev) // grouping
            ng = int(g[-1]) + 1
            pos = torch.zeros(ng, dtype=torch.float64, device=dev).index_add_(0, g, pos)
            neg = torch.zeros(ng, dtype=torch.float64, device=dev).index_add_(0, g, neg)
    return torch.cumsum(pos, 0), torch.cumsum(neg, 0)


def area_under_roc(scores, labels, weights=None, num_bins: int = 1000) -> float:
    tp, fp = binary_curve_points(scores, labels, weights, num_bins)
    P, N = float(tp[-1]), float(fp[-1])
    if P == 0 or N == 0:
        return float("nan") if (P == 0 and N == 0) else (1.0 if N == 0 else 0.0)
    x = torch.cat([torch.zeros(1, dtype=torch.float64, device=tp.device), fp / N,
                   torch.ones(1, dtype=torch.float64, device=tp.device)])
    y = torch.cat([torch.zeros(1, dtype=torch.float64, device=tp.device), tp / P,
                   torch.ones(1, dtype=torch.float64, device=tp.device)])
    return float(torch.sum((x[1:] - x[:-1]) * (y[1:] + y[:-1]) / 2.0))


def area_under_pr(scores, labels, weights=None, num_bins: int = 1000) -> float:
    tp, fp = binary_curve_points(scores, labels, weights, num_bins)
    P = float(tp[-1])
    if P == 0:
        return 0.0
    prec = tp / torch.clamp(tp + fp, min=1e-300)
    rec = tp / P
    x = torch.cat([torch.zeros(1, dtype=torch.float64, device=tp.device), rec])
    y = torch.cat([prec[:1], prec])
    return float(torch.sum((x[1:] - x[:-1]) * (y[1:] + y[:-1]) / 2.0))


class BinaryClassificationEvaluator(Params):
    _uid_prefix = "BinaryClassificationEvaluator"
    _java_class = "org.apache.spark.ml.evaluation.BinaryClassificationEvaluator"
    _params = [Param("metricName", "areaUnderROC|areaUnderPR", "areaUnderROC", str),
               Param("rawPredictionCol", "raw prediction column", "rawPrediction", str),
               Param("labelCol", "label column", "label", str),
               Param("weightCol", "weight column", None, str, has_default=False),
               Param("numBins", "curve down-sampling bins (0 = none)", 1000, int)]

    def evaluate(self, frame: Frame, params: Optional[dict] = None) -> float:
        ev = self.copy(params) if params else self
        col = frame.column(ev.getRawPredictionCol())
        s = _vec_col_to_tensor(col, 1)
        y = _labels(frame.column(ev.getLabelCol())).to(s.device)
        w = _labels(frame.column(ev.getWeightCol())).to(s.device) if ev.isSet("weightCol") else None
        if ev.getMetricName() == "areaUnderPR":
            return area_under_pr(s, y, w, ev.getNumBins())
        return area_under_roc(s, y, w, ev.getNumBins())

    def isLargerBetter(self) -> bool:  # noqa: N802
        return True


def confusion(labels: torch.Tensor, preds: torch.Tensor, weights: Optional[torch.Tensor] = None):
    """Weighted confusion matrix over the sorted union of label values (rows = actual)."""
    classes = torch.unique(torch.cat([labels, preds]), sorted=True)
    li = torch.searchsorted(classes, labels)
    pi = torch.searchsorted(classes, preds)
    k = classes.numel()
    w = torch.ones_like(labels) if weights is None else weights
    cm = torch.zeros(k * k, dtype=torch.float64, device=labels.device).index_add_(0, li * k + pi, w)
    return classes.cpu().numpy(), cm.view(k, k).cpu().numpy()


def multiclass_metrics(labels, preds, weights=None, beta: float = 1.0) -> dict:
    classes, cm = confusion(labels, preds, weights)
    total = cm.sum()
    label_count = cm.sum(1)
    pred_count = cm.sum(0)
    tp = np.diag(cm)
    present = label_count > 0
    prec = np.divide(tp, pred_count, out=np.zeros_like(tp), where=pred_count > 0)
    rec = np.divide(tp, label_count, out=np.zeros_like(tp), where=label_count > 0)
    fp = pred_count - tp
    neg = total - label_count
    fpr = np.divide(fp, neg, out=np.zeros_like(fp), where=neg > 0)
    b2 = beta * beta
    denom = b2 * prec + rec
    fm = np.divide((1 + b2) * prec * rec, denom, out=np.zeros_like(prec), where=denom > 0)
    frac = label_count / total if total > 0 else label_count
    w = lambda v: float(np.sum((v * frac)[present]))  # noqa: E731
    return {
        "classes": classes, "confusion": cm,
        "accuracy": float(tp.sum() / total) if total > 0 else 0.0,
        "weightedPrecision": w(prec), "weightedRecall": w(rec), "weightedTruePositiveRate": w(rec),
        "weightedFalsePositiveRate": w(fpr), "weightedFMeasure": w(fm), "f1": w(fm),
        "precisionByLabel": dict(zip(classes.tolist(), prec.tolist())),
        "recallByLabel": dict(zip(classes.tolist(), rec.tolist())),
        "fMeasureByLabel": dict(zip(classes.tolist(), fm.tolist())),
        "falsePositiveRateByLabel": dict(zip(classes.tolist(), fpr.tolist())),
        "hammingLoss": float(1.0 - tp.sum() / total) if total > 0 else 0.0,
    }


class MulticlassClassificationEvaluator(Params):
    _uid_prefix = "MulticlassClassificationEvaluator"
    _java_class = "org.apache.spark.ml.evaluation.MulticlassClassificationEvaluator"
    _params = [Param("metricName", "f1|accuracy|weightedPrecision|weightedRecall|...", "f1", str),
               Param("predictionCol", "prediction column", "prediction", str),
               Param("labelCol", "label column", "label", str),
               Param("probabilityCol", "probability column (logLoss)", "probability", str),
               Param("weightCol", "weight column", None, str, has_default=False),
               Param("metricLabel", "label for *ByLabel metrics", 0.0, float),
               Param("beta", "F-measure beta", 1.0, float),
               Param("eps", "logLoss clipping", 1e-15, float)]

    def evaluate(self, frame: Frame, params: Optional[dict] = None) -> float:
        ev = self.copy(params) if params else self
        name = ev.getMetricName()
        y = _labels(frame.column(ev.getLabelCol()))
        if name == "logLoss":
            prob = _vec_col_to_tensor(frame.column(ev.getProbabilityCol()))
            idx = y.to(prob.device).long()
            p = prob[torch.arange(prob.shape[0], device=prob.device), idx].clamp(ev.getEps(), 1 - ev.getEps())
            return float(-torch.log(p).mean())
        p = _labels(frame.column(ev.getPredictionCol())).to(y.device)
        w = _labels(frame.column(ev.getWeightCol())).to(y.device) if ev.isSet("weightCol") else None
        m = multiclass_metrics(y, p, w, ev.getBeta())
        if name.endswith("ByLabel"):
            base = {"truePositiveRateByLabel": "recallByLabel"}.get(name, name)
            return float(m[base].get(float(ev.getMetricLabel()), 0.0))
        if name == "weightedFMeasure":
            return m["weightedFMeasure"]
        return float(m[name])

    def isLargerBetter(self) -> bool:  # noqa: N802
        return self.getMetricName() not in ("weightedFalsePositiveRate", "falsePositiveRateByLabel", "hammingLoss",
                                            "logLoss")


def evaluate_all(frame: Frame, label_col: str = "labels") -> dict:
    """The reference's metric set (fraud_detection_spark.py:101-123) in one device pass."""
    y = _labels(frame.column(label_col))
    s = _vec_col_to_tensor(frame.column("rawPrediction"), 1).to(y.device)
    p = _labels(frame.column("prediction")).to(y.device)
    m = multiclass_metrics(y, p)
    return {"metrics": {"Accuracy": m["accuracy"], "Precision": m["weightedPrecision"],
                        "Recall": m["weightedRecall"], "F1": m["f1"], "AUC": area_under_roc(s, y)},
            "confusion_matrix": m["confusion"], "classes": m["classes"]}
