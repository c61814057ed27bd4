"""Fusion of a text pipeline's stages into one native launch.

``Tokenizer -> [StopWordsRemover] -> HashingTF|CountVectorizerModel -> [IDFModel] -> [classifier]``
(the shape of both the shipped ``dialogue_classification_model`` and the trainer's pipelines,
/root/reference/fraud_detection_spark.py:47-91) runs as ONE ``featurize_score`` call: raw UTF-8
bytes in, fp64 scores out. Intermediate columns (``words``, ``filtered_words``,
``raw_features``, ``features``) are attached lazily and only computed if read.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from ..ops.text import FeatureSpec, PackedText, featurize_score
from ..utils.config import default_device
from .classification import ClassificationModelBase
from .feature import CountVectorizerModel, HashingTF, IDFModel, StopWordsRemover, Tokenizer, native_vectors
from .frame import Frame, Lazy, TextColumn, TokenColumn
from .linalg import VectorColumn


class FusedPipeline:
    """Compiled text->score chain. ``predict`` returns (prediction, probability, rawPrediction)."""

    def __init__(self, tokenizer: Tokenizer, remover: Optional[StopWordsRemover], tf, idf: Optional[IDFModel],
                 model: Optional[ClassificationModelBase], device=None):
        self.tokenizer, self.remover, self.tf, self.idf, self.model = tokenizer, remover, tf, idf, model
        self.device = torch.device(device) if device is not None else default_device()
        kw = tf.spec_kwargs()
        self.stopwords = tuple(remover.getStopWords()) if remover is not None else None
        self._spec_raw = FeatureSpec(clean=False, stopwords=self.stopwords, **kw)
        self._spec_clean = FeatureSpec(clean=True, stopwords=self.stopwords, **kw)
        self.dim = self._spec_raw.dim
        if idf is not None and idf.idf.size < self.dim:
            raise ValueError("IDF vector is shorter than the TF feature space")
        if model is not None and model.numFeatures > self.dim:
            raise ValueError("classifier expects more features than the TF stage produces")
        self._idf_t = idf.idf_tensor(self.device) if idf is not None else None
        self._scorer = model.scorer() if model is not None else None

    @classmethod
    def from_stages(cls, stages: Sequence, device=None) -> "FusedPipeline":
        chain = match_chain(stages)
        if chain is None or chain[-1] != len(stages):
            raise ValueError("pipeline is not a fusable text->classifier chain")
        return cls(*chain[:5], device=device)

    def spec(self, clean: bool) -> FeatureSpec:
        return self._spec_clean if clean else self._spec_raw

    def run(self, texts, clean: bool = True, want_csr: bool = False, device=None):
        """Featurize + score. ``clean=True`` applies the reference's preprocess_text cleaning
        (agent_api.py:139-145) inside the kernel."""
        dev = torch.device(device) if device is not None else self.device
        packed = texts if isinstance(texts, PackedText) else PackedText.from_strings(list(texts))
        from .classification import LogisticRegressionModel
        from ..ops.text import LinearScorer

        lr = self._scorer if isinstance(self._scorer, LinearScorer) else None
        trees = None if lr is not None or self._scorer is None else self._scorer
        if lr is not None and lr.w.size < self.dim:
            import numpy as np

            lr = LinearScorer(np.concatenate([lr.w, np.zeros(self.dim - lr.w.size)]), lr.b)
            self._scorer = lr
        idf = self.idf.idf_tensor(dev) if self.idf is not None else None
        return featurize_score(packed, self.spec(clean), idf=idf, lr=lr, trees=trees, want_csr=want_csr, device=dev)

    def predict(self, texts, clean: bool = True, device=None):
        if self.model is None:
            raise ValueError("pipeline has no classifier stage")
        res = self.run(texts, clean=clean, device=device)
        rp, prob, pred = self.model.postprocess(res.raw)
        return pred, prob, rp


def match_chain(stages: Sequence):
    """Return (tokenizer, remover, tf, idf, model, n_stages_covered) or None."""
    if not stages or not isinstance(stages[0], Tokenizer):
        return None
    i = 1
    cur = stages[0].getOutputCol()
    remover = None
    if i < len(stages) and isinstance(stages[i], StopWordsRemover):
        r = stages[i]
        if r.getInputCol() != cur or r.getCaseSensitive():
            return None
        remover, cur, i = r, r.getOutputCol(), i + 1
    if i >= len(stages) or not isinstance(stages[i], (HashingTF, CountVectorizerModel)):
        return None
    tf = stages[i]
    if tf.getInputCol() != cur:
        return None
    cur, i = tf.getOutputCol(), i + 1
    idf = None
    if i < len(stages) and isinstance(stages[i], IDFModel) and stages[i].getInputCol() == cur:
        idf, cur, i = stages[i], stages[i].getOutputCol(), i + 1
    model = None
    if i < len(stages) and isinstance(stages[i], ClassificationModelBase) and stages[i].getFeaturesCol() == cur:
        model, i = stages[i], i + 1
    return tokenizer_tuple(stages[0], remover, tf, idf, model, i)


def tokenizer_tuple(*a):
    return a


class _Plan:
    def __init__(self, chain, frame: Frame):
        self.tok, self.rem, self.tf, self.idf, self.model, self.n = chain

    def run(self, frame: Frame, rest: Sequence = ()) -> Frame:
        tok, rem, tf, idf, model = self.tok, self.rem, self.tf, self.idf, self.model
        src = frame.column(tok.getInputCol())
        text = src if isinstance(src, TextColumn) else TextColumn([None if s is None else str(s) for s in src])
        raw, clean = text.lineage()
        n = len(frame)
        words = TokenColumn(text)
        frame = frame.withColumn(tok.getOutputCol(), words)
        tokens = words
        if rem is not None:
            tokens = TokenColumn(text, tuple(rem.getStopWords()))
            frame = frame.withColumn(rem.getOutputCol(), tokens)
        tf_col = Lazy(lambda: native_vectors(tokens, tf.spec_kwargs()), n)
        frame = frame.withColumn(tf.getOutputCol(), tf_col)
        if idf is not None:
            def _idf():
                vc = tf_col.get()
                ip, ix, v = vc.csr()
                w = idf.idf_tensor(v.device)
                return VectorColumn.scaled_counts(vc.size, ip, ix, v, w)
            frame = frame.withColumn(idf.getOutputCol(), Lazy(_idf, n))
        if model is not None:
            fp = FusedPipeline(tok, rem, tf, idf, model)
            res = fp.run(raw.packed(), clean=clean)
            frame = model.attach_outputs(frame, res.raw)
        for s in rest:
            frame = s.transform(frame)
        return frame


class _PlanWithRest:
    def __init__(self, plan: _Plan, rest):
        self.plan, self.rest = plan, rest

    def run(self, frame: Frame) -> Frame:
        return self.plan.run(frame, self.rest)


def plan_pipeline(stages: Sequence, frame: Frame):
    chain = match_chain(stages)
    if chain is None:
        return None
    src = frame.raw_column(stages[0].getInputCol()) if stages[0].getInputCol() in frame else None
    if src is None:
        return None
    return _PlanWithRest(_Plan(chain, frame), list(stages[chain[-1]:]))
