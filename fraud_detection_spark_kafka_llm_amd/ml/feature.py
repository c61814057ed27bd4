"""Feature stages: Tokenizer, StopWordsRemover, HashingTF, CountVectorizer(+Model), IDF(+Model).

Tokenizer/StopWordsRemover only record lineage (``TokenColumn``); HashingTF and CountVectorizerModel
consume it through the fused native featurizer (one gfx950 launch: clean -> split -> stop words ->
murmur3/vocab -> sparse vector), so token lists are never materialised on the hot path.
Reference usage: /root/reference/fraud_detection_spark.py:47-54 and shipped stages 0-3
(dialogue_classification_model/stages/{0_Tokenizer,1_StopWordsRemover,2_HashingTF,3_IDF}_*).
"""
from __future__ import annotations

from collections import Counter
from typing import Optional

import numpy as np
import torch

from ..io import spark_format as sf
from ..ops import oracle
from ..ops.text import FeatureSpec, featurize_score
from ..utils.config import default_device
from .base import Estimator, HasInOut, Model, Param, Transformer, register
from .frame import Frame, TextColumn, TokenColumn
from .linalg import VectorColumn
from .stopwords import load_default_stop_words


def _as_text(col) -> TextColumn:
    if isinstance(col, TextColumn):
        return col
    return TextColumn([None if c is None else str(c) for c in col])


def _tokens_of(col) -> list:
    if isinstance(col, TokenColumn):
        return col.tokens
    return [list(t) if t is not None else [] for t in col]


def native_vectors(col: TokenColumn, spec_kw: dict, device=None) -> VectorColumn:
    """Run the fused native featurizer over a fusable token lineage."""
    raw, clean = col.text.lineage()
    spec = FeatureSpec(clean=clean, stopwords=col.stopwords, **spec_kw)
    dev = torch.device(device) if device is not None else default_device()
    res = featurize_score(raw.packed(), spec, want_csr=True, device=dev)
    indptr, idx, val = res.csr()
    return VectorColumn(spec.dim, indptr, idx, val.to(torch.float64))


@register("org.apache.spark.ml.feature.Tokenizer")
class Tokenizer(HasInOut, Transformer):
    _uid_prefix = "Tokenizer"

    def _transform(self, frame: Frame) -> Frame:
        col = frame.column(self.getInputCol())
        return frame.withColumn(self.getOutputCol(), TokenColumn(_as_text(col)))


@register("org.apache.spark.ml.feature.StopWordsRemover")
class StopWordsRemover(HasInOut, Transformer):
    _uid_prefix = "StopWordsRemover"
    _params = [Param("caseSensitive", "case-sensitive comparison", False, bool),
               Param("locale", "locale for case-insensitive comparison", "en", str),
               Param("stopWords", "words to filter out", lambda: load_default_stop_words("english"), list)]

    @staticmethod
    def loadDefaultStopWords(language: str) -> list:  # noqa: N802
        return load_default_stop_words(language)

    def _default_hook(self) -> None:
        # Spark's JSON order: caseSensitive, locale, stopWords, outputCol
        out = f"{self.uid}__output"
        sw = self._defaultParamMap.pop("stopWords")
        self._defaultParamMap = {"caseSensitive": False, "locale": "en", "stopWords": sw, "outputCol": out}

    def _transform(self, frame: Frame) -> Frame:
        col = frame.column(self.getInputCol())
        sw = tuple(self.getStopWords())
        cs = bool(self.getCaseSensitive())
        if isinstance(col, TokenColumn) and col.fusable and col.stopwords is None and not cs:
            return frame.withColumn(self.getOutputCol(), TokenColumn(col.text, sw, cs))
        toks = [oracle.remove_stopwords(t, sw, cs) for t in _tokens_of(col)]
        text = col.text if isinstance(col, TokenColumn) else TextColumn([""] * len(toks))
        return frame.withColumn(self.getOutputCol(), TokenColumn(text, sw, cs, toks))


@register("org.apache.spark.ml.feature.HashingTF")
class HashingTF(HasInOut, Transformer):
    _uid_prefix = "HashingTF"
    _params = [Param("numFeatures", "number of features", 262144, int),
               Param("binary", "binary term frequencies", False, bool)]

    def _default_hook(self) -> None:
        self._defaultParamMap = {"outputCol": f"{self.uid}__output", "numFeatures": 262144, "binary": False}

    def indexOf(self, term: str) -> int:  # noqa: N802
        return oracle.term_index(term, self.getNumFeatures())

    def spec_kwargs(self) -> dict:
        return {"num_features": self.getNumFeatures(), "binary": bool(self.getBinary())}

    def _transform(self, frame: Frame) -> Frame:
        col = frame.column(self.getInputCol())
        n = self.getNumFeatures()
        if isinstance(col, TokenColumn) and col.fusable:
            vc = native_vectors(col, self.spec_kwargs())
        else:
            rows = [oracle.hashing_tf(t, n, self.getBinary()) for t in _tokens_of(col)]
            vc = _dict_rows_to_column(rows, n)
        return frame.withColumn(self.getOutputCol(), vc)


def _dict_rows_to_column(rows: list, size: int, device=None) -> VectorColumn:
    dev = torch.device(device) if device is not None else default_device()
    ptr = np.zeros(len(rows) + 1, dtype=np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    idx = np.fromiter((k for r in rows for k in r.keys()), dtype=np.int32, count=int(ptr[-1]))
    val = np.fromiter((v for r in rows for v in r.values()), dtype=np.float64, count=int(ptr[-1]))
    return VectorColumn(size, torch.from_numpy(ptr).to(dev), torch.from_numpy(idx).to(dev),
                        torch.from_numpy(val).to(dev))


class _CVParams:
    _params = [Param("vocabSize", "max vocabulary size", 262144, int),
               Param("minDF", "min documents a term must appear in", 1.0, float),
               Param("maxDF", "max documents a term may appear in", 9.223372036854776e18, float),
               Param("minTF", "min term count within a document", 1.0, float),
               Param("binary", "binary term frequencies", False, bool)]


@register("org.apache.spark.ml.feature.CountVectorizer")
class CountVectorizer(HasInOut, _CVParams, Estimator):
    _uid_prefix = "CountVectorizer"

    def _fit(self, frame: Frame) -> "CountVectorizerModel":
        col = frame.column(self.getInputCol())
        if isinstance(col, TokenColumn) and col.fusable and len(col):
            vocab = cv_fit_native(col, self.getVocabSize(), self.getMinDF(), self.getMaxDF())
        else:
            vocab = self._fit_python(_tokens_of(col))
        m = CountVectorizerModel(vocab, uid=self.uid)
        for k in ("inputCol", "outputCol", "minTF", "binary", "vocabSize", "minDF", "maxDF"):
            if self.isSet(k):
                m.set(k, self.getOrDefault(k))
        return m

    def _fit_python(self, toks: list) -> list:
        n_docs = len(toks)
        tf, df = Counter(), Counter()
        for t in toks:
            c = Counter(t)
            tf.update(c)
            df.update(c.keys())
        min_df = self.getMinDF()
        max_df = self.getMaxDF()
        lo = min_df if min_df >= 1.0 else min_df * n_docs
        hi = max_df if max_df >= 1.0 else max_df * n_docs
        cands = [(w, c) for w, c in tf.items() if lo <= df[w] <= hi]
        # top vocabSize by corpus term count (Spark `top(vocSize)(Ordering.by(count))`);
        # ties broken by the term itself for determinism.
        cands.sort(key=lambda wc: (-wc[1], wc[0]))
        return [w for w, _ in cands[: self.getVocabSize()]]


def _df_bounds(min_df: float, max_df: float, n_docs: int) -> tuple:
    return (min_df if min_df >= 1.0 else min_df * n_docs), (max_df if max_df >= 1.0 else max_df * n_docs)


def cv_fit_native(col: TokenColumn, vocab_size: int, min_df: float = 1.0, max_df: float = float(2 ** 63 - 1),
                  device=None) -> list:
    """CountVectorizer fit on the device (K-05, X-05): the fused text kernel emits a 64-bit key per
    kept token, a device sort yields corpus term counts and document frequencies, the minDF/maxDF
    filter and the top-``vocab_size`` selection run on device; only the selected terms are turned
    back into strings, from the first document containing each (host re-tokenisation of those
    documents only). Ordering: count descending, ties by term (same as the host fit)."""
    from ..ops.text import term_doc_counts, token_key, token_keys

    raw, clean = col.text.lineage()
    spec = FeatureSpec(clean=clean, stopwords=col.stopwords, num_features=1)
    dev = torch.device(device) if device is not None else default_device()
    keys, ntok = token_keys(raw.packed(), spec, dev)
    uk, tf, df, first = term_doc_counts(keys, ntok)
    lo, hi = _df_bounds(min_df, max_df, int(ntok.numel()))
    keep = (df.double() >= lo) & (df.double() <= hi)
    uk, tf, first = uk[keep], tf[keep], first[keep]
    if uk.numel() > vocab_size > 0:
        kth = torch.topk(tf, vocab_size).values[-1]
        sel = tf >= kth                                   # top-K plus the ties at the boundary
        uk, tf, first = uk[sel], tf[sel], first[sel]
    uk, tf, first = uk.cpu().numpy(), tf.cpu().numpy(), first.cpu().numpy()
    want = {int(k): None for k in uk}
    strings = raw.strings
    for d in np.unique(first):
        s = strings[int(d)] or ""
        toks = oracle.tokenize(oracle.clean_text(s) if clean else s)
        if col.stopwords is not None:
            toks = oracle.remove_stopwords(toks, col.stopwords)
        for t in toks:
            k = token_key(t)
            if k in want and want[k] is None:
                want[k] = t
    missing = [k for k, v in want.items() if v is None]
    if missing:
        raise RuntimeError(f"{len(missing)} token keys could not be mapped back to strings")
    cands = sorted(((want[int(k)], int(c)) for k, c in zip(uk, tf)), key=lambda wc: (-wc[1], wc[0]))
    return [w for w, _ in cands[:vocab_size]]


@register("org.apache.spark.ml.feature.CountVectorizerModel")
class CountVectorizerModel(HasInOut, _CVParams, Model):
    _uid_prefix = "CountVectorizer"

    def __init__(self, vocabulary: Optional[list] = None, **kw):
        super().__init__(**kw)
        self.vocabulary = list(vocabulary or [])

    def spec_kwargs(self) -> dict:
        return {"vocab": tuple(self.vocabulary), "min_tf": float(self.getMinTF()), "binary": bool(self.getBinary()),
                "num_features": max(1, len(self.vocabulary))}

    def _transform(self, frame: Frame) -> Frame:
        col = frame.column(self.getInputCol())
        if isinstance(col, TokenColumn) and col.fusable:
            vc = native_vectors(col, self.spec_kwargs())
        else:
            rows = [oracle.count_vectorize(t, self.vocabulary, self.getMinTF(), self.getBinary())
                    for t in _tokens_of(col)]
            vc = _dict_rows_to_column(rows, len(self.vocabulary))
        return frame.withColumn(self.getOutputCol(), vc)

    def _save_data(self, path) -> None:
        sf.write_data_parquet(path, [sf.Field.array("vocabulary", "string", contains_null=True)],
                              [{"vocabulary": self.vocabulary}])

    def _load_data(self, path, md) -> None:
        t = sf.read_data_parquet(path)
        self.vocabulary = list(t.column("vocabulary")[0].as_py())


@register("org.apache.spark.ml.feature.IDF")
class IDF(HasInOut, Estimator):
    _uid_prefix = "IDF"
    _params = [Param("minDocFreq", "min docs a term must appear in", 0, int)]

    def _default_hook(self) -> None:
        self._defaultParamMap = {"outputCol": f"{self.uid}__output", "minDocFreq": 0}

    def _fit(self, frame: Frame) -> "IDFModel":
        vc = frame.column(self.getInputCol())
        idf, df, n = idf_fit(vc, self.getMinDocFreq())
        m = IDFModel(idf, df, n, uid=self.uid)
        for k in ("inputCol", "outputCol", "minDocFreq"):
            if self.isSet(k):
                m.set(k, self.getOrDefault(k))
        return m


def idf_fit(vc: VectorColumn, min_doc_freq: int = 0, all_reduce=None):
    """docFreq = #rows with a non-zero entry; idf = ln((N+1)/(df+1)) or 0 below minDocFreq (X-06).
    ``all_reduce`` (optional) sums (docFreq, numDocs) across data-parallel ranks."""
    indptr, idx, val = vc.csr()
    nz = idx[val != 0].to(torch.int64)
    df = torch.bincount(nz, minlength=vc.size).to(torch.int64)
    n = torch.tensor([len(vc)], dtype=torch.int64, device=df.device)
    if all_reduce is not None:
        df, n = all_reduce(df), all_reduce(n)
    nd = int(n.item())
    idf = torch.log((nd + 1.0) / (df.to(torch.float64) + 1.0))
    idf = torch.where(df >= min_doc_freq, idf, torch.zeros_like(idf))
    return idf.cpu().numpy(), df.cpu().numpy(), nd


@register("org.apache.spark.ml.feature.IDFModel")
class IDFModel(HasInOut, Model):
    _uid_prefix = "IDF"
    _params = [Param("minDocFreq", "min docs a term must appear in", 0, int)]

    def _default_hook(self) -> None:
        self._defaultParamMap = {"outputCol": f"{self.uid}__output", "minDocFreq": 0}

    def __init__(self, idf=None, docFreq=None, numDocs: int = 0, **kw):  # noqa: N803
        super().__init__(**kw)
        self.idf = np.asarray(idf if idf is not None else [], dtype=np.float64)
        self.docFreq = np.asarray(docFreq if docFreq is not None else [], dtype=np.int64)
        self.numDocs = int(numDocs)
        self._dev: dict = {}

    def idf_tensor(self, device) -> torch.Tensor:
        key = str(device)
        if key not in self._dev:
            self._dev[key] = torch.from_numpy(self.idf).to(device)
        return self._dev[key]

    def _transform(self, frame: Frame) -> Frame:
        vc = frame.column(self.getInputCol())
        indptr, idx, val = vc.csr()
        w = self.idf_tensor(val.device)
        out = VectorColumn.scaled_counts(vc.size, indptr, idx, val, w)
        return frame.withColumn(self.getOutputCol(), out)

    def _save_data(self, path) -> None:
        sf.write_data_parquet(path, [sf.Field.vector("idf"), sf.Field.array("docFreq", "long"),
                                     sf.Field.simple("numDocs", "long")],
                              [{"idf": sf.dense_vector(self.idf), "docFreq": [int(x) for x in self.docFreq],
                                "numDocs": self.numDocs}])

    def _load_data(self, path, md) -> None:
        t = sf.read_data_parquet(path)
        row = t.to_pylist()[0]
        self.idf = sf.decode_vector(row["idf"])
        self.docFreq = np.asarray(row.get("docFreq") or [], dtype=np.int64)
        self.numDocs = int(row.get("numDocs") or 0)
        self._dev = {}
