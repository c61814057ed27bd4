"""A small columnar DataFrame with the subset of the Spark DataFrame API the reference uses.

Columns are typed containers rather than Python rows:

* ``TextColumn``  — strings, packed lazily into one UTF-8 buffer (``PackedText``) for the native
  featurizer; a cleaned column remembers its raw source (``lineage``) so the native kernel can
  apply ``regexp_replace(lower(x), "[^a-zA-Z ]", "")`` itself;
* ``TokenColumn`` — the *lineage* of Tokenizer/StopWordsRemover output (source text + stop
  words); token lists are only materialised if someone reads them, while HashingTF /
  CountVectorizer consume the lineage through the fused native op;
* ``VectorColumn`` (``ml.linalg``) — CSR or dense torch tensors on a device;
* numpy / torch arrays for scalars and ``[N, K]`` vector-valued outputs (``probability``);
* plain Python lists for anything else.

API mirrors pyspark where the reference calls it: ``withColumn, filter, select, randomSplit,
count, first, collect, limit, crosstab, toPandas`` (/root/reference/fraud_detection_spark.py:
30-45, 93-123, 338-344; utils/agent_api.py:139-175).
"""
from __future__ import annotations

import hashlib
from typing import Any, Callable, Iterable, Optional, Sequence

import numpy as np
import torch

from ..ops import oracle
from ..ops.text import PackedText
from .linalg import DenseVector, VectorColumn


# ----------------------------------------------------------------------------- columns
class TextColumn:
    def __init__(self, strings: Optional[Sequence] = None, source: Optional["TextColumn"] = None,
                 cleaned: bool = False):
        self._strings = list(strings) if strings is not None else None
        self.source = source          # raw column this one was cleaned from
        self.cleaned = cleaned
        self._packed: Optional[PackedText] = None

    @classmethod
    def cleaned_from(cls, raw: "TextColumn") -> "TextColumn":
        return cls(source=raw, cleaned=True)

    @property
    def strings(self) -> list:
        if self._strings is None:
            self._strings = [oracle.clean_text(s or "") for s in self.source.strings]
        return self._strings

    def __len__(self) -> int:
        return len(self.source) if self._strings is None else len(self._strings)

    def lineage(self) -> tuple["TextColumn", bool]:
        """(column whose bytes the native kernel should read, apply_clean?)."""
        if self.cleaned and self.source is not None:
            return self.source, True
        return self, False

    def packed(self) -> PackedText:
        if self._packed is None:
            self._packed = PackedText.from_strings(self.strings)
        return self._packed

    def take(self, rows: np.ndarray) -> "TextColumn":
        if self.cleaned and self.source is not None and self._strings is None:
            return TextColumn.cleaned_from(self.source.take(rows))
        s = self.strings
        out = TextColumn([s[i] for i in rows])
        if self.cleaned and self.source is not None:
            out.source, out.cleaned = self.source.take(rows), True
        return out


class TokenColumn:
    def __init__(self, text: TextColumn, stopwords: Optional[tuple] = None, case_sensitive: bool = False,
                 tokens: Optional[list] = None):
        self.text = text
        self.stopwords = stopwords
        self.case_sensitive = case_sensitive
        self._tokens = tokens

    @property
    def fusable(self) -> bool:
        return self._tokens is None and not self.case_sensitive

    @property
    def tokens(self) -> list:
        if self._tokens is None:
            toks = [oracle.tokenize(s or "") for s in self.text.strings]
            if self.stopwords is not None:
                toks = [oracle.remove_stopwords(t, self.stopwords, self.case_sensitive) for t in toks]
            self._tokens = toks
        return self._tokens

    def __len__(self) -> int:
        return len(self.text) if self._tokens is None else len(self._tokens)

    def take(self, rows: np.ndarray) -> "TokenColumn":
        if self._tokens is not None:
            return TokenColumn(self.text.take(rows), self.stopwords, self.case_sensitive,
                               [self._tokens[i] for i in rows])
        return TokenColumn(self.text.take(rows), self.stopwords, self.case_sensitive)


class Lazy:
    """A column computed on first access (e.g. intermediate features of a fused pipeline)."""

    def __init__(self, fn: Callable[[], Any], n: int):
        self.fn, self.n, self._v = fn, n, None

    def get(self):
        if self._v is None:
            self._v = self.fn()
        return self._v

    def __len__(self) -> int:
        return self.n


def _col_len(c) -> int:
    if isinstance(c, (torch.Tensor, np.ndarray)):
        return int(c.shape[0])
    return len(c)


def _take(c, rows: np.ndarray):
    if isinstance(c, Lazy):
        c = c.get()
    if isinstance(c, np.ndarray):
        return c[rows]
    if isinstance(c, torch.Tensor):
        return c[torch.as_tensor(rows, device=c.device, dtype=torch.int64)]
    if isinstance(c, (VectorColumn, TextColumn, TokenColumn)):
        return c.take(rows)
    return [c[i] for i in rows]


def _py(c, i: int):
    if isinstance(c, TextColumn):
        return c.strings[i]
    if isinstance(c, TokenColumn):
        return c.tokens[i]
    if isinstance(c, VectorColumn):
        return c.row(i)
    if isinstance(c, torch.Tensor):
        v = c[i]
        return DenseVector(v.detach().cpu().double().numpy()) if v.dim() else v.item()
    if isinstance(c, np.ndarray):
        v = c[i]
        return DenseVector(v) if getattr(v, "ndim", 0) else v.item()
    return c[i]


def _py_all(c) -> list:
    if isinstance(c, TextColumn):
        return list(c.strings)
    if isinstance(c, TokenColumn):
        return list(c.tokens)
    if isinstance(c, VectorColumn):
        return c.to_list()
    if isinstance(c, torch.Tensor):
        a = c.detach().cpu()
        if a.dim() > 1:
            return [DenseVector(r) for r in a.double().numpy()]
        return a.tolist()
    if isinstance(c, np.ndarray):
        if c.ndim > 1:
            return [DenseVector(r) for r in c.astype(np.float64)]
        return c.tolist()
    return list(c)


class Row(dict):
    """pyspark ``Row``: attribute, key and positional access."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __getitem__(self, k):
        if isinstance(k, int):
            return list(self.values())[k]
        return dict.__getitem__(self, k)

    def asDict(self) -> dict:  # noqa: N802
        return dict(self)


def _uniform(seed: int, n: int) -> np.ndarray:
    """Deterministic per-row uniforms in [0,1): splitmix64(seed, row)."""
    x = (np.arange(n, dtype=np.uint64) + np.uint64((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF))
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(11)).astype(np.float64) / float(1 << 53)


# ----------------------------------------------------------------------------- frame
class Frame:
    def __init__(self, columns: dict, order: Optional[list] = None, n: Optional[int] = None):
        self._cols = dict(columns)
        self._order = list(order) if order is not None else list(columns.keys())
        if n is None:
            n = _col_len(next(iter(self._cols.values()))) if self._cols else 0
        self._n = int(n)

    # ------------------------------------------------------------ construction
    @classmethod
    def from_pandas(cls, df, text_columns: Iterable[str] = ()) -> "Frame":
        cols = {}
        text_columns = set(text_columns)
        for c in df.columns:
            s = df[c]
            if c in text_columns or s.dtype == object:
                vals = [None if (isinstance(v, float) and np.isnan(v)) else v for v in s.tolist()]
                cols[c] = TextColumn(vals) if all(v is None or isinstance(v, str) for v in vals) else vals
            else:
                cols[c] = s.to_numpy()
        return cls(cols, list(df.columns), len(df))

    @classmethod
    def from_records(cls, rows: Sequence, schema: Sequence[str]) -> "Frame":
        cols = {}
        for j, name in enumerate(schema):
            vals = [r[j] if not isinstance(r, dict) else r[name] for r in rows]
            if vals and all(isinstance(v, str) or v is None for v in vals):
                cols[name] = TextColumn(vals)
            elif vals and all(isinstance(v, (int, float, np.number)) and not isinstance(v, bool) for v in vals):
                cols[name] = np.asarray(vals)
            else:
                cols[name] = vals
        return cls(cols, list(schema), len(rows))

    @classmethod
    def read_csv(cls, path, **kw) -> "Frame":
        import pandas as pd

        return cls.from_pandas(pd.read_csv(path, **kw))

    # ------------------------------------------------------------ schema / access
    @property
    def columns(self) -> list:
        return list(self._order)

    def __len__(self) -> int:
        return self._n

    def count(self) -> int:
        return self._n

    def column(self, name: str):
        c = self._cols[name]
        if isinstance(c, Lazy):
            c = c.get()
            self._cols[name] = c
        return c

    def __getitem__(self, name: str):
        return self.column(name)

    def __contains__(self, name: str) -> bool:
        return name in self._cols

    def raw_column(self, name: str):
        return self._cols[name]

    # ------------------------------------------------------------ transformations
    def withColumn(self, name: str, col) -> "Frame":  # noqa: N802
        if not isinstance(col, Lazy) and _col_len(col) != self._n:
            raise ValueError(f"column {name!r} has {_col_len(col)} rows, frame has {self._n}")
        cols = dict(self._cols)
        cols[name] = col
        order = self._order + ([name] if name not in self._cols else [])
        return Frame(cols, order, self._n)

    def withColumnRenamed(self, old: str, new: str) -> "Frame":  # noqa: N802
        cols = {(new if k == old else k): v for k, v in self._cols.items()}
        return Frame(cols, [new if k == old else k for k in self._order], self._n)

    def select(self, *names) -> "Frame":
        if len(names) == 1 and isinstance(names[0], (list, tuple)):
            names = tuple(names[0])
        return Frame({k: self._cols[k] for k in names}, list(names), self._n)

    def drop(self, *names) -> "Frame":
        keep = [k for k in self._order if k not in names]
        return Frame({k: self._cols[k] for k in keep}, keep, self._n)

    def take_rows(self, rows) -> "Frame":
        rows = np.asarray(rows, dtype=np.int64)
        return Frame({k: _take(v, rows) for k, v in self._cols.items()}, self._order, len(rows))

    def filter(self, cond) -> "Frame":
        """``cond``: boolean mask (array/tensor/list) or a predicate over ``Row``."""
        if callable(cond):
            mask = np.fromiter((bool(cond(r)) for r in self.collect()), dtype=bool, count=self._n)
        elif isinstance(cond, torch.Tensor):
            mask = cond.detach().cpu().numpy().astype(bool)
        else:
            mask = np.asarray(cond, dtype=bool)
        return self.take_rows(np.nonzero(mask)[0])

    where = filter

    def limit(self, n: int) -> "Frame":
        return self.take_rows(np.arange(min(n, self._n)))

    def randomSplit(self, weights: Sequence[float], seed: int = 0) -> list:  # noqa: N802
        """Per-row Bernoulli assignment by normalized cumulative weights (not stratified),
        deterministic in (seed, row). Spark's draw order depends on its partitioning, so the exact
        membership differs from Spark while the statistics match (fraud_detection_spark.py:338-339)."""
        w = np.asarray(weights, dtype=np.float64)
        bounds = np.cumsum(w / w.sum())
        u = _uniform(int(seed), self._n)
        which = np.searchsorted(bounds, u, side="right")
        which = np.minimum(which, len(w) - 1)
        return [self.take_rows(np.nonzero(which == i)[0]) for i in range(len(w))]

    def union(self, other: "Frame") -> "Frame":
        import pandas as pd

        return Frame.from_pandas(pd.concat([self.toPandas(), other.toPandas()], ignore_index=True))

    def cache(self) -> "Frame":
        return self

    persist = cache

    # ------------------------------------------------------------ actions
    def collect(self) -> list:
        cols = {k: _py_all(self.column(k)) for k in self._order}
        return [Row((k, cols[k][i]) for k in self._order) for i in range(self._n)]

    def first(self) -> Optional[Row]:
        if self._n == 0:
            return None
        return Row((k, _py(self.column(k), 0)) for k in self._order)

    def head(self, n: int = 1):
        return self.limit(n).collect() if n != 1 else self.first()

    def take(self, n: int) -> list:
        return self.limit(n).collect()

    def toPandas(self):  # noqa: N802
        import pandas as pd

        return pd.DataFrame({k: _py_all(self.column(k)) for k in self._order}, columns=self._order)

    def show(self, n: int = 20, truncate: bool = True) -> None:
        df = self.limit(n).toPandas()
        if truncate:
            df = df.map(lambda v: (str(v)[:17] + "...") if len(str(v)) > 20 else v)
        print(df.to_string(index=False))

    def crosstab(self, col1: str, col2: str):
        """Contingency table as pandas, first column ``{col1}_{col2}`` (Spark ``crosstab``)."""
        import pandas as pd

        a = _py_all(self.column(col1))
        b = _py_all(self.column(col2))
        ka = sorted(set(a), key=lambda v: (str(type(v)), v))
        kb = sorted(set(b), key=lambda v: (str(type(v)), v))
        counts = {(x, y): 0 for x in ka for y in kb}
        for x, y in zip(a, b):
            counts[(x, y)] += 1
        rows = [{f"{col1}_{col2}": _fmt(x), **{_fmt(y): counts[(x, y)] for y in kb}} for x in ka]
        return pd.DataFrame(rows, columns=[f"{col1}_{col2}"] + [_fmt(y) for y in kb])

    def __repr__(self) -> str:
        return f"Frame[{', '.join(self._order)}] ({self._n} rows)"


def _fmt(v) -> str:
    return str(v)


def fingerprint(frame: Frame) -> str:
    """Stable content hash (used for checkpoint/resume identity checks)."""
    h = hashlib.sha256()
    for k in frame.columns:
        h.update(k.encode())
        h.update(repr(_py_all(frame.column(k))[:1000]).encode())
    return h.hexdigest()[:16]
