"""``pyspark.ml.linalg``-compatible vectors plus the device-resident vector column.

Single rows are ``SparseVector``/``DenseVector`` (host, numpy); whole columns are
``VectorColumn`` — a CSR matrix (``indptr``/``indices``/``values`` torch tensors on the column's
device) or a dense ``[N, size]`` tensor — so pipelines never materialise per-row Python objects
on the hot path.
"""
from __future__ import annotations

from typing import Iterable, Optional, Sequence

import numpy as np
import torch


class Vector:
    size: int

    def toArray(self) -> np.ndarray:  # noqa: N802 (Spark API)
        raise NotImplementedError

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, i):
        return self.toArray()[i]


class DenseVector(Vector):
    def __init__(self, values: Iterable[float]):
        self.values = np.asarray(list(values) if not isinstance(values, np.ndarray) else values, dtype=np.float64)
        self.size = int(self.values.size)

    def toArray(self) -> np.ndarray:  # noqa: N802
        return self.values

    def __getitem__(self, i):
        return float(self.values[i])

    def dot(self, other) -> float:
        return float(np.dot(self.values, other.toArray()))

    def __eq__(self, other) -> bool:
        return isinstance(other, Vector) and np.array_equal(self.toArray(), other.toArray())

    def __repr__(self) -> str:
        return "DenseVector([" + ", ".join(repr(float(v)) for v in self.values) + "])"


class SparseVector(Vector):
    def __init__(self, size: int, indices: Sequence[int], values: Sequence[float]):
        self.size = int(size)
        idx = np.asarray(indices, dtype=np.int32)
        val = np.asarray(values, dtype=np.float64)
        order = np.argsort(idx, kind="stable")
        self.indices, self.values = idx[order], val[order]

    def toArray(self) -> np.ndarray:  # noqa: N802
        out = np.zeros(self.size, dtype=np.float64)
        out[self.indices] = self.values
        return out

    def __getitem__(self, i):
        j = np.searchsorted(self.indices, i)
        return float(self.values[j]) if j < self.indices.size and self.indices[j] == i else 0.0

    def numNonzeros(self) -> int:  # noqa: N802
        return int(np.count_nonzero(self.values))

    def dot(self, other) -> float:
        return float(np.dot(self.values, other.toArray()[self.indices]))

    def __eq__(self, other) -> bool:
        return isinstance(other, Vector) and np.array_equal(self.toArray(), other.toArray())

    def __repr__(self) -> str:
        return f"SparseVector({self.size}, {{" + ", ".join(
            f"{int(i)}: {float(v)!r}" for i, v in zip(self.indices, self.values)) + "})"


class Vectors:
    @staticmethod
    def dense(*values) -> DenseVector:
        if len(values) == 1 and not np.isscalar(values[0]):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size: int, *args) -> SparseVector:
        if len(args) == 1:
            d = dict(args[0]) if not isinstance(args[0], dict) else args[0]
            return SparseVector(size, list(d.keys()), list(d.values()))
        return SparseVector(size, args[0], args[1])


class VectorColumn:
    """A column of ``size``-dimensional vectors, CSR or dense, on one device."""

    def __init__(self, size: int, indptr: Optional[torch.Tensor] = None, indices: Optional[torch.Tensor] = None,
                 values: Optional[torch.Tensor] = None, dense: Optional[torch.Tensor] = None):
        self.size = int(size)
        self.indptr, self.indices, self._values, self.dense = indptr, indices, values, dense
        # TF-IDF columns built by the featurizer keep the integer term counts and the per-feature
        # IDF instead of fp64 values (8 B per entry, ~8 GB at 10M dialogues): the tree trainers
        # bin the counts directly, and ``values`` is only materialised if something asks for it
        self.tf_counts: Optional[torch.Tensor] = None
        self.tf_scale: Optional[torch.Tensor] = None
        self.count_bins = False
        if dense is None and indptr is None:
            raise ValueError("VectorColumn needs CSR arrays or a dense matrix")

    @property
    def values(self) -> Optional[torch.Tensor]:
        if self._values is None and self.tf_counts is not None and self.indices is not None:
            self._values = self.tf_counts.to(torch.float64) * self.tf_scale.to(
                device=self.indices.device, dtype=torch.float64)[self.indices.long()]
        return self._values

    @values.setter
    def values(self, v: Optional[torch.Tensor]) -> None:
        self._values = v

    @property
    def nnz(self) -> int:
        """Stored entries (sparse) or rows x size (dense)."""
        if self.indices is not None:
            return int(self.indices.numel())
        return int(self.dense.numel()) if self.dense is not None else 0

    @property
    def values_materialized(self) -> bool:
        return self._values is not None

    @classmethod
    def tfidf(cls, size: int, indptr: torch.Tensor, indices: torch.Tensor, counts: torch.Tensor,
              idf: torch.Tensor, feature_order=None, count_bins: bool = True) -> "VectorColumn":
        """A CSR TF-IDF column kept as (term counts, IDF vector): values = counts * idf[index]
        (fp64, bitwise the eager product), computed lazily (SURVEY §7.5 sizing: 4 B index + 4 B
        count per entry instead of + 8 B of values). ``count_bins``: the tree trainers bin the
        integer counts (bin = min(count, maxBins - 1)); False keeps Spark's value-space binning
        (midpoints between observed distinct values) on the materialised values."""
        vc = cls(size, indptr, indices, None)
        vc.tf_counts, vc.tf_scale = counts, idf
        vc.count_bins = bool(count_bins)
        if feature_order is not None:
            vc._feature_order = feature_order
        return vc

    @classmethod
    def scaled_counts(cls, size: int, indptr: torch.Tensor, indices: torch.Tensor, tf: torch.Tensor,
                      scale: torch.Tensor) -> "VectorColumn":
        """IDF of a term-frequency column: the TF values, when they are integral counts, are kept
        as int32 counts with the per-feature scale (lazy fp64 values, Spark value-space binning);
        otherwise the fp64 product is materialised."""
        if tf.numel() and tf.is_floating_point():
            integral = bool(torch.all((tf >= 0) & (tf == torch.round(tf)) & (tf < 2 ** 31)))
        else:
            integral = not tf.is_floating_point()
        if integral:
            return cls.tfidf(size, indptr, indices, tf.to(torch.int32), scale, count_bins=False)
        return cls(size, indptr, indices, tf.to(torch.float64) * scale[indices.to(torch.int64)])

    # -------------------------------------------------------------- construction
    @classmethod
    def from_rows(cls, rows: Sequence[Vector], size: Optional[int] = None, device="cpu") -> "VectorColumn":
        size = size if size is not None else (rows[0].size if rows else 0)
        ptr, idx, val = [0], [], []
        for r in rows:
            if isinstance(r, SparseVector):
                idx.append(r.indices.astype(np.int32))
                val.append(r.values.astype(np.float64))
            else:
                a = r.toArray() if isinstance(r, Vector) else np.asarray(r, dtype=np.float64)
                nz = np.nonzero(a)[0]
                idx.append(nz.astype(np.int32))
                val.append(a[nz])
            ptr.append(ptr[-1] + len(idx[-1]))
        ind = np.concatenate(idx) if idx else np.zeros(0, np.int32)
        vv = np.concatenate(val) if val else np.zeros(0, np.float64)
        return cls(size, torch.tensor(ptr, dtype=torch.int64, device=device),
                   torch.from_numpy(ind).to(device), torch.from_numpy(vv).to(device))

    # -------------------------------------------------------------- access
    def __len__(self) -> int:
        return int(self.dense.shape[0]) if self.dense is not None else int(self.indptr.numel()) - 1

    @property
    def device(self) -> torch.device:
        return (self.dense if self.dense is not None else self.indptr).device

    @property
    def is_sparse(self) -> bool:
        return self.dense is None

    def to(self, device) -> "VectorColumn":
        device = torch.device(device)
        if device == self.device:
            return self
        if self.dense is not None:
            return VectorColumn(self.size, dense=self.dense.to(device))
        if self._values is None and self.tf_counts is not None:
            return VectorColumn.tfidf(self.size, self.indptr.to(device), self.indices.to(device),
                                      self.tf_counts.to(device), self.tf_scale.to(device), count_bins=self.count_bins)
        return VectorColumn(self.size, self.indptr.to(device), self.indices.to(device), self.values.to(device))

    def csr(self):
        if self.dense is None:
            return self.indptr, self.indices, self.values
        d = self.dense
        nz = d != 0
        counts = nz.sum(1)
        indptr = torch.zeros(d.shape[0] + 1, dtype=torch.int64, device=d.device)
        torch.cumsum(counts, 0, out=indptr[1:])
        r, c = torch.nonzero(nz, as_tuple=True)
        return indptr, c.to(torch.int32), d[r, c]

    def take(self, rows) -> "VectorColumn":
        rows = torch.as_tensor(rows, dtype=torch.int64, device=self.device)
        if self.dense is not None:
            return VectorColumn(self.size, dense=self.dense[rows])
        start = self.indptr[rows]
        cnt = self.indptr[rows + 1] - start
        ptr = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=self.device)
        torch.cumsum(cnt, 0, out=ptr[1:])
        total = int(ptr[-1])
        r = torch.repeat_interleave(torch.arange(rows.numel(), device=self.device), cnt, output_size=total)
        pos = start[r] + (torch.arange(total, device=self.device) - ptr[r])
        return VectorColumn(self.size, ptr, self.indices[pos], self.values[pos])

    def row(self, i: int) -> Vector:
        if self.dense is not None:
            return DenseVector(self.dense[i].detach().cpu().double().numpy())
        a, b = int(self.indptr[i]), int(self.indptr[i + 1])
        return SparseVector(self.size, self.indices[a:b].cpu().numpy(), self.values[a:b].cpu().double().numpy())

    def to_list(self) -> list:
        if self.dense is not None:
            d = self.dense.detach().cpu().double().numpy()
            return [DenseVector(r) for r in d]
        ptr = self.indptr.cpu().numpy()
        ind = self.indices.cpu().numpy()
        val = self.values.cpu().double().numpy()
        return [SparseVector(self.size, ind[ptr[i]:ptr[i + 1]], val[ptr[i]:ptr[i + 1]]) for i in range(len(self))]

    def __getitem__(self, i):
        return self.row(i)

    def __iter__(self):
        return iter(self.to_list())
