"""Sparse ops over ``VectorColumn`` CSR data (native: ``csrc/sparse_kernels.hip`` / ``sparse_cpu.cpp``)."""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import native
from .text import LinearScorer, TreeArrays


def _csr(vc):
    indptr, idx, val = vc.csr()
    if val.dtype not in (torch.float32, torch.float64):
        val = val.to(torch.float64)
    return indptr.contiguous(), idx.to(torch.int32).contiguous(), val.contiguous()


def score_csr(vc, scorer, threads: int = 0) -> torch.Tensor:
    """Raw scores ``[N, K]`` fp64: LR margin (K=1) or tree-ensemble sums (K = leaf width)."""
    indptr, idx, val = _csr(vc)
    dev = indptr.device
    n = indptr.numel() - 1
    C = native.lib()
    if isinstance(scorer, LinearScorer):
        if scorer.w.size > vc.size:
            raise ValueError("coefficient vector longer than the feature space")
        out = torch.empty((n, 1), dtype=torch.float64, device=dev)
        w = scorer.weights(dev)
        if w.numel() < vc.size:   # features beyond the model's width contribute nothing
            w = torch.cat([w, torch.zeros(vc.size - w.numel(), dtype=torch.float64, device=dev)])
        C.score_csr(indptr, idx, val, w, scorer.b, None, 1, False, out, threads)
        return out
    if isinstance(scorer, TreeArrays):
        if scorer.max_feature() >= vc.size:
            raise ValueError("tree references a feature beyond the feature space")
        out = torch.empty((n, scorer.K), dtype=torch.float64, device=dev)
        C.score_csr(indptr, idx, val, None, 0.0, scorer.tensors(dev), scorer.K, scorer.cmp_less, out, threads)
        return out
    raise TypeError(f"unknown scorer {type(scorer)}")


def spmv(indptr, idx, val, x: torch.Tensor, threads: int = 0) -> torch.Tensor:
    y = torch.empty(indptr.numel() - 1, dtype=torch.float64, device=indptr.device)
    native.lib().spmv(indptr, idx, val, x, y, threads)
    return y


def spmv_t(indptr, idx, val, r: torch.Tensor, cols: int, threads: int = 0) -> torch.Tensor:
    g = torch.zeros(cols, dtype=torch.float64, device=indptr.device)
    native.lib().spmv_t(indptr, idx, val, r, g, threads)
    return g


def term_presence_by_label(vc, term_ids, labels, num_classes: int = 2) -> torch.Tensor:
    """K-19: documents containing each of ``term_ids`` per label, in one pass over the CSR
    (replaces the reference's one Spark job per word, fraud_detection_spark.py:256-269).
    Returns ``counts[len(term_ids), num_classes]`` (int64)."""
    indptr, idx, val = vc.csr()
    dev = indptr.device
    ids = torch.as_tensor(term_ids, dtype=torch.int64, device=dev)
    lab = torch.as_tensor(labels, device=dev).to(torch.int64)
    slot = torch.full((vc.size,), -1, dtype=torch.int64, device=dev)
    slot[ids] = torch.arange(ids.numel(), device=dev)
    row = torch.repeat_interleave(torch.arange(indptr.numel() - 1, device=dev), indptr[1:] - indptr[:-1],
                                  output_size=int(idx.numel()))
    s = slot[idx.to(torch.int64)]
    keep = (s >= 0) & (val != 0)
    key = s[keep] * num_classes + lab[row[keep]]
    return torch.bincount(key, minlength=ids.numel() * num_classes).view(ids.numel(), num_classes)


def doc_freq(idx: torch.Tensor, val: torch.Tensor, size: int) -> torch.Tensor:
    if idx.is_cuda:
        df = torch.zeros(size, dtype=torch.int64, device=idx.device)
        native.lib().doc_freq(idx.to(torch.int32).contiguous(), val.contiguous(), df)
        return df
    return torch.bincount(idx[val != 0].to(torch.int64), minlength=size)


@dataclass
class FeatureOrder:
    """Column-major (CSC) view of a count CSR: ``csc_row`` / ``csc_cnt`` (min(count, 255)) are
    views with >= 16 readable padding entries behind them, ``colptr`` [F+1], ``df`` document
    frequencies and ``maxc`` per-feature maximum count."""
    csc_row: torch.Tensor
    csc_cnt: torch.Tensor
    colptr: torch.Tensor
    df: torch.Tensor
    maxc: torch.Tensor
    # features whose entries were dropped from csc_row / csc_cnt (drop_features; df keeps them)
    dropped: Optional[torch.Tensor] = None

    def drop_features(self, drop: torch.Tensor) -> None:
        """Remove the entries of the features flagged in ``drop`` [F] (bool) IN PLACE: the kept
        columns slide left over the dropped ones, in order, so no second CSC is allocated (the
        trainers drop features whose values are all zero, e.g. IDF 0 for terms in every
        document, whose columns hold one entry per row: copying the rest of the CSC instead
        cost 5 B per entry of transient HBM). Every move copies ``chunk <= shift`` entries, so
        source and destination of one copy never overlap; copies run in stream order."""
        colptr = self.colptr.cpu().numpy()
        dmask = drop.cpu().numpy().astype(bool)
        lens = np.diff(colptr)
        dmask &= lens > 0
        if not dmask.any():
            return
        nnz = int(colptr[-1])
        # maximal runs of kept columns -> (src start, src end)
        edges = np.flatnonzero(np.diff(np.concatenate([[1], dmask.astype(np.int8), [1]])))
        dst = 0
        for a, b in zip(edges[0::2], edges[1::2]):          # kept features [a, b)
            s0, s1 = int(colptr[a]), int(colptr[b])
            n = s1 - s0
            if n and s0 != dst:
                shift = s0 - dst
                for off in range(0, n, shift):
                    c = min(shift, n - off)
                    self.csc_row[dst + off:dst + off + c].copy_(self.csc_row[s0 + off:s0 + off + c])
                    self.csc_cnt[dst + off:dst + off + c].copy_(self.csc_cnt[s0 + off:s0 + off + c])
            dst += n
        new_lens = np.where(dmask, 0, lens)
        newptr = np.concatenate([[0], np.cumsum(new_lens)]).astype(np.int64)
        assert int(newptr[-1]) == dst <= nnz
        self.colptr.copy_(torch.from_numpy(newptr))
        self.csc_row, self.csc_cnt = self.csc_row[:dst], self.csc_cnt[:dst]
        d = torch.from_numpy(dmask).to(self.maxc.device)
        self.dropped = d if self.dropped is None else (self.dropped | d)


# entries radix-sorted at once by feature_order: the device sort needs 24 B of temporaries per
# entry, so a 1.25B-entry shard sorts in row blocks of this size (each block's columns are copied
# into place; rows stay in row order within every column, exactly the one-shot CSC)
FO_BLOCK_ENTRIES = int(os.environ.get("FDX_FO_BLOCK_ENTRIES", 1 << 28))


def _feature_order_one(indptr, idx, counts, num_features: int, row_buf, cnt_buf) -> tuple:
    dev = idx.device
    nnz = int(idx.numel())
    colptr = torch.empty(num_features + 1, dtype=torch.int64, device=dev)
    df = torch.empty(num_features, dtype=torch.int64, device=dev)
    maxc = torch.empty(num_features, dtype=torch.int32, device=dev)
    native.lib().feature_order(indptr.contiguous(), idx.to(torch.int32).contiguous(), counts.contiguous(),
                               int(num_features), row_buf[:nnz], cnt_buf[:nnz], colptr, df, maxc)
    return colptr, df, maxc


def feature_order(indptr: torch.Tensor, idx: torch.Tensor, counts: torch.Tensor, num_features: int,
                  block_entries: Optional[int] = None) -> FeatureOrder:
    """CSR (rows, sorted unique feature ids per row, term counts) -> CSC by feature with a native
    radix sort; docFreq and the per-feature max count are segmented reductions (no atomics).
    Integer counts are sorted as int32 (no float copy). Above ``block_entries`` entries the rows
    are sorted in blocks, so the sort's temporaries stay bounded (HBM sizing)."""
    dev = idx.device
    nnz = int(idx.numel())
    if counts.dtype not in (torch.float32, torch.float64, torch.int32):
        counts = counts.to(torch.float32 if counts.is_floating_point() else torch.int32)
    pad = 16
    row_buf = torch.zeros(nnz + pad, dtype=torch.int32, device=dev)
    cnt_buf = torch.zeros(nnz + pad, dtype=torch.uint8, device=dev)
    block = int(block_entries or FO_BLOCK_ENTRIES)
    if nnz <= block:
        colptr, df, maxc = _feature_order_one(indptr, idx, counts, num_features, row_buf, cnt_buf)
        return FeatureOrder(row_buf[:nnz], cnt_buf[:nnz], colptr, df, maxc)
    N = int(indptr.numel() - 1)
    # row blocks of <= ~block entries (a single row larger than a block is its own block)
    targets = torch.arange(block, nnz, block, dtype=torch.int64, device=dev)
    cuts = torch.searchsorted(indptr, targets, right=True).clamp(1, N) - 1
    rcuts = sorted(set([0, N] + [int(c) for c in cuts.cpu().tolist() if 0 < int(c) < N]))
    C = native.lib()
    # pass 1: per-block column sizes (one bincount per block) -> every block's column offsets
    lens = []
    for r0, r1 in zip(rcuts[:-1], rcuts[1:]):
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        lens.append(torch.bincount(idx[e0:e1].to(torch.int64), minlength=num_features))
    tot = torch.stack(lens).sum(0)
    colptr = torch.zeros(num_features + 1, dtype=torch.int64, device=dev)
    torch.cumsum(tot, 0, out=colptr[1:])
    df = tot
    maxc = torch.zeros(num_features, dtype=torch.int32, device=dev)
    before = torch.zeros(num_features, dtype=torch.int64, device=dev)
    # pass 2: sort each block, add its first row, copy its columns into place (one block's
    # temporaries alive at a time; IncrementalFeatureOrder keeps every block until the end)
    for (r0, r1), ln in zip(zip(rcuts[:-1], rcuts[1:]), lens):
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        n = e1 - e0
        brow = torch.zeros(n + pad, dtype=torch.int32, device=dev)
        bcnt = torch.zeros(n + pad, dtype=torch.uint8, device=dev)
        bcol, _, bmax = _feature_order_one(indptr[r0:r1 + 1] - e0, idx[e0:e1], counts[e0:e1], num_features, brow, bcnt)
        brow[:n] += r0
        torch.maximum(maxc, bmax, out=maxc)
        C.copy_segments(brow[:n], bcnt[:n], bcol[:-1].contiguous(), (colptr[:-1] + before).contiguous(), ln,
                        row_buf[:nnz], cnt_buf[:nnz], None)
        before += ln
        del brow, bcnt, bcol
    return FeatureOrder(row_buf[:nnz], cnt_buf[:nnz], colptr, df, maxc)


class IncrementalFeatureOrder:
    """feature_order built one row block at a time, as the blocks arrive (e.g. each featurized
    chunk while the next chunk's raw text is still crossing PCIe): every block is sorted by
    feature on its own (``add``), and ``finish`` copies each block's columns into place behind the
    earlier blocks' entries of the same column. Rows stay ascending within every column, so the
    result equals the one-shot CSC of the concatenated CSR. Holds every block's sorted (row, count)
    pairs until ``finish`` (5 B per entry on top of the CSR, then the same again for the output)."""

    PAD = 16

    def __init__(self, num_features: int, device):
        self.F, self.dev = int(num_features), torch.device(device)
        self.blocks: list = []               # (block colptr, rows (global), counts u8, n entries)
        self.maxc = torch.zeros(self.F, dtype=torch.int32, device=self.dev)
        self.nnz = 0

    def add(self, indptr: torch.Tensor, idx: torch.Tensor, counts: torch.Tensor, first_row: int) -> None:
        """Sort one block: ``indptr`` local to the block (starts at 0), rows ``first_row + i``."""
        if counts.dtype not in (torch.float32, torch.float64, torch.int32):
            counts = counts.to(torch.float32 if counts.is_floating_point() else torch.int32)
        n = int(idx.numel())
        brow = torch.zeros(n + self.PAD, dtype=torch.int32, device=self.dev)
        bcnt = torch.zeros(n + self.PAD, dtype=torch.uint8, device=self.dev)
        bcol, _, bmax = _feature_order_one(indptr, idx, counts, self.F, brow, bcnt)
        if first_row:
            brow[:n] += int(first_row)
        torch.maximum(self.maxc, bmax, out=self.maxc)
        self.blocks.append((bcol, brow, bcnt, n))
        self.nnz += n

    def finish(self) -> FeatureOrder:
        nnz, dev = self.nnz, self.dev
        lens = [bcol[1:] - bcol[:-1] for bcol, _, _, _ in self.blocks]
        tot = torch.stack(lens).sum(0) if lens else torch.zeros(self.F, dtype=torch.int64, device=dev)
        colptr = torch.zeros(self.F + 1, dtype=torch.int64, device=dev)
        torch.cumsum(tot, 0, out=colptr[1:])
        if len(self.blocks) == 1:               # one block: its sort is the CSC
            _, brow, bcnt, n = self.blocks.pop()
            return FeatureOrder(brow[:n], bcnt[:n], colptr, tot, self.maxc)
        row_buf = torch.zeros(nnz + self.PAD, dtype=torch.int32, device=dev)
        cnt_buf = torch.zeros(nnz + self.PAD, dtype=torch.uint8, device=dev)
        before = torch.zeros(self.F, dtype=torch.int64, device=dev)
        C = native.lib()
        for (bcol, brow, bcnt, n), ln in zip(self.blocks, lens):
            C.copy_segments(brow[:n], bcnt[:n], bcol[:-1].contiguous(), (colptr[:-1] + before).contiguous(), ln,
                            row_buf[:nnz], cnt_buf[:nnz], None)
            before += ln
        self.blocks = []
        return FeatureOrder(row_buf[:nnz], cnt_buf[:nnz], colptr, tot, self.maxc)
