"""Feature binning + quantized CSC layout for the histogram tree engine (K-09, X-09/X-13).

Two binning paths:

* **count path** — HashingTF/CountVectorizer features (optionally IDF-scaled: value = tf * s_f with
  s_f > 0) are binned by the integer term count: bin = min(tf, max_bins - 1), the zero bin is 0.
  Because v = tf * s_f is monotone in tf, these bins give exactly the split candidates Spark's
  ``findSplitsForContinuousFeature`` produces for TF-IDF data (midpoints between consecutive
  distinct values) as long as a feature has < max_bins distinct counts; no sort is needed.
* **generic path** — arbitrary float features: distinct (feature, value) pairs via a sort; a
  feature with < max_bins distinct values gets one bin per value, otherwise equal-count groups.
  Values are keyed at float32 precision (XGBoost bins at float32 as well).

In both paths the thresholds are value-space midpoints, so the same tree scores raw feature
values with either ``x <= t`` (Spark) or ``x < t`` (XGBoost) semantics. Under data parallelism
the per-rank statistics (max counts / distinct values) are merged with collectives so every rank
holds identical bins.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import torch

from ..ops import native
from ..utils import tracing

CSC_PAD = 16

CHUNK = int(os.environ.get("FDX_HIST_CHUNK", 32768))   # entries per histogram work item (one wavefront)


@dataclass
class BinGroup:
    """Work items of the features of one MFMA tile shape: ``bt`` 0 = at most 16 bins (narrow
    16x16x32 tile), 1 / 2 = at most 32 / 64 bins (one or two 32-row 32x32x16 tiles)."""
    bt: int
    item_start: torch.Tensor     # int64 [I]
    item_end: torch.Tensor       # int64 [I]
    item_feat: torch.Tensor      # int32 [I]
    feat: torch.Tensor           # int32 [L]
    feat_item0: torch.Tensor     # int64 [L]
    feat_nitems: torch.Tensor    # int32 [L]
    item_blk: Optional[torch.Tensor] = None   # int32 [I] row block of the item (-1: whole column)
    _order: Optional[torch.Tensor] = None

    def subset(self, feat_mask: torch.Tensor) -> "BinGroup":
        """Restrict to features with ``feat_mask[fid]`` (RF per-level feature union)."""
        keep_items = feat_mask[self.item_feat.to(torch.int64)]
        keep_feat = feat_mask[self.feat.to(torch.int64)]
        item_start, item_end = self.item_start[keep_items], self.item_end[keep_items]
        item_feat = self.item_feat[keep_items]
        feat = self.feat[keep_feat]
        nitems = self.feat_nitems[keep_feat]
        item0 = torch.zeros_like(nitems, dtype=torch.int64)
        if nitems.numel():
            item0[1:] = torch.cumsum(nitems.to(torch.int64), 0)[:-1]
        blk = self.item_blk[keep_items] if self.item_blk is not None else None
        return BinGroup(self.bt, item_start, item_end, item_feat, feat, item0, nitems, blk)

    @property
    def num_items(self) -> int:
        return int(self.item_start.numel())

    def wave_order(self) -> torch.Tensor:
        """Item of every wave slot of the histogram / entry-statistics launches (-1: idle)."""
        if self._order is None:
            self._order = wave_order(self.item_blk, self.num_items, self.item_start.device)
        return self._order


def wave_order(item_blk: Optional[torch.Tensor], num_items: int, dev) -> torch.Tensor:
    """XCD-aware item placement. Workgroups are dealt round-robin over the 8 XCDs (observed
    dispatch, speed only), so workgroups b and b + 8 share an L2: the 4 wave slots of workgroup
    b = 8k + x get items of row blocks = x (mod 8) in block order, i.e. each XCD walks its own
    row blocks one after another and the block's 1-byte slot table and 8-byte row statistics
    (~1 MB) stay in that XCD's 4 MB L2. Whole-column items (row block -1) are spread round-robin
    and run last."""
    if num_items == 0:
        return torch.full((4,), -1, dtype=torch.int32, device=dev)
    idx = torch.arange(num_items, device=dev, dtype=torch.int64)
    if item_blk is None:
        blk = torch.full((num_items,), -1, dtype=torch.int64, device=dev)
    else:
        blk = item_blk.to(torch.int64)
    blocked = blk >= 0
    label = torch.where(blocked, blk % 8, idx % 8)
    phase = torch.where(blocked, blk // 8, torch.full_like(blk, 1 << 20))
    key = (label << 52) | (phase << 30) | idx
    order = torch.argsort(key)
    lab_sorted = label[order]
    counts = torch.bincount(lab_sorted, minlength=8)
    first = torch.cumsum(counts, 0) - counts
    pos = torch.arange(num_items, device=dev) - first[lab_sorted]
    per = int(counts.max())
    groups = (per + 3) // 4
    slot = (pos // 4) * 32 + lab_sorted * 4 + pos % 4
    out = torch.full((groups * 32,), -1, dtype=torch.int32, device=dev)
    out[slot] = order.to(torch.int32)
    return out


@dataclass
class Quantized:
    n_rows: int
    num_features: int
    fid_orig: torch.Tensor       # int64 [Fa]
    nbins: torch.Tensor          # int32 [Fa]
    zbin: torch.Tensor           # int32 [Fa]
    boff: torch.Tensor           # int64 [Fa+1]
    thresholds: np.ndarray       # float64 [TB]: split "bin <= b goes left" <=> "x <= thresholds[boff+b]"
    colptr: torch.Tensor         # int64 [Fa+1]
    csc_row: torch.Tensor        # int32 [nnz] (view; CSC_PAD readable entries follow)
    csc_bin: torch.Tensor        # uint8 [nnz] (view; CSC_PAD readable entries follow)
    groups: list = field(default_factory=list)
    _all_items: Optional[tuple] = None

    def all_items(self) -> tuple:
        """(item_start, item_end, wave_order) over the items of every group: one XCD-ordered launch
        for per-entry work that does not depend on the tile shape (entry statistics)."""
        if self._all_items is None:
            dev = self.csc_row.device
            gs = self.groups
            if not gs:
                z = torch.zeros(0, dtype=torch.int64, device=dev)
                self._all_items = (z, z, wave_order(None, 0, dev))
            else:
                st = torch.cat([g.item_start for g in gs])
                en = torch.cat([g.item_end for g in gs])
                blk = torch.cat([g.item_blk if g.item_blk is not None else
                                 torch.full((g.num_items,), -1, dtype=torch.int32, device=dev) for g in gs])
                self._all_items = (st, en, wave_order(blk, int(st.numel()), dev))
        return self._all_items
    boff_host: np.ndarray = None
    zbin_host: np.ndarray = None
    fid_host: np.ndarray = None

    @property
    def Fa(self) -> int:  # noqa: N802
        return int(self.nbins.numel())

    @property
    def TB(self) -> int:  # noqa: N802
        return int(self.boff_host[-1])

    @property
    def device(self) -> torch.device:
        return self.csc_row.device

    def threshold(self, fid: int, b: int) -> float:
        return float(self.thresholds[int(self.boff_host[fid]) + int(b)])


def _ordered_f32_bits(v: torch.Tensor) -> torch.Tensor:
    b = v.to(torch.float32).view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    neg = (b >> 31) == 1
    return torch.where(neg, b ^ 0xFFFFFFFF, b | 0x80000000)


def _decode_f32_bits(k: torch.Tensor) -> torch.Tensor:
    neg = (k >> 31) == 0
    b = torch.where(neg, k ^ 0xFFFFFFFF, k & 0x7FFFFFFF)
    b = torch.where(b >= (1 << 31), b - (1 << 32), b).to(torch.int32)
    return b.view(torch.float32).to(torch.float64)


def quantize(vc, max_bins: int = 32, counts: Optional[torch.Tensor] = None, scale: Optional[torch.Tensor] = None,
             all_reduce_max: Optional[Callable] = None, all_gather: Optional[Callable] = None,
             chunk: int = CHUNK, row_block: int = None, split_min: int = None) -> Quantized:
    """Bin a ``VectorColumn`` and build the CSC. ``counts``/``scale`` select the count path
    (per-entry integer counts and per-feature positive scale); integral non-negative values
    take it automatically with scale 1."""
    if max_bins < 2 or max_bins > 64:
        raise ValueError("max_bins must be in [2, 64] (bins are held in one or two 32-row MFMA tiles)")
    indptr, idx, val = vc.csr()
    dev = indptr.device
    N = int(indptr.numel() - 1)
    F = int(vc.size)
    idx64 = idx.to(torch.int64)
    val64 = val.to(torch.float64)
    if counts is None and val64.numel() and bool(torch.all(val64 >= 0)) and bool(torch.all(val64 == torch.round(val64))) \
            and float(val64.max()) < 65536:
        counts = val64
        scale = torch.ones(F, dtype=torch.float64, device=dev)
    if counts is not None and F < (1 << 31):
        Q = _quantize_counts(vc, indptr, idx, counts, scale, N, F, max_bins, all_reduce_max)
        with tracing.span("q.groups"):
            Q.groups = _make_groups(Q.colptr, Q.nbins, chunk, Q.csc_row, N, row_block or ROW_BLOCK,
                                    split_min or SPLIT_MIN)
        return Q
    with tracing.span("q.rows"):
        row = torch.repeat_interleave(torch.arange(N, device=dev, dtype=torch.int32), (indptr[1:] - indptr[:-1]),
                                      output_size=int(idx.numel()))
    with tracing.span("q.bins"):
        if counts is not None:
            q = _count_path(idx64, counts.to(torch.float64), scale.to(device=dev, dtype=torch.float64), F, max_bins,
                            all_reduce_max)
        else:
            q = _generic_path(idx64, val64, F, max_bins, all_gather)
    remap, nbins, zbin, thresholds, entry_bin, keep = q
    with tracing.span("q.filter"):
        fid = remap[idx64]
        keep = keep & (fid >= 0)
        fid, row, entry_bin = fid[keep], row[keep], entry_bin[keep]
    Fa = int(nbins.numel())
    with tracing.span("q.sort"):
        order = torch.sort(fid.to(torch.int32), stable=True).indices
    nnz = int(order.numel())
    # the histogram kernel loads 4-entry groups without per-lane branches: keep CSC_PAD readable
    # entries behind the end of both arrays (bin 0xff = no bin)
    sp = tracing.span("q.gather")
    sp.__enter__()
    csc_row = torch.zeros(nnz + CSC_PAD, dtype=torch.int32, device=dev)
    csc_row[:nnz] = row[order]
    csc_bin = torch.full((nnz + CSC_PAD,), 0xFF, dtype=torch.uint8, device=dev)
    csc_bin[:nnz] = entry_bin[order].to(torch.uint8)
    csc_row, csc_bin = csc_row[:nnz], csc_bin[:nnz]
    sp.__exit__(None, None, None)
    cnt = torch.bincount(fid, minlength=Fa)
    colptr = torch.zeros(Fa + 1, dtype=torch.int64, device=dev)
    torch.cumsum(cnt, 0, out=colptr[1:])
    boff = torch.zeros(Fa + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nbins.to(torch.int64), 0, out=boff[1:])
    fid_orig = torch.nonzero(remap >= 0).flatten()
    Q = Quantized(N, F, fid_orig, nbins.to(torch.int32).contiguous(), zbin.to(torch.int32).contiguous(), boff,
                  thresholds, colptr, csc_row, csc_bin)
    Q.boff_host = boff.cpu().numpy()
    Q.zbin_host = Q.zbin.cpu().numpy()
    Q.fid_host = fid_orig.cpu().numpy()
    with tracing.span("q.groups"):
        Q.groups = _make_groups(colptr, nbins, chunk, csc_row, N, row_block or ROW_BLOCK, split_min or SPLIT_MIN)
    return Q


def _quantize_counts(vc, indptr, idx, counts, scale, N, F, max_bins, all_reduce_max) -> "Quantized":
    """Count path on the native feature-major order (sort_kernels.hip): bins = min(count,
    max_bins - 1) with thresholds (k + 0.5) * scale_f; the CSC comes straight from the radix sort
    (cached on the VectorColumn as ``_feature_order`` when the caller already built it for IDF)."""
    from ..ops.sparse import feature_order

    dev = indptr.device
    fo = getattr(vc, "_feature_order", None)
    if fo is None or fo.colptr.numel() != F + 1 or fo.csc_row.device != dev:
        with tracing.span("q.order"):
            fo = feature_order(indptr, idx, counts, F)
    scale = scale.to(device=dev, dtype=torch.float64)
    maxb = torch.clamp(fo.maxc.to(torch.int64), max=max_bins - 1)
    maxb = torch.where(scale > 0, maxb, torch.zeros_like(maxb))
    if all_reduce_max is not None:
        maxb = all_reduce_max(maxb)
    active = maxb > 0
    Fa = int(active.sum())
    fid_orig = torch.nonzero(active).flatten()
    nbins = (maxb[active] + 1).to(torch.int32)
    nb = nbins.to(torch.int64)
    TB = int(nb.sum())
    f_of_bin = torch.repeat_interleave(torch.arange(Fa, device=dev), nb, output_size=TB)
    bstart = torch.cumsum(nb, 0) - nb
    k = torch.arange(TB, device=dev) - bstart[f_of_bin]
    thresholds = ((k.to(torch.float64) + 0.5) * scale[fid_orig][f_of_bin]).cpu().numpy()
    lens = fo.colptr[1:] - fo.colptr[:-1]
    nnz_all = int(fo.colptr[-1])
    with tracing.span("q.csc"):
        if int(lens[~active].sum()) == 0:        # every non-empty feature is active: the order is the CSC
            csc_row = fo.csc_row
            cnt = fo.csc_cnt
            colptr = torch.zeros(Fa + 1, dtype=torch.int64, device=dev)
            if Fa:
                colptr[:-1] = fo.colptr[:-1][active]
                colptr[-1] = fo.colptr[1:][active][-1]
        else:                                     # drop the entries of inactive features (scale 0)
            keep = torch.repeat_interleave(active, lens, output_size=nnz_all)
            n_keep = int(keep.sum())
            row_buf = torch.zeros(n_keep + CSC_PAD, dtype=torch.int32, device=dev)
            row_buf[:n_keep] = fo.csc_row[keep]
            csc_row = row_buf[:n_keep]
            cnt = fo.csc_cnt[keep]
            colptr = torch.zeros(Fa + 1, dtype=torch.int64, device=dev)
            torch.cumsum(lens[active], 0, out=colptr[1:])
        n = int(csc_row.numel())
        bin_buf = torch.full((n + CSC_PAD,), 0xFF, dtype=torch.uint8, device=dev)
        if cnt.is_cuda and cnt.data_ptr() % 16:           # compacted copy: realign for the native clamp
            cnt = cnt.clone()
        native.lib().clamp_u8(cnt.contiguous(), max_bins - 1, bin_buf[:n])
    boff = torch.zeros(Fa + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nb, 0, out=boff[1:])
    Q = Quantized(N, F, fid_orig, nbins.contiguous(), torch.zeros(Fa, dtype=torch.int32, device=dev), boff,
                  thresholds, colptr, csc_row, bin_buf[:n])
    Q.boff_host = boff.cpu().numpy()
    Q.zbin_host = Q.zbin.cpu().numpy()
    Q.fid_host = fid_orig.cpu().numpy()
    return Q


def _count_path(idx, counts, scale, F, max_bins, all_reduce_max):
    dev = idx.device
    keep = counts > 0
    b = torch.clamp(counts, max=max_bins - 1).to(torch.int64)
    maxb = torch.zeros(F, dtype=torch.int64, device=dev)
    maxb.scatter_reduce_(0, idx[keep], b[keep], reduce="amax")
    maxb = torch.where(scale > 0, maxb, torch.zeros_like(maxb))
    if all_reduce_max is not None:
        maxb = all_reduce_max(maxb)
    active = maxb > 0
    remap = torch.full((F,), -1, dtype=torch.int64, device=dev)
    Fa = int(active.sum())
    remap[active] = torch.arange(Fa, device=dev)
    nbins = (maxb[active] + 1).to(torch.int32)
    zbin = torch.zeros(Fa, dtype=torch.int32, device=dev)
    # thresholds: after bin k (count k) -> (k + 0.5) * s_f
    nb = nbins.to(torch.int64)
    TB = int(nb.sum())
    f_of_bin = torch.repeat_interleave(torch.arange(Fa, device=dev), nb, output_size=TB)
    start = torch.cumsum(nb, 0) - nb
    k = torch.arange(TB, device=dev) - start[f_of_bin]
    s = scale[active][f_of_bin]
    thresholds = ((k.to(torch.float64) + 0.5) * s).cpu().numpy()
    return remap, nbins, zbin, thresholds, b, keep


def _generic_path(idx, val, F, max_bins, all_gather):
    dev = idx.device
    keep = val != 0
    keys = (idx[keep] << 32) | _ordered_f32_bits(val[keep])
    uk, inv, cnt = torch.unique(keys, return_inverse=True, return_counts=True)
    if all_gather is not None:
        allk, allc = all_gather(uk, cnt)
        gk, ginv = torch.unique(allk, return_inverse=True)
        gc = torch.zeros(gk.numel(), dtype=torch.int64, device=dev).index_add_(0, ginv, allc)
        local_to_global = torch.searchsorted(gk, uk)
        inv = local_to_global[inv]
        uk, cnt = gk, gc
    ufeat = uk >> 32
    uval = _decode_f32_bits(uk & 0xFFFFFFFF)
    U = uk.numel()
    # per-feature segments of the sorted distinct keys
    fcnt = torch.bincount(ufeat, minlength=F)
    active = fcnt > 0
    remap = torch.full((F,), -1, dtype=torch.int64, device=dev)
    Fa = int(active.sum())
    remap[active] = torch.arange(Fa, device=dev)
    seg = remap[ufeat]
    nd = fcnt[active]                                          # distinct nonzero values per feature
    seg_start = torch.cumsum(nd, 0) - nd
    rank = torch.arange(U, device=dev) - seg_start[seg]
    # equal-count grouping for features with too many distinct values
    ccum = torch.cumsum(cnt, 0)
    seg_tot = torch.zeros(Fa, dtype=torch.int64, device=dev).index_add_(0, seg, cnt)
    seg_cstart = torch.zeros(Fa, dtype=torch.int64, device=dev)
    seg_cstart[1:] = torch.cumsum(seg_tot, 0)[:-1]
    before = ccum - cnt - seg_cstart[seg]
    slots = max_bins - 1
    grp = torch.where(nd[seg] <= slots, rank,
                      (before.to(torch.float64) * slots / seg_tot[seg].to(torch.float64)).to(torch.int64))
    # compact group ids per feature (monotone, may have gaps)
    key2 = seg * (1 << 20) + grp
    ug, ginv2 = torch.unique(key2, return_inverse=True)
    gseg = ug >> 20
    gcnt = torch.bincount(gseg, minlength=Fa)
    gstart = torch.cumsum(gcnt, 0) - gcnt
    grank = torch.arange(ug.numel(), device=dev) - gstart[gseg]
    # zero bin goes before the first positive group
    negg = torch.zeros(ug.numel(), dtype=torch.bool, device=dev)
    gmin = torch.full((ug.numel(),), float("inf"), dtype=torch.float64, device=dev)
    gmax = torch.full((ug.numel(),), float("-inf"), dtype=torch.float64, device=dev)
    gmin.scatter_reduce_(0, ginv2, uval, reduce="amin")
    gmax.scatter_reduce_(0, ginv2, uval, reduce="amax")
    negg = gmax < 0
    zb = torch.zeros(Fa, dtype=torch.int64, device=dev).index_add_(0, gseg, negg.to(torch.int64))
    gbin = grank + torch.where(negg, torch.zeros_like(grank), torch.ones_like(grank))
    nbins = (gcnt + 1).to(torch.int32)
    # bin value ranges (with the zero bin) -> midpoint thresholds
    nb = nbins.to(torch.int64)
    TB = int(nb.sum())
    boff = torch.cumsum(nb, 0) - nb
    bmin = torch.zeros(TB, dtype=torch.float64, device=dev)
    bmax = torch.zeros(TB, dtype=torch.float64, device=dev)
    gpos = boff[gseg] + gbin
    bmin[gpos] = gmin
    bmax[gpos] = gmax
    nxt = torch.roll(bmin, -1)
    thresholds = ((bmax + nxt) / 2.0).cpu().numpy()
    entry_group = ginv2[inv]
    entry_bin = gbin[entry_group]
    full_keep = keep.clone()
    eb = torch.zeros(idx.numel(), dtype=torch.int64, device=dev)
    eb[keep] = entry_bin
    return remap, nbins, zb.to(torch.int32), thresholds, eb, full_keep


ROW_BLOCK = int(os.environ.get("FDX_ROW_BLOCK", 1 << 17))   # rows per XCD row block: 1 B slot + 8 B statistics per row ~ 1.1 MB
SPLIT_MIN = int(os.environ.get("FDX_SPLIT_MIN", 1 << 13))   # columns with fewer entries stay whole (their gathers are few)


def _segments(colptr: torch.Tensor, csc_row: torch.Tensor, n_rows: int, row_block: int = ROW_BLOCK,
              split_min: int = SPLIT_MIN):
    """(start, end, feature, row block) of every column segment: columns with >= SPLIT_MIN entries
    are cut where the row block changes (rows are sorted inside a column, so a block's entries are
    contiguous); smaller columns are one segment with block -1."""
    dev = colptr.device
    Fa = colptr.numel() - 1
    n = colptr[1:] - colptr[:-1]
    nonempty = torch.nonzero(n > 0).flatten()
    starts = colptr[:-1][nonempty]
    feats = nonempty
    nblk = (n_rows + row_block - 1) // row_block
    split_cols = torch.nonzero(n >= split_min).flatten().to(torch.int32) if nblk > 1 else None
    if split_cols is not None and split_cols.numel():
        from ..ops import native

        S = int(split_cols.numel())
        bounds = torch.empty((S, nblk + 1), dtype=torch.int64, device=dev)
        native.lib().block_bounds(csc_row, colptr, split_cols, int(nblk), int(row_block), bounds)
        bounds[:, -1] = colptr[split_cols.to(torch.int64) + 1]
        b_start, b_end = bounds[:, :-1].reshape(-1), bounds[:, 1:].reshape(-1)
        b_feat = split_cols.to(torch.int64).repeat_interleave(nblk)
        b_blk = torch.arange(nblk, device=dev, dtype=torch.int64).repeat(S)
        ne = b_end > b_start
        unsplit = (n > 0) & (n < split_min)
        u_feat = torch.nonzero(unsplit).flatten()
        starts = torch.cat([colptr[:-1][u_feat], b_start[ne]])
        feats = torch.cat([u_feat, b_feat[ne]])
        seg_blk = torch.cat([torch.full_like(u_feat, -1), b_blk[ne]])
        starts, o = torch.sort(starts, stable=True)
        feats, seg_blk = feats[o], seg_blk[o]
    else:
        seg_blk = torch.full_like(starts, -1)
    ends = colptr[feats + 1]
    if starts.numel() > 1:
        nxt = starts[1:]
        same = feats[1:] == feats[:-1]
        ends = ends.clone()
        ends[:-1] = torch.where(same, nxt, ends[:-1])
    return starts, ends, feats, seg_blk


def _make_groups(colptr: torch.Tensor, nbins: torch.Tensor, chunk: int, csc_row: Optional[torch.Tensor] = None,
                 n_rows: int = 0, row_block: int = ROW_BLOCK, split_min: int = SPLIT_MIN) -> list:
    dev = colptr.device
    if csc_row is None:
        csc_row = torch.zeros(0, dtype=torch.int32, device=dev)
    s0, e0, f0, b0 = _segments(colptr, csc_row, n_rows, row_block, split_min)
    groups = []
    for bt in (0, 1, 2):    # 0: <= 16 bins (16x16x32 MFMA tile), 1: <= 32, 2: <= 64 bins
        lo, hi = ((0, 16), (17, 32), (33, 64))[bt]
        sel = (nbins[f0] >= lo) & (nbins[f0] <= hi)
        if not bool(sel.any()):
            continue
        s, e, f, b = s0[sel], e0[sel], f0[sel], b0[sel]
        nc = (e - s + chunk - 1) // chunk
        I = int(nc.sum())
        seg = torch.repeat_interleave(torch.arange(s.numel(), device=dev), nc, output_size=I)
        first = torch.cumsum(nc, 0) - nc
        k = torch.arange(I, device=dev) - first[seg]
        start = s[seg] + k * chunk
        end = torch.minimum(start + chunk, e[seg])
        item_feat = f[seg]
        feats, nitems = torch.unique_consecutive(item_feat, return_counts=True)
        item0 = torch.cumsum(nitems, 0) - nitems
        groups.append(BinGroup(bt, start.contiguous(), end.contiguous(), item_feat.to(torch.int32).contiguous(),
                               feats.to(torch.int32).contiguous(), item0.contiguous(),
                               nitems.to(torch.int32).contiguous(), b[seg].to(torch.int32).contiguous()))
    return groups
