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
values with either ``x <= t`` (Spark) or ``x < t`` (XGBoost) semantics.

Histogram layout (``_finish_items``): features present in >= HOT_DENSITY of the rows go to a
dense column-major bin block (their row state is streamed, not gathered; used for the shallow
levels where most rows are live). All features' entries are copied into a histogram CSC laid out
row-super-block-major (super-block = a range of
rows whose 1-byte slot and 8-byte digit slices fit one XCD's 4 MB L2; the XCD-ordered item
placement keeps each XCD inside one super-block at a time), as (row, key) with key = kbase + bin.
One wave of the i8 MFMA histogram kernel per work item: a chunk of one feature inside one
super-block, or several consecutive small features packed into one 64-key tile (``stride`` keys
per feature, kbase = position * stride), so the ~28K small text features do not each cost a wave. Under data parallelism
the per-rank statistics (max counts / distinct values) are merged with collectives so every rank
holds identical bins.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import torch

from ..ops import native
from ..utils import tracing
from ..utils.memory import RG_GROUP_MAX_ENTRIES

CSC_PAD = 16

# entries per histogram work item (one wavefront); 0: by the row count. A wave walks its item
# serially (the pass ends with its longest wave): RF 500 x depth 5 on a 1.25M-row shard 0.46 ->
# 0.41 s with 4K-entry items, on 10M rows 0.76 -> 0.72 s with 16K (profiles/r5/rf_chunk_sweep_*.jsonl)
CHUNK = int(os.environ.get("FDX_HIST_CHUNK", 0))


def default_chunk(n_rows: int) -> int:
    return CHUNK or (16384 if n_rows >= 4_000_000 else 4096)
# A work item's int32 MFMA accumulators gain at most 128 * 128 = 2^14 per entry, so one item may
# hold at most this many entries before a (key, column) sum could overflow (csrc/tree_kernels.hip)
MAX_ITEM_ENTRIES = (1 << 31) // (1 << 14) - 1
PACK_KEYS = 16   # keys of a packed multi-feature item (16 = one MFMA row tile)


@dataclass
class ItemGroup:
    """Work items of one MFMA row-tile count ``bt`` (16 * bt keys per item): a chunk of one
    feature (``meta`` stride 256, nfeat 1; ``koff`` windows for features with > 64 bins) or
    several whole small features packed into one tile."""
    bt: int
    item_start: torch.Tensor     # int64 [I]
    item_end: torch.Tensor       # int64 [I]
    item_f0: torch.Tensor        # int32 [I] first feature of the item
    item_meta: torch.Tensor      # int32 [I] stride_log2 | nfeat << 8 | koff << 16 (csrc/tree.h)
    item_blk: Optional[torch.Tensor] = None   # int32 [I] row block of the item (-1: whole column)
    _order: Optional[torch.Tensor] = None

    def subset(self, feat_mask: torch.Tensor) -> "ItemGroup":
        """Items with at least one feature in ``feat_mask`` (RF per-level feature union)."""
        cs = torch.zeros(feat_mask.numel() + 1, dtype=torch.int64, device=feat_mask.device)
        torch.cumsum(feat_mask.to(torch.int64), 0, out=cs[1:])
        f0 = self.item_f0.to(torch.int64)
        nf = (self.item_meta.to(torch.int64) >> 8) & 0xFF
        keep = (cs[f0 + nf] - cs[f0]) > 0
        blk = self.item_blk[keep] if self.item_blk is not None else None
        return ItemGroup(self.bt, self.item_start[keep], self.item_end[keep], self.item_f0[keep],
                         self.item_meta[keep], blk)

    @property
    def num_items(self) -> int:
        return int(self.item_start.numel())

    def wave_order(self) -> torch.Tensor:
        """Item of every wave slot of the histogram launches (-1: idle)."""
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


RG_BINS = int(os.environ.get("FDX_RG_BINS", 8192))   # local bins per row group: 8192 (1 workgroup per CU) or 4096 (2)
RG_MAX_GROUPS = 128
# workgroups per row-group pass: few and large -- every workgroup zeroes and flushes a whole
# 8192-bin table (up to 2 x 8192 int64 global atomics per slot it covers). 10M rows x 40 trees:
# 7.69 ms per tree at 2048, 6.19 at 512 (profiles/r4/gbdt_rg_work_sweep.txt); 1M rows x 100
# trees: 1.95 ms at 512, 1.67 at 256, 1.79 at 128 (profiles/r4/gbdt_1M_rg_wgs_sweep.txt). Since
# every pass stores per-workgroup tables instead (RgHistArgs part), more workgroups pay off: 1M rows
# fit 0.142 s at 128, 0.124 at 192, 0.116 at 256, 0.1145 at 384, 0.117 at 512; 10M rows 6.48 ms a
# tree at 512, 6.96 at 768, 6.68 at 1024 (profiles/r5/gbdt_rg_wgs_sweep_partials.txt). Default
# (FDX_RG_WGS unset): rows / 2731, in [128, 512], a multiple of 64.
RG_TARGET_WGS = int(os.environ.get("FDX_RG_WGS", 0))
# workgroups of the listed (level >= 1) passes, which cover fewer rows than the root's: 1M rows
# fit 0.1146 s at 384 (the root's), 0.1105-0.1114 at 256, 0.112 at 192, 0.120 at 128; 10M rows
# 6.40-6.45 ms a tree at 512 (the root's), 6.53-6.61 at 384 (profiles/r5/gbdt_rg_list_wgs_sweep.txt).
# Default (FDX_RG_LIST_WGS unset): rows / 4096, in [128, 512], a multiple of 64.
RG_LIST_WGS = int(os.environ.get("FDX_RG_LIST_WGS", 0))


def rg_default_wgs(n_rows: int) -> int:
    """Workgroups of a row-group pass over ``n_rows`` rows (see RG_TARGET_WGS)."""
    return int(min(512, max(128, round(n_rows * 1.5 / 4096 / 64) * 64)))


def rg_list_default_wgs(n_rows: int) -> int:
    """Workgroups of a listed (level >= 1) row-group pass (see RG_LIST_WGS)."""
    return int(min(512, max(128, round(n_rows / 4096 / 64) * 64)))
# work model of a (group, chunk) workgroup: cost ~ RG_ALPHA * rows + entries (a row costs its
# (ptr, digits) loads whether or not it has entries in the group)
RG_ALPHA = float(os.environ.get("FDX_RG_ALPHA", 16.0))
# groups with at least this many entries per row take lane-balanced batches (csrc/row_kernels.hip
# rg_batch); sparser ones a lane per row
RG_BAL_MIN = 8.0
# the sparse groups (gmode 0) also get a row per entry (4 B) for the entry-major pass of
# single-slot levels (csrc/row_kernels.hip rg_range_em); a listed level takes it when it lists at
# least RG_EM_MIN_FRAC of the rows (> 1: never). Bench corpus, half the rows listed: sparse groups
# 0.75 -> 0.48 ms; GBDT 10M x 40 trees 6.35 -> 6.28-6.32 ms per tree (profiles/r4)
RG_EM = True
RG_EM_MIN_FRAC = float(os.environ.get("FDX_RG_EM_MIN_FRAC", 0.3))


class _Ticker:
    """Device-synchronised phase timer (FDX_RG_TIMING=1)."""

    def __init__(self, dev, out: dict):
        import time as _t
        self._t, self.dev, self.out = _t, dev, out
        self._sync()
        self.t0 = _t.perf_counter()

    def _sync(self):
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def __call__(self, name: str) -> bool:
        self._sync()
        t = self._t.perf_counter()
        self.out[name] = round((t - self.t0) * 1e3, 2)
        self.t0 = t
        return True


class RowGroups:
    """Row-group CSR of the active features (csrc/tree.h "row-group histogram engine").

    Features are packed densest first into groups of at most ``RG_BINS`` local bins (a feature's
    bins contiguous); for group g the entries of row r are ``ent[gbase[g] + ptr[g, r] : gbase[g] +
    ptr[g, r + 1]]`` as uint16 local bins, and ``gbin[g, b]`` is the global histogram column of
    local bin b. Built on the device from the quantized CSC in two passes (count, place):
    4 B per (group, row) plus 2 B per entry. ``complete`` is False when the features with entries
    need more than ``RG_MAX_GROUPS`` groups (very wide vocabularies): the grower then keeps the
    CSC passes."""

    def __init__(self, Q: "Quantized", max_groups: int = None, bins: int = None, max_group_entries: int = None):
        C = native.lib()
        dev = Q.device
        self.timing: dict = {}
        tick = _Ticker(dev, self.timing) if os.environ.get("FDX_RG_TIMING") == "1" else None
        max_groups = RG_MAX_GROUPS if max_groups is None else max_groups
        self.bins = B = RG_BINS if bins is None else bins
        if B not in (4096, 8192):
            raise ValueError("row groups hold 4096 or 8192 bins")
        colptr = Q.colptr.cpu().numpy()
        cnt = np.diff(colptr)
        nb = Q.nbins.cpu().numpy().astype(np.int64)
        boff = np.asarray(Q.boff_host, dtype=np.int64)
        Fa = int(nb.size)
        tick and tick("d2h")
        order = np.argsort(-cnt, kind="stable")
        order = order[cnt[order] > 0]
        cum = np.concatenate([[0], np.cumsum(nb[order])])
        # a group's entry offsets are uint32 (ptr): a group closes before RG_GROUP_MAX_ENTRIES
        # entries, so a large shard gets more groups instead of a row limit (utils/memory.py)
        cum_e = np.concatenate([[0], np.cumsum(cnt[order])])
        cap_e = RG_GROUP_MAX_ENTRIES if max_group_entries is None else int(max_group_entries)
        fgroup = np.full(Fa, -1, dtype=np.int32)
        flocal = np.zeros(Fa, dtype=np.int32)
        starts = []
        i = 0
        while i < order.size and len(starts) < max_groups:
            j = int(np.searchsorted(cum, cum[i] + B, side="right")) - 1     # features [i, j) fit
            j = min(j, int(np.searchsorted(cum_e, cum_e[i] + cap_e, side="right")) - 1)
            j = max(j, i + 1)
            fs = order[i:j]
            fgroup[fs] = len(starts)
            flocal[fs] = (cum[i:j] - cum[i]).astype(np.int32)
            starts.append(i)
            i = j
        tick and tick("pack")
        self.complete = i >= order.size
        self.G = G = max(1, len(starts))
        self.n_rows = N = Q.n_rows
        # global column of every local bin
        gbin = np.full((G, B), -1, dtype=np.int32)
        sel = np.nonzero(fgroup >= 0)[0]
        if sel.size:
            rep = nb[sel]
            f_rep = np.repeat(sel, rep)
            k = np.arange(int(rep.sum()), dtype=np.int64) - np.repeat(np.cumsum(rep) - rep, rep)
            gbin[fgroup[f_rep], flocal[f_rep] + k] = (boff[f_rep] + k).astype(np.int32)
        tick and tick("gbin")
        egroup = np.zeros(G, dtype=np.int64)
        np.add.at(egroup, fgroup[sel], cnt[sel])
        if int(egroup.max(initial=0)) > RG_GROUP_MAX_ENTRIES:      # (one feature alone: > 2^31 rows)
            raise ValueError("row group over 2^31 - 1 entries: shard the rows over more ranks")
        pad = (egroup + 7) // 8 * 8                   # 16-byte aligned group starts
        gbase = np.concatenate([[0], np.cumsum(pad)]).astype(np.int64)
        self.entries = int(egroup.sum())
        self.group_entries = egroup
        gmode = (egroup >= RG_BAL_MIN * max(N, 1)).astype(np.uint8)
        self.gmode = torch.from_numpy(gmode).to(dev)
        self.fgroup_host, self.flocal_host = fgroup, flocal
        tick and tick("egroup")
        fg_t = torch.from_numpy(fgroup).to(dev)
        fl_t = torch.from_numpy(flocal).to(dev)
        self.gbase = torch.from_numpy(gbase).to(dev)
        self.gbin = torch.from_numpy(gbin).to(dev)
        tick and tick("plan")
        ptr = torch.empty((G, N + 1), dtype=torch.int32, device=dev) if N else torch.zeros((G, 1), dtype=torch.int32,
                                                                                            device=dev)
        # readable padding behind the end: the pass loads aligned 8-entry blocks
        self.ent = torch.empty(int(gbase[-1]) + 16, dtype=torch.int16, device=dev)[:int(gbase[-1])]
        # entry-major rows of the sparse tail: groups em_g0.. (every group after the last dense one)
        dense = np.nonzero(gmode != 0)[0]
        self.em_g0 = int(dense[-1]) + 1 if dense.size else 0
        self.ebase = int(gbase[self.em_g0])
        self.erow = None
        if RG_EM and self.em_g0 < G and N and int(gbase[-1]) > self.ebase:
            self.erow = torch.empty(int(gbase[-1]) - self.ebase, dtype=torch.int32, device=dev)
        tick and tick("alloc")
        csr = getattr(Q, "csr_src", None)
        if csr is not None and G <= 128:
            # rows of the count-path CSR: a wave per row, runs in CSR order, no global atomics
            indptr, idx, counts, max_bins = csr
            remap = torch.full((Q.num_features,), -1, dtype=torch.int32, device=dev)
            remap[Q.fid_orig] = torch.arange(Q.Fa, dtype=torch.int32, device=dev)
            work = torch.empty(G * C.tree_rg_build_csr_waves(N), dtype=torch.int32, device=dev)
            C.tree_rg_build_csr(indptr, idx, counts, remap, max_bins - 1, fg_t, fl_t, ptr, self.gbase, self.ent,
                                work, self.erow, self.em_g0, self.ebase)      # (erow written in the pass)
            self.ptr = ptr
            del work
            tick and tick("build")
        else:
            ptr.zero_()
            C.tree_rg_build(Q.csc_row, Q.csc_bin, Q.colptr, fg_t, fl_t, N, 0, ptr, None, None, None)
            self.ptr = torch.cumsum(ptr, dim=1, dtype=torch.int32)
            del ptr
            cursor = self.ptr[:, :N].clone(memory_format=torch.contiguous_format)   # (a view when G == 1)
            C.tree_rg_build(Q.csc_row, Q.csc_bin, Q.colptr, fg_t, fl_t, N, 1, None, cursor, self.gbase, self.ent)
            del cursor
            if self.erow is not None:
                C.tree_rg_erow(self.ptr, self.gbase, self.em_g0, self.erow)
                tick and tick("erow")
        self._work: dict = {}

    def work(self, target_wgs: int = 0, alpha: float = None) -> torch.Tensor:
        """Work table [3, n_wg] int32 (group, chunk, chunks of that group): each group's list is cut
        into chunks in proportion to its modelled cost alpha * rows + entries, so every workgroup
        carries about 1/target_wgs of the pass (the densest group holds ~79% of the entries on the
        bench corpus, but every group pays for every listed row)."""
        target_wgs = target_wgs or RG_TARGET_WGS or rg_default_wgs(self.n_rows)
        alpha = RG_ALPHA if alpha is None else alpha
        key = (target_wgs, alpha)
        t = self._work.get(key)
        if t is None:
            e = self.group_entries.astype(np.float64) + alpha * self.n_rows
            npg = np.maximum(1, np.rint(target_wgs * e / max(e.sum(), 1.0))).astype(np.int64)
            g = np.repeat(np.arange(self.G), npg)
            p = np.arange(int(npg.sum())) - np.repeat(np.cumsum(npg) - npg, npg)
            tab = np.stack([g, p, np.repeat(npg, npg)]).astype(np.int32)
            assert (tab[0] < self.G).all() and (tab[1] < tab[2]).all()
            t = self._work[key] = torch.from_numpy(tab).to(self.gbase.device)
        return t

    def list_work(self) -> torch.Tensor:
        """The work table of the listed (level >= 1) passes (RG_LIST_WGS)."""
        return self.work(RG_LIST_WGS or rg_list_default_wgs(self.n_rows))

    def list_work_first(self) -> torch.Tensor:
        return self.work_first(RG_LIST_WGS or rg_list_default_wgs(self.n_rows))

    def work_first(self, target_wgs: int = 0, alpha: float = None) -> torch.Tensor:
        """[G + 1] int32: the first work-table entry of each group (work() lists a group's chunks
        consecutively), for the reduction of a single-slot pass's partial tables."""
        tab = self.work(target_wgs, alpha)
        key = ("first", tab.data_ptr())
        t = self._work.get(key)
        if t is None:
            cnt = torch.bincount(tab[0].long(), minlength=self.G)
            t = self._work[key] = torch.cat([cnt.new_zeros(1), torch.cumsum(cnt, 0)]).to(torch.int32)
        return t

    @property
    def nbytes(self) -> int:
        em = self.erow.numel() * 4 if self.erow is not None else 0
        return int(self.ptr.numel() * 4 + self.ent.numel() * 2 + self.gbin.numel() * 4 + em)

    def em_args(self, emdig=None) -> dict:
        """Keyword arguments of tree_rg_hist for the entry-major sparse pass (empty: off). A listed
        single-slot level passes ``emdig``, the digit words zeroed outside its slot (tree_rg_list
        ``masked``), and takes the pass when it lists >= RG_EM_MIN_FRAC of the rows."""
        if self.erow is None:
            return {}
        kw = dict(erow=self.erow, ebase=self.ebase)
        if emdig is not None:
            kw.update(emdig=emdig, em_min_rows=max(1, int(RG_EM_MIN_FRAC * self.n_rows)))
        return kw


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
    # the CSC passes' histogram CSC and work items (built on first use: the row-group engine of
    # GBDT never reads them) -- see the properties below
    _kbase: torch.Tensor = None  # int32 [Fa] key base of each feature in its packed work item
    _groups: list = field(default_factory=list)
    _hot_groups: list = field(default_factory=list)  # CSC items of the dense-block features
    _h_row: torch.Tensor = None  # int32: histogram CSC (all features, super-block-major)
    _h_key: torch.Tensor = None  # uint8: kbase[f] + bin
    _n_super: int = 1            # row super-blocks of the histogram CSC
    # dense path for high-density features (K-10 dense variant): dense[d][row] = bin of feature
    # hot[d] (its zero bin when absent), rows padded to n_pad (multiple of 64)
    hot: np.ndarray = None       # int64 [Fh] Fa indices
    hot_bt: np.ndarray = None    # int64 [Fh] MFMA row tiles (16 bins each) of each hot feature
    dense: torch.Tensor = None   # uint8 [Fh, n_pad]
    boff_host: np.ndarray = None
    zbin_host: np.ndarray = None
    fid_host: np.ndarray = None
    _kbase_host: np.ndarray = None
    row0: int = 0                # global index of row 0 (data-parallel shards; bootstrap draws)

    @property
    def Fa(self) -> int:  # noqa: N802
        return int(self.nbins.numel())

    def _items(self) -> "Quantized":
        pend = getattr(self, "_items_pending", None)
        if pend is not None:
            self._items_pending = None
            with tracing.span("q.items"):
                _build_items(self, *pend)
        return self

    groups = property(lambda self: self._items()._groups)
    hot_groups = property(lambda self: self._items()._hot_groups)
    h_row = property(lambda self: self._items()._h_row)
    h_key = property(lambda self: self._items()._h_key)
    kbase = property(lambda self: self._items()._kbase)
    kbase_host = property(lambda self: self._items()._kbase_host)
    n_super = property(lambda self: self._items()._n_super)

    def rowgroups(self) -> RowGroups:
        """The row-group CSR of the row-group histogram engine (built on first use)."""
        r = getattr(self, "_rowgroups", None)
        if r is None:
            with tracing.span("q.rowgroups"):
                r = self._rowgroups = RowGroups(self)
        return r

    @property
    def n_pad(self) -> int:
        return (self.n_rows + 63) // 64 * 64

    @property
    def TB(self) -> int:  # noqa: N802
        return int(self.boff_host[-1])

    @property
    def device(self) -> torch.device:
        return self.csc_row.device

    def threshold(self, fid: int, b: int) -> float:
        return float(self.thresholds[int(self.boff_host[fid]) + int(b)])

    def bins_of(self, fid: int) -> torch.Tensor:
        """Bins of the entries of feature ``fid`` (feature-major CSC order)."""
        a, b = int(self.colptr[fid]), int(self.colptr[fid + 1])
        return self.csc_bin[a:b]


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
             chunk: int = None, super_rows: int = None, hot_density: float = None) -> Quantized:
    """Bin a ``VectorColumn`` and build the CSC. ``counts``/``scale`` select the count path
    (per-entry integer counts and per-feature positive scale); integral non-negative values
    take it automatically with scale 1."""
    if max_bins < 2 or max_bins > 256:
        raise ValueError("max_bins must be in [2, 256] (bins are one byte)")
    if counts is not None and vc.dense is None:
        indptr, idx, val = vc.indptr, vc.indices, None      # count path: the fp64 values are never read
    else:
        indptr, idx, val = vc.csr()
    dev = indptr.device
    N = int(indptr.numel() - 1)
    F = int(vc.size)
    chunk = chunk or default_chunk(N)       # (read at call time: experiments set the module value)
    val64 = val.to(torch.float64) if val is not None else None
    if counts is None and val64.numel() and bool(torch.all(val64 >= 0)) and bool(torch.all(val64 == torch.round(val64))) \
            and float(val64.max()) < 65536:
        counts = val64
        scale = torch.ones(F, dtype=torch.float64, device=dev)
    if counts is not None and F < (1 << 31):
        Q = _quantize_counts(vc, indptr, idx, counts, scale, N, F, max_bins, all_reduce_max)
        if idx.dtype == torch.int32 and counts.dtype in (torch.float32, torch.float64, torch.int32):
            Q.csr_src = (indptr, idx, counts, max_bins)     # (references) the row-group build reads rows
        with tracing.span("q.dense_block"):
            _finish_items(Q, chunk, super_rows or SUPER_ROWS, HOT_DENSITY if hot_density is None else hot_density)
        return Q
    idx64 = idx.to(torch.int64)      # generic path only (8 B per entry: never on the count path)
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
    with tracing.span("q.dense_block"):
        _finish_items(Q, chunk, super_rows or SUPER_ROWS, HOT_DENSITY if hot_density is None else hot_density)
    return Q


def _quantize_counts(vc, indptr, idx, counts, scale, N, F, max_bins, all_reduce_max) -> "Quantized":
    """Count path on the native feature-major order (sort_kernels.hip): bins = min(count,
    max_bins - 1) with thresholds (k + 0.5) * scale_f; the CSC comes straight from the radix sort
    (cached on the VectorColumn as ``_feature_order`` when the caller already built it for IDF)."""
    from ..ops.sparse import feature_order

    dev = indptr.device
    fo = getattr(vc, "_feature_order", None)
    scale = scale.to(device=dev, dtype=torch.float64)
    if fo is not None and fo.dropped is not None and bool((fo.dropped & (scale > 0)).any()):
        fo = None                        # (dropped columns are needed again: a fresh order)
    if fo is None or fo.colptr.numel() != F + 1 or fo.csc_row.device != dev:
        with tracing.span("q.order"):
            fo = feature_order(indptr, idx, counts, F)
    sp_h = tracing.span("q.head")
    sp_h.__enter__()
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
    if fo.dropped is not None and bool(((~active) & (lens > 0)).any()):
        # the order was already compacted in place for an earlier quantisation whose CSC may still
        # alias it: a larger drop set gets an order of its own instead of sliding entries under it
        with tracing.span("q.order"):
            fo = feature_order(indptr, idx, counts, F)
        lens = fo.colptr[1:] - fo.colptr[:-1]
    if bool(((~active) & (lens > 0)).any()):
        # the inactive features' entries (all-zero values: IDF 0 for terms in every document)
        # leave the shared feature order in place, so the order stays the CSC (no 5 B/entry copy)
        with tracing.span("q.drop"):
            fo.drop_features((~active) & (lens > 0))
        lens = fo.colptr[1:] - fo.colptr[:-1]
    nnz_all = int(fo.colptr[-1])
    sp_h.__exit__(None, None, None)
    with tracing.span("q.csc"):
        if int(lens[~active].sum()) == 0:        # every non-empty feature is active: the order is the CSC
            csc_row = fo.csc_row
            cnt = fo.csc_cnt
            colptr = torch.zeros(Fa + 1, dtype=torch.int64, device=dev)
            if Fa:
                colptr[:-1] = fo.colptr[:-1][active]
                colptr[-1] = fo.colptr[1:][active][-1]
        else:                                     # drop the entries of inactive features (scale 0)
            colptr = torch.zeros(Fa + 1, dtype=torch.int64, device=dev)
            torch.cumsum(lens[active], 0, out=colptr[1:])
            n_keep = int(colptr[-1])
            row_buf = torch.zeros(n_keep + CSC_PAD, dtype=torch.int32, device=dev)
            csc_row = row_buf[:n_keep]
            cnt = None
        n = int(csc_row.numel())
        bin_buf = torch.full((n + CSC_PAD,), 0xFF, dtype=torch.uint8, device=dev)
        if cnt is not None:
            if cnt.is_cuda and cnt.data_ptr() % 16:           # realign for the native clamp
                cnt = cnt.clone()
            native.lib().clamp_u8(cnt.contiguous(), max_bins - 1, bin_buf[:n])
        else:
            # bins of every entry in feature order, then one segment copy of the active features'
            # (row, bin) ranges (instead of a boolean mask over all nnz entries)
            full_bin = torch.empty(nnz_all + CSC_PAD, dtype=torch.uint8, device=dev)
            native.lib().clamp_u8(fo.csc_cnt[:nnz_all].contiguous(), max_bins - 1, full_bin[:nnz_all])
            if Fa:
                native.lib().copy_segments(fo.csc_row[:nnz_all], full_bin[:nnz_all], fo.colptr[:-1][active].contiguous(),
                                           colptr[:-1].contiguous(), lens[active].contiguous(), csc_row, bin_buf[:n],
                                           None)
            del full_bin
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


HOT_DENSITY = 0.1  # dense path for features in >= this fraction of rows


def _pow2_at_least(x: np.ndarray, lo: int = 1) -> np.ndarray:
    out = np.full(x.shape, lo, dtype=np.int64)
    while True:
        small = out < x
        if not small.any():
            return out
        out[small] *= 2


def _build_dense(Q: Quantized, hot: np.ndarray) -> None:
    """Column-major dense bins of the hot features (zero bin for rows absent from a column)."""
    Q.hot = hot.astype(np.int64)
    nb = Q.nbins.cpu().numpy()[Q.hot]
    Q.hot_bt = np.where(nb <= 16, 1, np.where(nb <= 32, 2, 4)).astype(np.int64)
    if not hot.size:
        Q.dense = None
        return
    dev = Q.device
    hot_t = torch.from_numpy(Q.hot).to(dev)
    # every column filled with its zero bin, then the hot features' CSC entries scattered: two
    # launches (a fill + index_copy per feature was ~290 launches, ~2 ms a fit)
    dense = Q.zbin[hot_t].to(torch.uint8)[:, None].expand(hot.size, Q.n_pad).contiguous()
    colptr = Q.colptr.cpu().numpy()
    seg_src = torch.from_numpy(colptr[Q.hot]).to(dev)
    lens = colptr[Q.hot + 1] - colptr[Q.hot]
    native.lib().dense_scatter(Q.csc_row, Q.csc_bin, seg_src, torch.from_numpy(lens).to(dev), dense, int(lens.max()))
    Q.dense = dense


COPY_PIECE = 8192      # entries per workgroup of the histogram CSC copy
LIGHT_ENTRIES = 0    # whole-column items up to this many entries (0: off; profiles/r4/rf500_light_entries_sweep.txt)
SUPER_ROWS = int(os.environ.get("FDX_SUPER_ROWS", 1 << 18))  # rows per super-block: 256 KB slots + 2 MB digits


def _split_items(st: torch.Tensor, en: torch.Tensor, per: torch.Tensor, blk: torch.Tensor, chunk: int) -> torch.Tensor:
    """Entry ranges [st, en) -> consecutive pieces of <= ``chunk`` entries, as item rows
    (start, end, *per, blk) -- per: [m, 5] (f0, sl2, nfeat, koff, bt) or [m, 1] (f0 only); item
    sums are order-free, so any split gives the same histogram. On the ranges' device."""
    nc = (en - st + chunk - 1) // chunk
    total = int(nc.sum())
    rep = torch.repeat_interleave(torch.arange(st.numel(), device=st.device), nc, output_size=total)
    k = torch.arange(total, device=st.device) - (torch.cumsum(nc, 0) - nc)[rep]
    s0 = st[rep] + k * chunk
    e0 = torch.minimum(s0 + chunk, en[rep])
    return torch.cat([s0[:, None], e0[:, None], per[rep], blk[rep][:, None]], 1)


def _finish_items(Q: Quantized, chunk: int = 0, super_rows: int = SUPER_ROWS, hot_density: float = HOT_DENSITY) \
        -> None:
    """Dense block now; histogram CSC and work items on first use (see the module docstring).

    * hot: features in >= ``hot_density`` of the rows with <= 64 bins -> dense block;
    * packed: consecutive features with <= 16 bins and few entries (<= ``chunk`` per super-block on
      average) share one <= 64-key item per super-block (stride = the largest pow2 bin count);
    * single: every other feature, per super-block, in chunks of <= ``chunk`` entries; features
      with > 64 bins get one item per 64-key window."""
    if not 0 < chunk <= MAX_ITEM_ENTRIES:
        raise ValueError(f"FDX_HIST_CHUNK must be in [1, {MAX_ITEM_ENTRIES}] (int32 MFMA accumulators)")
    colptr = Q.colptr.cpu().numpy().astype(np.int64)
    n = np.diff(colptr)
    nb = Q.nbins.cpu().numpy().astype(np.int64)
    Fa = int(nb.size)
    hot = (n >= hot_density * max(Q.n_rows, 1)) & (nb <= 64) & (n > 0) if hot_density > 0 else np.zeros(Fa, bool)
    with tracing.span("q.dense"):
        _build_dense(Q, np.nonzero(hot)[0])
    Q._items_pending = (chunk, super_rows, hot)


class _Checkpoints:
    """FDX_ITEMS_TIMING=1: synchronised wall time between named points of _build_items, printed
    once at its end (diagnostics: bench/probes/items_profile.py)."""

    def __init__(self):
        self.on = os.environ.get("FDX_ITEMS_TIMING") == "1"
        self.t = time.perf_counter()
        self.parts = []

    def __call__(self, name):
        if not self.on:
            return
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t = time.perf_counter()
        self.parts.append((name, round(1e3 * (t - self.t), 2)))
        self.t = t

    def report(self):
        if self.on:
            print("items timing (ms):", self.parts, flush=True)


def _build_items(Q: Quantized, chunk: int, super_rows: int, hot: np.ndarray) -> None:
    """The histogram CSC and work items of the CSC passes (first use of Q.groups & co.)."""
    from ..ops import native

    C = native.lib()
    dev = Q.device
    colptr = Q.colptr.cpu().numpy().astype(np.int64)
    ck = _Checkpoints()
    n = np.diff(colptr)
    nb = Q.nbins.cpu().numpy().astype(np.int64)
    Fa = int(nb.size)
    # hot features stay in the histogram CSC too (deep levels use it: only their live entries are
    # multiplied there, while the dense kernel masks every row); they are never packed
    cols = np.nonzero(n > 0)[0]
    ck("host_cols")
    sp_b = tracing.span("q.bounds")
    sp_b.__enter__()
    nsb = max(1, (Q.n_rows + super_rows - 1) // super_rows)
    sb_rows = (Q.n_rows + nsb - 1) // nsb if Q.n_rows else 1
    # --- per (super-block, feature) segments of the feature-major CSC and their new offsets
    S = int(cols.size)
    # light features (columns of <= LIGHT_ENTRIES entries) keep their whole column in row block 0:
    # one item per column instead of one per row block, so a sampled RF pass launches fewer
    # (mostly idle) wave slots; their entries are thousands of rows apart, so the row-block
    # locality that the heavy columns need buys them nothing
    ncol_all = n[cols]
    light = (ncol_all <= LIGHT_ENTRIES) & ~hot[cols] if LIGHT_ENTRIES > 0 else np.zeros(cols.size, bool)
    if S:
        cols_t = torch.from_numpy(cols.astype(np.int32)).to(dev)
        bounds = torch.empty((S, nsb + 1), dtype=torch.int64, device=dev)
        with tracing.span("q.bsearch"):
            C.block_bounds(Q.csc_row, Q.colptr, cols_t, int(nsb), int(sb_rows), bounds)
        ck("bsearch")
        bounds[:, -1] = Q.colptr[cols_t.to(torch.int64) + 1]
        if light.any() and nsb > 1:
            li = torch.from_numpy(np.nonzero(light)[0]).to(dev)
            bounds[li, 1:nsb] = bounds[li, nsb:nsb + 1]           # every entry in row block 0
        seg_src = bounds[:, :-1].t().contiguous()                    # [nsb, S]
        seg_len = (bounds[:, 1:] - bounds[:, :-1]).t().contiguous()
        flat = seg_len.reshape(-1)
        seg_dst = torch.cumsum(flat, 0) - flat
        total = int(flat.sum())
        ck("segments")
        with tracing.span("q.alloc"):
            h_row = torch.zeros(total + CSC_PAD, dtype=torch.int32, device=dev)
            h_key = torch.full((total + CSC_PAD,), 0xFF, dtype=torch.uint8, device=dev)
        ck("alloc")
        # [sb][i] start of cols[i] in super-block sb (on the device: the item table is built there,
        # no [nsb, S] host copies -- fresh host arrays of that size cost ~100 ms of page faults in
        # a process's first fit, profiles/r5/NOTES.md)
        hptr = torch.empty((nsb, S + 1), dtype=torch.int64, device=dev)
        hptr[:, :S] = seg_dst.view(nsb, S)
        if nsb > 1:
            hptr[:-1, S] = hptr[1:, 0]
        hptr[-1, S] = total
        seg_n = seg_len                                                 # [nsb, S]
    else:
        h_row = torch.zeros(CSC_PAD, dtype=torch.int32, device=dev)
        h_key = torch.full((CSC_PAD,), 0xFF, dtype=torch.uint8, device=dev)
        hptr = torch.zeros((nsb, 1), dtype=torch.int64, device=dev)
        seg_n = torch.zeros((nsb, 0), dtype=torch.int64, device=dev)
        total = 0
    sp_b.__exit__(None, None, None)
    ck("d2h_len")
    sp_p = tracing.span("q.pack")
    sp_p.__enter__()
    # --- packing (global: the same kbase in every super-block)
    ncol = n[cols]
    packable = (ncol <= chunk * nsb) & (nb[cols] <= 16) & ~hot[cols]
    stride = _pow2_at_least(nb[cols], 2)
    kbase = np.zeros(Fa, dtype=np.int64)
    # greedy runs of consecutive packable features (native: a Python loop over ~30K features cost
    # tens of ms): each run <= PACK_KEYS keys at the run's largest stride, <= chunk * nsb entries
    gp = native.lib().pack_runs(torch.from_numpy(packable.astype(np.uint8)), torch.from_numpy(stride.astype(np.int64)),
                                torch.from_numpy(ncol.astype(np.int64)), int(PACK_KEYS), int(chunk * nsb)).numpy()
    gp = np.asarray(gp, dtype=np.int64).reshape(-1, 3)
    if gp.shape[0]:       # kbase of feature j of a run = j << stride_log2 (vectorised over the runs)
        run_len = gp[:, 1] - gp[:, 0]
        pos = np.arange(int(run_len.sum())) - np.repeat(np.cumsum(run_len) - run_len, run_len)
        kbase[cols[np.repeat(gp[:, 0], run_len) + pos]] = pos << np.repeat(gp[:, 2], run_len)
    L = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.int64)).to(dev)   # noqa: E731
    sb_ids = torch.arange(nsb, dtype=torch.int64, device=dev)
    parts = []   # [m, 8] int64 (start, end, f0, sl2, nfeat, koff, bt, blk)
    if gp.shape[0]:
        i0s, i1s, sl2s = gp[:, 0], gp[:, 1], gp[:, 2]
        keys = (i1s - i0s) << sl2s
        bts = np.where(keys <= 16, 1, np.where(keys <= 32, 2, 4))
        G = gp.shape[0]
        st = hptr[:, L(i0s)].reshape(-1)                   # [nsb, G]: consecutive features are contiguous
        en = (hptr[:, L(i1s - 1)] + seg_n[:, L(i1s - 1)]).reshape(-1)
        per = torch.stack([L(cols[i0s]), L(sl2s), L(i1s - i0s), torch.zeros(G, dtype=torch.int64, device=dev),
                           L(bts)], 1).repeat(nsb, 1)      # [nsb * G, 5] (f0, sl2, nfeat, koff, bt)
        blk = sb_ids.repeat_interleave(G)
        keep = en > st
        parts.append(_split_items(st[keep], en[keep], per[keep], blk[keep], chunk))
    ck("pack_runs")
    single = np.nonzero(~packable)[0]
    if single.size:
        sg = L(single)
        st = hptr[:, sg].reshape(-1)                       # [nsb * len(single)]
        ln = seg_n[:, sg].reshape(-1)
        f_all = L(cols[single]).repeat(nsb)
        b_all = sb_ids.repeat_interleave(single.size)
        nbs = L(nb)
        keep = ln > 0
        one = torch.ones(1, dtype=torch.int64, device=dev)
        z = torch.zeros(1, dtype=torch.int64, device=dev)
        pieces = _split_items(st[keep], st[keep] + ln[keep], f_all[keep][:, None], b_all[keep], chunk)
        f_ = pieces[:, 2]
        for w in range(int((int(nb[cols[single]].max()) + 63) // 64)):
            sel = nbs[f_] > 64 * w
            pw = pieces[sel]
            nbw = torch.clamp(nbs[pw[:, 2]] - 64 * w, max=64)
            btw = torch.where(nbw <= 16, one, torch.where(nbw <= 32, one * 2, one * 4))
            m = pw.shape[0]
            parts.append(torch.stack([pw[:, 0], pw[:, 1], pw[:, 2], (z + 8).expand(m), one.expand(m),
                                      (z + 64 * w).expand(m), btw, pw[:, 3]], 1))
    ck("singles")
    items = torch.cat(parts) if parts else torch.zeros((0, 8), dtype=torch.int64, device=dev)
    if items.shape[0] and light.any():
        # items holding a whole (light) column: spread over the XCDs (row block -1)
        cl = L(np.concatenate([[0], np.cumsum(np.isin(np.arange(Fa), cols[light]))]))
        f0, nf = items[:, 2], items[:, 4]
        items[(cl[f0 + nf] - cl[f0]) > 0, 7] = -1
    sp_p.__exit__(None, None, None)
    ck("items")
    # --- the histogram CSC: (row, kbase + bin) of every (super-block, feature) segment
    if S:
        with tracing.span("q.copy"):
            # (the per-feature key bases copied once and tiled over the super-blocks on the device: a
            # host tile and its pageable copy cost ~25 ms in a process's first build)
            kb = torch.from_numpy(kbase[cols].astype(np.uint8)).to(dev).repeat(nsb) if kbase.any() else None
            # a workgroup per <= COPY_PIECE entries: the hot features' segments hold ~10^5 entries
            # each, and a workgroup per segment left the copy to its longest ones (~20 ms at 10M rows)
            src_p, dst_p, len_p = seg_src.reshape(-1), seg_dst, flat
            npc = (len_p + COPY_PIECE - 1) // COPY_PIECE
            npieces = int(npc.sum())
            if npieces > len_p.numel():
                rep = torch.repeat_interleave(torch.arange(len_p.numel(), device=dev), npc, output_size=npieces)
                k = (torch.arange(npieces, device=dev) - (torch.cumsum(npc, 0) - npc)[rep]) * COPY_PIECE
                src_p, dst_p = src_p[rep] + k, dst_p[rep] + k
                len_p = torch.minimum(len_p[rep] - k, torch.full_like(k, COPY_PIECE))
                kb = kb[rep] if kb is not None else None
            ck("copy_pieces")
            C.copy_segments(Q.csc_row, Q.csc_bin, src_p.contiguous(), dst_p.contiguous(), len_p.contiguous(),
                            h_row[:total], h_key[:total], kb.contiguous() if kb is not None else None)
    ck("copy")
    sp_g = tracing.span("q.groups")
    sp_g.__enter__()
    hot_d = torch.from_numpy(hot.astype(np.bool_)).to(dev)
    is_hot = hot_d[items[:, 2]] & (items[:, 4] == 1)
    groups = {False: [], True: []}
    # every group's items ordered by entry offset (stable: ties keep the table order)
    for hot_sel in (False, True):
        sel_h = is_hot if hot_sel else ~is_hot
        for bt in (1, 2, 4):
            ix = torch.nonzero(sel_h & (items[:, 6] == bt)).flatten()
            if ix.numel() == 0:
                continue
            ix = ix[torch.sort(items[ix, 0], stable=True).indices]
            g = items[ix]
            meta = g[:, 3] | (g[:, 4] << 8) | (g[:, 5] << 16)
            groups[hot_sel].append(ItemGroup(bt, g[:, 0].contiguous(), g[:, 1].contiguous(), g[:, 2].to(torch.int32),
                                             meta.to(torch.int32), g[:, 7].to(torch.int32)))
    ck("group_sort")

    Q._groups = groups[False]
    Q._hot_groups = groups[True]
    sp_g.__exit__(None, None, None)
    Q._h_row, Q._h_key = h_row[:total], h_key[:total]
    Q._n_super = nsb
    Q._kbase_host = kbase.astype(np.int32)
    Q._kbase = torch.from_numpy(Q._kbase_host).to(dev)
    ck("groups")
    ck.report()
