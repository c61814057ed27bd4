"""HBM sizing of training shards: how many rows one GPU can featurize and train.

The peak of a shard's pipeline is the larger of two moments, each modelled from what is live
(bytes per CSR entry "e", per row "r", per raw text byte of a featurization chunk "b"); the
numbers are the allocations of bench.py's path, measured stage by stage on the MI355X by
bench/probes/mem_probe.py (profiles/r4/mem_*.jsonl):

1. featurization, while the LAST chunk is processed (bench.featurize_shard with the feature
   order built per chunk):
     * the CSR being filled: int32 feature ids + fp32 term counts, capacity 1.05 x the entries
       plus one chunk (8 B/e), row pointer + labels (16 B/r);
     * the feature-order blocks of the chunks so far: int32 rows + uint8 counts (5 B/e);
     * the chunk's raw text in its two device staging buffers (2 B/b of the chunk),
       the fused kernel's CSR scratch (csrc/scoring.h csr_capacity: 1/2 slot per byte, 8 B a
       slot = 4 B/b) and the compaction's int64 step / position arrays and gathered entries
       (24 B per chunk entry), plus the chunk's radix-sort temporaries (24 B per chunk entry);
   or, at the end, the merged feature order (another 5 B/e) while the blocks are still held;
2. training (GBDT on the row-group engine; RF adds its CSC items, 5 B/e, on its own peak):
     * the CSR (8 B/e + slack), the feature order shared as the CSC (5 B/e of active entries),
       one uint8 bin per entry, the row-group entries (uint16: 2 B/e), and the row of every
       entry of the sparse groups (uint32, the entry-major root pass: 4 B per sparse entry, a
       fraction ``sparse_frac`` of the entries: ~21% on the bench corpus);
     * per row: pointer + labels (16 B), the row-group run starts (4 B per group), one byte per
       dense hot feature, the level loop's row state (digits, node, slot, list, margin, g, h,
       labels: 53 B);
     * the level histograms: (g, h) int64 per bin of each built node.

``max_rows_per_gpu`` inverts the model against ``torch.cuda.mem_get_info`` (or a given byte
budget), capped at the engine's index limits (ENGINE_MAX_ROWS; a row group's entry offsets are
kept below RG_GROUP_MAX_ENTRIES by splitting the group, which the model counts as extra groups);
``min_workers`` is the fewest equal shards that fit. bench.py reports the model next to
the measured peak of its timed GBDT phase (featurization + training).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

CSR_BYTES = 8.0             # int32 feature id + fp32 term count per entry
CSR_SLACK = 1.05            # featurize_shard's capacity estimate from the first chunk
ORDER_BYTES = 5.0           # feature order / CSC: int32 row + uint8 count per entry
BIN_BYTES = 1.0             # uint8 bin per active entry
RG_ENTRY_BYTES = 2.0        # row-group engine: uint16 local bin per entry
RG_EROW_BYTES = 4.0         # uint32 row per entry of the sparse groups (entry-major pass)
DEFAULT_SPARSE_FRAC = 0.21  # entries outside the dense row group (bench corpus: 205M of 968M)
ROW_BYTES = 16.0            # row pointer (int64) + labels (fp64) of the featurized shard
LEVEL_ROW_BYTES = 53.0      # level-loop row state (grower.Workspace + margins, g, h, labels)
CHUNK_TEXT_BYTES = 2.0      # two device staging buffers of one chunk's raw text
CHUNK_SCRATCH_BYTES = 4.0   # fused featurizer CSR scratch per text byte (scoring.h csr_capacity)
CHUNK_ENTRY_TEMP = 48.0     # per chunk entry: compaction int64 step + position + gathered entries,
                            # and the chunk's radix-sort temporaries
LEVEL_HIST_BYTES = 16.0     # (g, h) int64 sums per bin per node built in one level
RF_LANE_ROW_BYTES = 27.0    # RF: per tree in flight (models/forest_batch.py lanes), its workspace:
                            # digit words, masked digits, row -> node, packed row state, slots
                            # (~0.27 GB per lane at 10M rows, profiles/r4/rf500_sweep_*.json)
DEFAULT_HOT_FEATURES = 145  # dense-path features (>= 10 % of rows) of the bench dialogue corpus
DEFAULT_GROUPS = 11         # row groups of 8192 bins (bench corpus: ~90K bins over 2^18 buckets)
DEFAULT_BUILT_NODES = 32    # nodes built in the widest level (depth 6: 2^5)
DEFAULT_BYTES_PER_ROW = 1940.0   # raw UTF-8 bytes per dialogue of the bench corpus
DEFAULT_CHUNK_ROWS = 500_000     # bench featurization chunk
# index widths of the engine: int32 row ids (CSC rows, level row lists, entry-major rows, the
# partition's row pass), and uint32 entry offsets inside one row group (models/quantize.RowGroups
# splits a group before it reaches this many entries, so more rows mean more groups, not a limit)
ENGINE_MAX_ROWS = (1 << 31) - 1
RG_GROUP_MAX_ENTRIES = (1 << 31) - 1


def row_groups_for(nnz: int, groups: int = DEFAULT_GROUPS, sparse_frac: float = DEFAULT_SPARSE_FRAC) -> int:
    """Row groups of a shard with ``nnz`` entries: the bin-limited groups plus the extra groups the
    dense entries need under the per-group entry cap (RowGroups)."""
    dense = nnz * (1.0 - sparse_frac)
    return int(groups + max(0, math.ceil(dense / RG_GROUP_MAX_ENTRIES) - 1))


def featurize_bytes(rows: int, nnz: int, text_bytes_per_row: float = DEFAULT_BYTES_PER_ROW,
                    chunk_rows: int = DEFAULT_CHUNK_ROWS) -> float:
    """Peak bytes of featurizing ``rows`` rows into ``nnz`` CSR entries (model, see module doc)."""
    rows = max(int(rows), 0)
    chunk = min(rows, int(chunk_rows))
    chunk_entries = nnz * chunk / max(rows, 1)
    chunk_bytes = text_bytes_per_row * chunk
    csr = CSR_BYTES * (CSR_SLACK * nnz + chunk_entries) + ROW_BYTES * rows
    last_chunk = csr + ORDER_BYTES * nnz + (CHUNK_TEXT_BYTES + CHUNK_SCRATCH_BYTES) * chunk_bytes \
        + CHUNK_ENTRY_TEMP * chunk_entries
    merge = csr + 2 * ORDER_BYTES * nnz
    return max(last_chunk, merge)


def training_bytes(rows: int, nnz: int, hot_features: int = DEFAULT_HOT_FEATURES, total_bins: int = 0,
                   built_nodes: int = DEFAULT_BUILT_NODES, groups: int = DEFAULT_GROUPS,
                   sparse_frac: float = DEFAULT_SPARSE_FRAC, rf_lanes: int = 0) -> float:
    """Peak bytes of training (GBDT, row-group engine) on ``rows`` rows with ``nnz`` entries.
    ``rf_lanes`` > 0: a RandomForest with that many trees in flight instead (its CSC work items
    and a workspace per lane on top of the shared state)."""
    per_entry = CSR_BYTES * CSR_SLACK + ORDER_BYTES + BIN_BYTES + RG_ENTRY_BYTES + RG_EROW_BYTES * sparse_frac
    per_row = ROW_BYTES + 4.0 * row_groups_for(nnz, groups, sparse_frac) + hot_features + LEVEL_ROW_BYTES
    if rf_lanes > 0:
        per_entry += ORDER_BYTES
        per_row += RF_LANE_ROW_BYTES * rf_lanes
    return per_entry * nnz + per_row * rows + LEVEL_HIST_BYTES * total_bins * built_nodes * 2


def rf_lanes_that_fit(rows: int, want: int, free_bytes: int, headroom: float = 0.5) -> int:
    """Trees in flight whose workspaces fit ``headroom`` of ``free_bytes`` (at least 1, at most
    ``want``): the cap models/tree.fit_forest applies before building its lanes."""
    if free_bytes <= 0 or rows <= 0:
        return max(1, want)
    per = RF_LANE_ROW_BYTES * rows
    return int(max(1, min(want, (free_bytes * headroom) // max(per, 1.0))))


def pipeline_bytes(rows: int, nnz: int, **kw) -> float:
    """Peak bytes of featurization followed by training on one shard (the larger moment)."""
    fkw = {k: kw.pop(k) for k in ("text_bytes_per_row", "chunk_rows") if k in kw}
    return max(featurize_bytes(rows, nnz, **fkw), training_bytes(rows, nnz, **kw))


def device_budget(device=None, headroom: float = 0.9) -> int:
    """Bytes available to one training shard on ``device``: ``headroom`` of the free memory
    (``FDX_HBM_BUDGET_GB`` overrides; the CPU has no HBM budget: 0)."""
    env = os.environ.get("FDX_HBM_BUDGET_GB")
    if env:
        return int(float(env) * 2 ** 30)
    dev = torch.device(device) if device is not None else None
    if dev is None or dev.type != "cuda" or not torch.cuda.is_available():
        return 0
    free, _total = torch.cuda.mem_get_info(dev)
    return int(free * headroom)


def max_rows_per_gpu(nnz_per_row: float, device=None, budget_bytes: Optional[int] = None, **kw) -> int:
    """Largest row count whose modelled pipeline peak fits ``budget_bytes`` (default: 90 % of the
    device's free memory). 0 when there is no device budget. The model is piecewise linear in
    the row count (chunk terms saturate at one chunk), so the cap is found by bisection."""
    budget = device_budget(device) if budget_bytes is None else int(budget_bytes)
    if budget <= 0:
        return 0

    def fits(r: int) -> bool:
        return r <= ENGINE_MAX_ROWS and pipeline_bytes(r, int(r * nnz_per_row), **dict(kw)) <= budget

    lo, hi = 0, 1
    while fits(hi):
        lo, hi = hi, hi * 2
        if hi > 1 << 40:
            return lo
    while hi - lo > 1:
        mid = (lo + hi) // 2
        lo, hi = (mid, hi) if fits(mid) else (lo, mid)
    return lo


def min_workers(rows: int, nnz: int, device=None, budget_bytes: Optional[int] = None, rf_lanes: int = 0) -> int:
    """Fewest equal row shards that each fit one GPU (1 without a device budget); ``rf_lanes``:
    size for a RandomForest with that many trees in flight (training_bytes)."""
    if rows <= 0:
        return 1
    cap = max_rows_per_gpu(nnz / rows, device, budget_bytes, **({"rf_lanes": rf_lanes} if rf_lanes else {}))
    if cap <= 0:
        return 1
    return max(1, math.ceil(rows / cap))
