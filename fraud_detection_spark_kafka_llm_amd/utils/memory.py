"""HBM sizing of training shards: how many rows one GPU can train on.

A tree ensemble (GBDT / RF / DT) trained on a count TF-IDF ``VectorColumn`` keeps, per CSR entry:
  * the CSR itself: int32 feature ids + int32 term counts (8 B; the caller's features),
  * the feature-major order built for the IDF and reused as the CSC: int32 rows + uint8 capped
    counts (5 B),
  * the bins: uint8 (1 B),
  * the histogram CSC (super-block-major copy of the rows + uint8 keys: 5 B),
and per row: the CSR row pointer (8 B), labels, margins, gradients, digit words, node ids and
slot bytes (~40 B), plus one byte per hot (dense-path) feature. Transients on top: the feature
order's radix-sort temporaries, 29 B per entry of one sort block (ops/sparse.py
FO_BLOCK_ENTRIES), and the histogram buffers of one level.

``max_rows_per_gpu`` inverts that model against ``torch.cuda.mem_get_info`` (or a given byte
budget). bench.py reports it next to the measured peak HBM per row; the estimators' data-parallel
launcher raises the worker count when one GPU's shard would not fit.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

ENTRY_BYTES = 19.0          # persistent bytes per CSR entry (see the module docstring)
ROW_BYTES = 48.0            # persistent bytes per row, without the dense hot-feature block
SORT_TEMP_BYTES = 29.0      # radix-sort temporaries per entry of one feature-order block
LEVEL_HIST_BYTES = 16.0     # (g, h) int64 sums per bin per node built in one level
DEFAULT_HOT_FEATURES = 64   # dense-path features (>= 10 % of rows) of a dialogue corpus
DEFAULT_BUILT_NODES = 32    # nodes built in the widest level (depth 6: 2^5)


def training_bytes(rows: int, nnz: int, hot_features: int = DEFAULT_HOT_FEATURES, total_bins: int = 0,
                   built_nodes: int = DEFAULT_BUILT_NODES) -> float:
    """Model of the peak HBM bytes of training on ``rows`` rows with ``nnz`` CSR entries."""
    from ..ops.sparse import FO_BLOCK_ENTRIES

    block = min(nnz, FO_BLOCK_ENTRIES)
    return (ENTRY_BYTES * nnz + (ROW_BYTES + hot_features) * rows + SORT_TEMP_BYTES * block
            + LEVEL_HIST_BYTES * total_bins * built_nodes * 2)


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


def max_rows_per_gpu(nnz_per_row: float, device=None, budget_bytes: Optional[int] = None,
                     hot_features: int = DEFAULT_HOT_FEATURES, total_bins: int = 0,
                     built_nodes: int = DEFAULT_BUILT_NODES) -> int:
    """Largest row count whose modelled training peak fits ``budget_bytes`` (default: 90 % of the
    device's free memory). 0 when there is no device budget."""
    from ..ops.sparse import FO_BLOCK_ENTRIES

    budget = device_budget(device) if budget_bytes is None else int(budget_bytes)
    if budget <= 0:
        return 0
    fixed = SORT_TEMP_BYTES * FO_BLOCK_ENTRIES + LEVEL_HIST_BYTES * total_bins * built_nodes * 2
    per_row = ENTRY_BYTES * nnz_per_row + ROW_BYTES + hot_features
    return max(0, int((budget - fixed) // per_row))


def min_workers(rows: int, nnz: int, device=None, budget_bytes: Optional[int] = None) -> int:
    """Fewest equal row shards that each fit one GPU (1 without a device budget)."""
    if rows <= 0:
        return 1
    cap = max_rows_per_gpu(nnz / rows, device, budget_bytes)
    if cap <= 0:
        return 1
    return max(1, math.ceil(rows / cap))
