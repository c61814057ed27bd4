"""Multi-tree random-forest level passes (PAR-05).

Spark's RandomForest grows the nodes of many trees per pass over the data (node groups sized by
``maxMemoryInMB``; /root/reference/fraud_detection_spark.py:67-74 trains 100 trees). Here
``kRfTrees`` (8) trees grow in lockstep, level by level:

  * once per batch, ``tree_rf_rows`` writes each row's class counts for the 8 trees — the
    Poisson(1) bootstrap weight is drawn in-kernel from (seed, tree, global row) — as a 16-byte
    record, and the root totals;
  * per level, every open node of every tree samples its ⌈√F⌉ features on the device, the union
    mask selects the CSC work items, ``tree_rf_slots`` writes each row's 8 pass slots (one byte per
    tree) and ``tree_hist_rf`` builds the count histograms of up to 64 (tree, node) slots in one
    pass over the entries — two vector gathers per entry for all 8 trees;
  * one split launch covers all nodes (per-node tree index for the sampling key) and one
    device→host copy returns all best splits; rows are partitioned per tree.

The node tables are the same ``TreeTable`` the single-tree grower uses, so a batched forest is
bitwise identical to growing the trees one at a time (tested). Per-feature slot bit masks skip
the MFMA tiles of slots that did not sample an item's features.

Status: opt-in (``FDX_RF_BATCH=1``). On MI355X the per-tree passes win: they compact each pass to
one tree's live entries with a 1-byte slot and 2 count bytes per entry, while the batch carries
24 bytes of records per entry (measured in profiles/r2_rf_batch_ab.txt).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..ops import native
from ..utils import tracing
from .grower import GrowParams, TreeTable, Workspace, _best_splits, _partition_launch, _partition_stage
from .quantize import Quantized

K_RF_TREES = 8
MAX_PASS_SLOTS = 64
TILE_SKIP = os.environ.get("FDX_RF_TILE_SKIP", "1") != "0"


class BatchWorkspace:
    """Device buffers of one RF batch (reused across batches)."""

    def __init__(self, Q: Quantized):
        dev = Q.device
        self.rw = torch.empty((Q.n_rows, 2 * K_RF_TREES), dtype=torch.uint8, device=dev)
        self.rs = torch.empty((Q.n_rows, K_RF_TREES), dtype=torch.uint8, device=dev)
        self.row_node = torch.zeros((K_RF_TREES, Q.n_rows), dtype=torch.int32, device=dev)
        self.totals = torch.zeros((K_RF_TREES, 2), dtype=torch.int64, device=dev)
        self.kexp = torch.zeros(2, dtype=torch.int32, device=dev)       # integer counts: 2^0 steps


def _ct_for(cnt: int) -> int:
    ct = 1
    while ct * 8 < cnt:
        ct *= 2
    return ct


def grow_forest_batch(Q: Quantized, ws: Workspace, bw: BatchWorkspace, params: GrowParams, tree_ids: list,
                      label: torch.Tensor, bootstrap: bool) -> list:
    """Grow the trees ``tree_ids`` (at most K_RF_TREES) together; returns their Trees in order."""
    if not 0 < len(tree_ids) <= K_RF_TREES:
        raise ValueError("1..8 trees per batch")
    if params.mode == 0:
        raise ValueError("multi-tree batches grow classification (count) trees")
    C = native.lib()
    dev = Q.device
    T = len(tree_ids)
    tids = np.full(K_RF_TREES, -1, dtype=np.int32)
    tids[:T] = tree_ids
    tids_t = torch.from_numpy(tids).to(dev)
    with tracing.span("forest.batch_rows"):
        bw.totals.zero_()
        C.tree_rf_rows(label, tids_t, int(params.seed), bool(bootstrap), int(Q.row0), bw.rw, bw.totals)
        bw.row_node.zero_()
        tot = bw.totals.cpu().numpy()
    tabs = [TreeTable(tot[j].astype(np.int64)) for j in range(T)]
    levels = [[0] for _ in range(T)]
    scale = np.ones(2)
    max_nodes = 2 ** (params.max_depth + 1)
    TB = Q.TB
    groups = Q.groups + Q.hot_groups

    for d in range(params.max_depth + 1):
        opens = [[n for n in levels[j] if not tabs[j].is_leaf[n]] for j in range(T)]
        if d == params.max_depth or not any(opens):
            for j in range(T):
                for n in opens[j]:
                    tabs[j].is_leaf[n] = True
            break
        nodes = [(j, n) for j in range(T) for n in opens[j]]          # RF builds every open node
        nl = len(nodes)
        node_slot = np.full((K_RF_TREES, max_nodes), -1, dtype=np.int32)
        for k, (j, n) in enumerate(nodes):
            node_slot[j, n] = k
        stg = ws.staging
        h_ns = stg.add(node_slot.reshape(-1))
        h_ids = stg.add(np.array([n for _, n in nodes], dtype=np.int32))
        h_tree = stg.add(np.array([tree_ids[j] for j, _ in nodes], dtype=np.int32))
        h_slot_tree = stg.add(np.array([j for j, _ in nodes], dtype=np.int32))
        h_slot_node = stg.add(np.arange(nl, dtype=np.int32))
        h_tot = stg.add(np.stack([tabs[j].stats[n] for j, n in nodes]).astype(np.int64))
        up = stg.upload()
        # exact k-of-F sampling per (tree, node) on the device: thresholds per node; per pass, a
        # bit mask of the slots that sampled each feature selects work items and MFMA tiles
        feat_thr = torch.ones(nl, dtype=torch.float64, device=dev)
        if params.feat_k:
            m_all = torch.empty(Q.Fa, dtype=torch.uint8, device=dev)
            C.tree_rf_sample(int(params.seed), 0, up[h_ids], int(Q.num_features), int(params.feat_k), Q.fid_orig,
                             feat_thr, m_all, up[h_tree])                # every (tree, node) in one launch
            slot_bits = torch.empty(Q.Fa, dtype=torch.int64, device=dev)
            slot_any = torch.empty(Q.Fa, dtype=torch.uint8, device=dev)
        hist = torch.zeros((nl, TB, 2), dtype=torch.int64, device=dev)
        with tracing.span("forest.hist"):
            ns_dev = up[h_ns].view(K_RF_TREES, max_nodes)
            for s0 in range(0, nl, MAX_PASS_SLOTS):
                cnt = min(MAX_PASS_SLOTS, nl - s0)
                C.tree_rf_slots(bw.row_node, ns_dev, s0, cnt, bw.rs)
                ct = _ct_for(cnt)
                slot_node = up[h_slot_node][s0:s0 + cnt]
                slot_tree = up[h_slot_tree][s0:s0 + cnt]
                bits = anyf = None
                if params.feat_k:
                    C.tree_rf_slot_mask(int(params.seed), up[h_tree][s0:s0 + cnt], up[h_ids][s0:s0 + cnt],
                                        feat_thr[s0:s0 + cnt], Q.fid_orig, slot_bits, slot_any)
                    bits, anyf = (slot_bits if TILE_SKIP else None), slot_any
                for grp in groups:
                    if grp.num_items == 0:
                        continue
                    C.tree_hist_rf(grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(),
                                   Q.h_row, Q.h_key, bw.rs, bw.rw, Q.boff, Q.nbins, slot_node, slot_tree, hist, TB,
                                   grp.bt, ct, anyf, bits)
        with tracing.span("forest.split"):
            packed = _best_splits(C, hist, up[h_tot], Q.boff, Q.nbins, Q.zbin, Q.fid_orig, up[h_ids], bw.kexp, params,
                                  feat_thr if params.feat_k else None, 0, Q.Fa, 0, up[h_tree]).cpu().numpy()
        with tracing.span("forest.partition"):
            k0 = 0
            staged = []
            for j in range(T):
                cnt = len(opens[j])
                nxt, default_child, splits = tabs[j].apply_splits(opens[j], packed[k0:k0 + cnt], d, Q, params, scale,
                                                                  max_nodes)
                k0 += cnt
                if splits:
                    staged.append((j, _partition_stage(Q, stg, default_child, splits)))
                levels[j] = nxt
            if staged:                          # one upload for the 8 trees' partition tables
                up = stg.upload()
                for j, hs in staged:
                    _partition_launch(C, Q, up, hs, bw.row_node[j])
    return [tabs[j].build(Q, params, scale) for j in range(T)]
