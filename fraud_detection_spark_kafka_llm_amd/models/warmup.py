"""Untimed warm-up of the tree engine on a device (used by bench.py and bench/suite.py).

ROCm loads a kernel's code object lazily on its first launch, and the tree engine instantiates
many templated histogram kernels (row tiles x column tiles x digit planes, dense/CSC, root/non-root)
plus hipCUB/rocPRIM sorts: the first fit on a fresh process pays ~0.3-0.5 s for that, and the caching
allocators start cold. A small fit through the same path before a timed phase moves that cost out
of the measurement without skipping any work of the measured fit.
"""
from __future__ import annotations

import os

import torch

from ..data import synth
from ..ml.linalg import VectorColumn
from ..ml.stopwords import ENGLISH
from ..ops import text as T
from ..ops.sparse import feature_order

NUM_FEATURES = 1 << 18


def warm_tree_kernels(dev, rows: int = 1 << 16, gbdt_depth: int = 6, gbdt_max_bin: int = 256,
                      forest_depth: int = 0, forest_subset: str = "sqrt") -> None:
    """Featurize ``rows`` synthetic dialogues on ``dev`` and fit 2 GBDT trees (and 2 RF trees when
    ``forest_depth`` > 0) through the production path. Collective-free unless a process group is
    active, in which case every rank must call it (same rows on every rank)."""
    from .gbdt import GBDTParams, fit_gbdt
    from .tree import fit_forest

    dev = torch.device(dev)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=NUM_FEATURES)
    pt, y = synth.generate(synth.SynthConfig(n=rows, seed=5), device=dev, start=3 * 10**9)
    ip, ix, v = T.featurize_score(pt, spec, want_csr=True, device=dev).csr()
    fo = feature_order(ip, ix, v, NUM_FEATURES)
    idf = torch.log((rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(NUM_FEATURES, ip, ix, v, idf, fo)
    fault = os.environ.pop("FDX_FAULT", None)        # (injected faults target the measured fits)
    try:
        if gbdt_depth > 0:
            fit_gbdt(vc, y, GBDTParams(n_estimators=2, max_depth=gbdt_depth, max_bin=gbdt_max_bin), device=dev)
        if forest_depth > 0:
            fit_forest(vc, y, num_trees=2, max_depth=forest_depth, max_bins=32, bootstrap=True,
                       feature_subset=forest_subset, seed=1, device=dev)
    finally:
        if fault is not None:
            os.environ["FDX_FAULT"] = fault
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
