"""Random-forest per-node feature subsampling (X-10, K-14).

Spark samples exactly ``numFeaturesPerNode`` of the ``numFeatures`` feature indices without
replacement per node (``featureSubsetStrategy="auto"`` = ceil(sqrt(F)) for a forest;
/root/reference/fraud_detection_spark.py:67-74). Here every (tree, node, feature index) has a
counter-based priority (``feature_priority`` in csrc/tree.h, uniform in [0, 1)), and a node samples
the k features with the smallest priorities: exactly k, without replacement, no state, identical
on every rank and on host/device. ``node_thresholds`` finds each node's k-th smallest priority over
all F indices (the split kernel keeps a feature iff its priority <= the threshold);
``level_feature_mask`` is the union over the level's nodes, so histograms are only built for
features some node can actually split on.
"""
from __future__ import annotations

import math

import torch

_M = (1 << 64) - 1


def _u64(x: int) -> int:
    x &= _M
    return x - (1 << 64) if x >= (1 << 63) else x


_C1 = _u64(0x9E3779B97F4A7C15)
_C2 = _u64(0xBF58476D1CE4E5B9)
_C3 = _u64(0x94D049BB133111EB)


def _srl(x: torch.Tensor, s: int) -> torch.Tensor:
    return (x >> s) & ((1 << (64 - s)) - 1)


def mix64(x: torch.Tensor) -> torch.Tensor:
    x = x + _C1
    x = (x ^ _srl(x, 30)) * _C2
    x = (x ^ _srl(x, 27)) * _C3
    return x ^ _srl(x, 31)


def hash_uniform(a, b, c: torch.Tensor) -> torch.Tensor:
    """Vectorised twin of ``fdx::hash_uniform(a, b, c)`` (a, b scalars or tensors)."""
    x = mix64(torch.as_tensor(a, dtype=torch.int64, device=c.device) ^
              mix64(torch.as_tensor(b, dtype=torch.int64, device=c.device) ^ mix64(c)))
    return _srl(x, 11).to(torch.float64) * (1.0 / 9007199254740992.0)


def features_per_node(strategy: str, num_features: int) -> int:
    s = str(strategy).lower()
    if s in ("auto", "sqrt"):
        return int(math.ceil(math.sqrt(num_features)))
    if s == "all":
        return num_features
    if s == "onethird":
        return int(math.ceil(num_features / 3.0))
    if s == "log2":
        return max(1, int(math.ceil(math.log2(num_features))))
    v = float(s)
    return int(math.ceil(v * num_features)) if v <= 1.0 else min(num_features, int(v))


def _priorities(seed: int, tree_index: int, node: int, fid: torch.Tensor) -> torch.Tensor:
    a = _u64(int(seed) ^ 0x5BD1E995)
    b = _u64(((int(tree_index) & 0xFFFFFFFF) << 32) | (int(node) & 0xFFFFFFFF))
    return hash_uniform(a, b, fid)


def node_thresholds(num_features: int, seed: int, tree_index: int, nodes: list, k: int, dev) -> torch.Tensor:
    """[len(nodes)] float64: the k-th smallest priority of each node over feature indices 0..F-1
    (1.0 when k >= F: every feature)."""
    out = torch.ones(len(nodes), dtype=torch.float64, device=dev)
    if k >= num_features:
        return out
    fid = torch.arange(num_features, dtype=torch.int64, device=dev)
    for i, n in enumerate(nodes):
        out[i] = torch.kthvalue(_priorities(seed, tree_index, n, fid), k).values
    return out


def level_feature_mask(Q, seed: int, tree_index: int, nodes: list, thr: torch.Tensor) -> torch.Tensor:
    """[Fa] bool: active features sampled by at least one of ``nodes``."""
    fid = Q.fid_orig
    mask = torch.zeros(fid.numel(), dtype=torch.bool, device=fid.device)
    for i, n in enumerate(nodes):
        mask |= _priorities(seed, tree_index, n, fid) <= thr[i]
    return mask
