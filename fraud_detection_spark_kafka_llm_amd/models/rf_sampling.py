"""Random-forest per-node feature subsampling (X-10, K-14).

Spark samples ``numFeaturesPerNode`` features without replacement per node (``auto`` = sqrt for
classification). Here every (tree, node, feature) draws an independent counter-based uniform and
keeps the feature with probability ``k / numFeatures`` — same expected subset size, no state, and
identical on every rank and on host/device (``hash_uniform`` in csrc/tree.h). This module mirrors
that hash in torch to compute, per level, the union of sampled features so histograms are only
built for features some node can actually split on.
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


def node_feature_mask(Q, params, tree_index: int, nodes: list) -> torch.Tensor:
    fid = Q.fid_orig
    mask = torch.zeros(fid.numel(), dtype=torch.bool, device=fid.device)
    a = _u64(int(params.seed) ^ 0x5BD1E995)
    for n in nodes:
        b = _u64((int(tree_index) << 32) | (int(n) & 0xFFFFFFFF))
        mask |= hash_uniform(a, b, fid) < params.feat_prob
    return mask
