"""Binary logistic regression trainer (X-08): L-BFGS on the (weighted) mean log-loss.

Mirrors Spark ``LogisticRegression`` (binomial) as far as its semantics are defined: features are
standardized by their sample standard deviation when ``standardization=true`` (constant features
get coefficient 0), the L2 penalty ``regParam/2 * ||beta||^2`` acts on the standardized
coefficients, the intercept is unpenalised, L-BFGS keeps 10 correction pairs and stops after
``maxIter`` iterations or when the relative loss improvement falls below ``tol``. Spark's exact
iterate sequence (Breeze line search, virtual centering) is not reproduced, so coefficients match
Spark only at the optimum ("parity unpinned" for separable data, where both diverge until maxIter).

Hot ops run natively: margins ``X @ (s * beta)`` via ``csrc/sparse_kernels.hip::spmv_kernel`` and
the gradient ``X^T r`` as the same row-wise SpMV over ``X^T`` (built once per fit by a stable sort
of the entries by feature): every output is one fixed-order lane-strided dot product, no atomics,
so repeated fits are bitwise identical on the GPU. Under data parallelism each rank holds a row
shard and the gradient / loss / weight sums are all-reduced once per function evaluation (PAR-04).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from ..ml.linalg import VectorColumn
from ..ops.sparse import spmv
from ..parallel.dist import Collectives
from ..utils.config import default_device


def transpose_csr(indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, num_cols: int) -> tuple:
    """CSR of X^T: entries stably sorted by column, so each column keeps its rows ascending."""
    n = indptr.numel() - 1
    counts = indptr[1:] - indptr[:-1]
    rows = torch.repeat_interleave(torch.arange(n, dtype=torch.int32, device=idx.device), counts,
                                   output_size=int(idx.numel()))
    order = torch.sort(idx.to(torch.int64), stable=True).indices
    t_indptr = torch.zeros(num_cols + 1, dtype=torch.int64, device=idx.device)
    torch.cumsum(torch.bincount(idx.to(torch.int64), minlength=num_cols), 0, out=t_indptr[1:])
    return t_indptr, rows[order].contiguous(), val[order].contiguous()


def train_logistic_regression(features, labels, weights=None, max_iter: int = 100, tol: float = 1e-6,
                              reg_param: float = 0.0, elastic_net: float = 0.0, fit_intercept: bool = True,
                              standardization: bool = True, device=None, history_size: int = 10):
    if reg_param > 0 and elastic_net > 0:
        raise NotImplementedError("L1/elastic-net (OWL-QN) is not supported; use elasticNetParam=0")
    dev = torch.device(device) if device is not None else default_device()
    vc = features if isinstance(features, VectorColumn) else VectorColumn.from_rows(list(features))
    vc = vc.to(dev)
    indptr, idx, val = vc.csr()
    idx = idx.to(torch.int32).contiguous()
    val = val.to(torch.float64).contiguous()
    F = vc.size
    n = len(vc)
    y = torch.as_tensor(labels if isinstance(labels, (torch.Tensor, np.ndarray)) else
                        np.asarray([float(v) for v in labels])).to(device=dev, dtype=torch.float64)
    w = torch.ones(n, dtype=torch.float64, device=dev) if weights is None else \
        torch.as_tensor(np.asarray(weights, dtype=np.float64)).to(dev)
    coll = Collectives()
    wsum = float(coll.sum(w.sum().reshape(1))[0])
    t_indptr, t_idx, t_val = transpose_csr(indptr, idx, val, F)

    def xt(v: torch.Tensor, vals: Optional[torch.Tensor] = None) -> torch.Tensor:     # X^T v, fixed order
        return spmv(t_indptr, t_idx, t_val if vals is None else vals, v)

    # feature scaling (sample std over all ranks)
    if standardization:
        s1 = coll.sum(xt(w))
        s2 = coll.sum(xt(w, t_val * t_val))
        mean = s1 / wsum
        var = (s2 - wsum * mean * mean) / max(wsum - 1.0, 1.0)
        std = torch.sqrt(torch.clamp(var, min=0.0))
        scale = torch.where(std > 0, 1.0 / torch.where(std > 0, std, torch.ones_like(std)), torch.zeros_like(std))
    else:
        scale = torch.ones(F, dtype=torch.float64, device=dev)

    def fg(theta: torch.Tensor):
        beta, b = theta[:F], theta[F]
        m = spmv(indptr, idx, val, scale * beta) + (b if fit_intercept else 0.0)
        # stable log(1 + e^m) - y m
        loss_i = torch.clamp(m, min=0) - m * y + torch.log1p(torch.exp(-torch.abs(m)))
        r = w * (torch.sigmoid(m) - y)
        parts = torch.cat([(w * loss_i).sum().reshape(1), r.sum().reshape(1), xt(r)])
        parts = coll.sum(parts)
        loss = parts[0] / wsum + 0.5 * reg_param * torch.dot(beta, beta)
        g = torch.empty_like(theta)
        g[:F] = scale * parts[2:] / wsum + reg_param * beta
        g[F] = parts[1] / wsum if fit_intercept else 0.0
        return float(loss), g

    theta = torch.zeros(F + 1, dtype=torch.float64, device=dev)
    if fit_intercept:
        p = float(coll.sum((w * y).sum().reshape(1))[0]) / wsum
        if 0 < p < 1:
            theta[F] = math.log(p / (1 - p))
    loss, g = fg(theta)
    history = [loss]
    S, Y = [], []
    for it in range(max_iter):
        # two-loop recursion
        q = g.clone()
        alphas = []
        for s, yv in reversed(list(zip(S, Y))):
            rho = 1.0 / float(torch.dot(yv, s))
            a = rho * float(torch.dot(s, q))
            alphas.append((a, rho, s, yv))
            q -= a * yv
        if S:
            gamma = float(torch.dot(S[-1], Y[-1]) / torch.dot(Y[-1], Y[-1]))
            q *= gamma
        else:
            gn = float(torch.linalg.vector_norm(g))
            q *= 1.0 / max(gn, 1e-12)
        for a, rho, s, yv in reversed(alphas):
            bcoef = rho * float(torch.dot(yv, q))
            q += s * (a - bcoef)
        d = -q
        gd = float(torch.dot(g, d))
        if gd >= 0:         # not a descent direction: reset memory
            S, Y = [], []
            d = -g
            gd = float(torch.dot(g, d))
        step = 1.0
        new_loss, new_g = fg(theta + step * d)
        for _ in range(30):     # Armijo backtracking
            if new_loss <= loss + 1e-4 * step * gd:
                break
            step *= 0.5
            new_loss, new_g = fg(theta + step * d)
        s_vec = step * d
        y_vec = new_g - g
        if float(torch.dot(s_vec, y_vec)) > 1e-12:
            S.append(s_vec)
            Y.append(y_vec)
            if len(S) > history_size:
                S.pop(0)
                Y.pop(0)
        theta = theta + s_vec
        improvement = (loss - new_loss) / max(abs(new_loss), abs(loss), 1e-12)
        loss, g = new_loss, new_g
        history.append(loss)
        if abs(improvement) < tol or float(torch.linalg.vector_norm(g)) < 1e-9:
            break
    coef = (scale * theta[:F]).cpu().numpy()
    intercept = float(theta[F]) if fit_intercept else 0.0
    return coef, intercept, history
