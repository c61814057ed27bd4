"""Estimator-level data parallelism: ``SparkXGBClassifier(num_workers=N).fit(df)`` and
``RandomForestClassifier(numWorkers=N).fit(df)`` from a single Python process (PAR-01, X-13).

xgboost.spark turns ``num_workers`` into N Spark barrier tasks joined by a Rabit ring
(/root/reference/fraud_detection_spark.py:76-83). Here the estimator writes the feature matrix
once (CSR arrays as .npy in /dev/shm; a TF-IDF column goes as int32 indices + int32 term counts
+ the IDF vector, 8 B per entry -- the ranks rebuild the fp64 values bit for bit, lazily -- never
as 8-byte values), launches N rank processes through the elastic watchdog
(``run_elastic``: one process per GPU over RCCL when N GPUs are visible, gloo CPU ranks
otherwise), and every rank memory-maps its contiguous row shard and runs the same trainer as a
``torchrun`` job would: exact integer histograms reduce-scattered by feature shard, identical split
decisions on every rank, trees equal to ``num_workers=1`` bit for bit. Rank 0 returns the model.
Training checkpoints every ``checkpoint_every`` trees; if a rank dies the watchdog relaunches the
job with one rank fewer and it resumes from the checkpoint.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from .elastic import attempt, run_elastic


def _save(tmp: Path, vc, labels, weights) -> dict:
    """Stage the feature matrix for the ranks; returns the bytes written per array."""
    counts, scale = getattr(vc, "tf_counts", None), getattr(vc, "tf_scale", None)
    tfidf = counts is not None and scale is not None and vc.dense is None
    if tfidf:
        indptr, idx = vc.indptr, vc.indices
        np.save(tmp / "tf_counts.npy", counts.cpu().numpy().astype(np.int32))
        np.save(tmp / "tf_scale.npy", scale.cpu().numpy().astype(np.float64))
        (tmp / "count_bins").write_text("1" if getattr(vc, "count_bins", False) else "0")
    else:
        indptr, idx, val = vc.csr()
        np.save(tmp / "values.npy", val.cpu().numpy().astype(np.float64))
    np.save(tmp / "indptr.npy", indptr.cpu().numpy().astype(np.int64))
    np.save(tmp / "indices.npy", idx.cpu().numpy().astype(np.int32))
    y = labels.cpu().numpy() if isinstance(labels, torch.Tensor) else np.asarray(labels)
    np.save(tmp / "labels.npy", np.asarray(y, dtype=np.float32))
    if weights is not None:
        w = weights.cpu().numpy() if isinstance(weights, torch.Tensor) else np.asarray(weights)
        np.save(tmp / "weights.npy", np.asarray(w, dtype=np.float32))
    (tmp / "size").write_text(str(vc.size))
    return {p.name: p.stat().st_size for p in tmp.iterdir() if p.suffix == ".npy"}


def _load_shard(tmp: Path, rank: int, world: int):
    from ..ml.linalg import VectorColumn
    from .dist import shard_range

    indptr = np.load(tmp / "indptr.npy", mmap_mode="r")
    n = indptr.size - 1
    lo, hi = shard_range(n, rank, world)
    a, b = int(indptr[lo]), int(indptr[hi])
    ip = torch.from_numpy(np.asarray(indptr[lo:hi + 1]) - a)
    ix = torch.from_numpy(np.array(np.load(tmp / "indices.npy", mmap_mode="r")[a:b]))
    size = int((tmp / "size").read_text())
    if (tmp / "tf_counts.npy").exists():
        cnt = torch.from_numpy(np.array(np.load(tmp / "tf_counts.npy", mmap_mode="r")[a:b]))
        vc = VectorColumn.tfidf(size, ip, ix, cnt, torch.from_numpy(np.load(tmp / "tf_scale.npy")),
                                count_bins=(tmp / "count_bins").read_text() == "1")
    else:
        vv = torch.from_numpy(np.array(np.load(tmp / "values.npy", mmap_mode="r")[a:b]))
        vc = VectorColumn(size, ip, ix, vv)
    y = torch.from_numpy(np.array(np.load(tmp / "labels.npy", mmap_mode="r")[lo:hi]))
    w = None
    if (tmp / "weights.npy").exists():
        w = np.array(np.load(tmp / "weights.npy", mmap_mode="r")[lo:hi])
    return vc, y, w


def _worker(rank: int, world: int, tmp: str, kind: str, kw: dict, dev_kind: str, ckpt: str, every: int):
    tmp = Path(tmp)
    vc, y, w = _load_shard(tmp, rank, world)
    device = f"cuda:{rank % max(1, torch.cuda.device_count())}" if dev_kind == "cuda" else "cpu"
    resume = attempt() > 0
    if kind == "gbdt":
        from ..models.gbdt import GBDTParams, fit_gbdt

        res = fit_gbdt(vc, y, GBDTParams(**kw), device=device, weights=w, checkpoint_dir=ckpt,
                       checkpoint_every=every, resume=resume)
        return (res.trees, res.num_features, res.base_margin, res.train_seconds) if rank == 0 else None
    if kind == "rf":
        from ..models.tree import fit_forest

        res = fit_forest(vc, y, device=device, weights=w, checkpoint_dir=ckpt, checkpoint_every=every,
                         resume=resume, **kw)
        return (res.trees, res.num_features) if rank == 0 else None
    raise ValueError(kind)


def _resolve_device(device) -> torch.device:
    """The training device: the one passed, else the configured one (``FDX_DEVICE`` / the
    first GPU when present, utils.config.default_device)."""
    from ..utils.config import default_device

    return torch.device(device) if device is not None else default_device()


def effective_workers(num_workers: int, n_rows: int, device=None, nnz: int = 0, kind: str = "gbdt") -> int:
    """Rank processes worth launching: one per GPU at most when GPUs are used (never several
    ranks on one device), and none below ``FDX_DP_MIN_ROWS`` rows per rank (default 100000) —
    a process launch costs more than training such a shard, and the model is bitwise the same
    either way (exact histograms). With ``nnz`` given on a GPU, at least as many ranks as the
    HBM sizing rule needs for every shard to fit (utils/memory.py max_rows_per_gpu; ``kind`` "rf":
    with a workspace per tree in flight)."""
    n = int(num_workers)
    cuda = _resolve_device(device).type == "cuda"
    if cuda:
        n = min(n, max(1, torch.cuda.device_count()))
    min_rows = int(os.environ.get("FDX_DP_MIN_ROWS", "100000"))
    if min_rows > 0:
        n = min(n, max(1, n_rows // min_rows))
    if cuda and nnz > 0:
        from ..utils.memory import min_workers

        lanes = 0
        if kind == "rf":
            from ..models import forest_batch

            lanes = max(1, forest_batch.TREES_IN_FLIGHT)
        need = min_workers(n_rows, nnz, _resolve_device(device), rf_lanes=lanes)
        if need > n:
            n = min(need, max(1, torch.cuda.device_count()))
    return max(1, n)


def fit_data_parallel(kind: str, vc, labels, weights, kw: dict, num_workers: int, device=None,
                      checkpoint_dir: Optional[str] = None, checkpoint_every: int = 10, min_workers: int = 1):
    """Train ``kind`` ("gbdt" | "rf") on ``num_workers`` rank processes; returns rank 0's result
    tuple and the watchdog report (``rep.staged_bytes``: bytes staged through shared memory)."""
    use_gpu = _resolve_device(device).type == "cuda"
    n_gpu = torch.cuda.device_count() if use_gpu else 0
    backend = "nccl" if use_gpu and n_gpu >= num_workers else "gloo"
    dev_kind = "cuda" if use_gpu and n_gpu >= 1 else "cpu"
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    tmp = Path(tempfile.mkdtemp(prefix="fdx-dp-", dir=base))
    try:
        staged = _save(tmp, vc, labels, weights)
        ck = checkpoint_dir or str(tmp / "checkpoint")
        rep = run_elastic(_worker, num_workers, str(tmp), kind, kw, dev_kind, ck, checkpoint_every, backend=backend,
                          min_world=min_workers)
        rep.staged_bytes = staged
        return rep.results[0], rep
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
