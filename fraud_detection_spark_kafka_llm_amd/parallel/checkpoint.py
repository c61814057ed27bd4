"""Training checkpoints, resume and fault injection.

Ensembles are checkpointed every ``every`` trees as a Spark-layout model directory (the same
format as the final model, so a checkpoint is also a usable model) plus ``_resume.json``:
``{"kind", "trees_done", "base_margin", "num_features", "params", "world_size", "data_id"}``.
Written by rank 0 only as a complete versioned directory ``<dir>/ckpt-<trees>/``; the pointer
file ``<dir>/LATEST`` is then replaced atomically (``os.replace``), so a process killed at any
point (the elastic watchdog SIGKILLs survivors) leaves either the previous or the new checkpoint
readable, never none. Older versions are pruned after the pointer moves. On load, the stored
kind, data fingerprint (global rows / nnz / index and label sums: the same at any world size)
and tree-shaping parameters must match the run, or it fails loudly instead of replaying a
foreign ensemble.

Because histogram sums do not depend on how rows are sharded, a run may resume with a different
world size (elastic resume): the trees so far are replayed on each rank's new shard to rebuild
the margins (GBDT) and boosting continues.

Fault injection: ``FDX_FAULT="rank:R,tree:T"`` (or ``tree:T`` for every rank) raises
``InjectedFault`` right after tree T is grown on rank R — a stand-in for a GPU/rank failure in
tests of the recovery path; ``model:rf`` / ``model:gbdt`` limits it to one trainer.
"""
from __future__ import annotations

import json
import os
import shutil
from dataclasses import asdict, is_dataclass
from pathlib import Path
from typing import Optional

from . import dist


class InjectedFault(RuntimeError):
    pass


def parse_fault(spec: Optional[str] = None) -> Optional[dict]:
    spec = spec if spec is not None else os.environ.get("FDX_FAULT", "")
    if not spec:
        return None
    out = {}
    for part in spec.split(","):
        k, _, v = part.partition(":")
        k = k.strip()
        out[k] = v.strip() if k == "model" else int(v)
    return out


def maybe_fail(tree: int, fault: Optional[dict] = None, model: Optional[str] = None) -> None:
    """``attempt:A`` limits the fault to relaunch A of an elastic job; ``hard:1`` kills the
    process outright (``os._exit``) instead of raising, like a lost GPU or an OOM kill;
    ``model:M`` to the trainer ``model`` ("rf" / "gbdt")."""
    f = fault if fault is not None else parse_fault()
    if not f or "tree" not in f:
        return
    if "model" in f and f["model"] != model:
        return
    att = int(os.environ.get("FDX_ATTEMPT", "0"))
    if f["tree"] == tree and f.get("rank", dist.rank()) == dist.rank() and f.get("attempt", att) == att:
        if f.get("hard"):
            os._exit(17)
        raise InjectedFault(f"injected fault at tree {tree} on rank {dist.rank()}")


def data_fingerprint(vc, labels, coll=None) -> str:
    """World-size-independent id of a (features, labels) training set: global row / entry counts
    and sums of the feature indices, of the entry values' bit patterns (or term counts) and of the
    labels, all-reduced over the data-parallel ranks (any row sharding gives the same id)."""
    import torch

    y = labels.to(torch.float64) if isinstance(labels, torch.Tensor) else torch.as_tensor(labels, dtype=torch.float64)
    # every sum is taken in chunks: no full-size int64 / fp64 copy of the entries is allocated
    # (this runs right after prepare(), where the HBM sizing rule may have left little headroom)
    if getattr(vc, "dense", None) is not None:
        d = vc.dense
        parts = [d.shape[0], int((d != 0).sum()), 0, _chunked_sum(d, lambda c: (c.to(torch.float64) * 1024).round())]
    else:
        cnt = getattr(vc, "tf_counts", None)
        if cnt is not None:
            vsum = _chunked_sum(cnt, lambda c: c)
        else:
            vsum = _chunked_sum(vc.values, lambda c: (c.to(torch.float64) * 1024).round())
        parts = [len(vc), int(vc.indices.numel()), _chunked_sum(vc.indices, lambda c: c), vsum]
    parts.append(int((y.cpu() * 1024).round().sum()))
    t = torch.tensor(parts, dtype=torch.int64)
    if coll is not None and coll.active:
        dev = y.device if y.is_cuda else torch.device("cpu")
        t = coll.sum(t.to(dev)).cpu()
    return "-".join(str(int(x)) for x in t.tolist())


def _chunked_sum(x, fn, chunk: int = 1 << 24) -> int:
    """int(sum(fn(x))) accumulated in int64 over ``chunk``-element slices of the flattened x."""
    import torch

    flat = x.reshape(-1)
    total = 0
    for a in range(0, flat.numel(), chunk):
        total += int(fn(flat[a:a + chunk]).sum(dtype=torch.int64))
    return total


class EnsembleCheckpointer:
    """``params``: the tree-shaping parameters of the run (dict); a checkpoint whose stored
    params differ in any key except the ensemble size (and the intercept, stored on its own)
    is refused."""

    IGNORED = ("n_estimators", "num_trees", "base_score", "deterministic")

    def __init__(self, directory: str, every: int = 10, kind: str = "gbdt", data_id: str = "",
                 params: Optional[dict] = None):
        self.dir = Path(directory)
        self.every = max(1, int(every))
        self.kind = kind
        self.data_id = data_id
        self.params = params

    def _current(self) -> Optional[Path]:
        """Directory of the newest complete checkpoint (pointer first, then a scan, then the
        pre-versioning single-directory layout)."""
        ptr = self.dir / "LATEST"
        if ptr.exists():
            d = self.dir / ptr.read_text().strip()
            if (d / "_resume.json").exists():
                return d
        if self.dir.is_dir():
            # complete versions only: a ckpt-NNNNNN.tmp directory of a write killed before its
            # rename may already hold _resume.json, but is never a checkpoint
            vers = sorted((p for p in self.dir.glob("ckpt-*")
                           if p.name[5:].isdigit() and (p / "_resume.json").exists()),
                          key=lambda p: int(p.name[5:]))
            if vers:
                return vers[-1]
            if (self.dir / "_resume.json").exists():
                return self.dir
        return None

    @property
    def state_path(self) -> Path:
        cur = self._current()
        return (cur if cur is not None else self.dir) / "_resume.json"

    def load(self) -> Optional[dict]:
        cur = self._current()
        if cur is None:
            return None
        st = json.loads((cur / "_resume.json").read_text())
        if st.get("kind", self.kind) != self.kind:
            raise RuntimeError(f"checkpoint {cur} holds a {st.get('kind')} ensemble, not {self.kind}")
        if self.data_id and st.get("data_id") and st["data_id"] != self.data_id:
            raise RuntimeError(f"checkpoint {cur} was written for different data ({st['data_id']} != {self.data_id})")
        if self.params is not None and isinstance(st.get("params"), dict):
            diff = sorted(k for k in set(self.params) | set(st["params"])
                          if k not in self.IGNORED and self.params.get(k) != st["params"].get(k))
            if diff:
                raise RuntimeError(f"checkpoint {cur} was written with different parameters: {diff}")
        return st

    def load_trees(self) -> list:
        st = self.load()
        if st is None:
            return []
        from ..ml import classification, xgboost  # noqa: F401  (register the model readers)
        from ..ml.base import Params

        model = Params.load(self._current() / "model")
        return list(model.trees)[: st["trees_done"]]

    def maybe_save(self, trees_done: int, trees: list, base_margin: float, num_features: int, params=None,
                   force: bool = False) -> bool:
        if not force and trees_done % self.every != 0:
            return False
        if dist.rank() != 0:
            return False
        from ..ml.classification import RandomForestClassificationModel
        from ..ml.xgboost import SparkXGBClassifierModel

        self.dir.mkdir(parents=True, exist_ok=True)
        name = f"ckpt-{int(trees_done):06d}"
        tmp = self.dir / (name + ".tmp")
        if tmp.exists():
            shutil.rmtree(tmp)
        tmp.mkdir()
        if self.kind == "gbdt":
            m = SparkXGBClassifierModel(trees, num_features, base_margin)
        else:
            m = RandomForestClassificationModel(trees, num_features)
        m.save(tmp / "model")
        p = params if params is not None else self.params
        state = {"kind": self.kind, "trees_done": trees_done, "base_margin": base_margin,
                 "num_features": num_features, "world_size": dist.world_size(), "data_id": self.data_id,
                 "params": asdict(p) if is_dataclass(p) else p}
        _write_durable(tmp / "_resume.json", json.dumps(state, indent=1))
        final = self.dir / name
        if final.exists():
            shutil.rmtree(final)
        tmp.rename(final)
        _write_durable(self.dir / "LATEST.tmp", name)
        os.replace(self.dir / "LATEST.tmp", self.dir / "LATEST")       # the atomic switch
        for old in self.dir.glob("ckpt-*"):
            if old.name != name:
                shutil.rmtree(old, ignore_errors=True)
        return True


def _write_durable(path: Path, text: str) -> None:
    with open(path, "w") as f:
        f.write(text)
        f.flush()
        os.fsync(f.fileno())
