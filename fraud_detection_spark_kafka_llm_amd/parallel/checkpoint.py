"""Training checkpoints, resume and fault injection.

Ensembles are checkpointed every ``every`` trees as a Spark-layout model directory (the same
format as the final model, so a checkpoint is also a usable model) plus ``_resume.json``:
``{"kind", "trees_done", "base_margin", "num_features", "params", "world_size", "data_id"}``.
Written atomically (``.tmp`` dir + rename) by rank 0 only; every rank reads it on resume.

Because histogram sums do not depend on how rows are sharded, a run may resume with a different
world size (elastic resume): the trees so far are replayed on each rank's new shard to rebuild
the margins (GBDT) and boosting continues.

Fault injection: ``FDX_FAULT="rank:R,tree:T"`` (or ``tree:T`` for every rank) raises
``InjectedFault`` right after tree T is grown on rank R — a stand-in for a GPU/rank failure in
tests of the recovery path.
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
        out[k.strip()] = int(v)
    return out


def maybe_fail(tree: int, fault: Optional[dict] = None) -> None:
    """``attempt:A`` limits the fault to relaunch A of an elastic job; ``hard:1`` kills the
    process outright (``os._exit``) instead of raising, like a lost GPU or an OOM kill."""
    f = fault if fault is not None else parse_fault()
    if not f or "tree" not in f:
        return
    att = int(os.environ.get("FDX_ATTEMPT", "0"))
    if f["tree"] == tree and f.get("rank", dist.rank()) == dist.rank() and f.get("attempt", att) == att:
        if f.get("hard"):
            os._exit(17)
        raise InjectedFault(f"injected fault at tree {tree} on rank {dist.rank()}")


class EnsembleCheckpointer:
    def __init__(self, directory: str, every: int = 10, kind: str = "gbdt", data_id: str = ""):
        self.dir = Path(directory)
        self.every = max(1, int(every))
        self.kind = kind
        self.data_id = data_id

    @property
    def state_path(self) -> Path:
        return self.dir / "_resume.json"

    def load(self) -> Optional[dict]:
        if not self.state_path.exists():
            return None
        st = json.loads(self.state_path.read_text())
        if self.data_id and st.get("data_id") and st["data_id"] != self.data_id:
            raise RuntimeError(f"checkpoint {self.dir} was written for different data ({st['data_id']})")
        return st

    def load_trees(self) -> list:
        st = self.load()
        if st is None:
            return []
        from ..ml.base import Params

        model = Params.load(self.dir / "model")
        return list(model.trees)[: st["trees_done"]]

    def maybe_save(self, trees_done: int, trees: list, base_margin: float, num_features: int, params=None,
                   force: bool = False) -> bool:
        if not force and trees_done % self.every != 0:
            return False
        if dist.rank() != 0:
            return False
        from ..ml.classification import RandomForestClassificationModel
        from ..ml.xgboost import SparkXGBClassifierModel

        tmp = self.dir.with_name(self.dir.name + ".tmp")
        if tmp.exists():
            shutil.rmtree(tmp)
        tmp.mkdir(parents=True)
        if self.kind == "gbdt":
            m = SparkXGBClassifierModel(trees, num_features, base_margin)
        else:
            m = RandomForestClassificationModel(trees, num_features)
        m.save(tmp / "model")
        state = {"kind": self.kind, "trees_done": trees_done, "base_margin": base_margin,
                 "num_features": num_features, "world_size": dist.world_size(), "data_id": self.data_id,
                 "params": asdict(params) if is_dataclass(params) else params}
        (tmp / "_resume.json").write_text(json.dumps(state, indent=1))
        if self.dir.exists():
            old = self.dir.with_name(self.dir.name + ".old")
            if old.exists():
                shutil.rmtree(old)
            self.dir.rename(old)
            tmp.rename(self.dir)
            shutil.rmtree(old)
        else:
            tmp.rename(self.dir)
        return True
