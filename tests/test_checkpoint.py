"""Checkpoint / resume / fault injection / elastic resume for the GBDT trainer."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.parallel.checkpoint import InjectedFault, parse_fault
from fraud_detection_spark_kafka_llm_amd.parallel.launch import spawn


def _data(n=900, F=40, seed=2):
    rng = np.random.default_rng(seed)
    dense = (rng.random((n, F)) < 0.2) * rng.integers(1, 4, (n, F))
    y = ((dense[:, 1] > 0) | (dense[:, 5] > 1)).astype(np.float32)
    return dense.astype(np.float64), y


def _fit(dense, y, **kw):
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt

    vc = VectorColumn(dense.shape[1], dense=torch.from_numpy(dense))
    return fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=9, max_depth=3), device="cpu", **kw)


def _sig(res):
    """Exact: a resumed run replays the checkpointed trees in training order, so its margins and
    hence every later tree are bitwise those of the uninterrupted run."""
    return [(t.feature.tolist(), t.threshold.tolist(), t.stats[:, 0].tolist()) for t in res.trees]


def test_parse_fault():
    assert parse_fault("rank:1,tree:3") == {"rank": 1, "tree": 3}
    assert parse_fault("") is None


def test_fault_then_resume_equals_uninterrupted(tmp_path, monkeypatch):
    dense, y = _data()
    ref = _fit(dense, y)
    ck = tmp_path / "ck"
    monkeypatch.setenv("FDX_FAULT", "tree:5")
    with pytest.raises(InjectedFault):
        _fit(dense, y, checkpoint_dir=str(ck), checkpoint_every=3)
    monkeypatch.delenv("FDX_FAULT")
    from fraud_detection_spark_kafka_llm_amd.parallel.checkpoint import EnsembleCheckpointer

    st = EnsembleCheckpointer(str(ck)).load()
    assert st["trees_done"] == 6 and st["kind"] == "gbdt"
    assert (ck / "LATEST").read_text() == "ckpt-000006" and not list(ck.glob("ckpt-000003*"))
    res = _fit(dense, y, checkpoint_dir=str(ck), checkpoint_every=3, resume=True)
    assert len(res.trees) == 9
    assert _sig(res) == _sig(ref)
    assert res.base_margin == ref.base_margin


def _rank_fit(rank, world, ck, resume):
    from fraud_detection_spark_kafka_llm_amd.parallel.dist import shard_range

    dense, y = _data()
    lo, hi = shard_range(len(y), rank, world)
    return _sig(_fit(dense[lo:hi], y[lo:hi], checkpoint_dir=ck, checkpoint_every=3, resume=resume))


def test_elastic_resume_from_two_ranks_to_one(tmp_path, monkeypatch):
    dense, y = _data()
    ref = _sig(_fit(dense, y))
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("FDX_FAULT", "rank:1,tree:4")
    with pytest.raises(RuntimeError):
        spawn(_rank_fit, 2, ck, False, backend="gloo", timeout=120)
    monkeypatch.delenv("FDX_FAULT")
    # rank 0 wrote trees 0..2; resume on a single rank (world size changed 2 -> 1)
    out = _rank_fit(0, 1, ck, True)
    assert out == ref


def test_checkpoint_survives_kill_between_writes_and_refuses_foreign_runs(tmp_path):
    """A checkpoint interrupted after its directory was written but before the pointer moved
    (or mid-write) leaves the previous one loadable; a different kind, different data or
    different tree parameters are refused instead of silently replayed."""
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.parallel.checkpoint import EnsembleCheckpointer, data_fingerprint

    dense, y = _data()
    ck = tmp_path / "ck"
    _fit(dense, y, checkpoint_dir=str(ck), checkpoint_every=3)
    assert (ck / "LATEST").read_text() == "ckpt-000009"
    # a later save killed before its pointer switch: a half-written tmp dir and a complete dir
    (ck / "ckpt-000012.tmp" / "model").mkdir(parents=True)
    # (killed after its _resume.json was written, before the rename: still not a checkpoint)
    (ck / "ckpt-000012.tmp" / "_resume.json").write_text((ck / "ckpt-000009" / "_resume.json").read_text())
    vc = VectorColumn(dense.shape[1], dense=torch.from_numpy(dense))
    did = data_fingerprint(vc, torch.from_numpy(y))
    st = EnsembleCheckpointer(str(ck), kind="gbdt", data_id=did).load()
    assert st["trees_done"] == 9
    (ck / "LATEST").unlink()                    # pointer lost: the newest complete version is found
    assert EnsembleCheckpointer(str(ck)).load()["trees_done"] == 9
    with pytest.raises(RuntimeError, match="rf"):
        EnsembleCheckpointer(str(ck), kind="rf").load()
    other = data_fingerprint(VectorColumn(dense.shape[1], dense=torch.from_numpy(dense[:-1])), torch.from_numpy(y[:-1]))
    with pytest.raises(RuntimeError, match="different data"):
        EnsembleCheckpointer(str(ck), kind="gbdt", data_id=other).load()
    with pytest.raises(RuntimeError, match="max_depth"):
        _fit2 = __import__("fraud_detection_spark_kafka_llm_amd.models.gbdt", fromlist=["x"])
        _fit2.fit_gbdt(vc, torch.from_numpy(y), _fit2.GBDTParams(n_estimators=12, max_depth=4), device="cpu",
                       checkpoint_dir=str(ck), resume=True)
    # more trees with the same shape parameters: allowed (the ensemble grows from tree 9)
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt

    more = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=12, max_depth=3), device="cpu",
                    checkpoint_dir=str(ck), resume=True)
    full = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=12, max_depth=3), device="cpu")
    assert _sig(more) == _sig(full)


def _elastic_gbdt(rank, world, ck):
    from fraud_detection_spark_kafka_llm_amd.parallel.dist import shard_range
    from fraud_detection_spark_kafka_llm_amd.parallel.elastic import attempt

    dense, y = _data()
    lo, hi = shard_range(len(y), rank, world)
    return _sig(_fit(dense[lo:hi], y[lo:hi], checkpoint_dir=ck, checkpoint_every=3, resume=attempt() > 0)), world


def test_gbdt_watchdog_relaunch_is_bitwise_uninterrupted(tmp_path, monkeypatch):
    """a GBDT job relaunched by the elastic watchdog (world 3 -> 2 after a hard rank
    death) ends with exactly the trees and leaf values of an uninterrupted single-process run."""
    from fraud_detection_spark_kafka_llm_amd.parallel.elastic import run_elastic

    dense, y = _data()
    ref = _sig(_fit(dense, y))
    monkeypatch.setenv("FDX_FAULT", "rank:2,tree:4,hard:1,attempt:0")
    rep = run_elastic(_elastic_gbdt, 3, str(tmp_path / "ck"), backend="gloo", timeout=300)
    assert rep.attempts == 2 and rep.world_size == 2
    trees, world = rep.results[0]
    assert world == 2 and trees == ref
