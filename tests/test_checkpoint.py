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
    return [(t.feature.tolist(), np.round(t.stats[:, 0], 12).tolist()) for t in res.trees]


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
    import json

    st = json.loads((ck / "_resume.json").read_text())
    assert st["trees_done"] == 6 and st["kind"] == "gbdt"
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
    assert [f for f, _ in out] == [f for f, _ in ref]
    for (_, a), (_, b) in zip(out, ref):
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12)
