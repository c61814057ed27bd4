"""Device paths vs their host twins: CSR scoring, SpMV / SpMV^T (LR training), docFreq, L-BFGS LR,
the reference training flow on the GPU, and GBDT checkpoint / fault / resume on the GPU."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.ml.tree_model import ensemble_arrays
from fraud_detection_spark_kafka_llm_amd.ops import sparse as S
from fraud_detection_spark_kafka_llm_amd.ops.text import LinearScorer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _csr(n=3000, F=500, density=0.04, seed=0):
    rng = np.random.default_rng(seed)
    dense = (rng.random((n, F)) < density) * rng.integers(1, 7, (n, F)).astype(np.float64)
    y = ((dense[:, 3] > 0) | (dense[:, 7] > 2)).astype(np.float64)
    return VectorColumn(F, dense=torch.from_numpy(dense)), y


def test_score_csr_lr_and_trees_bitwise():
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt

    vc, y = _csr()
    lr = LinearScorer(np.random.default_rng(1).standard_normal(vc.size), 0.3)
    assert torch.equal(S.score_csr(vc, lr), S.score_csr(vc.to(DEV), lr).cpu())
    res = fit_gbdt(vc, torch.from_numpy(y.astype(np.float32)), GBDTParams(n_estimators=8, max_depth=4), device="cpu")
    arr = ensemble_arrays(res.trees, "value", cmp_less=True)
    assert torch.equal(S.score_csr(vc, arr), S.score_csr(vc.to(DEV), arr).cpu())


def test_spmv_spmv_t_and_doc_freq():
    vc, _ = _csr(seed=3)
    ip, ix, v = vc.csr()
    x = torch.randn(vc.size, dtype=torch.float64)
    r = torch.randn(len(vc), dtype=torch.float64)
    d = [t.to(DEV) for t in (ip, ix, v)]
    torch.testing.assert_close(S.spmv(*d, x.to(DEV)).cpu(), S.spmv(ip, ix, v, x), rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(S.spmv_t(*d, r.to(DEV), vc.size).cpu(), S.spmv_t(ip, ix, v, r, vc.size),
                               rtol=1e-12, atol=1e-12)
    assert torch.equal(S.doc_freq(d[1], d[2], vc.size).cpu(), S.doc_freq(ix, v, vc.size))


def test_logistic_regression_gpu_matches_host():
    from fraud_detection_spark_kafka_llm_amd.models.lr import train_logistic_regression

    vc, y = _csr(seed=4)
    a = train_logistic_regression(vc, y, max_iter=60, reg_param=0.01, device="cpu")
    b = train_logistic_regression(vc, y, max_iter=60, reg_param=0.01, device=DEV)
    np.testing.assert_allclose(np.asarray(b[0]), np.asarray(a[0]), rtol=1e-6, atol=1e-8)
    assert b[1] == pytest.approx(a[1], rel=1e-6, abs=1e-8)


def test_reference_training_flow_on_gpu(tmp_path, monkeypatch):
    from fraud_detection_spark_kafka_llm_amd import train

    monkeypatch.setenv("FDX_DEVICE", DEV)
    res = train.main(["--data", "", "--synthetic", "1600", "--no-plots", "--out-dir", str(tmp_path)])
    for model in ("DecisionTree", "RandomForest", "XGBoost"):
        assert res[model]["Test"]["Accuracy"] > 0.95, (model, res[model])
    assert (tmp_path / "fraud_detection_model" / "metadata" / "part-00000").exists()


def test_gbdt_fault_and_resume_on_gpu(tmp_path, monkeypatch):
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
    from fraud_detection_spark_kafka_llm_amd.parallel.checkpoint import InjectedFault

    vc, y = _csr(seed=5)
    yt = torch.from_numpy(y.astype(np.float32))
    p = GBDTParams(n_estimators=9, max_depth=4)
    ref = fit_gbdt(vc, yt, p, device=DEV)
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("FDX_FAULT", "tree:5")
    with pytest.raises(InjectedFault):
        fit_gbdt(vc, yt, p, device=DEV, checkpoint_dir=ck, checkpoint_every=3)
    monkeypatch.delenv("FDX_FAULT")
    res = fit_gbdt(vc, yt, p, device=DEV, checkpoint_dir=ck, checkpoint_every=3, resume=True)
    assert len(res.trees) == 9
    for a, b in zip(res.trees, ref.trees):
        np.testing.assert_array_equal(a.feature, b.feature)
        np.testing.assert_allclose(a.stats, b.stats, rtol=1e-12, atol=1e-15)
