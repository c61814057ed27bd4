"""LR training is deterministic: the gradient X^T r is a fixed-order SpMV over X^T (no atomics)."""
import numpy as np
import pytest
import torch


def _fit(device):
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.lr import train_logistic_regression

    rng = np.random.default_rng(11)
    n, F = 3000, 400
    dense = (rng.random((n, F)) < 0.05) * rng.random((n, F)) * 4
    y = (dense[:, :20].sum(1) + rng.normal(0, 0.3, n) > 1.0).astype(float)
    vc = VectorColumn(F, dense=torch.from_numpy(dense))
    return train_logistic_regression(vc, y, max_iter=40, reg_param=0.01, device=device)


def test_transpose_csr_matches_dense():
    from fraud_detection_spark_kafka_llm_amd.models.lr import transpose_csr

    rng = np.random.default_rng(0)
    d = (rng.random((50, 30)) < 0.2) * rng.random((50, 30))
    nz = np.nonzero(d)
    indptr = torch.from_numpy(np.concatenate([[0], np.cumsum((d != 0).sum(1))]).astype(np.int64))
    ti, tx, tv = transpose_csr(indptr, torch.from_numpy(nz[1].astype(np.int32)), torch.from_numpy(d[nz]), 30)
    back = np.zeros((30, 50))
    for c in range(30):
        back[c, tx[ti[c]:ti[c + 1]].numpy()] = tv[ti[c]:ti[c + 1]].numpy()
    np.testing.assert_array_equal(back, d.T)


def test_lr_fit_is_bitwise_repeatable_on_host():
    a, b = _fit("cpu"), _fit("cpu")
    np.testing.assert_array_equal(a[0], b[0])
    assert a[1] == b[1]


@pytest.mark.gpu
def test_gpu_lr_fit_is_bitwise_repeatable():
    a, b = _fit("cuda:0"), _fit("cuda:0")
    np.testing.assert_array_equal(a[0], b[0])
    assert a[1] == b[1] and a[2] == b[2]
    h = _fit("cpu")
    np.testing.assert_allclose(a[0], h[0], rtol=1e-6, atol=1e-9)
