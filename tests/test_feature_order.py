"""feature_order (ops/sparse.py): the row-blocked sort (bounded temporaries for large shards)
gives exactly the one-shot CSC, and int32 counts sort without a float copy."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order


def _csr(seed=0, n=5000, f=300):
    rng = np.random.default_rng(seed)
    rows = [np.sort(rng.choice(f, rng.integers(0, 40), replace=False)) for _ in range(n)]
    indptr = torch.tensor(np.concatenate([[0], np.cumsum([len(r) for r in rows])]), dtype=torch.int64)
    idx = torch.tensor(np.concatenate(rows), dtype=torch.int32)
    cnt = torch.tensor(rng.integers(1, 400, idx.numel()), dtype=torch.int32)
    return indptr, idx, cnt, f


def _same(a, b):
    for k in ("csc_row", "csc_cnt", "colptr", "df", "maxc"):
        assert torch.equal(getattr(a, k).cpu(), getattr(b, k).cpu()), k


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_row_blocked_feature_order_equals_one_shot(dev):
    indptr, idx, cnt, f = _csr()
    indptr, idx, cnt = indptr.to(dev), idx.to(dev), cnt.to(dev)
    one = feature_order(indptr, idx, cnt, f)
    for blk in (1000, 7777, 30000):
        _same(one, feature_order(indptr, idx, cnt, f, block_entries=blk))
    _same(one, feature_order(indptr, idx, cnt.float(), f))
    # against numpy: stable sort by feature keeps rows ascending within every column
    row = np.repeat(np.arange(indptr.numel() - 1), np.diff(indptr.cpu().numpy()))
    order = np.argsort(idx.cpu().numpy(), kind="stable")
    assert np.array_equal(one.csc_row.cpu().numpy(), row[order])
    assert np.array_equal(one.csc_cnt.cpu().numpy(), np.minimum(cnt.cpu().numpy()[order], 255))


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_incremental_feature_order_equals_one_shot(dev):
    """Blocks sorted as they arrive (bench featurize overlap) give exactly the one-shot CSC."""
    from fraud_detection_spark_kafka_llm_amd.ops.sparse import IncrementalFeatureOrder

    indptr, idx, cnt, f = _csr(seed=3)
    indptr, idx, cnt = indptr.to(dev), idx.to(dev), cnt.to(dev)
    one = feature_order(indptr, idx, cnt, f)
    for cuts in ([0, 5000], [0, 1, 1234, 1235, 4000, 5000], [0, 2500, 5000]):
        inc = IncrementalFeatureOrder(f, dev)
        for r0, r1 in zip(cuts[:-1], cuts[1:]):
            e0, e1 = int(indptr[r0]), int(indptr[r1])
            inc.add(indptr[r0:r1 + 1] - e0, idx[e0:e1], cnt[e0:e1], r0)
        _same(one, inc.finish())
