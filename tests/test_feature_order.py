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


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_drop_features_in_place_equals_order_without_them(dev):
    """FeatureOrder.drop_features slides the kept columns over the dropped ones in place: the
    result is the CSC of the CSR without those features (dense columns: every row, like a term
    in every document, and sparse ones, adjacent runs, the first and the last feature)."""
    indptr, idx, cnt, f = _csr(seed=5, n=3000, f=50)
    n = indptr.numel() - 1
    # make features 0, 7, 8 and 49 present in every row (IDF 0 in a TF-IDF column)
    rows = []
    ip, ix, c = indptr.numpy(), idx.numpy(), cnt.numpy()
    for r in range(n):
        cols = dict(zip(ix[ip[r]:ip[r + 1]].tolist(), c[ip[r]:ip[r + 1]].tolist()))
        for k in (0, 7, 8, 49):
            cols.setdefault(k, 1 + r % 5)
        rows.append(sorted(cols.items()))
    indptr = torch.tensor(np.concatenate([[0], np.cumsum([len(r) for r in rows])]), dtype=torch.int64)
    idx = torch.tensor([k for r in rows for k, _ in r], dtype=torch.int32)
    cnt = torch.tensor([v for r in rows for _, v in r], dtype=torch.int32)
    drop = torch.zeros(f, dtype=torch.bool)
    drop[[0, 7, 8, 20, 49]] = True
    fo = feature_order(indptr.to(dev), idx.to(dev), cnt.to(dev), f)
    fo.drop_features(drop.to(dev))
    keep = ~drop[idx.long()]
    kptr = torch.zeros(n + 1, dtype=torch.int64)
    torch.cumsum(torch.tensor([int(keep[indptr[r]:indptr[r + 1]].sum()) for r in range(n)]), 0, out=kptr[1:])
    ref = feature_order(kptr.to(dev), idx[keep].to(dev), cnt[keep].to(dev), f)
    assert torch.equal(fo.csc_row.cpu(), ref.csc_row.cpu())
    assert torch.equal(fo.csc_cnt.cpu(), ref.csc_cnt.cpu())
    assert torch.equal(fo.colptr.cpu(), ref.colptr.cpu())
    assert bool(fo.dropped.cpu()[0]) and not bool(fo.dropped.cpu()[1])


def test_trees_on_idf_zero_features_equal_trees_without_them():
    """A TF-IDF column whose terms in every row have IDF 0 trains the same GBDT / RF as the column
    without those terms (their entries are dropped from the shared feature order in place), and a
    second fit on the same column (RF after GBDT, as the bench does) reuses the dropped order."""
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest

    indptr, idx, cnt, f = _csr(seed=9, n=2000, f=60)
    ip, ix, c = indptr.numpy(), idx.numpy(), cnt.numpy() % 7 + 1
    rows = []
    for r in range(2000):
        cols = dict(zip(ix[ip[r]:ip[r + 1]].tolist(), c[ip[r]:ip[r + 1]].tolist()))
        cols.setdefault(3, 2)                  # a term in every row
        rows.append(sorted(cols.items()))
    indptr = torch.tensor(np.concatenate([[0], np.cumsum([len(r) for r in rows])]), dtype=torch.int64)
    idx = torch.tensor([k for r in rows for k, _ in r], dtype=torch.int32)
    cnt = torch.tensor([v for r in rows for _, v in r], dtype=torch.int32)
    y = torch.from_numpy(((idx.numpy()[indptr.numpy()[:-1]] % 2) == 0).astype(np.float32))
    df = torch.bincount(idx.long(), minlength=f)
    idf = torch.log((2000 + 1.0) / (df.double() + 1.0))
    assert float(idf[3]) == 0.0
    keep = idx != 3
    kptr = torch.zeros(2001, dtype=torch.int64)
    torch.cumsum(torch.tensor([int(keep[indptr[r]:indptr[r + 1]].sum()) for r in range(2000)]), 0, out=kptr[1:])
    full = VectorColumn.tfidf(f, indptr, idx, cnt, idf, feature_order(indptr, idx, cnt, f))
    ref = VectorColumn.tfidf(f, kptr, idx[keep], cnt[keep], idf)
    sig = lambda r: [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in r.trees]  # noqa: E731
    p = GBDTParams(n_estimators=3, max_depth=4)
    assert sig(fit_gbdt(full, y, p, device="cpu")) == sig(fit_gbdt(ref, y, p, device="cpu"))
    assert full._feature_order.dropped is not None
    kw = dict(num_trees=3, max_depth=4, bootstrap=True, feature_subset="sqrt", seed=1, device="cpu")
    assert sig(fit_forest(full, y, **kw)) == sig(fit_forest(ref, y, **kw))


def test_larger_drop_set_does_not_move_an_earlier_csc():
    """A second quantisation of the same column that needs MORE features dropped builds an order
    of its own: the first one's CSC (an alias of the shared, already compacted order) is left as
    it was, and both quantisations equal fresh ones."""
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize

    indptr, idx, cnt, f = _csr(seed=11, n=1500, f=40)
    cnt = cnt % 7 + 1
    idf1 = torch.ones(f, dtype=torch.float64)
    idf1[[3, 9]] = 0.0
    idf2 = idf1.clone()
    idf2[[5, 21]] = 0.0
    vc = VectorColumn.tfidf(f, indptr, idx, cnt, idf1, feature_order(indptr, idx, cnt, f))
    q1 = quantize(vc, max_bins=16, counts=vc.tf_counts, scale=idf1)
    row1, col1 = q1.csc_row.clone(), q1.colptr.clone()
    q2 = quantize(vc, max_bins=16, counts=vc.tf_counts, scale=idf2)
    assert torch.equal(q1.csc_row, row1) and torch.equal(q1.colptr, col1)
    for q, idf in ((q1, idf1), (q2, idf2)):
        fresh = quantize(VectorColumn.tfidf(f, indptr, idx, cnt, idf), max_bins=16, counts=cnt, scale=idf)
        assert torch.equal(q.csc_row, fresh.csc_row) and torch.equal(q.colptr, fresh.colptr)
