"""Data parallelism (PAR-01..PAR-04) with 2 CPU ranks over gloo: the DP models equal DP=1 models."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.parallel.launch import spawn


def _dataset(n=1200, F=80, seed=0):
    rng = np.random.default_rng(seed)
    dense = (rng.random((n, F)) < 0.15) * rng.integers(1, 5, (n, F))
    y = ((dense[:, 0] > 0) ^ (dense[:, 3] >= 2)).astype(np.float32)
    flip = rng.random(n) < 0.04
    y[flip] = 1 - y[flip]
    return dense.astype(np.float64), y


def _vc(dense):
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn

    return VectorColumn(dense.shape[1], dense=torch.from_numpy(dense))


def _train(rank, world, kind, device="cpu"):
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
    from fraud_detection_spark_kafka_llm_amd.models.lr import train_logistic_regression
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
    from fraud_detection_spark_kafka_llm_amd.parallel.dist import shard_range

    dense, y = _dataset()
    lo, hi = shard_range(len(y), rank, world)
    vc, yy = _vc(dense[lo:hi]), torch.from_numpy(y[lo:hi])
    if kind == "gbdt":
        r = fit_gbdt(vc, yy, GBDTParams(n_estimators=6, max_depth=4), device=device)
        return [(t.feature.tolist(), t.stats[:, 0].tolist()) for t in r.trees], r.base_margin
    if kind == "rf":
        r = fit_forest(vc, yy, num_trees=3, max_depth=4, bootstrap=False, feature_subset="sqrt", seed=5,
                       device=device)
        return [(t.feature.tolist(), t.stats.tolist()) for t in r.trees], 0.0
    if kind == "lr":
        coef, b, _ = train_logistic_regression(vc, yy.numpy(), max_iter=50, reg_param=0.01, device="cpu")
        return coef.tolist(), b
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["gbdt", "rf", "lr"])
def test_two_ranks_equal_single_process(kind):
    single = _train(0, 1, kind)
    outs = spawn(_train, 2, kind, backend="gloo")
    assert outs[0] == outs[1] or kind == "lr" and np.allclose(outs[0][0], outs[1][0])   # identical on both ranks
    dp = outs[0]
    if kind == "lr":
        np.testing.assert_allclose(dp[0], single[0], rtol=1e-6, atol=1e-8)
        assert dp[1] == pytest.approx(single[1], rel=1e-6)
        return
    for (f1, v1), (f2, v2) in zip(dp[0], single[0]):
        assert f1 == f2
        np.testing.assert_allclose(np.asarray(v1), np.asarray(v2), rtol=1e-6, atol=1e-9)
    assert dp[1] == pytest.approx(single[1])


def test_three_ranks_feature_sharded_split_equals_single_process():
    """world 3: uneven feature shards (reduce-scatter + all-gather of best splits) give the DP=1 trees."""
    single = _train(0, 1, "rf")
    outs = spawn(_train, 3, "rf", backend="gloo")
    assert outs[0] == outs[1] == outs[2]
    for (f1, v1), (f2, v2) in zip(outs[0][0], single[0]):
        assert f1 == f2
        np.testing.assert_allclose(np.asarray(v1), np.asarray(v2), rtol=1e-9)


def test_gbdt_is_bitwise_identical_across_world_sizes():
    """Exact int64 histograms of quantised g/h: DP=1, DP=2 and DP=3 produce bit-identical trees and
    leaf values."""
    single = _train(0, 1, "gbdt")
    for world in (2, 3):
        outs = spawn(_train, world, "gbdt", backend="gloo")
        assert all(o == outs[0] for o in outs)
        assert outs[0] == single, f"world {world} differs from single process"


def _idf_rank(rank, world):
    from fraud_detection_spark_kafka_llm_amd.ml.feature import idf_fit
    from fraud_detection_spark_kafka_llm_amd.parallel.dist import all_reduce_sum, shard_range

    dense, _ = _dataset()
    lo, hi = shard_range(len(dense), rank, world)
    idf, df, n = idf_fit(_vc(dense[lo:hi]), 0, all_reduce=all_reduce_sum)
    return idf.tolist(), df.tolist(), n


def test_distributed_idf_equals_global():
    from fraud_detection_spark_kafka_llm_amd.ml.feature import idf_fit

    dense, _ = _dataset()
    idf, df, n = idf_fit(_vc(dense))
    outs = spawn(_idf_rank, 3, backend="gloo")
    for o in outs:
        assert o[2] == n and o[1] == df.tolist()
        np.testing.assert_array_equal(np.asarray(o[0]), idf)


def test_parse_cpulist_and_bind_noop_without_gpu():
    from fraud_detection_spark_kafka_llm_amd.parallel.affinity import bind_to_gpu, parse_cpulist

    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []
    if not torch.cuda.is_available():
        assert bind_to_gpu(0)["bound"] is False


def _train_counting(rank, world, kind, device):
    """_train with the backend's reduce-scatter / all-gather / all-reduce calls counted."""
    import torch.distributed as td

    calls = {"reduce_scatter_tensor": 0, "all_gather_into_tensor": 0, "all_gather": 0, "all_reduce": 0}
    for name in calls:
        orig = getattr(td, name)

        def wrapped(*a, _orig=orig, _name=name, **k):
            calls[_name] += 1
            return _orig(*a, **k)

        setattr(td, name, wrapped)
    from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

    D.reset_bytes()
    trees = _train(rank, world, kind, device)
    # (the native GBDT runner calls RCCL itself on the process group's communicator: counted by
    # the runner into D.CALLS, not seen by torch.distributed)
    return trees, dict(calls, direct_rs=D.CALLS.get("reduce_scatter", 0) - calls["reduce_scatter_tensor"],
                       direct_ag=D.CALLS.get("all_gather", 0) - calls["all_gather_into_tensor"])


@pytest.mark.parametrize("kind", ["gbdt", "rf"])
def test_forced_collectives_at_world_one_equal_plain_path(kind, monkeypatch):
    """FDX_FORCE_COLLECTIVES=1 runs the feature-sharded reduce-scatter / all-gather split path on
    a world-size-1 group (gloo here; RCCL on the GPU box): same trees as the plain path."""
    single = _train(0, 1, kind)
    monkeypatch.setenv("FDX_FORCE_COLLECTIVES", "1")
    (forced, calls), = spawn(_train_counting, 1, kind, "cpu", backend="gloo")
    # gloo runs the same reduce_scatter_tensor / all_gather_into_tensor calls as RCCL
    assert calls["reduce_scatter_tensor"] > 0 and calls["all_gather_into_tensor"] > 0
    assert forced == single


@pytest.mark.gpu
def test_gpu_rccl_forced_collectives_trees_equal_non_dp(monkeypatch):
    """RCCL (backend nccl) at world size 1: reduce_scatter_tensor / all_gather_into_tensor carry
    the int64 histogram partials and best-split tuples; the trees equal the non-DP GPU trees."""
    single = spawn(_train, 1, "gbdt", "cuda:0", backend="gloo")[0]
    monkeypatch.setenv("FDX_FORCE_COLLECTIVES", "1")
    (forced, calls), = spawn(_train_counting, 1, "gbdt", "cuda:0", backend="nccl")
    assert calls["reduce_scatter_tensor"] + calls["direct_rs"] > 0, calls
    assert calls["all_gather_into_tensor"] + calls["direct_ag"] > 0, calls
    assert forced == single


def _tfidf_dataset(n=1500, F=300, seed=1):
    """Sparse term-count rows (a few frequent terms, a long tail) + labels tied to two terms."""
    rng = np.random.default_rng(seed)
    p = 0.6 / (1.0 + np.arange(F)) ** 0.8
    counts = (rng.random((n, F)) < p) * rng.integers(1, 4, (n, F))
    y = ((counts[:, 1] > 0) ^ (counts[:, 7] >= 2)).astype(np.float32)
    flip = rng.random(n) < 0.05
    y[flip] = 1 - y[flip]
    return counts, y


def _train_tfidf(rank, world, kind):
    """The bench shape: a TF-IDF column kept as (counts, idf), row-sharded, with the
    collectives counted (world > 1 must run reduce_scatter_tensor itself)."""
    import torch.distributed as td

    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
    from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

    calls = {"reduce_scatter_tensor": 0}
    if td.is_initialized():
        orig = td.reduce_scatter_tensor

        def rs(*a, **k):
            calls["reduce_scatter_tensor"] += 1
            return orig(*a, **k)

        td.reduce_scatter_tensor = rs
    counts, y = _tfidf_dataset()
    df = (counts > 0).sum(0)
    idf = torch.from_numpy(np.log((len(y) + 1.0) / (df + 1.0)))
    lo, hi = D.shard_range(len(y), rank, world)
    c = counts[lo:hi]
    nz = c != 0
    indptr = torch.from_numpy(np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64))
    rr, cc = np.nonzero(nz)
    vc = VectorColumn.tfidf(counts.shape[1], indptr, torch.from_numpy(cc.astype(np.int32)),
                            torch.from_numpy(c[rr, cc].astype(np.int32)), idf)
    yy = torch.from_numpy(y[lo:hi])
    D.reset_bytes()
    if kind == "rf":
        r = fit_forest(vc, yy, num_trees=4, max_depth=5, max_bins=32, bootstrap=True, feature_subset="sqrt", seed=42,
                       device="cpu")
        out = [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in r.trees]
    else:
        r = fit_gbdt(vc, yy, GBDTParams(n_estimators=5, max_depth=6), device="cpu")
        out = [(t.feature.tolist(), t.threshold.tolist(), t.stats[:, 0].tolist()) for t in r.trees]
    assert not vc.values_materialized          # the count path never builds the fp64 values
    return out, calls["reduce_scatter_tensor"], D.BYTES["reduce_scatter"]


@pytest.mark.parametrize("kind", ["rf", "gbdt"])
def test_tfidf_dp_world2_trees_equal_single_process(kind):
    """BASELINE configs 3 (RF, bootstrap + sqrt features) and 4 (XGB-compatible GBDT) on the
    bench's TF-IDF column: 2 gloo ranks running reduce_scatter_tensor give bitwise the DP=1 trees."""
    single, _, _ = _train_tfidf(0, 1, kind)
    outs = spawn(_train_tfidf, 2, kind, backend="gloo")
    for trees, n_rs, nbytes in outs:
        assert n_rs > 0 and nbytes > 0
        assert trees == single


def _train_rf_lanes(rank, world, device="cpu"):
    """RF with several trees in flight (PAR-05) and the level collectives counted: returns the
    trees, the lanes used and the sequence of collective calls this rank issued."""
    import torch.distributed as td

    from fraud_detection_spark_kafka_llm_amd.models import grower
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
    from fraud_detection_spark_kafka_llm_amd.parallel.dist import shard_range

    seq = []
    if td.is_initialized():
        for name in ("reduce_scatter_tensor", "all_gather_into_tensor", "all_reduce"):
            orig = getattr(td, name)

            def wrapped(out, *a, _orig=orig, _name=name, **k):
                seq.append((_name, tuple(out.shape)))
                return _orig(out, *a, **k)

            setattr(td, name, wrapped)
    dense, y = _dataset(n=1500, F=120, seed=3)
    lo, hi = shard_range(len(y), rank, world)
    grower.reset_level_stats()
    r = fit_forest(_vc(dense[lo:hi]), torch.from_numpy(y[lo:hi]), num_trees=9, max_depth=5, bootstrap=True,
                   feature_subset="sqrt", seed=11, device=device)
    trees = [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in r.trees]
    return trees, r.lanes, seq, grower.LEVEL_STATS["coll_calls"]


@pytest.mark.parametrize("world", [2, 3])
def test_rf_trees_in_flight_under_dp_equal_single_process(world, monkeypatch):
    """PAR-05 under data parallelism (BASELINE config 3): 4 trees in flight per rank, lanes advanced
    in FIFO order so that every rank issues the same reduce-scatter / all-gather sequence; the
    forest is bitwise the DP=1 one-tree-at-a-time forest."""
    monkeypatch.setenv("FDX_RF_INFLIGHT", "1")
    serial = spawn(_train_rf_lanes, 1, backend="gloo")[0]
    assert serial[1] == 1
    monkeypatch.setenv("FDX_RF_INFLIGHT", "4")
    outs = spawn(_train_rf_lanes, world, backend="gloo")
    for trees, lanes, seq, n_coll in outs:
        assert lanes == 4
        assert trees == serial[0]
        assert n_coll > 0
        assert any(name == "reduce_scatter_tensor" for name, _ in seq)
    # the same collective sequence (names and payload shapes) on every rank
    assert all(o[2] == outs[0][2] for o in outs)


def _train_rf_uneven_caps(rank, world):
    """Ranks whose own lane cap differs (e.g. different free HBM): rank 0 can hold 1 lane, the
    others 4."""
    from fraud_detection_spark_kafka_llm_amd.models import tree as T

    T._local_lane_cap = lambda Q: 1 if rank == 0 else 4
    return _train_rf_lanes(rank, world)


def test_rf_lane_count_agreed_across_ranks_with_uneven_caps(monkeypatch):
    """the trees in flight follow the smallest rank's cap, so ranks with different free
    memory still take the same path and issue the same collective sequence (no hang, no
    mismatched reduce-scatter), and the forest is the DP=1 forest."""
    monkeypatch.setenv("FDX_RF_INFLIGHT", "1")
    serial = spawn(_train_rf_lanes, 1, backend="gloo")[0]
    outs = spawn(_train_rf_uneven_caps, 2, backend="gloo")
    for trees, lanes, seq, n_coll in outs:
        assert lanes == 1
        assert trees == serial[0]
    assert outs[0][2] == outs[1][2]


@pytest.mark.gpu
def test_gpu_rccl_forced_collectives_rf_lanes_equal_serial(monkeypatch):
    """RCCL at world 1 with 4 RF trees in flight: the lanes' reduce-scatters / all-gathers queue on
    the communicator's stream behind each lane's kernels; the forest equals the one-tree-at-a-time
    non-DP GPU forest (and the shared CSC items are built before the lanes fork: cold Q)."""
    monkeypatch.setenv("FDX_RF_INFLIGHT", "1")
    serial = spawn(_train_rf_lanes, 1, "cuda:0", backend="gloo")[0]
    monkeypatch.setenv("FDX_RF_INFLIGHT", "4")
    monkeypatch.setenv("FDX_FORCE_COLLECTIVES", "1")
    monkeypatch.setenv("FDX_RF_COMPACT", "1")         # the compact-level layout on the device too
    (trees, lanes, seq, n_coll), = spawn(_train_rf_lanes, 1, "cuda:0", backend="nccl")
    # (the lockstep batch calls RCCL itself on the process group's communicator: its level
    # collectives are counted in n_coll, not seen by torch.distributed)
    assert lanes == 4 and n_coll > 0
    assert trees == serial[0]


def _rf_rs_bytes(rank, world):
    from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

    D.reset_bytes()
    trees, lanes, seq, n_coll = _train_rf_lanes(rank, world)
    return trees, D.BYTES["reduce_scatter"]


def test_rf_compact_levels_send_only_sampled_bins(monkeypatch):
    """RF levels under DP reduce-scatter only the bins of the level's union feature sample
    (FeatureShards.compact): far fewer bytes, bitwise the same forest."""
    monkeypatch.setenv("FDX_RF_COMPACT", "0")
    full = spawn(_rf_rs_bytes, 2, backend="gloo")
    monkeypatch.setenv("FDX_RF_COMPACT", "1")
    comp = spawn(_rf_rs_bytes, 2, backend="gloo")
    assert comp[0][0] == full[0][0] == comp[1][0]
    assert comp[0][1] < 0.7 * full[0][1], (comp[0][1], full[0][1])


def _count_calls(rank, world, kind, groups):
    """Per-kind collective calls of one fit (parallel.dist.CALLS), with the trees."""
    import os

    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
    from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

    os.environ["FDX_RF_GROUPS"] = str(groups)
    from fraud_detection_spark_kafka_llm_amd.models import forest_batch

    forest_batch.LANE_GROUPS = groups
    dense, y = _dataset(n=1500, F=120, seed=3)
    lo, hi = D.shard_range(len(y), rank, world)
    vc, yy = _vc(dense[lo:hi]), torch.from_numpy(y[lo:hi])
    if kind == "rf":
        from fraud_detection_spark_kafka_llm_amd.models.tree import prepare

        prepare(vc, yy, "cpu")                 # quantisation's own collectives, counted apart
        D.reset_bytes()
        r = fit_forest(vc, yy, num_trees=8, max_depth=5, bootstrap=True, feature_subset="sqrt", seed=11, device="cpu")
        trees = [(t.feature.tolist(), t.stats.tolist()) for t in r.trees]
    else:
        D.reset_bytes()
        r = fit_gbdt(vc, yy, GBDTParams(n_estimators=4, max_depth=6), device="cpu")
        trees = [(t.feature.tolist(), t.stats[:, 0].tolist()) for t in r.trees]
    return trees, dict(D.CALLS)


def test_rf_lanes_share_one_collective_per_level_batch(monkeypatch):
    """Under DP the trees in flight batch their levels: one reduce-scatter + one all-gather per
    group-level (not per tree-level), the root totals ride in the first reduce-scatter (no
    per-tree all-reduce), and the forest is unchanged."""
    monkeypatch.setenv("FDX_RF_INFLIGHT", "4")
    serial_env = spawn(_count_calls, 2, "rf", 1, backend="gloo")
    outs = spawn(_count_calls, 2, "rf", 2, backend="gloo")
    assert outs[0][0] == outs[1][0] == serial_env[0][0]
    quant = 2                                      # (quantize: counted before the fit, see prepare)
    for trees, calls in serial_env:
        # 8 trees x <= 5 levels in batches of 4: at most ~2 x 5 + stragglers per kind
        assert calls["reduce_scatter"] <= 14, calls
        assert calls["all_gather"] <= 14 + quant, calls
        assert calls["all_reduce"] <= quant, calls
    for trees, calls in outs:                      # 2 groups of 2 lanes
        assert calls["reduce_scatter"] <= 24, calls


def test_gbdt_dp_collectives_per_tree_at_most_13():
    """GBDT under DP: per tree one all-reduce (the quantisation max) + a reduce-scatter and an
    all-gather per level (6 levels) = 13; the root totals ride in the root reduce-scatter."""
    outs = spawn(_count_calls, 2, "gbdt", 1, backend="gloo")
    single = _count_calls(0, 1, "gbdt", 1)
    assert outs[0][0] == outs[1][0] == single[0]
    calls = outs[0][1]
    n_trees = 4
    # (+ the base-score all-reduce of fit_gbdt and quantisation's max / key gathers)
    assert calls["reduce_scatter"] + calls["all_gather"] <= 12 * n_trees + 4, calls
    assert calls["all_reduce"] <= n_trees + 3, calls


def _train_gbdt_checked(rank, world, depth):
    """GBDT under DP with the level checks on (every open node built or subtracted before the
    split search reads its histogram row: grower.LEVEL_CHECKS in the device loop, always in the
    host loop taken by trees deeper than 6)."""
    from fraud_detection_spark_kafka_llm_amd.models import grower
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
    from fraud_detection_spark_kafka_llm_amd.parallel.dist import shard_range

    assert grower.LEVEL_CHECKS
    dense, y = _dataset(n=1500, F=120, seed=4)
    lo, hi = shard_range(len(y), rank, world)
    r = fit_gbdt(_vc(dense[lo:hi]), torch.from_numpy(y[lo:hi]), GBDTParams(n_estimators=3, max_depth=depth),
                 device="cpu")
    return [(t.feature.tolist(), t.stats[:, 0].tolist()) for t in r.trees]


@pytest.mark.parametrize("depth", [6, 7])
def test_gbdt_dp_level_checks_every_open_node_built_or_subtracted(depth, monkeypatch):
    """VERDICT r5 hygiene: the DP levels leave the level histogram uninitialised on the promise
    n_build + n_sub == n_open; the check runs (device loop at depth 6, host loop at depth 7) and
    the trees equal DP=1."""
    monkeypatch.setenv("FDX_LEVEL_CHECKS", "1")
    single = spawn(_train_gbdt_checked, 1, depth, backend="gloo")[0]
    outs = spawn(_train_gbdt_checked, 2, depth, backend="gloo")
    assert outs[0] == outs[1] == single
