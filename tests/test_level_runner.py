"""The native per-level runner (csrc/bindings_level.cpp RfLevels) and the kernels it brought:
same forests and boosters as the Python-driven levels, multi-workgroup compact layout equal to
the host twin."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ops import native


def _forest(device, n=6000, F=400, trees=6, depth=5, seed=7, rows=None):
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest

    rng = np.random.default_rng(seed)
    p = 0.5 / (1.0 + np.arange(F)) ** 0.7
    counts = (rng.random((n, F)) < p) * rng.integers(1, 4, (n, F))
    y = ((counts[:, 1] > 0) ^ (counts[:, 5] >= 2)).astype(np.float32)
    flip = rng.random(n) < 0.05
    y[flip] = 1 - y[flip]
    if rows is not None:                                     # (this rank's shard)
        counts, y = counts[rows[0]:rows[1]], y[rows[0]:rows[1]]
    vc = VectorColumn(F, dense=torch.from_numpy(counts.astype(np.float64)))
    r = fit_forest(vc, torch.from_numpy(y), num_trees=trees, max_depth=depth, bootstrap=True, feature_subset="sqrt",
                   seed=seed, device=device)
    return [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in r.trees]


@pytest.mark.gpu
@pytest.mark.parametrize("inflight", [1, 4])
def test_gpu_native_levels_equal_python_levels(inflight, monkeypatch):
    from fraud_detection_spark_kafka_llm_amd.models import forest_batch, grower

    monkeypatch.setattr(forest_batch, "TREES_IN_FLIGHT", inflight)
    monkeypatch.setattr(grower, "NATIVE_LEVELS", False)
    ref = _forest("cuda:0")
    monkeypatch.setattr(grower, "NATIVE_LEVELS", True)
    assert _forest("cuda:0") == ref                           # the lockstep batch (RfBatch)
    monkeypatch.setattr(forest_batch, "BATCH", False)         # the generic loop on the runner, per tree
    assert _forest("cuda:0") == ref
    monkeypatch.setattr(forest_batch, "BATCH", True)
    for presel, fused in ((False, True), (True, False)):
        monkeypatch.setattr(grower, "PRESELECT", presel)
        monkeypatch.setattr(grower, "FUSED_PACK", fused)
        assert _forest("cuda:0") == ref
    assert _forest("cpu") == ref


@pytest.mark.gpu
@pytest.mark.parametrize("inflight,depth", [(2, 5), (3, 3), (8, 5), (16, 6)])
def test_gpu_rf_lockstep_batch_equals_per_tree_lanes(inflight, depth, monkeypatch):
    """the trees in flight grown in lockstep batches (csrc/bindings_level.cpp
    RfBatch: one lane-batched launch per stage of a level, the level loop in C++) are bitwise the
    per-tree lanes' forest, with and without preselected item lists."""
    from fraud_detection_spark_kafka_llm_amd.models import forest_batch, grower

    monkeypatch.setattr(forest_batch, "TREES_IN_FLIGHT", inflight)
    for presel in (True, False):
        monkeypatch.setattr(grower, "PRESELECT", presel)
        monkeypatch.setattr(forest_batch, "BATCH", False)
        ref = _forest("cuda:0", trees=7, depth=depth)
        monkeypatch.setattr(forest_batch, "BATCH", True)
        assert _forest("cuda:0", trees=7, depth=depth) == ref, presel


def _dp_forest(rank, world, device, batch, compact):
    """One rank's forest under data parallelism (lockstep batches or per-tree lanes)."""
    from fraud_detection_spark_kafka_llm_amd.models import forest_batch, grower
    from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

    forest_batch.BATCH = batch
    forest_batch.TREES_IN_FLIGHT = 4
    grower.RF_COMPACT = compact
    lo, hi = D.shard_range(6000, rank, world)
    D.reset_bytes()
    grower.reset_level_stats()
    trees = _forest(device, trees=7, rows=(lo, hi))
    return trees, dict(D.CALLS), grower.LEVEL_STATS["coll_calls"]


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend,compact", [(1, "nccl", "1"), (1, "nccl", "0"), (2, "gloo", "auto")])
def test_gpu_rf_lockstep_batch_dp_equals_single_process(world, backend, compact, monkeypatch):
    """The lockstep batches under data parallelism: ONE reduce-scatter and ONE all-gather per
    batch-level (RCCL from the batch on the process group's communicator at world 1; Python
    callbacks over gloo with two ranks on this GPU), compact and full layouts: the single-process
    forest bit for bit."""
    from fraud_detection_spark_kafka_llm_amd.models import forest_batch
    from fraud_detection_spark_kafka_llm_amd.parallel.launch import spawn

    monkeypatch.setattr(forest_batch, "BATCH", False)
    monkeypatch.setattr(forest_batch, "TREES_IN_FLIGHT", 4)
    ref = _forest("cuda:0", trees=7)
    monkeypatch.setenv("FDX_FORCE_COLLECTIVES", "1")
    outs = spawn(_dp_forest, world, "cuda:0", True, compact, backend=backend)
    for trees, calls, level_calls in outs:
        assert trees == ref
        # 7 trees, 4 lanes in forest_batch.BATCHES batches, 5 levels: 2 per batch-level
        per = -(-4 // max(1, min(forest_batch.BATCHES, 4)))
        assert 0 < level_calls <= 2 * -(-7 // per) * 5, level_calls
        assert calls["reduce_scatter"] <= -(-7 // per) * 5, calls
    assert all(o[1] == outs[0][1] for o in outs)


def _booster(device, n=5000, F=300, trees=8, depth=6, seed=11, rows=None):
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt

    rng = np.random.default_rng(seed)
    p = 0.5 / (1.0 + np.arange(F)) ** 0.6
    vals = (rng.random((n, F)) < p) * rng.integers(1, 6, (n, F))        # (counts: the row-group engine)
    y = ((vals[:, 0] >= 2) ^ (vals[:, 3] >= 3)).astype(np.float32)
    flip = rng.random(n) < 0.05
    y[flip] = 1 - y[flip]
    if rows is not None:                                     # (this rank's shard)
        vals, y = vals[rows[0]:rows[1]], y[rows[0]:rows[1]]
    vc = VectorColumn(F, dense=torch.from_numpy(vals.astype(np.float64)))
    r = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=trees, max_depth=depth, learning_rate=0.3),
                 device=device)
    return [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in r.trees]


@pytest.mark.gpu
def test_gpu_gbdt_native_round_equals_python_levels(monkeypatch):
    """The fused boosting round (gradient prologue, split + plan, partition zeroing, leaf update
    from the node table; csrc/bindings_level.cpp) grows the same trees, bit for bit, as the
    Python-issued levels and as the host."""
    from fraud_detection_spark_kafka_llm_amd.models import grower

    monkeypatch.setattr(grower, "NATIVE_LEVELS", False)
    ref = _booster("cuda:0")
    monkeypatch.setattr(grower, "NATIVE_LEVELS", True)
    assert _booster("cuda:0") == ref                         # the level loop in the runner (C++)
    monkeypatch.setattr(grower, "GBDT_CXX_LEVELS", False)    # the generic Python loop on the runner
    assert _booster("cuda:0") == ref
    monkeypatch.setattr(grower, "GBDT_CXX_LEVELS", True)
    for flag in ("RG_PARTIALS", "PARTITION_COUNTS"):
        monkeypatch.setattr(grower, flag, False)
        assert _booster("cuda:0") == ref, flag
        monkeypatch.setattr(grower, flag, True)
    assert _booster("cpu") == ref
    for depth in (1, 3):                                     # (a one-level tree: gbdt_root only)
        monkeypatch.setattr(grower, "NATIVE_LEVELS", False)
        ref_d = _booster("cuda:0", depth=depth)
        monkeypatch.setattr(grower, "NATIVE_LEVELS", True)
        assert _booster("cuda:0", depth=depth) == ref_d, depth


@pytest.mark.gpu
def test_gpu_gbdt_large_shard_paths_equal_host(monkeypatch):
    """the >4M-row regime on small data -- the list kernels' 2048-row waves, no
    partition row counts (partition_counts_ok false) and the fewest-rows sibling choice -- grows
    the host's trees bit for bit, with the choice on and off, on the C++ and the Python level loop."""
    from fraud_detection_spark_kafka_llm_amd.models import grower

    C = native.lib()
    ref = _booster("cpu")
    ref8 = _booster("cpu", depth=8)            # (levels with more than 64 next-level nodes)
    old = C.tree_set_list_big_rows(1000)
    try:
        assert C.tree_rg_list_rows(5000) == 2048 and not C.tree_partition_counts_ok(5000)
        for cxx in (True, False):
            monkeypatch.setattr(grower, "GBDT_CXX_LEVELS", cxx)
            for choose in (True, False):
                monkeypatch.setattr(grower, "GBDT_CHOOSE_ROWS", choose)
                assert _booster("cuda:0") == ref, (cxx, choose)
                assert _booster("cuda:0", depth=8) == ref8, (cxx, choose, 8)
    finally:
        C.tree_set_list_big_rows(old)
    assert C.tree_rg_list_rows(5000) == 512


def _dp_booster(rank, world, device, cxx, direct=True, big=False):
    """One rank's booster under data parallelism, with its collective calls counted (big: the
    >4M-row list regime on this small shard -- 2048-row list waves, the partition's per-node
    counts instead of the lists' counting pass)."""
    from fraud_detection_spark_kafka_llm_amd.models import grower
    from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

    if big:
        native.lib().tree_set_list_big_rows(1000)
    grower.GBDT_CXX_LEVELS = cxx
    grower.DP_DIRECT_RCCL = direct
    lo, hi = D.shard_range(5000, rank, world)
    D.reset_bytes()
    trees = _booster(device, rows=(lo, hi))
    return trees, dict(D.CALLS), grower.LEVEL_STATS["coll_calls"]


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend", [(1, "nccl"), (2, "gloo")])
def test_gpu_gbdt_dp_runner_levels_equal_single_process(world, backend, monkeypatch):
    """the data-parallel GBDT level loop in the runner (RfLevels.gbdt_dp_levels:
    the level's reduce-scatter / all-gather / the quantisation max as callbacks, the sibling
    subtraction inside the shard's split search) grows the single-process trees bit for bit -- at
    world 1 through RCCL and at world 2 (two ranks on this GPU over gloo: 2 feature shards) -- as
    does the Python-issued DP level loop; 13 collectives per tree."""
    from fraud_detection_spark_kafka_llm_amd.parallel.launch import spawn

    ref = _booster("cuda:0")
    monkeypatch.setenv("FDX_FORCE_COLLECTIVES", "1")
    trees = 8
    # (the runner calls RCCL itself on the process group's communicator; direct=False: through
    # the Python callbacks, as on gloo)
    for cxx, direct, big in ((True, True, False), (True, False, False), (False, True, False), (True, True, True)):
        outs = spawn(_dp_booster, world, "cuda:0", cxx, direct, big, backend=backend)
        for got, calls, level_calls in outs:
            assert got == ref, (cxx, direct, big, world)
            assert level_calls > 0
            # (+ fit_gbdt's base score and the quantisation's max / key gathers)
            assert calls["reduce_scatter"] + calls["all_gather"] <= 12 * trees + 4, calls
            assert calls["all_reduce"] <= trees + 3, calls


@pytest.mark.gpu
def test_gpu_rf_compact_chunked_equals_host():
    C = native.lib()
    rng = np.random.default_rng(3)
    Fa = 20000
    nbins = torch.from_numpy(rng.integers(1, 33, Fa).astype(np.int32))
    mask = torch.from_numpy((rng.random(Fa) < 0.07).astype(np.uint8))
    fs = torch.tensor([0, 3000, 3000, 15000, Fa], dtype=torch.int64)      # an empty shard too
    S = fs.numel() - 1
    ref_local = torch.zeros(Fa + 1, dtype=torch.int64)
    ref_sizes = torch.zeros(S, dtype=torch.int64)
    C.tree_rf_compact(mask, nbins, fs, ref_local, ref_sizes)
    dev = torch.device("cuda:0")
    for chunks in (0, int((fs[1:] - fs[:-1]).max())):
        local = torch.full((Fa + 1,), -7, dtype=torch.int64, device=dev)
        sizes = torch.full((S,), -7, dtype=torch.int64, device=dev)
        C.tree_rf_compact(mask.to(dev), nbins.to(dev), fs.to(dev), local, sizes, chunks)
        assert torch.equal(local.cpu(), ref_local) and torch.equal(sizes.cpu(), ref_sizes), chunks
