"""Estimator-level data parallelism and the elastic watchdog (CPU gloo ranks).

SparkXGBClassifier(num_workers=N) / RandomForestClassifier(numWorkers=N) launch N rank processes
from one Python process; the trees must equal num_workers=1 exactly. A rank killed mid-training
is detected by the parent watchdog, which relaunches at a smaller world size from the checkpoint.
"""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ml.classification import RandomForestClassifier
from fraud_detection_spark_kafka_llm_amd.ml.frame import Frame
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.ml.xgboost import SparkXGBClassifier


def _frame(n=900, F=60, seed=4):
    rng = np.random.default_rng(seed)
    dense = (rng.random((n, F)) < 0.15) * rng.integers(1, 5, (n, F)).astype(np.float64)
    y = ((dense[:, 2] > 0) ^ (dense[:, 7] >= 2)).astype(np.float64)
    flip = rng.random(n) < 0.05
    y[flip] = 1 - y[flip]
    return Frame({"features": VectorColumn(F, dense=torch.from_numpy(dense)), "label": y})


def _sig(model):
    return [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in model.trees]


@pytest.fixture(autouse=True)
def _dp_on_small_data(monkeypatch):
    monkeypatch.setenv("FDX_DP_MIN_ROWS", "0")      # launch ranks even for these tiny frames


def test_effective_workers_policy(monkeypatch):
    from fraud_detection_spark_kafka_llm_amd.parallel.estimator_dp import effective_workers

    assert effective_workers(4, 10, "cpu") == 4
    monkeypatch.setenv("FDX_DP_MIN_ROWS", "1000")
    assert effective_workers(4, 2500, "cpu") == 2 and effective_workers(4, 500, "cpu") == 1


@pytest.mark.parametrize("workers", [2, 3])
def test_xgb_num_workers_trains_identical_trees(workers):
    df = _frame()
    kw = dict(features_col="features", label_col="label", n_estimators=5, max_depth=4)
    single = SparkXGBClassifier(**kw).fit(df)
    multi = SparkXGBClassifier(num_workers=workers, **kw).fit(df)
    assert _sig(multi) == _sig(single)
    assert multi.base_margin == single.base_margin


def test_rf_num_workers_trains_identical_trees():
    df = _frame()
    kw = dict(featuresCol="features", labelCol="label", numTrees=4, maxDepth=4, seed=9)
    single = RandomForestClassifier(**kw).fit(df)
    multi = RandomForestClassifier(numWorkers=2, **kw).fit(df)
    assert _sig(multi) == _sig(single)
    assert "numWorkers" not in multi._paramMap


def _elastic_rf(rank, world, ck):
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
    from fraud_detection_spark_kafka_llm_amd.parallel.dist import shard_range
    from fraud_detection_spark_kafka_llm_amd.parallel.elastic import attempt

    df = _frame()
    vc, y = df.column("features"), df.column("label")
    lo, hi = shard_range(len(y), rank, world)
    res = fit_forest(vc.take(np.arange(lo, hi)), torch.from_numpy(y[lo:hi]), num_trees=8, max_depth=4,
                     bootstrap=True, feature_subset="sqrt", seed=3, device="cpu", checkpoint_dir=ck,
                     checkpoint_every=2, resume=attempt() > 0)
    return [(t.feature.tolist(), t.stats.tolist()) for t in res.trees], world, attempt()


def test_watchdog_relaunches_smaller_world_from_checkpoint(tmp_path, monkeypatch):
    """world 3, rank 1 dies hard (os._exit) after tree 4 of the first launch: the watchdog kills
    the survivors, relaunches with world 2, training resumes from the tree-4 checkpoint and the
    forest equals an uninterrupted single-process one."""
    from fraud_detection_spark_kafka_llm_amd.parallel.elastic import run_elastic

    ck = str(tmp_path / "ck")
    ref, _, _ = _elastic_rf(0, 1, None)
    monkeypatch.setenv("FDX_FAULT", "rank:1,tree:4,hard:1,attempt:0")
    rep = run_elastic(_elastic_rf, 3, ck, backend="gloo", timeout=300)
    assert rep.attempts == 2 and rep.world_size == 2
    assert rep.failures[0][1] == 3 and rep.failures[0][2] == 1 and "exit" in rep.failures[0][3]
    trees, world, att = rep.results[0]
    assert world == 2 and att == 1
    assert trees == ref
    assert rep.results[1][0] == ref


def test_rf_checkpoint_resume_equals_uninterrupted(tmp_path, monkeypatch):
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
    from fraud_detection_spark_kafka_llm_amd.parallel.checkpoint import InjectedFault

    df = _frame()
    vc, y = df.column("features"), torch.from_numpy(df.column("label"))
    kw = dict(num_trees=6, max_depth=4, bootstrap=True, feature_subset="sqrt", seed=1, device="cpu")
    ref = fit_forest(vc, y, **kw)
    ck = str(tmp_path / "rf")
    monkeypatch.setenv("FDX_FAULT", "tree:3")
    with pytest.raises(InjectedFault):
        fit_forest(vc, y, checkpoint_dir=ck, checkpoint_every=2, **kw)
    monkeypatch.delenv("FDX_FAULT")
    res = fit_forest(vc, y, checkpoint_dir=ck, checkpoint_every=2, resume=True, **kw)
    assert [(t.feature.tolist(), t.stats.tolist()) for t in res.trees] == \
        [(t.feature.tolist(), t.stats.tolist()) for t in ref.trees]


def test_tfidf_estimator_dp_stages_counts_not_values_and_matches_single():
    """SparkXGBClassifier(num_workers=N) on a HashingTF -> IDF column stages int32
    indices + int32 term counts (8 B per entry) and the IDF vector through shared memory -- no
    fp64 values -- and the ranks rebuild the values bitwise (trees equal num_workers=1)."""
    from fraud_detection_spark_kafka_llm_amd.data import synth
    from fraud_detection_spark_kafka_llm_amd.ml import (IDF, HashingTF, Pipeline, StopWordsRemover, TextColumn,
                                                         Tokenizer)

    pt, y = synth.generate(synth.SynthConfig(n=3000, seed=8))
    raw = TextColumn(pt.strings())
    df = Frame({"dialogue": raw, "clean_text": TextColumn.cleaned_from(raw), "labels": y.numpy().astype(np.float64)})
    feats = Pipeline(stages=[Tokenizer(inputCol="clean_text", outputCol="words"),
                             StopWordsRemover(inputCol="words", outputCol="filtered_words"),
                             HashingTF(inputCol="filtered_words", outputCol="raw_features", numFeatures=1 << 12),
                             IDF(inputCol="raw_features", outputCol="features")]).fit(df).transform(df)
    col = feats.column("features")
    assert col.tf_counts is not None and not col.values_materialized
    kw = dict(features_col="features", label_col="labels", n_estimators=4, max_depth=4)
    single = SparkXGBClassifier(**kw).fit(feats)
    est = SparkXGBClassifier(num_workers=2, **kw)
    multi = est.fit(feats)
    assert _sig(multi) == _sig(single) and multi.base_margin == single.base_margin
    staged = est.last_dp_report.staged_bytes
    nnz, n = int(col.indices.numel()), len(col)
    assert "values.npy" not in staged
    assert staged["indices.npy"] + staged["tf_counts.npy"] <= 8 * nnz + 256
    per_row = (staged["indptr.npy"] + staged["labels.npy"] - 256) / n
    assert per_row <= 12.5


def test_estimator_dp_follows_the_configured_device(monkeypatch):
    """FDX_DEVICE=cpu keeps num_workers CPU ranks even where GPUs are visible."""
    from fraud_detection_spark_kafka_llm_amd.parallel import estimator_dp as E

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("FDX_DEVICE", "cpu")
    assert E.effective_workers(4, 10) == 4 and E._resolve_device(None).type == "cpu"
    monkeypatch.setenv("FDX_DEVICE", "cuda:0")
    assert E.effective_workers(4, 10) == 1
