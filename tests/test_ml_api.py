"""ML API: pipelines end to end (fit/transform/save/load), evaluators vs brute force, LR trainer."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.data import synth
from fraud_detection_spark_kafka_llm_amd.ml import (IDF, CountVectorizer, DecisionTreeClassifier, Frame, HashingTF,
                                                     LogisticRegression, Pipeline, PipelineModel,
                                                     RandomForestClassifier, StopWordsRemover, TextColumn, Tokenizer)
from fraud_detection_spark_kafka_llm_amd.ml.evaluation import (BinaryClassificationEvaluator,
                                                                MulticlassClassificationEvaluator, area_under_roc)
from fraud_detection_spark_kafka_llm_amd.ml.xgboost import SparkXGBClassifier, SparkXGBClassifierModel


@pytest.fixture(scope="module")
def frames():
    pt, y = synth.generate(synth.SynthConfig(n=900, seed=5))
    raw = TextColumn(pt.strings())
    df = Frame({"dialogue": raw, "clean_text": TextColumn.cleaned_from(raw), "labels": y.numpy()})
    return df.randomSplit([0.7, 0.3], seed=42)


def exact_auc(s, y):
    pos, neg = s[y == 1], s[y == 0]
    gt = (pos[:, None] > neg[None, :]).sum() + 0.5 * (pos[:, None] == neg[None, :]).sum()
    return gt / (len(pos) * len(neg))


def test_auc_matches_mann_whitney():
    rng = np.random.default_rng(0)
    s = np.round(rng.random(500), 2)
    y = (rng.random(500) < 0.4).astype(float)
    assert area_under_roc(torch.from_numpy(s), torch.from_numpy(y), num_bins=0) == pytest.approx(exact_auc(s, y))
    # <1000 distinct scores -> no down-sampling even with the default numBins
    assert area_under_roc(torch.from_numpy(s), torch.from_numpy(y)) == pytest.approx(exact_auc(s, y))


def test_multiclass_weighted_metrics():
    y = np.array([0, 0, 0, 1, 1, 1, 1, 0], dtype=float)
    p = np.array([0, 1, 0, 1, 1, 0, 1, 0], dtype=float)
    df = Frame({"label": y, "prediction": p})
    ev = MulticlassClassificationEvaluator(labelCol="label")
    # class 0: tp=3 fp=1 fn=1 ; class 1: tp=3 fp=1 fn=1 -> all 0.75
    assert ev.evaluate(df, {"metricName": "accuracy"}) == pytest.approx(0.75)
    assert ev.evaluate(df, {"metricName": "weightedPrecision"}) == pytest.approx(0.75)
    assert ev.evaluate(df, {"metricName": "weightedRecall"}) == pytest.approx(0.75)
    assert ev.evaluate(df) == pytest.approx(0.75)


def _feature_stages(cv=False):
    tf = CountVectorizer(inputCol="filtered_words", outputCol="raw_features", vocabSize=20000) if cv else \
        HashingTF(inputCol="filtered_words", outputCol="raw_features", numFeatures=4096)
    return [Tokenizer(inputCol="clean_text", outputCol="words"),
            StopWordsRemover(inputCol="words", outputCol="filtered_words"), tf,
            IDF(inputCol="raw_features", outputCol="features")]


@pytest.mark.parametrize("make", [
    lambda: DecisionTreeClassifier(featuresCol="features", labelCol="labels", maxDepth=5),
    lambda: RandomForestClassifier(featuresCol="features", labelCol="labels", numTrees=10, maxDepth=4, seed=42),
    lambda: SparkXGBClassifier(features_col="features", label_col="labels", max_depth=4, n_estimators=15),
    lambda: LogisticRegression(featuresCol="features", labelCol="labels", maxIter=30, regParam=0.01),
])
@pytest.mark.parametrize("cv", [False, True])
def test_pipeline_fit_transform_save_load(frames, tmp_path, make, cv):
    train, test = frames
    model = Pipeline(stages=_feature_stages(cv) + [make()]).fit(train)
    out = model.transform(test)
    auc = BinaryClassificationEvaluator(labelCol="labels").evaluate(out)
    acc = MulticlassClassificationEvaluator(labelCol="labels", metricName="accuracy").evaluate(out)
    assert auc > 0.85 and acc > 0.8, (auc, acc)
    path = tmp_path / "m"
    model.write().overwrite().save(str(path))
    again = PipelineModel.load(str(path))
    out2 = again.transform(test)
    np.testing.assert_allclose(out2.column("probability").cpu().numpy(), out.column("probability").cpu().numpy(),
                               rtol=1e-9, atol=1e-12)
    # the fused serving path agrees with the staged transform
    pred, prob, _ = again.compile().predict(test.column("dialogue").strings, clean=True)
    np.testing.assert_allclose(prob.cpu().numpy(), out.column("probability").cpu().numpy(), rtol=1e-9, atol=1e-12)


def test_xgboost_json_roundtrip(frames, tmp_path):
    train, test = frames
    model = Pipeline(stages=_feature_stages() + [SparkXGBClassifier(features_col="features", label_col="labels",
                                                                       n_estimators=5, max_depth=3)]).fit(train)
    xgbm = model.stages[-1]
    js = xgbm.to_xgboost_json()
    back = SparkXGBClassifierModel.from_xgboost_json(js)
    feats = model.stages[-2].transform(model.stages[-3].transform(
        model.stages[1].transform(model.stages[0].transform(test)))).column("features")
    from fraud_detection_spark_kafka_llm_amd.ops.sparse import score_csr

    a = score_csr(feats, xgbm.scorer())
    b = score_csr(feats, back.scorer())
    np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-6)
    assert back.base_margin == pytest.approx(xgbm.base_margin, abs=1e-6)


def test_xgboost_spark_writer_layout_and_legacy_reader(frames, tmp_path):
    """SparkXGBClassifierModel.save writes xgboost.spark's layout (metadata/ + model/part-00000 with
    the booster JSON); reload is bitwise; the round-1 data/ layout still loads."""
    import json

    train, test = frames
    feats_model = Pipeline(stages=_feature_stages()).fit(train)
    tr, te = feats_model.transform(train), feats_model.transform(test)
    m = SparkXGBClassifier(features_col="features", label_col="labels", n_estimators=6, max_depth=3).fit(tr)
    path = tmp_path / "xgb"
    m.save(str(path))
    assert (path / "metadata" / "part-00000").exists() and (path / "model" / "part-00000").exists()
    assert not (path / "data").exists()
    md = json.loads((path / "metadata" / "part-00000").read_text().splitlines()[0])
    assert md["class"] == "xgboost.spark.core.SparkXGBClassifierModel"
    booster = json.loads((path / "model" / "part-00000").read_text().splitlines()[0])
    assert booster["learner"]["objective"]["name"] == "binary:logistic"
    assert len(booster["learner"]["gradient_booster"]["model"]["trees"]) == 6
    back = SparkXGBClassifierModel.load(str(path))
    np.testing.assert_array_equal(back.transform(te).column("probability").cpu().numpy(),
                                  m.transform(te).column("probability").cpu().numpy())
    # a booster without this engine's attributes (as xgboost writes it) loads through the JSON trees
    del booster["learner"]["attributes"]["fdx_trees"], booster["learner"]["attributes"]["fdx_base_margin"]
    (path / "model" / "part-00000").write_text(json.dumps(booster) + "\n")
    plain = SparkXGBClassifierModel.load(str(path))
    np.testing.assert_allclose(plain.transform(te).column("probability").cpu().numpy(),
                               m.transform(te).column("probability").cpu().numpy(), rtol=1e-6)
    # legacy layout
    legacy = tmp_path / "legacy"
    m._save_metadata(legacy)
    m._save_data_legacy(legacy)
    old = SparkXGBClassifierModel.load(str(legacy))
    np.testing.assert_array_equal(old.transform(te).column("probability").cpu().numpy(),
                                  m.transform(te).column("probability").cpu().numpy())


def test_lr_trainer_converges_on_separable_margin():
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.models.lr import train_logistic_regression

    rng = np.random.default_rng(3)
    X = rng.normal(size=(400, 5))
    wtrue = np.array([1.5, -2.0, 0.0, 0.5, 1.0])
    y = (rng.random(400) < 1 / (1 + np.exp(-(X @ wtrue - 0.3)))).astype(float)
    vc = VectorColumn(5, dense=torch.from_numpy(X))
    coef, b, hist = train_logistic_regression(vc, y, max_iter=100, tol=1e-10, device="cpu")
    # compare with a plain Newton solve of the same (unregularised) objective
    Xb = np.hstack([X, np.ones((400, 1))])
    th = np.zeros(6)
    for _ in range(50):
        p = 1 / (1 + np.exp(-Xb @ th))
        H = Xb.T @ (Xb * (p * (1 - p))[:, None])
        th -= np.linalg.solve(H, Xb.T @ (p - y))
    np.testing.assert_allclose(coef, th[:5], rtol=1e-4, atol=1e-4)
    assert b == pytest.approx(th[5], abs=1e-4)
    assert hist[-1] <= hist[0]


def _cv_corpus(n=400, seed=3):
    from fraud_detection_spark_kafka_llm_amd.data import synth

    pt, _ = synth.generate(synth.SynthConfig(n=n, seed=seed))
    docs = pt.strings()
    docs[3] = "Ünïcödé Straße CAFÉ café the THE"      # non-ASCII
    docs[7] = ""                                     # empty
    docs[11] = " ".join(["longword%d" % (i % 50) for i in range(1200)])   # > 4 KB (device cap)
    return docs


@pytest.mark.parametrize("clean", [True, False])
def test_count_vectorizer_native_fit_equals_python_fit(clean):
    from fraud_detection_spark_kafka_llm_amd.ml import CountVectorizer, StopWordsRemover, Tokenizer
    from fraud_detection_spark_kafka_llm_amd.ml.frame import TokenColumn

    raw = TextColumn(_cv_corpus())
    text = TextColumn.cleaned_from(raw) if clean else raw
    df = Frame({"t": text})
    df = Tokenizer(inputCol="t", outputCol="w").transform(df)
    df = StopWordsRemover(inputCol="w", outputCol="f").transform(df)
    col = df.column("f")
    assert isinstance(col, TokenColumn) and col.fusable
    for kw in (dict(vocabSize=300), dict(vocabSize=50, minDF=3.0), dict(vocabSize=10_000, minDF=0.05, maxDF=0.9)):
        cv = CountVectorizer(inputCol="f", outputCol="v", **kw)
        native = cv.fit(df).vocabulary
        python = cv._fit_python(col.tokens)
        assert native == python, kw


@pytest.mark.gpu
def test_count_vectorizer_fit_on_gpu_equals_python_fit():
    from fraud_detection_spark_kafka_llm_amd.ml import CountVectorizer, StopWordsRemover, Tokenizer
    from fraud_detection_spark_kafka_llm_amd.ml.feature import cv_fit_native

    raw = TextColumn(_cv_corpus(2000, 5))
    df = Frame({"t": TextColumn.cleaned_from(raw)})
    df = Tokenizer(inputCol="t", outputCol="w").transform(df)
    df = StopWordsRemover(inputCol="w", outputCol="f").transform(df)
    col = df.column("f")
    cv = CountVectorizer(inputCol="f", outputCol="v", vocabSize=500, minDF=2.0)
    assert cv_fit_native(col, 500, 2.0, device="cuda:0") == cv._fit_python(col.tokens)
