"""PAR-07: the reference's three classifiers fitted concurrently (one thread + HIP stream each)
give the same models as sequential fits."""
import pytest


def _sigs(models):
    out = {}
    for name, pm in models.items():
        m = pm.stages[-1]
        out[name] = [(t.feature.tolist(), t.stats.tolist()) for t in m.trees]
    return out


def _train(concurrent):
    from fraud_detection_spark_kafka_llm_amd import train

    spark = train.initialize_spark()
    df = train.load_and_clean_data(spark, None, 800, 42)
    return train.train_models(df, train.build_feature_pipeline(2000), train.make_classifiers(12, 4, 42),
                              concurrent=concurrent)


def test_sequential_fits_are_repeatable():
    assert _sigs(_train(False)) == _sigs(_train(False))


@pytest.mark.gpu
def test_gpu_concurrent_fits_equal_sequential(monkeypatch):
    monkeypatch.setenv("FDX_DEVICE", "cuda:0")
    assert _sigs(_train(True)) == _sigs(_train(False))
