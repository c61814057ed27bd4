"""Appendix A golden values of the shipped LR pipeline: margins to 1e-13 on the
host path and on the fused HIP featurize+score kernel on cuda:0."""
import numpy as np
import pytest

from fraud_detection_spark_kafka_llm_amd.data import fixtures
from shipped_model import shipped_pipeline


def _margins(device):
    pm = shipped_pipeline()
    texts = [fixtures.golden_text(n) for n, *_ in fixtures.GOLDEN]
    pred, prob, rp = pm.compile(device=device).predict(texts, clean=True)
    return pred.cpu().numpy(), prob.cpu().numpy(), rp.cpu().numpy()


def _check(pred, prob, rp):
    for i, (name, margin, p, label) in enumerate(fixtures.GOLDEN):
        assert pred[i] == label, name
        assert abs(rp[i, 1] - margin) <= 1e-13, (name, rp[i, 1], margin)
        assert prob[i, 1] == pytest.approx(p, rel=1e-12), name


def test_fixture_equals_reference_model(shipped_model_path):
    from fraud_detection_spark_kafka_llm_amd.ml import PipelineModel

    ref = PipelineModel.load(shipped_model_path)
    mine = shipped_pipeline()
    np.testing.assert_array_equal(ref.stages[-1].coefficients, mine.stages[-1].coefficients)
    np.testing.assert_array_equal(ref.stages[3].idf, mine.stages[3].idf)
    assert ref.stages[1].getStopWords() == mine.stages[1].getStopWords()


def test_golden_margins_host():
    _check(*_margins("cpu"))


@pytest.mark.gpu
def test_gpu_golden_margins_on_cuda():
    pred, prob, rp = _margins("cuda:0")
    _check(pred, prob, rp)
    hp, hprob, hrp = _margins("cpu")
    np.testing.assert_array_equal(rp, hrp)          # device and host kernels agree bitwise
