"""The training application (reference main() flow) end to end on a small synthetic corpus."""
import json

import numpy as np

import fraud_detection_spark as app
from fraud_detection_spark_kafka_llm_amd.io import spark_format as sf
from fraud_detection_spark_kafka_llm_amd.ml import PipelineModel
from fraud_detection_spark_kafka_llm_amd.ml.classification import DecisionTreeClassificationModel


def test_main_flow(tmp_path):
    summary = app.main(["--data", "", "--synthetic", "700", "--out-dir", str(tmp_path), "--num-trees", "12",
                        "--vocab-size", "3000"])
    assert set(summary) == {"DecisionTree", "RandomForest", "XGBoost"}
    for name, res in summary.items():
        assert res["Test"]["Accuracy"] > 0.85, (name, res)
        assert 0.9 < res["Test"]["AUC"] <= 1.0
    for f in ("metrics_comparison.png", "confusion_matrices_decisiontree.png", "word_associations_randomforest.png",
              "word_associations_decisiontree.png", "results.json"):
        assert (tmp_path / f).exists(), f
    out = json.loads((tmp_path / "results.json").read_text())
    assert sum(out["split"]) == 700
    ws = out["word_stats"]["DecisionTree"]
    assert ws and set(ws[0]) == {"word", "scam_count", "non_scam_count", "scam_ratio", "importance"}
    # the saved DT pipeline is a Spark-layout directory that loads back
    path = tmp_path / "fraud_detection_model"
    assert sf.verify_tree(path) == []
    md = sf.read_metadata(path / "stages" / sorted(p.name for p in (path / "stages").iterdir())[-1])
    assert md["class"] == "org.apache.spark.ml.classification.DecisionTreeClassificationModel"
    assert md["numFeatures"] > 0 and md["numClasses"] == 2
    pm = PipelineModel.load(str(path))
    assert isinstance(pm.stages[-1], DecisionTreeClassificationModel)
    assert [type(s).__name__ for s in pm.stages[:4]] == ["Tokenizer", "StopWordsRemover", "CountVectorizerModel",
                                                          "IDFModel"]
    pred, prob, raw = pm.compile().predict(["Innocent: hello. Suspect: please verify your social security number "
                                            "immediately or your account will be suspended"])
    assert prob.shape == (1, 2) and np.isclose(float(prob.sum()), 1.0)


def test_load_and_clean_filters_labels(tmp_path):
    import pandas as pd

    p = tmp_path / "d.csv"
    pd.DataFrame({"dialogue": ["Hi there!", "123 !!!", "Verify now", "x"], "personality": ["a"] * 4,
                  "type": ["t"] * 4, "labels": ["1", "0", " 0", "bad"]}).to_csv(p, index=False)
    spark = app.initialize_spark()
    df = app.load_and_clean_data(spark, str(p))
    # "123 !!!" cleans to " " (kept: not empty), "x" row dropped for its label
    assert df.count() == 3
    assert list(df.column("labels")) == [1.0, 0.0, 0.0]
    assert df.column("clean_text").strings == ["hi there", " ", "verify now"]
