"""The reference's shipped LR pipeline rebuilt from ``fixtures/shipped_lr.npz`` (see
fixtures/make_shipped_lr_fixture.py): usable where /root/reference is not mounted (GPU box)."""
import json
from pathlib import Path

import numpy as np

FIXTURE = Path(__file__).with_name("fixtures") / "shipped_lr.npz"


def shipped_pipeline():
    from fraud_detection_spark_kafka_llm_amd.ml import PipelineModel
    from fraud_detection_spark_kafka_llm_amd.ml.classification import LogisticRegressionModel
    from fraud_detection_spark_kafka_llm_amd.ml.feature import HashingTF, IDFModel, StopWordsRemover, Tokenizer

    z = np.load(FIXTURE)                      # allow_pickle=False (default)
    cols = json.loads(str(z["columns"]))
    stages = [Tokenizer(inputCol=cols["tok"][0], outputCol=cols["tok"][1]),
              StopWordsRemover(inputCol=cols["sw"][0], outputCol=cols["sw"][1], stopWords=[str(s) for s in z["stopWords"]],
                               caseSensitive=cols["caseSensitive"]),
              HashingTF(inputCol=cols["tf"][0], outputCol=cols["tf"][1], numFeatures=cols["numFeatures"],
                        binary=cols["binary"]),
              IDFModel(z["idf"], z["docFreq"], int(z["numDocs"]), inputCol=cols["idf"][0], outputCol=cols["idf"][1]),
              LogisticRegressionModel(z["coefficients"], float(z["intercept"]), featuresCol=cols["lr"][0])]
    return PipelineModel(stages)
