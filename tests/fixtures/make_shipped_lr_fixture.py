"""Regenerate ``shipped_lr.npz`` from the reference's shipped ``dialogue_classification_model``.

The GPU box has no /root/reference, so the golden-value tests there run on the shipped model's
arrays (coefficients, intercept, IDF, HashingTF width, stop words, column names) saved as a plain
npz (no pickle), read back by ``tests/shipped_model.py``. Run here with the reference mounted:
``python tests/fixtures/make_shipped_lr_fixture.py``.
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from fraud_detection_spark_kafka_llm_amd.ml import PipelineModel  # noqa: E402


def main(src="/root/reference/dialogue_classification_model", out=Path(__file__).with_name("shipped_lr.npz")):
    pm = PipelineModel.load(src)
    tok, sw, tf, idf, lr = pm.stages
    cols = {"tok": [tok.getInputCol(), tok.getOutputCol()], "sw": [sw.getInputCol(), sw.getOutputCol()],
            "tf": [tf.getInputCol(), tf.getOutputCol()], "idf": [idf.getInputCol(), idf.getOutputCol()],
            "lr": [lr.getFeaturesCol()], "numFeatures": tf.getNumFeatures(), "binary": bool(tf.getBinary()),
            "caseSensitive": bool(sw.getCaseSensitive())}
    np.savez_compressed(out, coefficients=lr.coefficients, intercept=np.float64(lr.intercept), idf=idf.idf,
                        docFreq=idf.docFreq, numDocs=np.int64(idf.numDocs),
                        stopWords=np.asarray(sw.getStopWords(), dtype=str), columns=np.asarray(json.dumps(cols)))
    print(f"wrote {out}")


if __name__ == "__main__":
    main()
