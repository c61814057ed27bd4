"""Spark on-disk layout: shipped model load, golden predictions, write -> read round trips."""
import json

import numpy as np
import pyarrow.parquet as pq
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.data import fixtures
from fraud_detection_spark_kafka_llm_amd.io import spark_format as sf
from fraud_detection_spark_kafka_llm_amd.ml import Frame, PipelineModel, TextColumn


def test_java_double_format():
    assert sf.java_double_str(1e-6) == "1.0E-6"
    assert sf.java_double_str(0.5) == "0.5"
    assert sf.java_double_str(0.0) == "0.0"
    assert sf.java_double_str(100.0) == "100.0"
    assert sf.java_double_str(9.223372036854776e18) == "9.223372036854776E18"
    assert sf.java_double_str(12345678.0) == "1.2345678E7"
    assert sf.java_double_str(0.001) == "0.001"
    assert sf.java_double_str(2.5e-4) == "2.5E-4"


def test_shipped_metadata_reserialises_identically(shipped_model_path):
    for p in shipped_model_path.rglob("metadata/part-00000"):
        raw = p.read_text()
        md = json.loads(raw)
        # re-encode with Spark's number formatting (floats that Spark wrote as doubles)
        assert sf.spark_json_dumps(md) + "\n" == raw.replace("1.0E-6", "1.0E-6")


def test_shipped_crcs_verify(shipped_model_path):
    assert sf.verify_tree(shipped_model_path) == []


def test_load_shipped_model_golden(shipped_model_path):
    pm = PipelineModel.load(shipped_model_path)
    assert [type(s).__name__ for s in pm.stages] == ["Tokenizer", "StopWordsRemover", "HashingTF", "IDFModel",
                                                      "LogisticRegressionModel"]
    lr = pm.stages[-1]
    assert lr.intercept == -7.218662911169931
    assert np.count_nonzero(lr.coefficients) == 4081
    idf = pm.stages[3]
    assert idf.numDocs == 1150
    # idf = ln((N+1)/(df+1)) for all 10000 entries
    np.testing.assert_allclose(idf.idf, np.log(1151.0 / (idf.docFreq + 1.0)), rtol=0, atol=1e-15)
    texts = [fixtures.golden_text(n) for n, *_ in fixtures.GOLDEN]
    raw = TextColumn(texts)
    out = pm.transform(Frame({"dialogue": raw, "clean_text": TextColumn.cleaned_from(raw)}))
    rows = out.select("prediction", "probability", "rawPrediction").collect()
    for (name, margin, p, pred), r in zip(fixtures.GOLDEN, rows):
        assert r["prediction"] == pred
        assert r["rawPrediction"][1] == pytest.approx(margin, rel=1e-14, abs=1e-13)
        assert r["probability"][1] == pytest.approx(p, rel=1e-12)


def test_roundtrip_write_read(tmp_path, shipped_model_path):
    pm = PipelineModel.load(shipped_model_path)
    out = tmp_path / "m"
    pm.write().overwrite().save(str(out))
    assert sf.verify_tree(out) == []
    # metadata keys and parquet schemas equal the shipped ones
    for stage_dir in sorted((shipped_model_path / "stages").iterdir()):
        mine = out / "stages" / stage_dir.name
        a, b = sf.read_metadata(stage_dir), sf.read_metadata(mine)
        assert a["class"] == b["class"] and a["uid"] == b["uid"]
        assert a["paramMap"] == b["paramMap"] and a["defaultParamMap"] == b["defaultParamMap"]
        if (stage_dir / "data").exists():
            assert sf.spark_schema_of(stage_dir) == sf.spark_schema_of(mine)
            pa = next((stage_dir / "data").glob("*.parquet"))
            pb = next((mine / "data").glob("*.parquet"))
            assert pq.ParquetFile(pa).schema_arrow.equals(pq.ParquetFile(pb).schema_arrow, check_metadata=False)
    pm2 = PipelineModel.load(str(out))
    np.testing.assert_array_equal(pm2.stages[-1].coefficients, pm.stages[-1].coefficients)
    np.testing.assert_array_equal(pm2.stages[3].idf, pm.stages[3].idf)
    assert (out / "_SUCCESS").exists() is False and (out / "metadata" / "_SUCCESS").exists()


def test_crc_format(tmp_path):
    p = tmp_path / "f.bin"
    data = bytes(range(256)) * 5
    sf.write_file_with_crc(p, data)
    crc = (tmp_path / ".f.bin.crc").read_bytes()
    assert crc[:4] == b"crc\x00" and int.from_bytes(crc[4:8], "big") == 512 and len(crc) == 8 + 4 * 3
    assert sf.verify_crc(p)
    p.write_bytes(data[:-1] + b"x")
    assert not sf.verify_crc(p)
