"""Serving: LLM client + stub server, agent on the shipped model, JSON extraction, streaming engine."""
import importlib
import json
import sys

import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.data import fixtures
from fraud_detection_spark_kafka_llm_amd.serve.agent import ClassificationAgent
from fraud_detection_spark_kafka_llm_amd.serve.llm import Analyzer, ChatClient, LLMError, RetryPolicy, StubLLM
from fraud_detection_spark_kafka_llm_amd.serve.llm_stub import StubServer
from fraud_detection_spark_kafka_llm_amd.stream import fake_kafka
from fraud_detection_spark_kafka_llm_amd.stream.engine import StreamingEngine, extract_texts
from fraud_detection_spark_kafka_llm_amd.stream.ring import PinnedRing


def test_chat_client_against_stub_server_with_retry():
    sleeps = []
    with StubServer(fail_first=2) as srv:
        c = ChatClient(api_key="k", base_url=srv.url, retry=RetryPolicy(attempts=3), sleep=sleeps.append)
        out = c.generate("Potentially Fraudulent ... verify your social security")
        assert "red flags" in out and "verify" in out
        assert len(srv.requests) == 3 and sleeps == [2.0, 2.0]   # exponential wait clamped to min 2s
        body = srv.requests[-1]
        assert body["model"] == "deepseek-chat" and body["max_tokens"] == 1000
        assert body["messages"][0]["role"] == "system"
    with StubServer(fail_first=5) as srv:
        c = ChatClient(base_url=srv.url, retry=RetryPolicy(attempts=3), sleep=lambda s: None)
        with pytest.raises(LLMError):
            c.generate("x")
        assert len(srv.requests) == 3


def test_chat_client_does_not_retry_client_errors(monkeypatch):
    c = ChatClient(base_url="http://127.0.0.1:9/v1", retry=RetryPolicy(attempts=3, min_wait=0), sleep=lambda s: None)
    with pytest.raises(LLMError):   # connection refused -> retried then LLMError (not a bare Exception)
        c.generate("x")


def test_prompt_contents():
    p = Analyzer.create_prompt("Hello", 1.0, 0.987)
    assert "Potentially Fraudulent" in p and "(Confidence Score: 0.99)" in p and "**Dialogue**" in p
    assert "Non-Fraudulent (Safe)" in Analyzer.create_prompt("Hi", 0)


def test_agent_on_shipped_model(shipped_model_path, tmp_path):
    agent = ClassificationAgent(str(shipped_model_path), llm=StubLLM(), device="cpu")
    r = agent.predict_and_get_label(fixtures.SCAM_SAMPLE)
    assert r["prediction"] == 1.0 and r["confidence"] == pytest.approx(0.9999999999165088, rel=1e-12)
    rb = agent.predict_batch([fixtures.BENIGN_SAMPLE, "", fixtures.SCAM_SAMPLE])
    assert [x["prediction"] for x in rb] == [0.0, 0.0, 1.0]
    assert rb[1]["confidence"] == pytest.approx(0.000732244982553525, rel=1e-12)
    out = agent.classify_and_explain(fixtures.SCAM_SAMPLE)
    assert set(out) == {"prediction", "confidence", "analysis", "historical_insight"}
    assert "stub-llm" in out["analysis"] and out["historical_insight"] is None
    # historical similarity: the closest historical dialogue ranks first
    import pandas as pd

    hist = pd.DataFrame({"dialogue": ["I am calling about your dentist appointment on Friday",
                                      "Verify your social security number now or face arrest",
                                      "Your package will be delivered tomorrow"], "label": [0, 1, 0]})
    agent.historical_data = hist
    cases = agent.find_similar_historical_cases("please verify your social security number", n=2)
    assert cases[0]["dialogue"].startswith("Verify your social")
    out = agent.classify_and_explain("please verify your social security number")
    assert out["historical_insight"] is not None


def test_dropin_agent_api_with_stub_backend(shipped_model_path, monkeypatch):
    monkeypatch.setenv("FDX_LLM_BACKEND", "stub")
    monkeypatch.delenv("DEEPSEEK_API_KEY", raising=False)
    sys.modules.pop("utils.agent_api", None)
    api = importlib.import_module("utils.agent_api")
    agent = api.DeepSeekClassificationAgent(model_path=str(shipped_model_path), device="cpu")
    res = agent.classify_and_explain(fixtures.SCAM_SAMPLE)
    assert res["prediction"] == 1.0 and res["analysis"]
    assert isinstance(api.DeepSeekAnalyzer("k").llm, StubLLM)


def test_dropin_agent_api_requires_key_for_deepseek(monkeypatch):
    monkeypatch.setenv("FDX_LLM_BACKEND", "deepseek")
    monkeypatch.delenv("DEEPSEEK_API_KEY", raising=False)
    sys.modules.pop("utils.agent_api", None)
    with pytest.raises(ValueError):
        importlib.import_module("utils.agent_api")
    sys.modules.pop("utils.agent_api", None)


def test_json_extraction_edge_cases():
    ring = PinnedRing(slots=1, max_docs=16, max_bytes=4096, pin=False)
    vals = [json.dumps({"text": "plain"}).encode(),
            json.dumps({"id": 7, "meta": {"text": "nested-not-top"}, "text": "a\"b\\c\né\U0001F600"}).encode(),
            b'{"text": 5}', b'not json', b'{"other": "x"}', json.dumps({"text": ""}).encode(),
            b'  {"text" : "sp\\u00e9ced" , "x":[1,{"y":"}"}]}  ']
    st = extract_texts(vals, ring.slots[0])
    assert st.tolist() == [0, 0, 1, 1, 1, 0, 0]
    s = ring.slots[0]
    o = s.offsets.numpy()
    got = [bytes(s.data.numpy()[o[i]:o[i + 1]]).decode() for i in range(len(vals))]
    assert got[0] == "plain" and got[1] == "a\"b\\c\né\U0001F600" and got[5] == "" and got[6] == "spéced"


def test_streaming_engine_end_to_end(shipped_model_path, monkeypatch):
    monkeypatch.setenv("KAFKA_BOOTSTRAP_SERVERS", "memory://engine-test")
    monkeypatch.setenv("KAFKA_INPUT_TOPIC", "customer-dialogues-raw")
    monkeypatch.setenv("KAFKA_OUTPUT_TOPIC", "dialogues-classified")
    from utils.kafka_utils import get_kafka_consumer, get_kafka_producer

    broker = fake_kafka.broker_for("memory://engine-test")
    broker.create_topic("customer-dialogues-raw", 3)
    prod = get_kafka_producer()
    texts = [fixtures.SCAM_SAMPLE, fixtures.BENIGN_SAMPLE] * 60
    for i, t in enumerate(texts):
        prod.produce("customer-dialogues-raw", key=f"id-{i}", value=json.dumps({"text": t}))
    prod.produce("customer-dialogues-raw", key="bad", value=b"{broken")
    prod.flush()
    broker.inject_error("customer-dialogues-raw")
    agent = ClassificationAgent(str(shipped_model_path), llm=StubLLM(), device="cpu")
    consumer, producer = get_kafka_consumer(), get_kafka_producer()
    eng = StreamingEngine.from_agent(agent, consumer, producer, "dialogues-classified", batch_max=32,
                                     max_latency_ms=1, explain="none")
    stats = eng.run(idle_timeout_s=0.2)
    assert stats["messages"] == len(texts) + 1 and stats["bad_messages"] == 1 and stats["broker_errors"] == 1
    out = broker.messages("dialogues-classified")
    assert len(out) == len(texts)
    by_key = {m.key(): json.loads(m.value()) for m in out}
    r0, r1 = by_key[b"id-0"], by_key[b"id-1"]
    assert r0["prediction"] == 1.0 and r1["prediction"] == 0.0
    assert r0["original_text"] == fixtures.SCAM_SAMPLE
    assert set(r0) == {"prediction", "confidence", "analysis", "historical_insight", "original_text"}
    # commit-after-produce: the group's committed offsets cover every partition's log end
    committed = consumer.committed_offsets()
    for p in range(3):
        assert committed[("customer-dialogues-raw", p)] == len(broker.topics["customer-dialogues-raw"][p])


def test_streaming_engine_async_explanations(shipped_model_path):
    broker = fake_kafka.broker_for("memory://async-test")
    broker.create_topic("in", 1)
    p = fake_kafka.Producer({"bootstrap.servers": "memory://async-test"})
    for i in range(5):
        p.produce("in", key=str(i), value=json.dumps({"text": fixtures.SCAM_SAMPLE}))
    c = fake_kafka.Consumer({"bootstrap.servers": "memory://async-test", "group.id": "g",
                             "auto.offset.reset": "earliest", "enable.auto.commit": False})
    c.subscribe(["in"])
    agent = ClassificationAgent(str(shipped_model_path), llm=StubLLM(), device="cpu")
    eng = StreamingEngine.from_agent(agent, c, p, "out", batch_max=8, max_latency_ms=1, explain="async")
    eng.run(idle_timeout_s=0.2)
    recs = [json.loads(m.value()) for m in broker.messages("out")]
    assert sum(1 for r in recs if r.get("type") == "explanation") == 5
    assert sum(1 for r in recs if "original_text" in r) == 5


def _trained_model_dir(tmp_path, kind="xgb"):
    """A small HashingTF->IDF->classifier pipeline trained on synthetic dialogues (self-contained:
    the GPU box has no /root/reference)."""
    from fraud_detection_spark_kafka_llm_amd.data import synth
    from fraud_detection_spark_kafka_llm_amd.ml import (IDF, Frame, HashingTF, LogisticRegression, Pipeline,
                                                         StopWordsRemover, TextColumn, Tokenizer)
    from fraud_detection_spark_kafka_llm_amd.ml.xgboost import SparkXGBClassifier

    pt, y = synth.generate(synth.SynthConfig(n=800, seed=21))
    raw = TextColumn(pt.strings())
    df = Frame({"dialogue": raw, "clean_text": TextColumn.cleaned_from(raw), "labels": y.numpy()})
    clf = SparkXGBClassifier(features_col="features", label_col="labels", n_estimators=20, max_depth=4) \
        if kind == "xgb" else LogisticRegression(featuresCol="features", labelCol="labels", maxIter=20)
    model = Pipeline(stages=[Tokenizer(inputCol="clean_text", outputCol="words"),
                             StopWordsRemover(inputCol="words", outputCol="filtered_words"),
                             HashingTF(inputCol="filtered_words", outputCol="raw_features", numFeatures=1 << 18),
                             IDF(inputCol="raw_features", outputCol="features"), clf]).fit(df)
    path = tmp_path / f"model_{kind}"
    model.save(str(path))
    return str(path)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["xgb", "lr"])
def test_gpu_streaming_engine_matches_host(tmp_path, kind):
    model_dir = _trained_model_dir(tmp_path, kind)
    broker = fake_kafka.broker_for(f"memory://gpu-test-{kind}")
    broker.create_topic("in", 3)
    p = fake_kafka.Producer({"bootstrap.servers": f"memory://gpu-test-{kind}"})
    from fraud_detection_spark_kafka_llm_amd.data import synth

    pt, _ = synth.generate(synth.SynthConfig(n=3000, seed=9))
    for i, t in enumerate(pt.strings()):
        p.produce("in", key=str(i), value=json.dumps({"text": t}))
    c = fake_kafka.Consumer({"bootstrap.servers": f"memory://gpu-test-{kind}", "group.id": "g",
                             "auto.offset.reset": "earliest", "enable.auto.commit": False})
    c.subscribe(["in"])
    agent = ClassificationAgent(model_dir, llm=StubLLM(), device="cuda:0")
    eng = StreamingEngine.from_agent(agent, c, p, "out", batch_max=512, max_latency_ms=2)
    stats = eng.run(idle_timeout_s=0.5)
    assert stats["produced"] == 3000
    host = ClassificationAgent(model_dir, llm=StubLLM(), device="cpu")
    recs = {int(m.key()): json.loads(m.value()) for m in broker.messages("out")}
    texts = pt.strings()
    ref = host.predict_batch(texts)
    for i in range(0, 3000, 97):
        assert recs[i]["prediction"] == ref[i]["prediction"]
        assert recs[i]["confidence"] == pytest.approx(ref[i]["confidence"], rel=1e-12, abs=1e-15)


def test_multi_scorer_round_robin_keeps_submission_order(tmp_path):
    from fraud_detection_spark_kafka_llm_amd.ops.text import FeatureSpec, LinearScorer
    from fraud_detection_spark_kafka_llm_amd.stream.gpu_worker import HostScorer, MultiGpuScorer
    from fraud_detection_spark_kafka_llm_amd.stream.ring import PinnedRing

    spec = FeatureSpec(clean=True, num_features=64)
    w = np.arange(64, dtype=np.float64) / 64.0
    scorers = [HostScorer(spec, None, LinearScorer(w, 0.1), max_docs=8, depth=2) for _ in range(3)]
    multi = MultiGpuScorer(scorers)
    assert multi.depth == 6
    ring = PinnedRing(slots=6, max_docs=8, max_bytes=4096, pin=False)
    single = HostScorer(spec, None, LinearScorer(w, 0.1), max_docs=8)
    want, got = [], []
    for i, slot in enumerate(ring.slots):
        slot.fill([f"message {i} number {j} bank" for j in range(i + 1)])
        want.append(single.score_packed(slot))
        multi.submit(slot)
    assert multi.inflight == 6
    while multi.inflight:
        got.append(multi.collect()[1])
    for a, b in zip(want, got):
        np.testing.assert_array_equal(a, b)


def test_serve_cli_consumes_classifies_and_commits(tmp_path, monkeypatch):
    from fraud_detection_spark_kafka_llm_amd.stream import serve

    model_dir = _trained_model_dir(tmp_path, "lr")
    url = "memory://serve-cli"
    monkeypatch.setenv("KAFKA_BOOTSTRAP_SERVERS", url)
    monkeypatch.setenv("KAFKA_OUTPUT_TOPIC", "out")
    broker = fake_kafka.broker_for(url)
    broker.create_topic("customer-dialogues-raw", 3)
    broker.create_topic("out", 3)
    p = fake_kafka.Producer({"bootstrap.servers": url})
    texts = ["please verify your bank account now", "see you at the dentist on friday", "urgent gift card payment"]
    for i in range(300):
        p.produce("customer-dialogues-raw", key=str(i), value=json.dumps({"text": texts[i % 3]}))
    assert serve.main(["--model", model_dir, "--gpus", "0", "--max-messages", "300", "--idle-timeout", "2"]) == 0
    c = fake_kafka.Consumer({"bootstrap.servers": url, "group.id": "check", "auto.offset.reset": "earliest"})
    c.subscribe(["out"])
    outs = c.consume(num_messages=1000, timeout=0.5)
    assert len(outs) == 300
    rec = json.loads(outs[0].value())
    assert set(rec) >= {"prediction", "confidence", "analysis", "historical_insight", "original_text"}


def test_native_record_encoding_is_byte_identical_to_json_dumps():
    import random

    import torch

    from fraud_detection_spark_kafka_llm_amd.ops import native

    C = native.lib()
    raw = [t.encode("utf-8") for t in ["say \"hi\" \\ \n\t\r\b\f \x01 \x7f é 中文 😀", "", "plain text"]]
    raw += [b"bad \xff utf8", b"\xed\xa0\x80 surrogate", b"over \xc0\xaf long", b"trunc \xe4\xb8"]
    vals = [0.0, 1.0, 0.0001, 1e-05, 4.13167538969518e-05, 0.9999999999165088, 1e16, 9999999999999998.0, 5e-324,
            float("nan"), float("inf"), -0.0, 0.1 + 0.2, 1.7976931348623157e308]
    rng = random.Random(1)
    vals += [rng.choice([rng.random(), rng.random() * 1e-6, 10 ** rng.uniform(-320, 300)]) for _ in range(3000)]
    n = len(vals)
    texts = [raw[i % len(raw)] for i in range(n)]
    data = torch.from_numpy(np.frombuffer(b"".join(texts) + b"\0" * 16, dtype=np.uint8).copy())
    off = torch.from_numpy(np.concatenate([[0], np.cumsum([len(t) for t in texts])]).astype(np.int64))
    pred, conf = torch.tensor(vals, dtype=torch.float64), torch.tensor(vals[::-1], dtype=torch.float64)
    skip = torch.zeros(n, dtype=torch.int32)
    skip[5] = 1
    out, oo, st = torch.empty(16, dtype=torch.uint8), torch.empty(n + 1, dtype=torch.int64), torch.empty(n, dtype=torch.int32)
    need = C.encode_records(pred, conf, data, off, skip, out, oo, st, 0)
    assert need < 0                                        # buffer too small -> required size
    out = torch.empty(-need, dtype=torch.uint8)
    assert C.encode_records(pred, conf, data, off, skip, out, oo, st, 0) == -need
    for i in range(n):
        if i == 5:
            assert st[i] == 2
            continue
        try:
            text = texts[i].decode("utf-8")
        except UnicodeDecodeError:
            assert st[i] == 1
            continue
        want = json.dumps({"prediction": vals[i], "confidence": vals[::-1][i], "analysis": None,
                           "historical_insight": None, "original_text": text})
        assert bytes(out[oo[i]:oo[i + 1]].numpy()).decode("ascii") == want


@pytest.mark.gpu
def test_gpu_scorer_long_dialogues_match_host():
    from fraud_detection_spark_kafka_llm_amd.ops.text import FeatureSpec, LinearScorer
    from fraud_detection_spark_kafka_llm_amd.stream.gpu_worker import GpuScorer, HostScorer
    from fraud_detection_spark_kafka_llm_amd.stream.ring import PinnedRing

    rng = np.random.default_rng(0)
    words = ["bank", "verify", "account", "please", "hello", "prize", "meeting", "doctor"]
    docs = [" ".join(rng.choice(words, int(k))) for k in rng.integers(1, 3000, 200)]   # up to ~20 KB
    docs += ["x" * 80000, "short one"]
    F = 1 << 12
    spec = FeatureSpec(clean=True, num_features=F)
    lr = LinearScorer(rng.standard_normal(F), -0.1)
    idf = rng.random(F)
    ring = PinnedRing(slots=1, max_docs=256, max_bytes=1 << 20)
    ring.slots[0].fill(docs)
    gpu = GpuScorer(spec, idf, lr, "cuda:0", max_docs=256, max_bytes=1 << 20)
    host = HostScorer(spec, idf, lr, max_docs=256, max_bytes=1 << 20)
    np.testing.assert_array_equal(gpu.score_packed(ring.slots[0]), host.score_packed(ring.slots[0]))


def test_serve_group_clients_refuses_in_memory_broker(tmp_path, monkeypatch):
    """--group-clients runs the Kafka clients in other processes: an in-process memory:// broker
    cannot be shared with them, so the CLI refuses it instead of serving an empty topic."""
    from fraud_detection_spark_kafka_llm_amd.stream import serve

    model_dir = _trained_model_dir(tmp_path, "lr")
    monkeypatch.setenv("KAFKA_BOOTSTRAP_SERVERS", "memory://serve-group")
    with pytest.raises(SystemExit, match="real Kafka bootstrap"):
        serve.main(["--model", model_dir, "--gpus", "0", "--group-clients", "2", "--max-messages", "10"])
