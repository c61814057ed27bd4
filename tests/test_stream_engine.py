"""Streaming engine v2: per-partition readers, carry-over of slot overflow, delivery-gated commits,
the in-memory broker's confluent-compatible contracts (test strategy: SURVEY.md §4, X-20)."""
import json

import numpy as np
import pytest

from fraud_detection_spark_kafka_llm_amd.data import fixtures
from fraud_detection_spark_kafka_llm_amd.serve.agent import ClassificationAgent
from fraud_detection_spark_kafka_llm_amd.serve.llm import StubLLM
from fraud_detection_spark_kafka_llm_amd.stream import fake_kafka, kafka
from fraud_detection_spark_kafka_llm_amd.stream.engine import LatencyHistogram, StreamingEngine


def _conf(url, group="g"):
    return {"bootstrap.servers": url, "group.id": group, "auto.offset.reset": "earliest",
            "enable.auto.commit": False}


def _fill(url, topic, texts, parts=3):
    broker = fake_kafka.broker_for(url)
    broker.create_topic(topic, parts)
    p = fake_kafka.Producer({"bootstrap.servers": url})
    for i, t in enumerate(texts):
        p.produce(topic, key=f"k{i}", value=json.dumps({"text": t}))
    return broker


@pytest.fixture(scope="module")
def agent(shipped_model_path):
    return ClassificationAgent(str(shipped_model_path), llm=StubLLM(), device="cpu")


def test_commit_contract_matches_confluent():
    url = "memory://contract"
    broker = _fill(url, "t", ["a", "b"], parts=1)
    c = fake_kafka.Consumer(_conf(url))
    c.subscribe(["t"])
    m = c.poll(0.1)
    with pytest.raises(TypeError):
        c.commit(message=object())               # confluent type-checks cimpl.Message
    with pytest.raises(TypeError):
        c.commit(offsets=[("t", 0, 1)])
    c.commit(offsets=[fake_kafka.TopicPartition("t", 0, m.offset() + 1)])
    assert c.committed([fake_kafka.TopicPartition("t", 0)])[0].offset == 1
    assert len(broker.topics["t"][0]) == 2


def test_columnar_consume_and_produce_records():
    url = "memory://columnar"
    broker = _fill(url, "t", [f"m{i}" for i in range(10)], parts=1)
    c = fake_kafka.Consumer(_conf(url))
    c.assign([fake_kafka.TopicPartition("t", 0)])
    rbs = c.consume_batches(7, 0.1)
    assert sum(r.n for r in rbs) == 7 and rbs[0].base_offset == 0
    rest = c.consume_batches(100, 0.1)
    assert sum(r.n for r in rest) == 3 and rest[0].base_offset == 7
    assert json.loads(rest[-1].value(rest[-1].n - 1))["text"] == "m9"
    p = fake_kafka.Producer({"bootstrap.servers": url})
    got = []
    keys, ko, _ = fake_kafka.pack([b"x", b"yy"])
    vals, vo, _ = fake_kafka.pack([b"1", b"22"])
    p.produce_records("o", 0, keys, ko, vals, vo, on_delivery=lambda err, rb: got.append((err, rb.n)))
    assert got == []                      # delivery reports are served by poll/flush
    p.flush()
    assert got == [(None, 2)]
    assert [(m.key(), m.value()) for m in broker.messages("o")] == [(b"x", b"1"), (b"yy", b"22")]


def test_partition_readers_commit_only_delivered(agent, monkeypatch):
    url = "memory://readers"
    texts = [fixtures.SCAM_SAMPLE, fixtures.BENIGN_SAMPLE, "hello there"] * 100
    broker = _fill(url, "in", texts)
    monkeypatch.setenv("KAFKA_BOOTSTRAP_SERVERS", url)
    consumers = kafka.get_partition_consumers("in", group="g2")
    assert len(consumers) == 3
    prod = fake_kafka.Producer({"bootstrap.servers": url})
    eng = StreamingEngine.from_agent(agent, consumers, prod, "out", batch_max=64, max_latency_ms=2)
    st = eng.run(idle_timeout_s=0.3)
    assert st["messages"] == 300 and st["produced"] == 300 and st["delivery_errors"] == 0
    assert st["p50_ms"] > 0 and st["p95_ms"] >= st["p50_ms"]
    committed = consumers[0].committed_offsets()
    for p in range(3):
        assert committed[("in", p)] == len(broker.topics["in"][p])
    recs = {m.key(): json.loads(m.value()) for m in broker.messages("out")}
    assert recs[b"k0"]["prediction"] == 1.0 and recs[b"k0"]["original_text"] == fixtures.SCAM_SAMPLE


@pytest.mark.parametrize("inline", ["", "0"])
def test_confluent_surface_clients_take_the_per_record_path(agent, monkeypatch, inline):
    """FDX_KAFKA_COLUMNAR=0: clients expose only the confluent_kafka API (per-record Messages and
    produce calls) — the path a librdkafka client takes (native pack_messages / produce_each).
    Default: the partition reader runs on the engine thread (inline); "0": reader threads."""
    monkeypatch.setenv("FDX_STREAM_INLINE", inline)
    url = "memory://confluent-surface" + inline
    texts = [fixtures.SCAM_SAMPLE, fixtures.BENIGN_SAMPLE, "hello there"] * 40
    broker = _fill(url, "in", texts)
    nullkey = fake_kafka.Producer({"bootstrap.servers": url})
    nullkey.produce("in", key=None, value=json.dumps({"text": "no key here"}), partition=0)
    nullkey.produce("in", key=b"bad", value=b"{not json", partition=1)
    monkeypatch.setenv("KAFKA_BOOTSTRAP_SERVERS", url)
    monkeypatch.setenv("FDX_KAFKA_COLUMNAR", "0")
    c = kafka.get_kafka_consumer(["in"], group="cs")        # one consumer over all 3 partitions
    prod = kafka.get_kafka_producer()
    assert not hasattr(c, "consume_batches") and not hasattr(prod, "produce_records")
    eng = StreamingEngine.from_agent(agent, c, prod, "out", batch_max=32, max_latency_ms=1)
    st = eng.run(idle_timeout_s=0.3)
    assert st["messages"] == 122 and st["produced"] == 121 and st["bad_messages"] == 1
    assert st["delivery_errors"] == 0
    out = broker.messages("out")
    recs = {m.key(): json.loads(m.value()) for m in out}
    assert all(recs[f"k{i}".encode()]["original_text"] == texts[i] for i in range(len(texts)))
    assert recs[b"k0"]["prediction"] == 1.0
    assert [json.loads(m.value())["original_text"] for m in out if m.key() is None] == ["no key here"]
    got = c.committed([fake_kafka.TopicPartition("in", p) for p in range(3)])
    assert [tp.offset for tp in got] == [len(broker.topics["in"][p]) for p in range(3)]


def test_failed_delivery_blocks_that_partitions_commit(agent):
    url = "memory://faildeliver"
    broker = _fill(url, "in", ["a b c"] * 30, parts=1)
    c = fake_kafka.Consumer(_conf(url))
    c.subscribe(["in"])
    prod = fake_kafka.Producer({"bootstrap.servers": url})
    prod.fail_next = 1                    # the first micro-batch's output is rejected
    eng = StreamingEngine.from_agent(agent, c, prod, "out", batch_max=8, max_latency_ms=1)
    st = eng.run(idle_timeout_s=0.2)
    assert st["delivery_errors"] == 1 and st["produced"] == 30 - 8
    # at-least-once: nothing past the failed segment is committed, so a restart re-reads it
    assert c.committed_offsets().get(("in", 0), 0) == 0


@pytest.mark.parametrize("inline", ["", "1"])
def test_slot_overflow_is_carried_over_not_lost(agent, monkeypatch, inline):
    monkeypatch.setenv("FDX_STREAM_INLINE", inline)
    url = "memory://overflow" + inline
    texts = [("word " * 150)[:700] + str(i) for i in range(40)] + ["x" * 5000]
    broker = _fill(url, "in", texts, parts=1)
    c = fake_kafka.Consumer(_conf(url))
    c.subscribe(["in"])
    prod = fake_kafka.Producer({"bootstrap.servers": url})
    eng = StreamingEngine.from_agent(agent, c, prod, "out", batch_max=32, max_latency_ms=1, max_bytes=4096)
    st = eng.run(idle_timeout_s=0.2)
    # 40 records of ~700 bytes do not fit a 4 KB slot in one go: every one is carried over and
    # scored; the 5 KB record can never fit and is rejected as a bad message (and committed)
    assert st["messages"] == 41 and st["produced"] == 40 and st["bad_messages"] == 1
    out = {m.key(): json.loads(m.value())["original_text"] for m in broker.messages("out")}
    assert all(out[f"k{i}".encode()] == texts[i] for i in range(40))
    assert c.committed_offsets()[("in", 0)] == 41


def test_max_messages_quota_is_exact(agent):
    url = "memory://quota"
    broker = _fill(url, "in", ["some dialogue text"] * 200)
    consumers = []
    for p in range(3):
        c = fake_kafka.Consumer(_conf(url, "q"))
        c.assign([fake_kafka.TopicPartition("in", p)])
        consumers.append(c)
    prod = fake_kafka.Producer({"bootstrap.servers": url})
    eng = StreamingEngine.from_agent(agent, consumers, prod, "out", batch_max=16, max_latency_ms=1)
    st = eng.run(max_messages=50, idle_timeout_s=0.2)
    assert st["messages"] == 50 and broker.size("out") == 50
    assert sum(consumers[0].committed_offsets().values()) == 50


def test_async_explanations_are_sampled_and_bounded(agent):
    url = "memory://explain-sample"
    _fill(url, "in", [fixtures.SCAM_SAMPLE] * 40, parts=1)
    c = fake_kafka.Consumer(_conf(url))
    c.subscribe(["in"])
    prod = fake_kafka.Producer({"bootstrap.servers": url})
    eng = StreamingEngine.from_agent(agent, c, prod, "out", batch_max=16, max_latency_ms=1, explain="async",
                                     explain_every=10)
    st = eng.run(idle_timeout_s=0.2)
    recs = [json.loads(m.value()) for m in fake_kafka.broker_for(url).messages("out")]
    assert st["explanations"] == 4 and sum(1 for r in recs if r.get("type") == "explanation") == 4


def test_real_bootstrap_without_client_library_raises(monkeypatch):
    try:
        import confluent_kafka  # noqa: F401
        pytest.skip("confluent_kafka installed")
    except ImportError:
        pass
    monkeypatch.setenv("KAFKA_BOOTSTRAP_SERVERS", "broker-1:9092")
    monkeypatch.delenv("FDX_KAFKA", raising=False)
    with pytest.raises(ImportError):
        kafka.get_kafka_producer()
    monkeypatch.setenv("FDX_KAFKA", "memory")
    assert isinstance(kafka.get_kafka_producer(), fake_kafka.Producer)


def test_latency_histogram_percentiles():
    h = LatencyHistogram()
    h.add(np.linspace(1.0, 100.0, 10000))
    assert h.percentile(50) == pytest.approx(50.5, rel=0.02)
    assert h.percentile(95) == pytest.approx(95.05, rel=0.02)


def test_pack_messages_reads_any_message_class_and_reuses_buffers():
    """pack_messages: the in-memory Message's items directly, any other class through its methods
    (as cimpl.Message), errors listed apart; values into a caller buffer when it is large enough."""
    from fraud_detection_spark_kafka_llm_amd.ops import native

    class Msg:                                    # method surface only (like confluent_kafka's)
        def __init__(self, t, p, o, k, v, err=None):
            self._f = (t, p, o, k, v, err)

        def topic(self):
            return self._f[0]

        def partition(self):
            return self._f[1]

        def offset(self):
            return self._f[2]

        def key(self):
            return self._f[3]

        def value(self):
            return self._f[4]

        def error(self):
            return self._f[5]

        def timestamp(self):
            return (1, 1234)

    fake_kafka._native()                          # registers the in-memory Message class
    a = tuple.__new__(fake_kafka.Message, ("t", 0, 5, b"k1", b"value-one", None, 99))     # ts in ms
    b = Msg("t", 0, 6, None, b"v2")
    e = Msg("t", 0, -1, None, None, err=fake_kafka.KafkaError(1, "boom"))
    c = tuple.__new__(fake_kafka.Message, ("t", 1, 7, b"k3", b"third", None, None))
    for buf in (None, np.zeros(64, dtype=np.uint8), np.zeros(3, dtype=np.uint8)):
        part_of, parts, kb, ko, nk, vb, vo, offs, ts, errs = native.lib().pack_messages([a, b, e, c], buf)
        assert [tuple(x) for x in parts] == [("t", 0), ("t", 1)] and part_of.tolist() == [0, 0, 1]
        assert bytes(vb) == b"value-onev2third" and vo.tolist() == [0, 9, 11, 16]
        assert bytes(kb) == b"k1k3" and ko.tolist() == [0, 2, 2, 4] and nk.tolist() == [0, 1, 0]
        assert offs.tolist() == [5, 6, 7] and ts.tolist() == [99, 1234, -1]
        assert [i for i, _ in errs] == [2]
        if buf is not None and buf.size >= 16:
            assert bytes(buf[:16]) == b"value-onev2third"      # written in place


def test_extract_from_value_references_equals_packed_extraction():
    """extract_json_field_refs (values read in place) gives the packed path's bytes and statuses."""
    import torch

    from fraud_detection_spark_kafka_llm_amd.ops import native

    vals = [json.dumps({"text": f"doc {i} " + "w" * (i % 7), "n": i}).encode() for i in range(50)]
    vals[3], vals[9], vals[17] = None, b"{not json", json.dumps({"other": 1}).encode()
    C = native.lib()
    buf, off, _ = fake_kafka.pack([v if v is not None else b"" for v in vals])
    outs = []
    for refs in (False, True):
        out = torch.zeros(4096, dtype=torch.uint8)
        oo = torch.zeros(len(vals) + 1, dtype=torch.int64)
        st = np.zeros(len(vals), dtype=np.int32)
        if refs:
            total = C.extract_json_field_refs(vals, len(vals), "text", out, oo, torch.from_numpy(st), 0)
        else:
            total = C.extract_json_field(torch.from_numpy(buf), torch.from_numpy(off), "text", out, oo,
                                         torch.from_numpy(st), 0)
        outs.append((bytes(out[:total].numpy()), oo.tolist(), st.tolist()))
    assert outs[0] == outs[1]
    assert outs[1][2][3] == outs[1][2][9] == outs[1][2][17] == 1 and outs[1][2][0] == 0
