"""Kafka consumer/producer factories (R-18, R-19), reading the reference's environment variables.

``KAFKA_BOOTSTRAP_SERVERS`` (default ``localhost:9092``), ``KAFKA_CONSUMER_GROUP``
(``dialogue-classifier-group``), ``KAFKA_INPUT_TOPIC`` (``customer-dialogues-raw``),
``KAFKA_SECURITY_PROTOCOL=SASL_SSL`` + ``KAFKA_USERNAME``/``KAFKA_PASSWORD`` (SASL PLAIN);
consumer: ``auto.offset.reset=earliest``, ``enable.auto.commit=False`` (/root/reference/utils/
kafka_utils.py:11-49). The backend is confluent_kafka (librdkafka) when importable and the
bootstrap is a real address; ``memory://...`` bootstraps (or ``FDX_KAFKA=memory``) select the
in-memory broker of ``fake_kafka`` — used by tests, benchmarks and offline demos.
``FDX_KAFKA_COLUMNAR=0`` hands out in-memory clients restricted to the confluent_kafka surface
(per-record Messages / produce calls, no columnar batches): the path a real librdkafka client
takes through the streaming engine, measurable without a broker.
"""
from __future__ import annotations

import os
from typing import Optional

from . import fake_kafka

DEFAULT_BOOTSTRAP = "localhost:9092"
DEFAULT_GROUP = "dialogue-classifier-group"
DEFAULT_INPUT = "customer-dialogues-raw"
DEFAULT_OUTPUT = "dialogues-classified"


def _security(conf: dict) -> dict:
    if os.getenv("KAFKA_SECURITY_PROTOCOL") == "SASL_SSL":
        conf.update({"security.protocol": "SASL_SSL", "sasl.mechanisms": "PLAIN",
                     "sasl.username": os.getenv("KAFKA_USERNAME"), "sasl.password": os.getenv("KAFKA_PASSWORD")})
    return conf


def _use_memory(bootstrap: str) -> bool:
    """In-memory broker only when asked for (``memory://`` or ``FDX_KAFKA=memory``): a real
    bootstrap without confluent_kafka is an error, never a silent switch to a private broker."""
    if bootstrap.startswith("memory://") or os.getenv("FDX_KAFKA", "").lower() == "memory":
        return True
    try:
        import confluent_kafka  # noqa: F401
    except ImportError as e:
        raise ImportError(f"confluent_kafka is required for bootstrap {bootstrap!r}; install it, or use a "
                          "memory:// bootstrap / FDX_KAFKA=memory for the in-memory broker") from e
    return False


def _columnar() -> bool:
    return os.getenv("FDX_KAFKA_COLUMNAR", "1") != "0"


def _mem_consumer(conf: dict):
    c = fake_kafka.Consumer(conf)
    return c if _columnar() else fake_kafka.ConfluentConsumer(c)


def _mem_producer(conf: dict):
    p = fake_kafka.Producer(conf)
    return p if _columnar() else fake_kafka.ConfluentProducer(p)


def consumer_config(group: Optional[str] = None) -> dict:
    return _security({"bootstrap.servers": os.getenv("KAFKA_BOOTSTRAP_SERVERS", DEFAULT_BOOTSTRAP),
                      "group.id": group or os.getenv("KAFKA_CONSUMER_GROUP", DEFAULT_GROUP),
                      "auto.offset.reset": "earliest", "enable.auto.commit": False})


def producer_config() -> dict:
    return _security({"bootstrap.servers": os.getenv("KAFKA_BOOTSTRAP_SERVERS", DEFAULT_BOOTSTRAP)})


def get_kafka_consumer(topics=None, group: Optional[str] = None):
    conf = consumer_config(group)
    if _use_memory(conf["bootstrap.servers"]):
        c = _mem_consumer(conf)
    else:
        from confluent_kafka import Consumer

        c = Consumer(conf)
    c.subscribe(list(topics) if topics else [os.getenv("KAFKA_INPUT_TOPIC", DEFAULT_INPUT)])
    return c


def get_partition_consumers(topic: Optional[str] = None, group: Optional[str] = None) -> list:
    """One consumer per partition of ``topic`` (static ``assign``, same group): the streaming
    engine runs one reader thread per consumer. Starting offsets are the group's commits."""
    conf = consumer_config(group)
    topic = topic or os.getenv("KAFKA_INPUT_TOPIC", DEFAULT_INPUT)
    if _use_memory(conf["bootstrap.servers"]):
        nparts = fake_kafka.broker_for(conf["bootstrap.servers"]).partitions(topic)
        out = []
        for p in range(nparts):
            c = _mem_consumer(conf)
            c.assign([fake_kafka.TopicPartition(topic, p)])
            out.append(c)
        return out
    from confluent_kafka import Consumer, TopicPartition

    probe = Consumer(conf)
    nparts = len(probe.list_topics(topic, timeout=10).topics[topic].partitions)
    probe.close()
    out = []
    for p in range(nparts):
        c = Consumer(conf)
        c.assign([TopicPartition(topic, p)])
        out.append(c)
    return out


def get_kafka_producer():
    conf = producer_config()
    if _use_memory(conf["bootstrap.servers"]):
        return _mem_producer(conf)
    from confluent_kafka import Producer

    return Producer(conf)


def output_topic() -> Optional[str]:
    return os.getenv("KAFKA_OUTPUT_TOPIC")


def kafka_exception_class():
    try:
        from confluent_kafka import KafkaException

        return KafkaException
    except ImportError:
        return fake_kafka.KafkaException
