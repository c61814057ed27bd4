"""Kafka load generation and end-to-end measurement for the streaming engine (BASELINE config 5).

The reference measures nothing (its Streamlit loop handles one message per iteration,
/root/reference/app_ui.py:168-248); here two measurements run against the in-memory broker:

  * ``throughput_run`` — a topic pre-filled with N ``{"text": ...}`` records over P partitions;
    the engine (one reader per partition) consumes, scores, produces and commits all of them.
    dialogues/s = N / (first consume -> last delivery + commit).
  * ``latency_run`` — a paced producer thread appends records at a fixed rate (one columnar batch
    per partition every ``tick_ms``, stamped with its append time) while the engine runs; the
    per-message latency (append -> output delivered) percentiles come from the engine's histogram.

Records are views of a pool of distinct dialogues (no per-message Python objects anywhere).
"""
from __future__ import annotations

import json
import threading
import time
from typing import Callable

import numpy as np

from . import fake_kafka


class MessagePool:
    """``{"text": t}`` JSON values and ``id-i`` keys of distinct dialogues, columnar."""

    def __init__(self, texts: list):
        self.vals, self.voff, _ = fake_kafka.pack([json.dumps({"text": t}).encode() for t in texts])
        self.keys, self.koff, _ = fake_kafka.pack([f"id-{i}".encode() for i in range(len(texts))])
        self.n = len(texts)

    @property
    def avg_bytes(self) -> float:
        return float(self.voff[-1]) / max(self.n, 1)

    def batch(self, start: int, count: int, topic: str = "", partition: int = 0, ts=None) -> fake_kafka.RecordBatch:
        """Records [start, start+count) of the pool (wrapping), as views when they do not wrap."""
        s = start % self.n
        if s + count <= self.n:
            vo, ko = self.voff[s:s + count + 1], self.koff[s:s + count + 1]
            return fake_kafka.RecordBatch(topic, partition, 0, self.keys[ko[0]:ko[-1]], ko - ko[0],
                                          self.vals[vo[0]:vo[-1]], vo - vo[0], None, ts)
        a = self.batch(s, self.n - s)
        b = self.batch(0, count - (self.n - s))
        return fake_kafka.RecordBatch(topic, partition, 0, np.concatenate([a.keys, b.keys]),
                                      np.concatenate([a.key_off, b.key_off[1:] + a.key_off[-1]]),
                                      np.concatenate([a.values, b.values]),
                                      np.concatenate([a.val_off, b.val_off[1:] + a.val_off[-1]]), None, ts)


def prefill(broker: fake_kafka.Broker, topic: str, pool: MessagePool, n: int, partitions: int = 3,
            batch: int = 8192) -> None:
    broker.create_topic(topic, partitions)
    with broker.lock:
        for i, s in enumerate(range(0, n, batch)):
            p = i % partitions
            rb = pool.batch(s, min(batch, n - s), topic, p)
            broker.topics[topic][p].append(rb)
        broker.cond.notify_all()


class PacedProducer(threading.Thread):
    """Appends ``rate`` records/s for ``duration_s`` as one batch per partition per tick."""

    def __init__(self, broker: fake_kafka.Broker, topic: str, pool: MessagePool, rate: float, duration_s: float,
                 partitions: int = 3, tick_ms: float = 1.0):
        super().__init__(name="fdx-paced-producer", daemon=True)
        self.broker, self.topic, self.pool = broker, topic, pool
        self.rate, self.duration, self.parts, self.tick = rate, duration_s, partitions, tick_ms / 1000.0
        self.sent = 0
        broker.create_topic(topic, partitions)

    def run(self) -> None:
        t0 = time.perf_counter()
        nxt = t0
        while True:
            now = time.perf_counter()
            if now - t0 >= self.duration:
                return
            due = int((now - t0) * self.rate) - self.sent
            if due > 0:
                per = [due // self.parts + (1 if p < due % self.parts else 0) for p in range(self.parts)]
                with self.broker.lock:
                    for p, k in enumerate(per):
                        if k:
                            rb = self.pool.batch(self.sent, k, self.topic, p, ts=time.perf_counter())
                            self.broker.topics[self.topic][p].append(rb)
                            self.sent += k
                    self.broker.cond.notify_all()
            nxt += self.tick
            time.sleep(max(0.0, nxt - time.perf_counter()))


def _consumers(url: str, topic: str, partitions: int, group: str, confluent: bool = False) -> list:
    out = []
    for p in range(partitions):
        c = fake_kafka.Consumer({"bootstrap.servers": url, "group.id": group, "auto.offset.reset": "earliest",
                                 "enable.auto.commit": False})
        c.assign([fake_kafka.TopicPartition(topic, p)])
        out.append(fake_kafka.ConfluentConsumer(c) if confluent else c)
    return out


def _producer(url: str, confluent: bool):
    p = fake_kafka.Producer({"bootstrap.servers": url})
    return fake_kafka.ConfluentProducer(p) if confluent else p


def _committed(consumers: list) -> int:
    c = consumers[0]
    return sum(getattr(c, "_inner", c).committed_offsets().values())


def throughput_run(make_engine: Callable, pool: MessagePool, n: int, partitions: int = 3,
                   url: str = "memory://loadgen-tp", confluent: bool = False) -> dict:
    """``make_engine(consumers, producer, output_topic)`` -> StreamingEngine. ``confluent``: the
    clients expose only the confluent_kafka surface (per-record Messages and produce calls)."""
    broker = fake_kafka.broker_for(url)
    prefill(broker, "in", pool, n, partitions)
    broker.create_topic("out", partitions)
    consumers = _consumers(url, "in", partitions, "tp", confluent)
    eng = make_engine(consumers, _producer(url, confluent), "out")
    t0 = time.perf_counter()
    st = eng.run(max_messages=n, idle_timeout_s=5.0)
    dt = time.perf_counter() - t0
    committed = _committed(consumers)
    out_n = broker.size("out")
    _drop(url)
    return {"dialogues_per_s": n / dt, "sec": dt, "messages": st["messages"], "produced": st["produced"],
            "committed": committed, "output_records": out_n, "p50_ms": st["p50_ms"], "p95_ms": st["p95_ms"],
            "batches": st["batches"]}


def latency_run(make_engine: Callable, pool: MessagePool, rate: float, duration_s: float, partitions: int = 3,
                url: str = "memory://loadgen-lat", warmup_s: float = 0.3, confluent: bool = False) -> dict:
    broker = fake_kafka.broker_for(url)
    broker.create_topic("in", partitions)
    broker.create_topic("out", partitions)
    consumers = _consumers(url, "in", partitions, "lat", confluent)
    eng = make_engine(consumers, _producer(url, confluent), "out")
    gen = PacedProducer(broker, "in", pool, rate, duration_s + warmup_s, partitions)
    res = {}

    def reset_after_warmup():
        time.sleep(warmup_s)
        eng.stats.latency.reset()

    threading.Thread(target=reset_after_warmup, daemon=True).start()
    gen.start()
    t0 = time.perf_counter()
    st = eng.run(idle_timeout_s=0.5)
    gen.join()
    res.update({"offered_per_s": rate, "sent": gen.sent, "messages": st["messages"], "produced": st["produced"],
                "p50_ms": st["p50_ms"], "p95_ms": st["p95_ms"], "p99_ms": st["p99_ms"],
                "p50_batch_ms": st["p50_batch_ms"], "batches": st["batches"], "sec": time.perf_counter() - t0,
                "committed": _committed(consumers)})
    _drop(url)
    return res


def _drop(url: str) -> None:
    fake_kafka._BROKERS.pop(url, None)
