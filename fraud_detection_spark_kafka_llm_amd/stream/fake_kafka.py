"""In-memory Kafka broker with the confluent_kafka Consumer/Producer surface (test double, X-20).

Implements what the reference and the streaming engine use: topics with N partitions, keyed
partitioning (murmur-free: stable hash of the key), consumer groups with committed offsets,
``auto.offset.reset`` earliest/latest, ``enable.auto.commit``, ``subscribe / poll / consume /
commit / committed / close``, ``produce(topic, value, key, on_delivery) / poll / flush``,
``Message.key/value/topic/partition/offset/error``. Fault injection: ``broker.inject_error``
makes the next poll of a topic return an error message (the reference kills its loop on these,
app_ui.py:200-201; the engine skips and logs them).
"""
from __future__ import annotations

import threading
import time
import zlib
from collections import defaultdict
from typing import Callable, Optional


class KafkaError:
    _PARTITION_EOF = -191
    UNKNOWN = -1

    def __init__(self, code: int = -1, reason: str = "error", fatal: bool = False):
        self._code, self._reason, self._fatal = code, reason, fatal

    def code(self) -> int:
        return self._code

    def str(self) -> str:  # noqa: A003
        return self._reason

    def fatal(self) -> bool:
        return self._fatal

    def __repr__(self) -> str:
        return f"KafkaError({self._code}, {self._reason!r})"


class KafkaException(Exception):
    pass


class Message:
    __slots__ = ("_topic", "_partition", "_offset", "_key", "_value", "_error", "_ts")

    def __init__(self, topic, partition, offset, key, value, error=None):
        self._topic, self._partition, self._offset = topic, partition, offset
        self._key, self._value, self._error = key, value, error
        self._ts = time.time()

    def topic(self):
        return self._topic

    def partition(self):
        return self._partition

    def offset(self):
        return self._offset

    def key(self):
        return self._key

    def value(self):
        return self._value

    def error(self):
        return self._error

    def timestamp(self):
        return (1, int(self._ts * 1000))


def _b(v) -> Optional[bytes]:
    if v is None:
        return None
    return v.encode("utf-8") if isinstance(v, str) else bytes(v)


class Broker:
    def __init__(self):
        self.lock = threading.RLock()
        self.topics: dict = {}
        self.committed: dict = defaultdict(dict)    # group -> {(topic, part): next offset}
        self._errors: dict = defaultdict(int)
        self.cond = threading.Condition(self.lock)

    def create_topic(self, name: str, partitions: int = 3) -> None:
        with self.lock:
            self.topics.setdefault(name, [[] for _ in range(partitions)])

    def partitions(self, topic: str) -> int:
        with self.lock:
            self.create_topic(topic)
            return len(self.topics[topic])

    def append(self, topic: str, key, value, partition: Optional[int] = None) -> Message:
        with self.lock:
            self.create_topic(topic)
            parts = self.topics[topic]
            if partition is None or partition < 0:
                partition = (zlib.crc32(key) if key else zlib.crc32(value or b"") ^ len(parts[0])) % len(parts)
            m = Message(topic, partition, len(parts[partition]), key, value)
            parts[partition].append(m)
            self.cond.notify_all()
            return m

    def append_many(self, topic: str, keys: list, values: list) -> None:
        """Batch append (one lock / one wake-up for the whole batch); same partitioning as append."""
        with self.lock:
            self.create_topic(topic)
            parts = self.topics[topic]
            np_ = len(parts)
            for key, value in zip(keys, values):
                partition = (zlib.crc32(key) if key else zlib.crc32(value or b"") ^ len(parts[0])) % np_
                parts[partition].append(Message(topic, partition, len(parts[partition]), key, value))
            self.cond.notify_all()

    def inject_error(self, topic: str, count: int = 1) -> None:
        with self.lock:
            self._errors[topic] += count

    def take_error(self, topic: str) -> bool:
        with self.lock:
            if self._errors[topic] > 0:
                self._errors[topic] -= 1
                return True
            return False

    def size(self, topic: str) -> int:
        with self.lock:
            return sum(len(p) for p in self.topics.get(topic, []))

    def messages(self, topic: str) -> list:
        with self.lock:
            return [m for p in self.topics.get(topic, []) for m in p]


_DEFAULT = Broker()
_BROKERS: dict = {}


def broker_for(bootstrap: str) -> Broker:
    if not bootstrap or bootstrap.startswith("memory://default"):
        return _DEFAULT
    return _BROKERS.setdefault(bootstrap, Broker())


class Consumer:
    def __init__(self, config: dict, broker: Optional[Broker] = None):
        self.config = dict(config)
        self.broker = broker or broker_for(self.config.get("bootstrap.servers", ""))
        self.group = self.config.get("group.id", "default")
        self.auto_commit = bool(self.config.get("enable.auto.commit", True))
        self.reset = self.config.get("auto.offset.reset", "latest")
        self.topics: list = []
        self.positions: dict = {}
        self.closed = False
        self._rr = 0

    def subscribe(self, topics, on_assign=None, on_revoke=None) -> None:
        self.topics = list(topics)
        with self.broker.lock:
            for t in self.topics:
                for p in range(self.broker.partitions(t)):
                    c = self.broker.committed[self.group].get((t, p))
                    if c is None:
                        c = 0 if self.reset in ("earliest", "smallest", "beginning") else len(self.broker.topics[t][p])
                    self.positions[(t, p)] = c

    def assignment(self) -> list:
        return list(self.positions)

    def _next(self) -> Optional[Message]:
        with self.broker.lock:
            for t in self.topics:
                if self.broker.take_error(t):
                    return Message(t, -1, -1, None, None, KafkaError(KafkaError.UNKNOWN, "injected broker error"))
            keys = list(self.positions)
            for i in range(len(keys)):
                k = keys[(self._rr + i) % len(keys)]
                t, p = k
                log = self.broker.topics[t][p]
                if self.positions[k] < len(log):
                    m = log[self.positions[k]]
                    self.positions[k] += 1
                    self._rr = (self._rr + i + 1) % len(keys)
                    if self.auto_commit:
                        self.broker.committed[self.group][k] = self.positions[k]
                    return m
        return None

    def poll(self, timeout: float = -1) -> Optional[Message]:
        if self.closed:
            raise RuntimeError("Consumer closed")
        deadline = time.time() + (timeout if timeout and timeout > 0 else 0)
        while True:
            m = self._next()
            if m is not None or time.time() >= deadline:
                return m
            with self.broker.cond:
                self.broker.cond.wait(timeout=min(0.05, max(0.0, deadline - time.time())))

    def consume(self, num_messages: int = 1, timeout: float = -1) -> list:
        out = []
        deadline = time.time() + (timeout if timeout and timeout > 0 else 0)
        while len(out) < num_messages:
            m = self._next()
            if m is None:
                if time.time() >= deadline:
                    break
                with self.broker.cond:
                    self.broker.cond.wait(timeout=min(0.05, max(0.0, deadline - time.time())))
                continue
            out.append(m)
            if m.error():
                break
        return out

    def commit(self, message: Optional[Message] = None, offsets=None, asynchronous: bool = True):
        with self.broker.lock:
            if message is not None:
                self.broker.committed[self.group][(message.topic(), message.partition())] = message.offset() + 1
            elif offsets:
                for tp in offsets:
                    self.broker.committed[self.group][(tp.topic, tp.partition)] = tp.offset
            else:
                for k, v in self.positions.items():
                    self.broker.committed[self.group][k] = v
        return None

    def committed_offsets(self) -> dict:
        with self.broker.lock:
            return dict(self.broker.committed[self.group])

    def close(self) -> None:
        if self.auto_commit:
            self.commit()
        self.closed = True


class Producer:
    def __init__(self, config: dict, broker: Optional[Broker] = None):
        self.config = dict(config)
        self.broker = broker or broker_for(self.config.get("bootstrap.servers", ""))
        self._pending: list = []
        self.lock = threading.Lock()

    def produce(self, topic: str, value=None, key=None, partition: int = -1, on_delivery: Optional[Callable] = None,
                callback: Optional[Callable] = None, **kw) -> None:
        if topic is None:
            raise TypeError("topic must be a str (KAFKA_OUTPUT_TOPIC unset?)")
        m = self.broker.append(topic, _b(key), _b(value), partition)
        cb = on_delivery or callback
        if cb is not None:
            with self.lock:
                self._pending.append((cb, m))

    def produce_batch(self, topic: str, keys: list, values: list) -> None:
        """Many messages at once (no delivery callbacks): what the streaming engine uses when the
        producer offers it; librdkafka producers get per-message ``produce`` calls instead."""
        if topic is None:
            raise TypeError("topic must be a str (KAFKA_OUTPUT_TOPIC unset?)")
        self.broker.append_many(topic, [_b(k) for k in keys], [_b(v) for v in values])

    def poll(self, timeout: float = 0) -> int:
        with self.lock:
            pend, self._pending = self._pending, []
        for cb, m in pend:
            cb(None, m)
        return len(pend)

    def flush(self, timeout: float = -1) -> int:
        self.poll(0)
        return 0

    def __len__(self) -> int:
        return len(self._pending)
