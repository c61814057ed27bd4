"""In-memory Kafka broker with the confluent_kafka Consumer/Producer surface (test double, X-20).

Implements what the reference and the streaming engine use: topics with N partitions, keyed
partitioning (stable crc32 of the key), consumer groups with committed offsets,
``auto.offset.reset`` earliest/latest, ``enable.auto.commit``, ``subscribe / assign / poll /
consume / commit / committed / close``, ``produce(topic, value, key, on_delivery) / poll / flush``,
``Message.key/value/topic/partition/offset/error``, ``TopicPartition``. Fault injection:
``broker.inject_error`` makes the next poll of a topic return an error message (the reference
kills its loop on these, app_ui.py:200-201; the engine skips and logs them).

Partitions store columnar record batches (keys / values as one byte buffer + offsets each, like
Kafka's own record batches), so the streaming engine can move a whole micro-batch per call
(``Consumer.consume_batches``, ``Producer.produce_records``) without a Python object per message;
``poll``/``consume`` materialise per-message ``Message`` objects for the reference-style API.
``Consumer.commit`` type-checks like confluent_kafka: ``message=`` must be a ``Message``; offsets go
through ``offsets=[TopicPartition(topic, partition, next_offset)]``.
"""
from __future__ import annotations

import bisect
import threading
import time
import zlib
from collections import defaultdict
from typing import Callable, Optional
from zlib import crc32

import numpy as np


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


class TopicPartition:
    """confluent_kafka.TopicPartition: (topic, partition, offset)."""

    def __init__(self, topic: str, partition: int = -1, offset: int = -1001):
        self.topic, self.partition, self.offset = topic, int(partition), int(offset)

    def __repr__(self) -> str:
        return f"TopicPartition({self.topic!r}, {self.partition}, {self.offset})"

    def __eq__(self, o) -> bool:
        return (self.topic, self.partition, self.offset) == (o.topic, o.partition, o.offset)

    def __hash__(self) -> int:
        return hash((self.topic, self.partition, self.offset))


class Message(tuple):
    """confluent_kafka.Message: (topic, partition, offset, key, value, error, timestamp ms), a tuple
    underneath so a consume of many records builds them without a Python __init__ per record."""
    __slots__ = ()

    def __new__(cls, topic, partition, offset, key, value, error=None, ts=None):
        return tuple.__new__(cls, (topic, partition, offset, key, value, error,
                                   int((time.time() if ts is None else ts) * 1000)))

    def topic(self):
        return self[0]

    def partition(self):
        return self[1]

    def offset(self):
        return self[2]

    def key(self):
        return self[3]

    def value(self):
        return self[4]

    def error(self):
        return self[5]

    def timestamp(self):
        return (1, self[6])


_NATIVE = [False, None]


def _native():
    """The native core's broker fast paths (C-speed Message accessors, batch -> Messages, per-record
    produce), as a librdkafka client would run them; None without the built extension or with
    FDX_KAFKA_NATIVE=0 (the pure-Python broker)."""
    if not _NATIVE[0]:
        _NATIVE[0] = True
        import os
        if os.environ.get("FDX_KAFKA_NATIVE", "1") != "0":
            try:
                from ..ops import native
                lib = native.lib()
                lib.install_message_accessors(Message)
                _NATIVE[1] = lib
            except Exception:                    # noqa: BLE001 (no extension: pure Python)
                _NATIVE[1] = None
    return _NATIVE[1]


def _b(v) -> Optional[bytes]:
    if v is None:
        return None
    return v.encode("utf-8") if isinstance(v, str) else bytes(v)


def pack(items: list) -> tuple:
    """bytes-like items (None allowed) -> (uint8 buffer, int64 offsets [n+1], null mask or None)."""
    null = [v is None for v in items]
    bs = [b"" if v is None else _b(v) for v in items]
    off = np.zeros(len(bs) + 1, dtype=np.int64)
    np.cumsum(np.fromiter((len(v) for v in bs), dtype=np.int64, count=len(bs)), out=off[1:])
    buf = np.frombuffer(b"".join(bs), dtype=np.uint8).copy() if bs else np.zeros(0, np.uint8)
    return buf, off, (np.asarray(null) if any(null) else None)


class RecordBatch:
    """Columnar records of one partition: keys/values as byte buffers + offsets, consecutive
    offsets from ``base_offset``, one append timestamp (seconds, ``time.perf_counter`` clock)."""
    __slots__ = ("topic", "partition", "base_offset", "keys", "key_off", "values", "val_off", "null_keys", "ts")

    def __init__(self, topic, partition, base_offset, keys, key_off, values, val_off, null_keys=None, ts=None):
        self.topic, self.partition, self.base_offset = topic, partition, base_offset
        self.keys, self.key_off, self.values, self.val_off = keys, key_off, values, val_off
        self.null_keys = null_keys
        self.ts = time.perf_counter() if ts is None else ts

    @property
    def n(self) -> int:
        return int(self.val_off.size - 1)

    @property
    def last_offset(self) -> int:
        return self.base_offset + self.n - 1

    def slice(self, a: int, b: int) -> "RecordBatch":
        """Records [a, b) (views of the byte buffers, rebased offsets)."""
        ko, vo = self.key_off[a:b + 1], self.val_off[a:b + 1]
        nk = self.null_keys[a:b] if self.null_keys is not None else None
        return RecordBatch(self.topic, self.partition, self.base_offset + a, self.keys[ko[0]:ko[-1]], ko - ko[0],
                           self.values[vo[0]:vo[-1]], vo - vo[0], nk, self.ts)

    def key(self, i: int) -> Optional[bytes]:
        if self.null_keys is not None and self.null_keys[i]:
            return None
        return self.keys[self.key_off[i]:self.key_off[i + 1]].tobytes()

    def value(self, i: int) -> bytes:
        return self.values[self.val_off[i]:self.val_off[i + 1]].tobytes()

    def message(self, i: int) -> Message:
        return Message(self.topic, self.partition, self.base_offset + i, self.key(i), self.value(i))

    def messages(self) -> list:
        """Every record as a ``Message`` (bytes sliced out of the buffers; one C loop when the
        native core is loaded)."""
        ms = int((self.ts + (time.time() - time.perf_counter())) * 1000)
        fast = _native()
        if fast is not None:
            return fast.build_messages(Message, self.topic, self.partition, self.base_offset,
                                       np.ascontiguousarray(self.keys), np.ascontiguousarray(self.key_off),
                                       np.ascontiguousarray(self.values), np.ascontiguousarray(self.val_off),
                                       self.null_keys, ms)
        vb, kb = self.values.tobytes(), self.keys.tobytes()
        vo, ko = self.val_off.tolist(), self.key_off.tolist()
        nk = self.null_keys
        t, p, b = self.topic, self.partition, self.base_offset
        new = tuple.__new__
        return [new(Message, (t, p, b + i, None if (nk is not None and nk[i]) else kb[ko[i]:ko[i + 1]],
                              vb[vo[i]:vo[i + 1]], None, ms)) for i in range(len(vo) - 1)]


class _Partition:
    """Stored record batches plus a tail of single appends (``produce``), sealed into one columnar
    batch when the partition is next read: a per-record produce costs two list appends."""

    def __init__(self, topic: str = "", index: int = 0):
        self.batches: list = []
        self.starts: list = []
        self.size = 0
        self.topic, self.index = topic, index
        self._tk: list = []
        self._tv: list = []
        self._tts = 0.0

    def append_one(self, key: Optional[bytes], value: Optional[bytes]) -> int:
        if not self._tk:
            self._tts = time.perf_counter()
        self._tk.append(key)
        self._tv.append(value)
        self.size += 1
        return self.size - 1

    def _seal(self) -> None:
        if self._tk:
            kb, ko, nk = pack(self._tk)
            vb, vo, _ = pack(self._tv)
            n = len(self._tk)
            self._tk, self._tv = [], []
            rb = RecordBatch(self.topic, self.index, self.size - n, kb, ko, vb, vo, nk, self._tts)
            self.batches.append(rb)
            self.starts.append(self.size - n)

    def append(self, rb: RecordBatch) -> None:
        self._seal()
        rb.base_offset = self.size
        self.batches.append(rb)
        self.starts.append(self.size)
        self.size += rb.n

    def read(self, pos: int, max_n: int) -> Optional[RecordBatch]:
        """Records from offset ``pos`` (at most ``max_n``, never across stored batches)."""
        if pos >= self.size:
            return None
        self._seal()
        i = bisect.bisect_right(self.starts, pos) - 1
        rb = self.batches[i]
        a = pos - rb.base_offset
        return rb.slice(a, min(rb.n, a + max_n)) if (a or max_n < rb.n) else rb

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, off: int) -> Message:
        self._seal()
        rb = self.batches[bisect.bisect_right(self.starts, off) - 1]
        return rb.message(off - rb.base_offset)


class Broker:
    def __init__(self):
        self.lock = threading.RLock()
        self.topics: dict = {}
        self.committed: dict = defaultdict(dict)    # group -> {(topic, part): next offset}
        self._errors: dict = defaultdict(int)
        self.cond = threading.Condition(self.lock)
        self.waiting = 0          # consumers blocked in cond.wait (appends notify only then)

    def create_topic(self, name: str, partitions: int = 3) -> None:
        with self.lock:
            if name not in self.topics:
                self.topics[name] = [_Partition(name, i) for i in range(partitions)]

    def partitions(self, topic: str) -> int:
        with self.lock:
            self.create_topic(topic)
            return len(self.topics[topic])

    @staticmethod
    def _route(key, value, nparts: int) -> int:
        return (zlib.crc32(key) if key else zlib.crc32(value or b"")) % nparts

    def append(self, topic: str, key, value, partition: Optional[int] = None, want_message: bool = True):
        """One record (the per-record ``produce`` path: kept to a few list appends under the lock)."""
        with self.lock:
            parts = self.topics.get(topic)
            if parts is None:
                self.create_topic(topic)
                parts = self.topics[topic]
            if partition is None or partition < 0:
                partition = (crc32(key) if key else crc32(value or b"")) % len(parts)
            off = parts[partition].append_one(key, value)
            if self.waiting:
                self.cond.notify_all()
        return tuple.__new__(Message, (topic, partition, off, key, value, None, int(time.time() * 1000))) \
            if want_message else None

    def append_records(self, topic: str, partition: int, keys, key_off, values, val_off, null_keys=None,
                       copy: bool = True) -> RecordBatch:
        """One columnar batch into one partition (the buffers are copied unless ``copy=False``)."""
        with self.lock:
            self.create_topic(topic)
            parts = self.topics[topic]
            if partition is None or partition < 0:
                partition = 0
            partition %= len(parts)
            cp = (lambda a: np.array(a, copy=True)) if copy else np.asarray
            rb = RecordBatch(topic, partition, 0, cp(keys), cp(key_off), cp(values), cp(val_off),
                             None if null_keys is None else cp(null_keys))
            parts[partition].append(rb)
            self.cond.notify_all()
            return rb

    def append_many(self, topic: str, keys: list, values: list) -> None:
        """Batch append with keyed partitioning (one columnar batch per partition)."""
        with self.lock:
            self.create_topic(topic)
            np_ = len(self.topics[topic])
            by: dict = defaultdict(lambda: ([], []))
            for k, v in zip(keys, values):
                k, v = _b(k), _b(v)
                kk, vv = by[self._route(k, v, np_)]
                kk.append(k)
                vv.append(v)
            for p, (kk, vv) in sorted(by.items()):
                kb, ko, nk = pack(kk)
                vb, vo, _ = pack(vv)
                self.topics[topic][p].append(RecordBatch(topic, p, 0, kb, ko, vb, vo, nk))
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
            for p in self.topics.get(topic, []):
                p._seal()
            return [rb.message(i) for p in self.topics.get(topic, []) for rb in p.batches for i in range(rb.n)]


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

    def _start(self, t: str, p: int) -> int:
        c = self.broker.committed[self.group].get((t, p))
        if c is None:
            c = 0 if self.reset in ("earliest", "smallest", "beginning") else len(self.broker.topics[t][p])
        return c

    def subscribe(self, topics, on_assign=None, on_revoke=None) -> None:
        self.topics = list(topics)
        with self.broker.lock:
            for t in self.topics:
                for p in range(self.broker.partitions(t)):
                    self.positions[(t, p)] = self._start(t, p)

    def assign(self, partitions: list) -> None:
        """Static assignment (one consumer per partition, as the engine's partition readers use)."""
        with self.broker.lock:
            for tp in partitions:
                self.broker.create_topic(tp.topic)
                if tp.topic not in self.topics:
                    self.topics.append(tp.topic)
                self.positions[(tp.topic, tp.partition)] = tp.offset if tp.offset >= 0 else \
                    self._start(tp.topic, tp.partition)

    def assignment(self) -> list:
        return [TopicPartition(t, p) for t, p in self.positions]

    def _error(self) -> Optional[Message]:
        for t in self.topics:
            if self.broker.take_error(t):
                return Message(t, -1, -1, None, None, KafkaError(KafkaError.UNKNOWN, "injected broker error"))
        return None

    def _take(self, max_n: int) -> Optional[RecordBatch]:
        keys = list(self.positions)
        for i in range(len(keys)):
            k = keys[(self._rr + i) % len(keys)]
            t, p = k
            rb = self.broker.topics[t][p].read(self.positions[k], max_n)
            if rb is not None:
                self.positions[k] += rb.n
                self._rr = (self._rr + i + 1) % len(keys)
                if self.auto_commit:
                    self.broker.committed[self.group][k] = self.positions[k]
                return rb
        return None

    def _wait(self, deadline: float) -> bool:
        now = time.time()
        if now >= deadline:
            return False
        with self.broker.cond:
            self.broker.waiting += 1
            try:
                self.broker.cond.wait(timeout=min(0.05, deadline - now))
            finally:
                self.broker.waiting -= 1
        return True

    def poll(self, timeout: float = -1) -> Optional[Message]:
        if self.closed:
            raise RuntimeError("Consumer closed")
        deadline = time.time() + (timeout if timeout and timeout > 0 else 0)
        while True:
            with self.broker.lock:
                err = self._error()
                if err is not None:
                    return err
                rb = self._take(1)
            if rb is not None:
                return rb.message(0)
            if not self._wait(deadline):
                return None

    def consume(self, num_messages: int = 1, timeout: float = -1) -> list:
        out = []
        for item in self.consume_batches(num_messages, timeout):
            if isinstance(item, Message):
                out.append(item)
            else:
                out.extend(item.messages())
        return out

    def consume_batches(self, max_messages: int = 1, timeout: float = -1) -> list:
        """Up to ``max_messages`` records as columnar ``RecordBatch`` views (an error, if any, is
        returned as a ``Message`` with ``error()`` set, last)."""
        if self.closed:
            raise RuntimeError("Consumer closed")
        out, n = [], 0
        deadline = time.time() + (timeout if timeout and timeout > 0 else 0)
        while n < max_messages:
            with self.broker.lock:
                err = self._error()
                if err is not None:
                    out.append(err)
                    break
                rb = self._take(max_messages - n)
            if rb is not None:
                out.append(rb)
                n += rb.n
                continue
            if n or not self._wait(deadline):
                break
        return out

    def commit(self, message: Optional[Message] = None, offsets=None, asynchronous: bool = True):
        if message is not None and not isinstance(message, Message):
            raise TypeError("expected message=Message (confluent_kafka type-checks cimpl.Message)")
        with self.broker.lock:
            if message is not None:
                self.broker.committed[self.group][(message.topic(), message.partition())] = message.offset() + 1
            elif offsets:
                for tp in offsets:
                    if not isinstance(tp, TopicPartition):
                        raise TypeError("offsets must be TopicPartition objects")
                    self.broker.committed[self.group][(tp.topic, tp.partition)] = tp.offset
            else:
                for k, v in self.positions.items():
                    self.broker.committed[self.group][k] = v
        return None

    def committed(self, partitions: list, timeout: float = -1) -> list:
        with self.broker.lock:
            return [TopicPartition(tp.topic, tp.partition,
                                   self.broker.committed[self.group].get((tp.topic, tp.partition), -1001))
                    for tp in partitions]

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
        self.fail_next = 0            # fault injection: fail the next N deliveries
        fast = _native()
        if fast is not None:          # per-record produce in C (falls back to _produce_py itself)
            self.produce = fast.make_fast_produce(self, self.broker, Message)

    def _deliver_later(self, cb, err, what) -> None:
        if cb is not None:
            with self.lock:
                self._pending.append((cb, err, what))

    def _maybe_fail(self):
        with self.lock:
            if self.fail_next > 0:
                self.fail_next -= 1
                return KafkaError(KafkaError.UNKNOWN, "injected delivery failure")
        return None

    def produce(self, topic: str, value=None, key=None, partition: int = -1, on_delivery: Optional[Callable] = None,
                callback: Optional[Callable] = None, **kw) -> None:
        self._produce_py(topic, value, key, partition, on_delivery, callback, **kw)

    def _produce_py(self, topic: str, value=None, key=None, partition: int = -1,
                    on_delivery: Optional[Callable] = None, callback: Optional[Callable] = None, **kw) -> None:
        if topic is None:
            raise TypeError("topic must be a str (KAFKA_OUTPUT_TOPIC unset?)")
        cb = on_delivery or callback
        err = self._maybe_fail() if self.fail_next else None
        if type(key) is not bytes and key is not None:
            key = _b(key)
        if type(value) is not bytes and value is not None:
            value = _b(value)
        m = None if err else self.broker.append(topic, key, value, partition, cb is not None)
        if cb is not None:
            self._pending.append((cb, err, m))     # list.append is atomic under the GIL

    def produce_batch(self, topic: str, keys: list, values: list) -> None:
        """Many messages at once, keyed partitioning, no delivery callbacks."""
        if topic is None:
            raise TypeError("topic must be a str (KAFKA_OUTPUT_TOPIC unset?)")
        self.broker.append_many(topic, keys, values)

    def produce_records(self, topic: str, partition: int, keys, key_off, values, val_off, null_keys=None,
                        on_delivery: Optional[Callable] = None, copy: bool = True) -> None:
        """One columnar batch into one partition; ``on_delivery(err, RecordBatch)`` from poll/flush.
        ``copy=False`` hands the buffers to the broker (the caller must not reuse them)."""
        if topic is None:
            raise TypeError("topic must be a str (KAFKA_OUTPUT_TOPIC unset?)")
        err = self._maybe_fail()
        rb = None if err else self.broker.append_records(topic, partition, keys, key_off, values, val_off, null_keys,
                                                         copy=copy)
        self._deliver_later(on_delivery, err, rb)

    def poll(self, timeout: float = 0) -> int:
        with self.lock:
            pend, self._pending = self._pending, []
        fast = _native() if pend else None
        if fast is not None:
            fast.deliver_reports(pend)          # the same calls, in order, from a C loop
        else:
            for cb, err, what in pend:
                cb(err, what)
        return len(pend)

    def flush(self, timeout: float = -1) -> int:
        self.poll(0)
        return 0

    def __len__(self) -> int:
        return len(self._pending)


class ConfluentConsumer:
    """Only the confluent_kafka.Consumer surface of an in-memory consumer (no columnar
    ``consume_batches``): what the streaming engine sees with a real librdkafka client. Selected
    by ``FDX_KAFKA_COLUMNAR=0`` (stream/kafka.py) and by the loadgen's confluent-API runs."""
    _API = frozenset(("subscribe", "assign", "assignment", "poll", "consume", "commit", "committed", "close",
                      "unsubscribe", "position"))

    def __init__(self, inner: Consumer):
        self._inner = inner

    def __getattr__(self, name):
        if name in ConfluentConsumer._API:
            return getattr(self._inner, name)
        raise AttributeError(name)


class ConfluentProducer:
    """Only the confluent_kafka.Producer surface (per-record ``produce`` with delivery callbacks,
    ``poll``, ``flush``; no columnar ``produce_records``)."""
    _API = frozenset(("produce", "poll", "flush"))

    def __init__(self, inner: Producer):
        self._inner = inner

    def __getattr__(self, name):
        if name in ConfluentProducer._API:
            return getattr(self._inner, name)
        raise AttributeError(name)

    def __len__(self) -> int:
        return len(self._inner)
