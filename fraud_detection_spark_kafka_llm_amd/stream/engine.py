"""Streaming classification engine: Kafka -> native JSON extraction -> pinned ring -> GPU -> Kafka.

Replaces the reference's strictly serial Streamlit loop (/root/reference/app_ui.py:168-248: one
message per iteration, two Spark jobs + an LLM call each, ``flush()`` per message, no offset
commit, loop dies on the first broker error) with a batched, pipelined engine:

  * one reader thread per consumer (``get_partition_consumers`` gives one per partition) pulls
    columnar record batches (``Consumer.consume_batches``; confluent consumers are packed into the
    same columnar form) and extracts ``value.text`` in C++ (GIL released) straight into a pinned
    ring slot. Records that do not fit the slot (extraction status 2) are carried over to the
    next slot, never dropped or committed unprocessed.
  * the engine thread submits full slots to the GpuScorer (H2D / fused featurize+score on HIP
    streams), collects finished batches as soon as their event fires, encodes the output records
    in C++ (``{prediction, confidence, analysis, historical_insight, original_text}``, the
    reference's schema, json.dumps-identical bytes) and produces them asynchronously, one columnar
    batch per input partition segment (``Producer.produce_records``; per-record ``produce`` with a
    counting callback on confluent producers). There is no flush per batch.
  * offsets are committed from the producer's delivery callbacks, per partition, only up to the
    end of the contiguous delivered prefix (``commit(offsets=[TopicPartition(t, p, last + 1)])``):
    at-least-once — a failed delivery stops that partition's commits at the failed segment, so a
    restart re-consumes it.

Broker errors and undecodable messages are counted and skipped (undecodable ones are committed:
there is nothing to retry). Per-message latency (broker append -> output delivered) is tracked in
a log-binned histogram (``p50_ms`` / ``p95_ms`` / ``p99_ms``). LLM explanations: ``"none"``
(analysis null), ``"sync"`` (inline, reference behaviour) or ``"async"`` (classification produced
immediately; every ``explain_every``-th message is explained on a bounded thread pool and the
explanation follows as a second record with the same key and ``"type": "explanation"``).
"""
from __future__ import annotations

import concurrent.futures as cf
import functools
import gc
import json
import os
import queue
import sys
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from ..ops import native
from ..ops.text import PAD
from ..utils.logging import get_logger
from ..utils.metrics import REGISTRY
from . import fake_kafka
from .ring import PinnedRing, Slot

log = get_logger("stream")

_LAT_LO, _LAT_BINS_PER_DECADE = 1e-3, 133         # ms; ~1.7 % wide log bins from 1 us to 1000 s
_LAT_EDGES = _LAT_LO * 10.0 ** (np.arange(9 * _LAT_BINS_PER_DECADE + 1) / _LAT_BINS_PER_DECADE)


class LatencyHistogram:
    """Per-message latency in milliseconds, log-binned (percentiles at ~1.7 % resolution)."""

    def __init__(self):
        self.counts = np.zeros(_LAT_EDGES.size + 1, dtype=np.int64)
        self.n = 0
        self.lock = threading.Lock()

    def add(self, ms: np.ndarray) -> None:
        idx = np.log10(np.maximum(ms, _LAT_LO) / _LAT_LO)
        idx *= _LAT_BINS_PER_DECADE
        k = np.minimum(np.ceil(idx).astype(np.int64), self.counts.size - 1)
        c = np.bincount(k, minlength=self.counts.size)
        with self.lock:
            self.counts += c
            self.n += int(ms.size)

    def percentile(self, q: float) -> float:
        with self.lock:
            if self.n == 0:
                return 0.0
            k = int(np.searchsorted(np.cumsum(self.counts), q / 100.0 * self.n))
        lo = _LAT_EDGES[max(k - 1, 0)]
        hi = _LAT_EDGES[min(k, _LAT_EDGES.size - 1)]
        return float(np.sqrt(lo * hi))

    def reset(self) -> None:
        with self.lock:
            self.counts[:] = 0
            self.n = 0


@dataclass
class EngineStats:
    messages: int = 0
    batches: int = 0
    produced: int = 0
    broker_errors: int = 0
    bad_messages: int = 0
    committed: int = 0
    delivery_errors: int = 0
    explanations: int = 0
    explain_dropped: int = 0
    batch_latency_ms: list = field(default_factory=list)
    latency: LatencyHistogram = field(default_factory=LatencyHistogram)

    def summary(self) -> dict:
        lat = np.asarray(self.batch_latency_ms[-100000:] or [0.0])
        return {"messages": self.messages, "batches": self.batches, "produced": self.produced,
                "broker_errors": self.broker_errors, "bad_messages": self.bad_messages, "committed": self.committed,
                "delivery_errors": self.delivery_errors, "explanations": self.explanations,
                "explain_dropped": self.explain_dropped,
                "p50_ms": self.latency.percentile(50), "p95_ms": self.latency.percentile(95),
                "p99_ms": self.latency.percentile(99),
                "p50_batch_ms": float(np.percentile(lat, 50)), "p95_batch_ms": float(np.percentile(lat, 95)),
                "p99_batch_ms": float(np.percentile(lat, 99))}


# ---------------------------------------------------------------------------------------------- input
class _Piece:
    """Records of one partition waiting to be placed into a slot: a columnar batch, optional
    per-record offsets (None = consecutive from ``rb.base_offset``) and append time(s)."""
    __slots__ = ("rb", "offs", "ts")

    def __init__(self, rb, offs=None, ts=None):
        self.rb, self.offs = rb, offs
        self.ts = rb.ts if ts is None else ts

    def split(self, j: int) -> tuple:
        a = _Piece(self.rb.slice(0, j), None if self.offs is None else self.offs[:j],
                   self.ts if np.isscalar(self.ts) else self.ts[:j])
        b = _Piece(self.rb.slice(j, self.rb.n), None if self.offs is None else self.offs[j:],
                   self.ts if np.isscalar(self.ts) else self.ts[j:])
        return a, b

    def last_offset(self) -> int:
        return int(self.offs[-1]) if self.offs is not None else self.rb.base_offset + self.rb.n - 1


@dataclass
class _Segment:
    """Consecutive slot records [a, b) of one input partition."""
    topic: str
    partition: int
    a: int
    b: int
    hi: int                    # last input offset
    keys: np.ndarray
    key_off: np.ndarray
    null_keys: Optional[np.ndarray]
    ts: np.ndarray             # append time per record (perf_counter seconds)
    reader: int
    n_out: int = 0

    def key(self, i: int) -> Optional[bytes]:
        if self.null_keys is not None and self.null_keys[i]:
            return None
        return self.keys[self.key_off[i]:self.key_off[i + 1]].tobytes()


@dataclass
class _Batch:
    segments: list
    status: np.ndarray         # 0 ok, 1 bad JSON / no text field / oversize
    t_ready: float


def _concat_keys(pieces: list) -> tuple:
    if len(pieces) == 1:
        rb = pieces[0].rb
        return rb.keys, rb.key_off, rb.null_keys
    keys = np.concatenate([p.rb.keys for p in pieces])
    lens = np.concatenate([np.diff(p.rb.key_off) for p in pieces])
    off = np.zeros(lens.size + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    nulls = None
    if any(p.rb.null_keys is not None for p in pieces):
        nulls = np.concatenate([p.rb.null_keys if p.rb.null_keys is not None else np.zeros(p.rb.n, bool)
                                for p in pieces])
    return keys, off, nulls


def _subset(buf: np.ndarray, off: np.ndarray, keep: np.ndarray) -> tuple:
    """Columnar byte array restricted to the records where ``keep``."""
    lens = np.diff(off)
    sel = np.repeat(keep, lens)
    new = np.zeros(int(keep.sum()) + 1, dtype=np.int64)
    np.cumsum(lens[keep], out=new[1:])
    return buf[off[0]:off[-1]][sel], new


class _RefBatch(fake_kafka.RecordBatch):
    """A RecordBatch whose values are a list of the consumed messages' own bytes objects
    (``val_off`` still counts their bytes): the text field is extracted from them in place."""
    __slots__ = ()

    def slice(self, a: int, b: int) -> "_RefBatch":
        ko, vo = self.key_off[a:b + 1], self.val_off[a:b + 1]
        nk = self.null_keys[a:b] if self.null_keys is not None else None
        return _RefBatch(self.topic, self.partition, self.base_offset + a, self.keys[ko[0]:ko[-1]], ko - ko[0],
                         self.values[a:b], vo - vo[0], nk, self.ts)

    def value(self, i: int) -> bytes:
        v = self.values[i]
        return b"" if v is None else v


def _to_pieces(msgs: list) -> tuple:
    """confluent Messages -> (per-partition columnar pieces in consume order, [(index, error)]).
    One native pass over the list (csrc/bindings_kafka.cpp pack_messages): the per-message method
    calls (error, topic, partition, key, value, offset, timestamp) run from C, not bytecode; the
    values are not copied (by_ref: _RefBatch), the text is extracted from them in place."""
    part_of, parts, kb, ko, nk, vb, vo, offs, ts_ms, errors = native.lib().pack_messages(msgs, None, True)
    now = time.perf_counter()
    ts = np.where(ts_ms > 0, ts_ms / 1000.0 - (time.time() - now), now)
    out = []
    for pi, (t, p) in enumerate(parts):
        if len(parts) == 1:
            sel = None
            kk, kof, vv, vof, nn, oo, tt = kb, ko, vb, vo, nk, offs, ts
        else:                                   # several partitions in one consume: split
            sel = np.flatnonzero(part_of == pi)
            kk, kof = _subset(kb, ko, part_of == pi)
            vv = [vb[i] for i in sel.tolist()]
            vof = np.zeros(sel.size + 1, dtype=np.int64)
            np.cumsum(np.diff(vo)[sel], out=vof[1:])
            nn, oo, tt = nk[sel], offs[sel], ts[sel]
        nulls = nn.astype(bool) if nn.any() else None
        rb = _RefBatch(t, p, int(oo[0]), kk, kof, vv, vof, nulls, float(tt.min()))
        out.append(_Piece(rb, oo, tt))
    return out, errors


def extract_into(slot: Slot, pos: int, n: int, rb, field_name: str, status: np.ndarray) -> int:
    """Native extraction of ``field_name`` for the records of ``rb`` into ``slot`` at byte ``pos``
    / document ``n``; returns the byte count written (``status`` 2 = did not fit)."""
    k = status.size
    cap = slot.data.numel() - PAD
    if isinstance(rb.values, list):         # _RefBatch: the messages' own value buffers
        total = native.lib().extract_json_field_refs(rb.values, k, field_name, slot.data[pos:cap],
                                                     slot.offsets[n: n + k + 1], torch.from_numpy(status), 0)
    else:
        vo = rb.val_off[: k + 1]
        total = native.lib().extract_json_field(torch.from_numpy(rb.values), torch.from_numpy(np.ascontiguousarray(vo)),
                                                field_name, slot.data[pos:cap], slot.offsets[n: n + k + 1],
                                                torch.from_numpy(status), 0)
    if pos:
        slot.offsets[n: n + k + 1] += pos
    return int(total)


def extract_texts(values: list, slot: Slot, field_name: str = "text") -> np.ndarray:
    """Bulk JSON extraction of ``field_name`` for a list of message values into an empty slot;
    returns the per-message status (0 ok, 1 missing / not a string / bad JSON, 2 did not fit)."""
    vb, vo, _ = fake_kafka.pack([v if v is not None else b"" for v in values])
    kb, ko, _ = fake_kafka.pack([b""] * len(values))
    rb = fake_kafka.RecordBatch("", 0, 0, kb, ko, vb, vo)
    status = np.zeros(len(values), dtype=np.int32)
    total = extract_into(slot, 0, 0, rb, field_name, status)
    slot.data[total: total + PAD] = 0
    slot.n_docs, slot.n_bytes = len(values), total
    return status


SWITCH_INTERVAL_S = float(os.environ.get("FDX_SWITCH_INTERVAL_MS", 0.5)) / 1e3


class _Reader(threading.Thread):
    """One consumer -> pinned slots. Holds at most one slot at a time."""

    def __init__(self, eng: "StreamingEngine", idx: int, consumer):
        super().__init__(name=f"fdx-reader-{idx}", daemon=True)
        self.eng, self.idx, self.consumer = eng, idx, consumer
        self.columnar = hasattr(consumer, "consume_batches")
        self.carry: deque = deque()

    def run(self) -> None:
        try:
            while True:
                if self.eng._readers_stop.is_set() and not self.carry:
                    return
                slot = self.eng.ring.acquire_free(timeout=0.05)
                if slot is None:
                    continue
                if self._fill(slot):
                    self.eng.ring.publish(slot)
                else:
                    self.eng.ring.release(slot)
                    if self.eng._quota_done():
                        return
        except BaseException as e:  # surfaced by the engine thread
            self.eng._reader_error = e

    def _poll(self, want: int, timeout: float) -> None:
        eng = self.eng
        want = eng._claim(want)
        if want == 0:
            if not eng._inline_on:
                time.sleep(0.0005)    # another reader holds the remaining quota
            return
        if eng._quota is not None:    # never hold a reservation across a blocking wait
            timeout = 0
        got = 0
        try:
            if self.columnar:
                items = self.consumer.consume_batches(want, timeout)
            else:
                items = self.consumer.consume(num_messages=want, timeout=timeout)
            if self.columnar:
                for it in items:
                    if isinstance(it, fake_kafka.RecordBatch):
                        self.carry.append(_Piece(it))
                        got += it.n
                    elif it.error() is not None:
                        eng._count("broker_errors", 1)
                        log.warning("kafka error: %s", it.error())
            elif items:
                pieces, errors = _to_pieces(items if isinstance(items, list) else list(items))
                for _, err in errors:
                    eng._count("broker_errors", 1)
                    log.warning("kafka error: %s", err)
                self.carry.extend(pieces)
                got += sum(pc.rb.n for pc in pieces)
        finally:
            eng._settle(want, got)
        if not got and timeout == 0 and not eng._inline_on:
            time.sleep(0.001)
        if got:
            eng._last_read = time.time()

    def _fill(self, slot: Slot) -> bool:
        eng = self.eng
        cap_b = slot.data.numel() - PAD
        cap_d = min(slot.offsets.numel() - 1, eng.batch_max)
        n = pos = 0
        placed: list = []
        deadline = None
        slot.offsets[0] = 0
        polled = False
        while n < cap_d:
            if not self.carry:
                now = time.time()
                if (deadline is not None and now >= deadline) or eng._readers_stop.is_set() or eng._quota_done():
                    break
                if polled and deadline is None and eng._inline_on:
                    break                 # inline: nothing arrived, back to the engine loop
                polled = True
                first = eng.poll_s if not eng._inline_busy() else 0.0005
                self._poll(cap_d - n, first if deadline is None else deadline - now)
                continue
            pc = self.carry.popleft()
            k = min(pc.rb.n, cap_d - n)
            if k < pc.rb.n:
                pc, rest = pc.split(k)
                self.carry.appendleft(rest)
            status = np.zeros(k, dtype=np.int32)
            extract_into(slot, pos, n, pc.rb, eng.field, status)
            over = np.flatnonzero(status == 2)
            if over.size:
                j = int(over[0])
                if j == 0 and n == 0:        # one record larger than a whole slot: reject it
                    status[0] = 1
                    slot.offsets[1] = 0
                    j = 1
                if j < k:
                    pc, rest = pc.split(j)
                    self.carry.appendleft(rest)
                    status = status[:j]
                    k = j
                if k == 0:
                    break
            placed.append((pc, status))
            n += k
            pos = int(slot.offsets[n])
            if deadline is None:
                deadline = time.time() + eng.max_latency_s
            if over.size:
                break                     # slot full by bytes
        if n == 0:
            return False
        slot.data[pos: pos + PAD] = 0
        slot.n_docs, slot.n_bytes = n, pos
        slot.meta = self._meta(placed)
        return True

    def _meta(self, placed: list) -> _Batch:
        segs, status = [], []
        a = 0
        i = 0
        while i < len(placed):
            j = i
            t, p = placed[i][0].rb.topic, placed[i][0].rb.partition
            while j + 1 < len(placed) and placed[j + 1][0].rb.topic == t and placed[j + 1][0].rb.partition == p:
                j += 1
            group = [placed[x][0] for x in range(i, j + 1)]
            cnt = sum(g.rb.n for g in group)
            keys, koff, nulls = _concat_keys(group)
            ts = np.concatenate([np.full(g.rb.n, g.ts) if np.isscalar(g.ts) else g.ts for g in group])
            segs.append(_Segment(t, p, a, a + cnt, group[-1].last_offset(), keys, koff, nulls, ts, self.idx))
            status.extend(placed[x][1] for x in range(i, j + 1))
            a += cnt
            i = j + 1
        return _Batch(segs, np.concatenate(status), time.perf_counter())


# ---------------------------------------------------------------------------------------------- commits
class _CommitTracker:
    """Per partition, segments in consume order; the commit point is the end of the delivered
    prefix (a failed segment blocks it: at-least-once)."""

    def __init__(self):
        self.q: dict = {}
        self.lock = threading.Lock()

    def add(self, seg: _Segment) -> list:
        e = [seg.hi, 0]
        with self.lock:
            self.q.setdefault((seg.topic, seg.partition), deque()).append(e)
        return e

    def resolve(self, key: tuple, entry: list, ok: bool) -> Optional[int]:
        with self.lock:
            entry[1] = 1 if ok else -1
            dq = self.q[key]
            hi = None
            while dq and dq[0][1] == 1:
                hi = dq.popleft()[0]
            return hi


# ---------------------------------------------------------------------------------------------- engine
class StreamingEngine:
    def __init__(self, scorer, postprocess, consumer, producer, output_topic: Optional[str],
                 batch_max: int = 4096, max_latency_ms: float = 5.0, explain: str = "none", agent=None,
                 slots: int = 0, max_bytes: int = 64 << 20, field_name: str = "text", commit: bool = True,
                 explain_every: int = 1, explain_max_pending: int = 1024, poll_ms: float = 20.0,
                 ring: Optional[PinnedRing] = None):
        if explain != "none" and agent is None:
            raise ValueError("explain requires an agent (LLM analyzer)")
        if output_topic is None:
            raise TypeError("output_topic must be a str (KAFKA_OUTPUT_TOPIC unset?)")
        self.scorer, self.postprocess = scorer, postprocess
        self.consumers = list(consumer) if isinstance(consumer, (list, tuple)) else [consumer]
        self.consumer = self.consumers[0]
        self.producer = producer
        self.topic = output_topic
        self.batch_max = min(batch_max, scorer.max_docs)
        self.max_latency_s = max_latency_ms / 1000.0
        self.poll_s = poll_ms / 1000.0
        self.explain, self.agent = explain, agent
        self.explain_every, self.explain_max_pending = max(1, explain_every), explain_max_pending
        self.field = field_name
        self.commit = commit
        nslots = max(slots, scorer.depth + len(self.consumers) + 2)
        if ring is not None:     # e.g. a consumer-group client's shared-memory slots (stream/group.py)
            if len(ring.slots) < scorer.depth + 1 or ring.slots[0].offsets.numel() - 1 < self.batch_max:
                raise ValueError("ring too small for the scorer depth / batch_max")
            self.ring = ring
        else:
            self.ring = PinnedRing(slots=nslots, max_docs=self.batch_max, max_bytes=min(max_bytes, scorer.max_bytes))
        self.stats = EngineStats()
        self.tracker = _CommitTracker()
        self._stop = threading.Event()
        self._readers_stop = threading.Event()
        self._reader_error: Optional[BaseException] = None
        self._lock = threading.Lock()
        self._quota: Optional[int] = None
        self._claimed = 0
        self._last_read = time.time()
        # partition readers run on the engine thread itself (no reader threads) for per-record
        # (confluent-surface) consumers: their work holds the GIL, so threads only convoy on it.
        # None: inline exactly when no consumer has the columnar consume_batches.
        env = os.environ.get("FDX_STREAM_INLINE", "")
        self.inline = None if env == "" else env == "1"
        self._inline_on = False
        self._pool = cf.ThreadPoolExecutor(max_workers=8) if explain == "async" else None
        self._explain_pending = 0
        self._seen = 0
        self._m_msgs = REGISTRY.counter("stream_messages_total")
        self._m_lat = REGISTRY.histogram("stream_batch_latency_ms")
        self._enc_meta = (torch.empty(self.batch_max + 1, dtype=torch.int64),
                          torch.empty(self.batch_max, dtype=torch.int32))
        self._columnar_out = hasattr(producer, "produce_records")
        self._out_parts = producer.broker.partitions(output_topic) if isinstance(producer, fake_kafka.Producer) else 1
        self._tp_cls = [fake_kafka.TopicPartition if isinstance(c, fake_kafka.Consumer) else _confluent_tp()
                        for c in self.consumers]

    @classmethod
    def from_agent(cls, agent, consumer, producer, output_topic, device=None, devices=None, **kw) -> "StreamingEngine":
        """``devices``: several GPUs of this process (round-robin micro-batches, MultiGpuScorer)."""
        from .gpu_worker import make_multi_scorer

        fp = agent.fused
        idf = fp.idf.idf if fp.idf is not None else None
        devs = list(devices) if devices else [device or agent.device]
        scorer = make_multi_scorer(fp.spec(True), idf, fp.model.scorer(), devs,
                                   max_docs=kw.get("batch_max", 4096), max_bytes=kw.get("max_bytes", 64 << 20))
        return cls(scorer, fp.model.postprocess_numpy, consumer, producer, output_topic, agent=agent, **kw)

    def stop(self) -> None:
        self._stop.set()

    # ------------------------------------------------------------------ reader coordination
    def _claim(self, want: int) -> int:
        """Reserve up to ``want`` of the remaining ``max_messages`` before a consume call."""
        with self._lock:
            if self._quota is None:
                return want
            g = min(want, self._quota)
            self._quota -= g
            self._claimed += g
            return g

    def _settle(self, claimed: int, got: int) -> None:
        """Return the unused part of a reservation once its consume call is done."""
        with self._lock:
            if self._quota is not None:
                self._quota += claimed - got
                self._claimed -= claimed

    def _quota_done(self) -> bool:
        """All of ``max_messages`` consumed (reservations in flight may still be returned)."""
        with self._lock:
            return self._quota is not None and self._quota <= 0 and self._claimed == 0

    def _inline_busy(self) -> bool:
        """Inline readers with micro-batches in flight: poll briefly, results are waiting."""
        return self._inline_on and self.scorer.inflight > 0

    def _count(self, name: str, k: int) -> None:
        with self._lock:
            setattr(self.stats, name, getattr(self.stats, name) + k)

    # ------------------------------------------------------------------ main loop
    def run(self, max_messages: Optional[int] = None, idle_timeout_s: float = 1.0) -> dict:
        # long-lived objects (model, tables, torch/numpy internals) leave the collector's young
        # generations: full collections would otherwise stall the readers for 50-100 ms
        gc.freeze()
        # the readers, the engine thread and a client's own threads share the GIL: a 5 ms default
        # switch interval shows up directly in per-message latency (p50 ~2 ms at 300K msgs/s)
        if sys.getswitchinterval() > SWITCH_INTERVAL_S:
            sys.setswitchinterval(SWITCH_INTERVAL_S)
        self._quota = max_messages
        self._readers_stop.clear()
        self._last_read = time.time()
        readers = [_Reader(self, i, c) for i, c in enumerate(self.consumers)]
        inline = self.inline if self.inline is not None else not any(r.columnar for r in readers)
        self._inline_on = inline
        if not inline:
            for r in readers:
                r.start()
        rr = 0
        try:
            while True:
                if self._reader_error is not None:
                    raise self._reader_error
                if inline and self.scorer.inflight < self.scorer.depth:
                    # one slot from the next partition reader, on this thread
                    free = self.ring.acquire_free(timeout=0)
                    if free is not None:
                        r = readers[rr]
                        rr = (rr + 1) % len(readers)
                        if r._fill(free):
                            self.ring.publish(free)
                        else:
                            self.ring.release(free)
                slot = self.ring.acquire_full(timeout=0 if inline else (0.0005 if self.scorer.inflight else 0.005))
                if slot is not None:
                    while self.scorer.inflight >= self.scorer.depth:
                        self._finish_one()
                    self._submit(slot)
                while self.scorer.inflight and self.scorer.ready():
                    self._finish_one()
                self.producer.poll(0)
                if slot is None and not self.scorer.inflight:
                    if self._stop.is_set():
                        break
                    alive = (not self._quota_done() or any(r.carry for r in readers)) if inline else \
                        any(r.is_alive() for r in readers)
                    if not alive or time.time() - self._last_read > max(idle_timeout_s, 2 * self.max_latency_s):
                        if self.ring._full.empty():
                            break
        finally:
            self._readers_stop.set()
            for r in readers:
                if r.is_alive():
                    r.join(timeout=10.0)
            while True:                                  # slots the readers published while stopping
                slot = self.ring.acquire_full(timeout=0)
                if slot is None:
                    break
                while self.scorer.inflight >= self.scorer.depth:
                    self._finish_one()
                self._submit(slot)
            while self.scorer.inflight:
                self._finish_one()
            if self._pool:
                self._pool.shutdown(wait=True)
                self._pool = cf.ThreadPoolExecutor(max_workers=8)
            self.producer.flush()
            self.producer.poll(0)
        if self._reader_error is not None:
            raise self._reader_error
        return self.stats.summary()

    def _submit(self, slot: Slot) -> None:
        b: _Batch = slot.meta
        b.entries = [self.tracker.add(s) for s in b.segments]
        self.stats.messages += slot.n_docs
        self._m_msgs.inc(slot.n_docs)
        self.scorer.submit(slot)

    def _finish_one(self) -> None:
        slot, raw = self.scorer.collect(copy=False)
        b: _Batch = slot.meta
        n = slot.n_docs
        pred, p1 = self.postprocess(raw)
        status = b.status
        bad = status != 0
        self.stats.bad_messages += int(bad.sum())
        data = slot.data.numpy()
        offs = slot.offsets.numpy()
        if self.explain == "sync":
            enc = None
        else:
            enc = self._encode(status, pred, p1, slot)
        for seg, entry in zip(b.segments, b.entries):
            self._produce_segment(seg, entry, status, pred, p1, data, offs, enc)
        if self.explain == "async":
            self._submit_explanations(b, status, pred, p1, data, offs)
        self._seen += n
        dt = (time.perf_counter() - b.t_ready) * 1e3
        self.stats.batch_latency_ms.append(dt)
        self._m_lat.observe(dt)
        self.stats.batches += 1
        slot.meta = None
        self.ring.release(slot)

    def _encode(self, status, pred, p1, slot: Slot) -> tuple:
        """Native json.dumps-identical output records for the whole micro-batch."""
        n = slot.n_docs
        C = native.lib()
        pred_t = torch.from_numpy(np.ascontiguousarray(pred, dtype=np.float64))
        conf_t = torch.from_numpy(np.ascontiguousarray(p1, dtype=np.float64))
        skip = torch.from_numpy(np.ascontiguousarray(status != 0, dtype=np.int32))
        out_off, st = self._enc_meta
        if out_off.numel() < n + 1:
            out_off, st = torch.empty(n + 1, dtype=torch.int64), torch.empty(n, dtype=torch.int32)
            self._enc_meta = (out_off, st)
        out_off, st = out_off[: n + 1], st[:n]
        # a fresh buffer per batch, handed to the producer without a copy (the in-memory broker
        # keeps it as the log segment; librdkafka copies on produce)
        buf = torch.empty(slot.n_bytes + 160 * n + 4096, dtype=torch.uint8)
        need = C.encode_records(pred_t, conf_t, slot.data, slot.offsets, skip, buf, out_off, st, 0)
        if need < 0:
            buf = torch.empty(-need, dtype=torch.uint8)
            need = C.encode_records(pred_t, conf_t, slot.data, slot.offsets, skip, buf, out_off, st, 0)
        return buf.numpy(), out_off.numpy(), st.numpy()

    @staticmethod
    def _record_py(pred, conf, text: str, analysis=None, insight=None) -> bytes:
        return json.dumps({"prediction": float(pred), "confidence": float(conf), "analysis": analysis,
                           "historical_insight": insight, "original_text": text}).encode()

    def _produce_segment(self, seg: _Segment, entry, status, pred, p1, data, offs, enc) -> None:
        a, b = seg.a, seg.b
        if enc is not None and not np.any(enc[2][a:b] == 1):
            buf, oo, st = enc
            keep = st[a:b] == 0
            vals = buf[oo[a]:oo[b]]
            if keep.all():
                voff = oo[a:b + 1] - oo[a]
                keys, koff, nulls = seg.keys, seg.key_off, seg.null_keys
                if koff[0] != 0:
                    keys, koff = keys[koff[0]:koff[-1]], koff - koff[0]
            else:                           # skipped records encode to zero bytes
                voff = np.append(oo[a:b][keep], oo[b]) - oo[a]
                keys, koff = _subset(seg.keys, seg.key_off, keep)
                nulls = seg.null_keys[keep] if seg.null_keys is not None else None
            seg.n_out = int(keep.sum())
        else:                               # sync explanations or invalid UTF-8 text: Python path
            kl, vl = [], []
            for i in range(a, b):
                if status[i] != 0:
                    continue
                text = bytes(data[offs[i]:offs[i + 1]]).decode("utf-8", "replace")
                if enc is None:
                    r = self.agent.classify_and_explain(text, prediction={"prediction": float(pred[i]),
                                                                          "confidence": float(p1[i])})
                    vl.append(self._record_py(pred[i], p1[i], text, r["analysis"], r["historical_insight"]))
                elif enc[2][i] == 0:
                    vl.append(bytes(enc[0][enc[1][i]:enc[1][i + 1]]))
                else:
                    vl.append(self._record_py(pred[i], p1[i], text))
                kl.append(seg.key(i - a))
            keys, koff, nulls = fake_kafka.pack(kl)
            vals, voff, _ = fake_kafka.pack(vl)
            seg.n_out = len(vl)
        if seg.n_out == 0:
            self._on_delivery(seg, entry, None)
            return
        if self._columnar_out:
            try:
                self.producer.produce_records(self.topic, seg.partition % self._out_parts, keys, koff, vals, voff,
                                              nulls, on_delivery=functools.partial(self._on_delivery_cb, seg, entry),
                                              copy=False)
            except Exception as e:
                log.error("produce failed: %s", e)
                self._on_delivery(seg, entry, e)
            return
        self._produce_each(seg, entry, keys, koff, nulls, vals, voff)

    def _produce_each(self, seg, entry, keys, koff, nulls, vals, voff) -> None:
        """Per-record produce (confluent producers): the segment resolves when every record's
        delivery report has arrived; any error fails it."""
        # one C callable counts the segment's reports (first error kept) and resolves it at the last
        cb = native.lib().DeliveryCounter(seg.n_out, functools.partial(self._on_delivery, seg, entry))

        # one C loop of produce() calls (BufferError: poll(0.05) and retry; other errors: cb(err))
        native.lib().produce_each(self.producer, self.topic, np.ascontiguousarray(keys, dtype=np.uint8),
                                  np.ascontiguousarray(koff, dtype=np.int64),
                                  None if nulls is None else np.ascontiguousarray(nulls, dtype=np.uint8),
                                  np.ascontiguousarray(vals, dtype=np.uint8), np.ascontiguousarray(voff, dtype=np.int64),
                                  cb)

    def _on_delivery_cb(self, seg, entry, err, _msg) -> None:
        self._on_delivery(seg, entry, err)

    def _on_delivery(self, seg: _Segment, entry, err) -> None:
        key = (seg.topic, seg.partition)
        if err is not None:
            self.stats.delivery_errors += 1
            log.error("delivery failed for %s[%d] up to offset %d: %s", seg.topic, seg.partition, seg.hi, err)
            self.tracker.resolve(key, entry, False)
            return
        self.stats.produced += seg.n_out
        self.stats.latency.add((time.perf_counter() - seg.ts) * 1e3)
        hi = self.tracker.resolve(key, entry, True)
        if hi is not None and self.commit:
            tp = self._tp_cls[seg.reader](seg.topic, seg.partition, hi + 1)
            try:
                self.consumers[seg.reader].commit(offsets=[tp], asynchronous=True)
                self.stats.committed += 1
            except Exception as e:       # the next delivered segment commits past this point
                log.warning("commit failed: %s", e)

    # ------------------------------------------------------------------ explanations
    def _submit_explanations(self, b: _Batch, status, pred, p1, data, offs) -> None:
        every = self.explain_every
        for seg in b.segments:
            first = (-(self._seen + seg.a)) % every
            for i in range(seg.a + first, seg.b, every):
                if status[i] != 0:
                    continue
                with self._lock:
                    if self._explain_pending >= self.explain_max_pending:
                        self.stats.explain_dropped += 1
                        continue
                    self._explain_pending += 1
                text = bytes(data[offs[i]:offs[i + 1]]).decode("utf-8", "replace")
                self._pool.submit(self._explain_async, seg.key(i - seg.a), text, float(pred[i]), float(p1[i]))

    def _explain_async(self, key, text, pred, conf) -> None:
        try:
            analysis = self.agent.analyzer.analyze_prediction(text, pred, conf)
        except Exception as e:   # the classification was already produced
            analysis = f"explanation failed: {e}"
        try:
            self.producer.produce(self.topic, key=key, value=json.dumps({"type": "explanation", "prediction": pred,
                                                                          "confidence": conf, "analysis": analysis}))
        finally:
            with self._lock:
                self._explain_pending -= 1
                self.stats.explanations += 1


def _confluent_tp():
    try:
        from confluent_kafka import TopicPartition
        return TopicPartition
    except ImportError:
        return fake_kafka.TopicPartition
