"""Streaming classification engine: Kafka -> native JSON extraction -> pinned ring -> GPU -> Kafka.

Replaces the reference's strictly serial Streamlit loop (/root/reference/app_ui.py:168-248: one
message per iteration, two Spark jobs + an LLM call each, ``flush()`` per message, no offset
commit, loop dies on the first broker error) with a batched, pipelined engine:

  consume(batch) -> extract ``value.text`` for the whole batch in C++ straight into a pinned ring
  slot -> GpuScorer (H2D / fused featurize+score / D2H overlapped on 3 HIP streams) -> results
  produced with the original key (``{prediction, confidence, analysis, historical_insight,
  original_text}``, the reference's output schema) -> offsets committed only after the
  producer has delivered the batch (at-least-once; the reference never commits).

Broker errors and undecodable messages are counted and skipped instead of terminating the
loop. LLM explanations: ``explain="none"`` (analysis null), ``"sync"`` (inline, reference
behaviour) or ``"async"`` (classification is produced immediately; the explanation follows as a
second record with the same key and ``"type": "explanation"`` once the LLM answers).
Multiple engines (one per GPU / per partition subset) can share a consumer group.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
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
from .gpu_worker import GpuScorer
from .ring import PinnedRing, Slot

log = get_logger("stream")


@dataclass
class EngineStats:
    messages: int = 0
    batches: int = 0
    produced: int = 0
    broker_errors: int = 0
    bad_messages: int = 0
    committed: int = 0
    batch_latency_ms: list = field(default_factory=list)

    def summary(self) -> dict:
        lat = np.asarray(self.batch_latency_ms or [0.0])
        return {"messages": self.messages, "batches": self.batches, "produced": self.produced,
                "broker_errors": self.broker_errors, "bad_messages": self.bad_messages, "committed": self.committed,
                "p50_batch_ms": float(np.percentile(lat, 50)), "p95_batch_ms": float(np.percentile(lat, 95)),
                "p99_batch_ms": float(np.percentile(lat, 99))}


def extract_texts(values: list, slot: Slot, field_name: str = "text") -> np.ndarray:
    """Native bulk JSON extraction of ``field_name`` into ``slot``; returns per-message status."""
    n = len(values)
    enc = [v if isinstance(v, (bytes, bytearray)) else (v or b"") for v in values]
    lens = np.fromiter((len(v) for v in enc), dtype=np.int64, count=n)
    in_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=in_off[1:])
    buf = np.frombuffer(b"".join(enc), dtype=np.uint8) if n else np.zeros(0, np.uint8)
    status = np.zeros(n, dtype=np.int32)
    cap = slot.data.numel() - PAD
    total = native.lib().extract_json_field(torch.from_numpy(buf.copy() if not buf.flags.writeable else buf),
                                            torch.from_numpy(in_off), field_name, slot.data[:cap],
                                            slot.offsets[: n + 1], torch.from_numpy(status), 0)
    slot.data[total: total + PAD] = 0
    slot.n_docs, slot.n_bytes = n, int(total)
    return status


class StreamingEngine:
    def __init__(self, scorer, postprocess, consumer, producer, output_topic: Optional[str],
                 batch_max: int = 4096, max_latency_ms: float = 5.0, explain: str = "none", agent=None,
                 slots: int = 4, max_bytes: int = 64 << 20, field_name: str = "text", commit: bool = True):
        if explain != "none" and agent is None:
            raise ValueError("explain requires an agent (LLM analyzer)")
        self.scorer, self.postprocess = scorer, postprocess
        self.consumer, self.producer = consumer, producer
        self.topic = output_topic
        self.batch_max = min(batch_max, scorer.max_docs)
        self.max_latency_s = max_latency_ms / 1000.0
        self.explain, self.agent = explain, agent
        self.field = field_name
        self.commit = commit
        self.ring = PinnedRing(slots=max(slots, scorer.depth + 1), max_docs=self.batch_max,
                               max_bytes=min(max_bytes, scorer.max_bytes))
        self.stats = EngineStats()
        self._stop = threading.Event()
        self._pool = cf.ThreadPoolExecutor(max_workers=8) if explain == "async" else None
        self._m_msgs = REGISTRY.counter("stream_messages_total")
        self._m_lat = REGISTRY.histogram("stream_batch_latency_ms")
        self._enc_buf = torch.empty(1 << 22, dtype=torch.uint8)

    @classmethod
    def from_agent(cls, agent, consumer, producer, output_topic, device=None, devices=None, **kw) -> "StreamingEngine":
        """``devices``: several GPUs of this process (round-robin micro-batches, MultiGpuScorer)."""
        from .gpu_worker import make_multi_scorer

        fp = agent.fused
        idf = fp.idf.idf if fp.idf is not None else None
        devs = list(devices) if devices else [device or agent.device]
        scorer = make_multi_scorer(fp.spec(True), idf, fp.model.scorer(), devs,
                                   max_docs=kw.get("batch_max", 4096), max_bytes=kw.get("max_bytes", 64 << 20))
        return cls(scorer, fp.model.postprocess, consumer, producer, output_topic, agent=agent, **kw)

    def stop(self) -> None:
        self._stop.set()

    # ------------------------------------------------------------------ main loop
    def run(self, max_messages: Optional[int] = None, idle_timeout_s: float = 1.0) -> dict:
        idle_since = time.time()
        while not self._stop.is_set():
            if max_messages is not None and self.stats.messages >= max_messages:
                break
            want = self.batch_max if max_messages is None else min(self.batch_max, max_messages - self.stats.messages)
            msgs = self.consumer.consume(num_messages=want, timeout=self.max_latency_s)
            good = []
            for m in msgs:
                if m.error() is not None:
                    self.stats.broker_errors += 1
                    log.warning("kafka error: %s", m.error())
                    continue
                good.append(m)
            if not good:
                if self.scorer.inflight:
                    self._finish_one()
                elif time.time() - idle_since > idle_timeout_s:
                    break
                continue
            idle_since = time.time()
            slot = self.ring.acquire_free(timeout=None)
            t0 = time.perf_counter()
            status = extract_texts([m.value() for m in good], slot, self.field)
            slot.meta = {"msgs": good, "status": status, "t0": t0}
            self.stats.messages += len(good)
            self._m_msgs.inc(len(good))
            if self.scorer.inflight == self.scorer.depth:
                self._finish_one()
            self.scorer.submit(slot)
        while self.scorer.inflight:
            self._finish_one()
        if self._pool:
            self._pool.shutdown(wait=True)
        self.producer.flush()
        return self.stats.summary()

    def _finish_one(self) -> None:
        slot, raw = self.scorer.collect()
        meta = slot.meta
        msgs, status = meta["msgs"], meta["status"]
        _, prob, pred = self.postprocess(torch.from_numpy(raw))
        pred = pred.numpy()
        p1 = prob[:, 1].numpy()
        offs = slot.offsets.numpy()
        data = slot.data.numpy()
        self.stats.bad_messages += int(np.sum(status != 0))
        if self.explain == "sync":
            keys, values = [], []
            for i, m in enumerate(msgs):
                if status[i] != 0:
                    continue
                text = bytes(data[offs[i]:offs[i + 1]]).decode("utf-8", "replace")
                r = self.agent.classify_and_explain(text, prediction={"prediction": float(pred[i]),
                                                                      "confidence": float(p1[i])})
                keys.append(m.key())
                values.append(json.dumps({"prediction": float(pred[i]), "confidence": float(p1[i]),
                                          "analysis": r["analysis"], "historical_insight": r["historical_insight"],
                                          "original_text": text}))
        else:
            keys, values = self._encode_outputs(msgs, status, pred, p1, slot.data, slot.offsets)
        if hasattr(self.producer, "produce_batch"):
            self.producer.produce_batch(self.topic, keys, values)
        else:
            for k, v in zip(keys, values):
                self.producer.produce(self.topic, key=k, value=v)
        if self.explain == "async":
            for i, m in enumerate(msgs):
                if status[i] == 0:
                    text = bytes(data[offs[i]:offs[i + 1]]).decode("utf-8", "replace")
                    self._pool.submit(self._explain_async, m.key(), text, float(pred[i]), float(p1[i]))
        self.producer.poll(0)
        self.producer.flush()
        self.stats.produced += int(np.sum(status == 0))
        if self.commit:
            last = {}
            for m in msgs:
                k = (m.topic(), m.partition())
                last[k] = max(last.get(k, -1), m.offset())
            for (t, p), off in last.items():
                self.consumer.commit(message=_Pos(t, p, off))
                self.stats.committed += 1
        dt = (time.perf_counter() - meta["t0"]) * 1e3
        self.stats.batch_latency_ms.append(dt)
        self._m_lat.observe(dt)
        self.stats.batches += 1
        slot.meta = None
        self.ring.release(slot)

    def _encode_outputs(self, msgs, status, pred, p1, data: torch.Tensor, offsets: torch.Tensor) -> tuple:
        """Output values {prediction, confidence, analysis: null, historical_insight: null,
        original_text} for the whole micro-batch in one native call (json.dumps-identical bytes);
        records whose text is not valid UTF-8 are encoded here with the "replace" decoding."""
        n = len(msgs)
        C = native.lib()
        pred_t = torch.from_numpy(np.ascontiguousarray(pred, dtype=np.float64))
        conf_t = torch.from_numpy(np.ascontiguousarray(p1, dtype=np.float64))
        skip = torch.from_numpy(np.ascontiguousarray(status != 0, dtype=np.int32))
        out_off = torch.empty(n + 1, dtype=torch.int64)
        st = torch.empty(n, dtype=torch.int32)
        need = C.encode_records(pred_t, conf_t, data, offsets, skip, self._enc_buf, out_off, st, 0)
        if need < 0:
            self._enc_buf = torch.empty(int(-need * 1.25) + 4096, dtype=torch.uint8)
            need = C.encode_records(pred_t, conf_t, data, offsets, skip, self._enc_buf, out_off, st, 0)
        buf = self._enc_buf.numpy()
        oo = out_off.numpy()
        st = st.numpy()
        offs = offsets.numpy()
        keys, values = [], []
        for i, m in enumerate(msgs):
            if st[i] == 0:
                values.append(buf[oo[i]:oo[i + 1]].tobytes())
            elif st[i] == 1:
                text = bytes(data.numpy()[offs[i]:offs[i + 1]]).decode("utf-8", "replace")
                values.append(json.dumps({"prediction": float(pred[i]), "confidence": float(p1[i]), "analysis": None,
                                          "historical_insight": None, "original_text": text}))
            else:
                continue
            keys.append(m.key())
        return keys, values

    def _explain_async(self, key, text, pred, conf) -> None:
        try:
            analysis = self.agent.analyzer.analyze_prediction(text, pred, conf)
        except Exception as e:   # the classification was already produced
            analysis = f"explanation failed: {e}"
        self.producer.produce(self.topic, key=key, value=json.dumps({"type": "explanation", "prediction": pred,
                                                                      "confidence": conf, "analysis": analysis}))


class _Pos:
    """Minimal message-like object for ``Consumer.commit(message=...)``."""

    def __init__(self, topic, partition, offset):
        self._t, self._p, self._o = topic, partition, offset

    def topic(self):
        return self._t

    def partition(self):
        return self._p

    def offset(self):
        return self._o
