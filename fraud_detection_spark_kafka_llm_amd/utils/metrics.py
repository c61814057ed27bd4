"""Metrics registry: counters, gauges and latency histograms.

Thread-safe, dependency-free; ``REGISTRY.snapshot()`` returns a dict (p50/p95/p99 for histograms)
and ``to_prometheus()`` renders the Prometheus text exposition format so a serving process can
expose ``/metrics`` (the streaming engine records messages, batch latency, errors).
"""
from __future__ import annotations

import threading
from collections import deque

import numpy as np


class Counter:
    def __init__(self, name: str):
        self.name, self.value, self._lock = name, 0.0, threading.Lock()

    def inc(self, v: float = 1.0) -> None:
        with self._lock:
            self.value += v


class Gauge:
    def __init__(self, name: str):
        self.name, self.value = name, 0.0

    def set(self, v: float) -> None:
        self.value = float(v)


class Histogram:
    BUCKETS = (0.1, 0.25, 0.5, 1, 2.5, 5, 10, 25, 50, 100, 250, 500, 1000, 2500, 5000, float("inf"))

    def __init__(self, name: str, window: int = 10000):
        self.name = name
        self._vals: deque = deque(maxlen=window)
        self.count = 0
        self.sum = 0.0
        self.buckets = [0] * len(self.BUCKETS)
        self._lock = threading.Lock()

    def observe(self, v: float) -> None:
        with self._lock:
            self._vals.append(float(v))
            self.count += 1
            self.sum += float(v)
            for i, b in enumerate(self.BUCKETS):
                if v <= b:
                    self.buckets[i] += 1
                    break

    def quantiles(self) -> dict:
        with self._lock:
            a = np.asarray(self._vals) if self._vals else np.zeros(1)
        return {"p50": float(np.percentile(a, 50)), "p95": float(np.percentile(a, 95)),
                "p99": float(np.percentile(a, 99))}


class Registry:
    def __init__(self):
        self._m: dict = {}
        self._lock = threading.Lock()

    def _get(self, cls, name):
        with self._lock:
            m = self._m.get(name)
            if m is None:
                m = self._m[name] = cls(name)
            return m

    def counter(self, name: str) -> Counter:
        return self._get(Counter, name)

    def gauge(self, name: str) -> Gauge:
        return self._get(Gauge, name)

    def histogram(self, name: str) -> Histogram:
        return self._get(Histogram, name)

    def snapshot(self) -> dict:
        out = {}
        for name, m in list(self._m.items()):
            if isinstance(m, Histogram):
                out[name] = {"count": m.count, "sum": m.sum, **m.quantiles()}
            else:
                out[name] = m.value
        return out

    def to_prometheus(self) -> str:
        lines = []
        for name, m in sorted(self._m.items()):
            n = "fdx_" + name
            if isinstance(m, Counter):
                lines += [f"# TYPE {n} counter", f"{n} {m.value}"]
            elif isinstance(m, Gauge):
                lines += [f"# TYPE {n} gauge", f"{n} {m.value}"]
            else:
                lines.append(f"# TYPE {n} histogram")
                acc = 0
                for b, c in zip(m.BUCKETS, m.buckets):
                    acc += c
                    le = "+Inf" if b == float("inf") else repr(b)
                    lines.append(f'{n}_bucket{{le="{le}"}} {acc}')
                lines += [f"{n}_sum {m.sum}", f"{n}_count {m.count}"]
        return "\n".join(lines) + "\n"


REGISTRY = Registry()
