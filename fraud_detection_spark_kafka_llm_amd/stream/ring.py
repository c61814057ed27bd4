"""Pinned-host micro-batch ring (C-03).

A fixed set of page-locked slots; each slot holds one packed micro-batch (UTF-8 bytes +
int64 offsets + the message keys on the host side). Producers (Kafka consumer threads) fill free
slots; GPU workers take full slots, issue an async H2D copy from them and release them when the
copy's event has completed. Slots are recycled, so steady-state streaming allocates nothing and
every H2D is a DMA from pinned memory (no staging copy by the driver).
"""
from __future__ import annotations

import queue
import threading
from dataclasses import dataclass, field
from typing import Any, Optional, Sequence

import numpy as np
import torch

from ..ops.text import PAD


@dataclass
class Slot:
    index: int
    data: torch.Tensor          # uint8 pinned [max_bytes + PAD]
    offsets: torch.Tensor       # int64 pinned [max_docs + 1]
    n_docs: int = 0
    n_bytes: int = 0
    keys: list = field(default_factory=list)
    meta: Any = None

    def fill(self, texts: Sequence[str], keys: Optional[Sequence] = None) -> int:
        """Pack as many of ``texts`` as fit; returns the number consumed."""
        cap_b = self.data.numel() - PAD
        cap_d = self.offsets.numel() - 1
        buf = self.data.numpy()
        off = self.offsets.numpy()
        off[0] = 0
        pos = 0
        n = 0
        for t in texts:
            if n >= cap_d:
                break
            b = t.encode("utf-8") if isinstance(t, str) else bytes(t)
            if pos + len(b) > cap_b:
                if n == 0:
                    raise ValueError(f"a single message of {len(b)} bytes exceeds the slot capacity {cap_b}")
                break
            buf[pos:pos + len(b)] = np.frombuffer(b, dtype=np.uint8)
            pos += len(b)
            n += 1
            off[n] = pos
        buf[pos:pos + PAD] = 0
        self.n_docs, self.n_bytes = n, pos
        self.keys = list(keys[:n]) if keys is not None else []
        return n

    def fill_packed(self, data: np.ndarray, offsets: np.ndarray) -> None:
        n = len(offsets) - 1
        nb = int(offsets[-1] - offsets[0])
        if n > self.offsets.numel() - 1 or nb > self.data.numel() - PAD:
            raise ValueError("packed batch exceeds slot capacity")
        self.data.numpy()[:nb] = data[int(offsets[0]):int(offsets[-1])]
        self.data.numpy()[nb:nb + PAD] = 0
        self.offsets.numpy()[: n + 1] = offsets - offsets[0]
        self.n_docs, self.n_bytes = n, nb


class PinnedRing:
    def __init__(self, slots: int = 4, max_docs: int = 65536, max_bytes: int = 256 << 20, pin: bool = True):
        pin = pin and torch.cuda.is_available()
        self.slots = []
        for i in range(slots):
            d = torch.zeros(max_bytes + PAD, dtype=torch.uint8)
            o = torch.zeros(max_docs + 1, dtype=torch.int64)
            if pin:
                d, o = d.pin_memory(), o.pin_memory()
            self.slots.append(Slot(i, d, o))
        self._free: "queue.Queue[Slot]" = queue.Queue()
        self._full: "queue.Queue[Slot]" = queue.Queue()
        for s in self.slots:
            self._free.put(s)
        self.closed = threading.Event()

    def acquire_free(self, timeout: Optional[float] = None) -> Optional[Slot]:
        try:
            return self._free.get(timeout=timeout)
        except queue.Empty:
            return None

    def publish(self, slot: Slot) -> None:
        self._full.put(slot)

    def acquire_full(self, timeout: Optional[float] = None) -> Optional[Slot]:
        try:
            return self._full.get(timeout=timeout)
        except queue.Empty:
            return None

    def release(self, slot: Slot) -> None:
        slot.n_docs = slot.n_bytes = 0
        slot.keys = []
        self._free.put(slot)

    def close(self) -> None:
        self.closed.set()
