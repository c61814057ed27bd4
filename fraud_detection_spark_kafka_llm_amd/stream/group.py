"""Consumer-group streaming: P client processes (one per partition) around ONE GPU scoring process.

A librdkafka-shaped client costs ~1-2 us of interpreter work per record on each side (a Message
object per consumed record, one ``produce`` call + delivery report per output record), all of it
under one GIL: a single-process engine tops out near 0.6 M dialogues/s however fast the GPU is
(profiles/r3s3/NOTES.md). Kafka's own answer is the consumer group, and that is the layout here —
the reference's topics have 3 partitions (/root/reference/README.md:110-121), its loop consumes
them one message at a time in one process (/root/reference/app_ui.py:196-226):

  * each **client process** (``python -m ...stream.group``, started as a child that never touches
    the GPU) runs an ordinary :class:`~.engine.StreamingEngine` over its partition(s): poll ->
    native JSON extraction -> produce + delivery-gated commits, its own latency histogram. Its
    ring slots live in a shared-memory segment, and its scorer is a :class:`RemoteScorer` that
    only passes slot indices over a socket;
  * the **GPU process** (:class:`ConsumerGroup`) maps every client's segment, page-locks it
    (``hipHostRegister``: the H2D DMA reads the client's slot directly, no staging copy), feeds
    the slots of all clients through one :class:`~.gpu_worker.GpuScorer` copy/compute pipeline
    and writes (prediction, P(scam)) back into the slot's result rows.

Per micro-batch the IPC is two 16-byte socket messages; the text bytes are written once (by the
client's extraction) and read once (by the DMA engine).

**Several scoring processes, one per GPU** (BASELINE config 5: "3-partition topic -> 8-GPU batched
inference"). Under torchrun every rank is one process on its own GPU; no process opens another
rank's device. Rank 0 runs the :class:`ConsumerGroup` (it creates the segments and starts the
clients); every other rank runs a :class:`ScorerPeer`, which maps the same segments, page-locks
them for ITS device and serves micro-batches over a Unix socket per client. The rendezvous
(segment names, the peers' socket names) goes through the process group's key-value store
(:class:`GroupRendezvous`), never through a device collective. Each client's
:class:`RemoteScorer` sends every micro-batch to the scoring process with the fewest of its
batches outstanding (ties rotate), and hands results back to its engine in submission order.
The peers stop when every client has closed its connection (the group's close).
"""
from __future__ import annotations

import json
import os
import pickle
import socket
import struct
import subprocess
import sys
import time
from collections import deque
from multiprocessing.connection import Connection, wait as mp_wait
from multiprocessing import shared_memory
from typing import Optional

import numpy as np
import torch

from ..ops.text import PAD
from .ring import PinnedRing, Slot

_SUB, _DONE, _CTL = b"S", b"D", b"C"
_HDR = struct.Struct("<iiq")            # slot index, documents, bytes
_HELLO = struct.Struct("<i")            # client index on a peer connection (-1: abort)
_ALIGN = 4096


def _round(x: int) -> int:
    return (x + _ALIGN - 1) // _ALIGN * _ALIGN


def slot_layout(slots: int, max_docs: int, max_bytes: int) -> dict:
    """Byte layout of one client's segment: per slot the text bytes, the int64 offsets and the
    [max_docs, 2] float64 result rows, each page aligned."""
    d, o, r = _round(max_bytes + PAD), _round((max_docs + 1) * 8), _round(max_docs * 16)
    return {"slots": slots, "max_docs": max_docs, "max_bytes": max_bytes, "data": d, "offs": o, "res": r,
            "stride": d + o + r, "size": slots * (d + o + r)}


def _views(buf, lay: dict) -> list:
    """(data uint8, offsets int64, result float64 [max_docs, 2]) tensors per slot over ``buf``."""
    whole = torch.frombuffer(buf, dtype=torch.uint8, count=lay["size"])
    out = []
    for i in range(lay["slots"]):
        b = i * lay["stride"]
        data = whole[b: b + lay["max_bytes"] + PAD]
        offs = whole[b + lay["data"]: b + lay["data"] + (lay["max_docs"] + 1) * 8].view(torch.int64)
        res = whole[b + lay["data"] + lay["offs"]: b + lay["data"] + lay["offs"] + lay["max_docs"] * 16] \
            .view(torch.float64).view(lay["max_docs"], 2)
        out.append((data, offs, res))
    return out


class SharedRing(PinnedRing):
    """The engine's slot ring over a shared-memory segment (same free/full queues as PinnedRing)."""

    def __init__(self, views: list):
        import queue
        import threading

        self.slots = [Slot(i, d, o) for i, (d, o, _) in enumerate(views)]
        self.results = [r for _, _, r in views]
        self._free, self._full = queue.Queue(), queue.Queue()
        for s in self.slots:
            self._free.put(s)
        self.closed = threading.Event()


class RemoteScorer:
    """Client-side scorer over one or more scoring processes (``conns[0]``: the group's own, the
    others: ScorerPeers). ``submit`` sends the slot index to the scorer with the fewest of this
    client's batches outstanding; ``collect`` returns the (prediction, P(scam)) rows written into
    the oldest submitted slot (FIFO over all scorers, like GpuScorer)."""

    def __init__(self, conns, ring: SharedRing, max_docs: int, max_bytes: int, depth: int = 2, first: int = 0):
        self.conns = list(conns) if isinstance(conns, (list, tuple)) else [conns]
        self.conn, self.ring = self.conns[0], ring
        self.max_docs, self.max_bytes, self._depth = max_docs, max_bytes, depth
        self._q: deque = deque()                  # (slot, scorer) in submission order
        self._out = [0] * len(self.conns)         # outstanding batches per scorer
        self._done: set = set()                   # slot indices whose results arrived
        self._rr = first % len(self.conns)        # clients start on different scorers
        self.sent = [0] * len(self.conns)         # batches sent per scorer (stats)

    @property
    def depth(self) -> int:
        return self._depth

    @property
    def inflight(self) -> int:
        return len(self._q)

    def submit(self, slot: Slot) -> None:
        if len(self._q) >= self._depth:
            raise RuntimeError("pipeline full: call collect() first")
        n = len(self.conns)
        best = self._rr
        for j in range(1, n):
            k = (self._rr + j) % n
            if self._out[k] < self._out[best]:
                best = k
        self._rr = (best + 1) % n
        self.conns[best].send_bytes(_SUB + _HDR.pack(slot.index, slot.n_docs, slot.n_bytes))
        self._out[best] += 1
        self.sent[best] += 1
        self._q.append((slot, best))

    def _recv(self, k: int) -> None:
        try:
            m = self.conns[k].recv_bytes()
        except EOFError:
            raise RuntimeError(f"scoring process {k} closed its connection") from None
        if m[:1] != _DONE:
            raise RuntimeError(f"unexpected message from scoring process {k}: {m[:1]!r}")
        self._done.add(_HDR.unpack_from(m, 1)[0])
        self._out[k] -= 1

    def _pump(self, block: bool) -> None:
        pending = [k for k in range(len(self.conns)) if self._out[k]]
        if not pending:
            return
        if block:
            ready = mp_wait([self.conns[k] for k in pending])
            pending = [k for k in pending if self.conns[k] in ready]
        for k in pending:
            while self._out[k] and self.conns[k].poll(0):
                self._recv(k)

    def ready(self) -> bool:
        if self._q and self._q[0][0].index not in self._done:
            self._pump(block=False)
        return bool(self._q) and self._q[0][0].index in self._done

    def collect(self, copy: bool = True) -> tuple:
        if not self._q:
            raise RuntimeError("nothing in flight")
        slot, _ = self._q[0]
        while slot.index not in self._done:
            self._pump(block=True)
        self._q.popleft()
        self._done.discard(slot.index)
        res = self.ring.results[slot.index][: slot.n_docs].numpy()
        return slot, res.copy() if copy else res


def remote_postprocess(res: np.ndarray) -> tuple:
    """The GPU process already post-processed: rows are (prediction, P(scam))."""
    return res[:, 0], res[:, 1]


# ---------------------------------------------------------------------------------------------- GPU side
class _Client:
    """A client as seen by a scoring process: its segment's slot views and its data connection."""

    def __init__(self, idx: int, shm, lay: dict, conn: Optional[Connection] = None, proc=None):
        self.idx, self.shm, self.lay, self.proc = idx, shm, lay, proc
        self.conn = conn
        self.views = _views(shm.buf, lay)
        self.slots = [Slot(i, d, o) for i, (d, o, _) in enumerate(self.views)]
        self.registered: list = []
        self.reply = None


def _register(cl: _Client) -> None:
    """Page-lock the client's slot views for this process's device (hipHostRegister): the H2D DMA
    reads the client's bytes in place."""
    from ..ops import native

    for d, o, r in cl.views:
        for t in (d, o, r):
            native.lib().host_register(t)
            cl.registered.append(t)


def _unregister(cl: _Client) -> None:
    if cl.registered:
        from ..ops import native

        for t in cl.registered:
            native.lib().host_unregister(t)
        cl.registered = []


class _ScoreLoop:
    """The data plane of one scoring process: micro-batches from the clients' slots through one
    scorer pipeline; (prediction, P(scam)) written back into the slot, then a DONE message."""

    def __init__(self, scorer, postprocess, clients: list, batch_max: int, max_bytes: int):
        self.scorer, self.postprocess, self.clients = scorer, postprocess, clients
        self.batch_max, self.max_bytes = batch_max, max_bytes
        self.batches = self.docs = 0

    def submit(self, cl: _Client, m: bytes) -> None:
        i, n, nb = _HDR.unpack_from(m, 1)
        if not (0 <= i < len(cl.slots)) or n > self.batch_max or nb > self.max_bytes:
            raise RuntimeError(f"client {cl.idx}: bad slot header {(i, n, nb)}")
        sc = self.scorer
        while sc.inflight >= sc.depth:
            self.finish()
        s = cl.slots[i]
        s.n_docs, s.n_bytes, s.meta = n, nb, (cl.idx, i)
        sc.submit(s)
        self.batches += 1
        self.docs += n

    def finish(self) -> None:
        slot, raw = self.scorer.collect(copy=False)
        c, i = slot.meta
        slot.meta = None
        pred, p1 = self.postprocess(raw)
        cl = self.clients[c]
        res = cl.views[i][2][: slot.n_docs].numpy()
        res[:, 0] = pred
        res[:, 1] = p1
        cl.conn.send_bytes(_DONE + _HDR.pack(i, slot.n_docs, slot.n_bytes))

    def pump(self) -> None:
        while self.scorer.inflight and self.scorer.ready():
            self.finish()

    def drain(self) -> None:
        while self.scorer.inflight:
            self.finish()


def single_host_group() -> bool:
    """A consumer group's scoring processes share POSIX shared-memory segments and abstract Unix
    sockets, which exist on one host only: every rank of the job must be on this node
    (LOCAL_WORLD_SIZE == WORLD_SIZE under torchrun)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world


class GroupRendezvous:
    """Rank 0 <-> peer scoring processes: the group's segment config and the peers' socket names
    through a key-value store (the process group's TCPStore under torchrun). ``key`` must be the
    same on every rank and unique per group."""

    def __init__(self, store, key: str, world: int, rank: int, timeout_s: float = 600.0):
        self.store, self.key, self.world, self.rank, self.timeout_s = store, key, world, rank, timeout_s

    @classmethod
    def from_process_group(cls, key: str, timeout_s: float = 600.0) -> "GroupRendezvous":
        import torch.distributed as td

        store = td.distributed_c10d._get_default_store()
        return cls(store, f"fdx-group/{key}", td.get_world_size(), td.get_rank(), timeout_s)

    @property
    def n_peers(self) -> int:
        return self.world - 1

    def _wait(self, k: str) -> bytes:
        import datetime

        self.store.wait([k], datetime.timedelta(seconds=self.timeout_s))
        return self.store.get(k)

    def publish_config(self, cfg: dict) -> None:
        self.store.set(f"{self.key}/cfg", json.dumps(cfg))

    def config(self) -> dict:
        return json.loads(self._wait(f"{self.key}/cfg"))

    def publish_socket(self, name: str) -> None:
        self.store.set(f"{self.key}/sock/{self.rank}", name)

    def publish_socket_error(self, why: str) -> None:
        """A peer that failed to start says so in its socket key, so the coordinator's wait ends
        at once (instead of at the rendezvous timeout)."""
        self.store.set(f"{self.key}/sock/{self.rank}", "!" + why)

    def sockets(self) -> list:
        """Every peer's socket name (waits for each); raises if a peer published a start error."""
        vals = [self._wait(f"{self.key}/sock/{r}").decode() for r in range(1, self.world)]
        errs = [f"rank {r}: {v[1:]}" for r, v in enumerate(vals, 1) if v.startswith("!")]
        if errs:
            raise RuntimeError("scoring peers failed to start: " + "; ".join(errs))
        return vals

    def published_sockets(self) -> list:
        """The socket names published so far (no waiting; start errors skipped)."""
        out = []
        for r in range(1, self.world):
            k = f"{self.key}/sock/{r}"
            try:
                if self.store.check([k]):
                    v = self.store.get(k).decode()
                    if not v.startswith("!"):
                        out.append(v)
            except Exception:                      # noqa: BLE001 (best effort)
                pass
        return out

    def publish_stats(self, stats: dict) -> None:
        self.store.set(f"{self.key}/stats/{self.rank}", json.dumps(stats))

    def stats(self) -> list:
        return [json.loads(self._wait(f"{self.key}/stats/{r}")) for r in range(1, self.world)]


# Client placement (the consumer-group rate fell between two boxes with nothing in the
# record to explain it). With FDX_GROUP_PIN=1 (default) every client process gets CPUs of its own
# from the end of this process's allowed set and the scoring process keeps the rest, so a client
# never competes with the scorer's Python threads for a core; the record carries each client's
# CPUs, NUMA node, CPU seconds and rate, and the cgroup's CPU quota and throttling during the run.
# Measured on the 1-GPU boxes (profiles/r6/kafka/NOTES.md): a confluent-surface client keeps ~2.2
# CPUs busy (its poll / extraction / delivery threads), so 2 logical CPUs of its own cut it to
# 1.14-1.24 M/s for the group, 2-3 whole cores of its own to 1.24-1.39; the clients sharing 8 whole
# cores each (24 cores, SMT siblings included) away from the scorer's gave 1.65-1.74 M/s against
# 1.59-1.63 unpinned. Columnar clients (per-batch work) ran faster unpinned: only confluent-surface
# groups are pinned.
GROUP_PIN = os.environ.get("FDX_GROUP_PIN", "1") == "1"
GROUP_CPUS_PER_CLIENT = int(os.environ.get("FDX_GROUP_CPUS_PER_CLIENT", "8"))
GROUP_WHOLE_CORES = os.environ.get("FDX_GROUP_WHOLE_CORES", "1") == "1"
GROUP_SHARED = os.environ.get("FDX_GROUP_SHARED", "1") == "1"


def cpu_list_str(cpus) -> str:
    """Compact sorted CPU list: [0, 1, 2, 5, 128, 129] -> "0-2,5,128-129"."""
    out, run = [], []
    for c in sorted(cpus):
        if run and c == run[-1] + 1:
            run.append(c)
            continue
        if run:
            out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
        run = [c]
    if run:
        out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out)


def core_siblings(cpu: int, sysfs: str = "/sys/devices/system/cpu") -> tuple:
    """The logical CPUs sharing ``cpu``'s physical core (SMT siblings), ``(cpu,)`` if unknown."""
    try:
        with open(os.path.join(sysfs, f"cpu{cpu}", "topology", "thread_siblings_list")) as fh:
            out = []
            for part in fh.read().strip().split(","):
                a, _, b = part.partition("-")
                out.extend(range(int(a), int(b or a) + 1))
            return tuple(sorted(out)) or (cpu,)
    except (OSError, ValueError):
        return (cpu,)


def client_cpu_plan(allowed: list, n_clients: int, per_client: int = GROUP_CPUS_PER_CLIENT,
                    siblings=None, shared: bool = GROUP_SHARED) -> tuple:
    """(per-client CPU lists, the scorer's CPUs): clients take ``per_client`` physical cores each
    (every allowed SMT sibling of a core goes with it, so a client never shares a core with the
    scorer's threads) from the end of ``allowed``, when at least as many cores remain for the
    scorer; else no pinning (None). ``siblings(cpu)`` gives a CPU's core (default: sysfs; with
    FDX_GROUP_WHOLE_CORES=0 every logical CPU counts as a core of its own). ``shared``: the clients
    pool their cores (every client may run on all of them)."""
    allowed = sorted(allowed)
    if siblings is None:
        siblings = core_siblings if GROUP_WHOLE_CORES else (lambda c: (c,))
    cores, seen = [], set()
    for c in allowed:
        if c in seen:
            continue
        core = [s for s in siblings(c) if s in allowed and s not in seen] or [c]
        seen.update(core)
        cores.append(core)
    cores.sort(key=lambda core: core[0])
    if n_clients <= 0 or per_client <= 0:
        return None, None
    if shared:                       # (a smaller machine: fewer cores each, the scorer keeps half)
        per_client = min(per_client, len(cores) // (2 * n_clients))
        if per_client <= 0:
            return None, None
    need = n_clients * per_client
    if len(cores) < 2 * need:
        return None, None
    tail = cores[len(cores) - need:]
    plan = [sorted(c for core in tail[i * per_client:(i + 1) * per_client] for c in core) for i in range(n_clients)]
    if shared:
        plan = [sorted(c for p in plan for c in p)] * n_clients
    return plan, sorted(c for core in cores[:len(cores) - need] for c in core)


def numa_node_of(cpu: int, sysfs: str = "/sys/devices/system/cpu") -> int:
    try:
        for name in os.listdir(os.path.join(sysfs, f"cpu{cpu}")):
            if name.startswith("node") and name[4:].isdigit():
                return int(name[4:])
    except OSError:
        pass
    return -1


def cgroup_cpu(root: str = "/sys/fs/cgroup") -> dict:
    """The cgroup v2 CPU quota (cpus) of this process and the throttling counters of the level that
    sets it: the process's own cgroup and its ancestors up to ``root`` are read, the tightest
    ``cpu.max`` wins (a box's quota usually sits above the process's own cgroup). Empty if unknown."""
    out: dict = {}
    try:
        with open("/proc/self/cgroup") as fh:
            rel = fh.read().strip().split("::")[-1].strip().strip("/")
    except OSError:
        rel = ""
    parts = rel.split("/") if rel else []
    best = None
    for k in range(len(parts), -1, -1):
        base = os.path.join(root, *parts[:k])
        try:
            with open(os.path.join(base, "cpu.max")) as fh:
                q, per = fh.read().split()
        except (OSError, ValueError):
            continue
        cpus = None if q == "max" else int(q) / int(per)
        if best is None or (cpus is not None and (best[0] is None or cpus < best[0])):
            best = (cpus, base)
    if best is None:
        return out
    out["quota_cpus"] = None if best[0] is None else round(best[0], 2)
    try:
        with open(os.path.join(best[1], "cpu.stat")) as fh:
            for line in fh:
                k, v = line.split()
                if k in ("nr_throttled", "throttled_usec", "usage_usec"):
                    out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def host_cpu_times(path: str = "/proc/stat") -> tuple:
    """(busy, total) jiffies of the whole host from ``/proc/stat`` (other tenants' work included):
    the busy-CPU count over an interval is d(busy) / d(total) * CPUs."""
    try:
        with open(path) as fh:
            v = [int(x) for x in fh.readline().split()[1:]]
    except (OSError, ValueError):
        return 0, 0
    idle = v[3] + (v[4] if len(v) > 4 else 0)
    return sum(v) - idle, sum(v)


class ConsumerGroup:
    """The coordinating scoring process of a consumer group: ``n_clients`` client processes, this
    process's scorer and, with ``rendezvous``, one :class:`ScorerPeer` per other rank.

    ``postprocess(raw) -> (pred, p1)`` runs in the scoring processes (the clients hold no model).
    ``pool`` (a loadgen.MessagePool) is shared with the clients for the in-memory broker runs."""

    def __init__(self, scorer, postprocess, n_clients: int, batch_max: int = 16384, max_latency_ms: float = 5.0,
                 max_bytes: int = 64 << 20, client_depth: int = 2, pool=None, confluent: bool = True,
                 register: Optional[bool] = None, env: Optional[dict] = None,
                 rendezvous: Optional[GroupRendezvous] = None):
        self.scorer, self.postprocess = scorer, postprocess
        self.batch_max = min(batch_max, scorer.max_docs)
        max_bytes = min(max_bytes, scorer.max_bytes)
        self.rdv = rendezvous if (rendezvous is not None and rendezvous.n_peers > 0) else None
        self.n_scorers = 1 + (self.rdv.n_peers if self.rdv is not None else 0)
        # enough batches in flight per client to keep every scoring process busy
        client_depth = max(client_depth, -(-2 * self.n_scorers // max(n_clients, 1)))
        slots = client_depth + 3
        self.lay = slot_layout(slots, self.batch_max, max_bytes)
        self.clients: list = []
        self._pool_shm = None
        self._published = False
        self.peer_sockets: list = []
        pool_lay = None
        dev = getattr(scorer, "dev", None)
        self.register = (dev is not None and dev.type == "cuda") if register is None else register
        try:
            if pool is not None:
                pool_lay, self._pool_shm = _share_pool(pool)
            segs = [shared_memory.SharedMemory(create=True, size=self.lay["size"]) for _ in range(n_clients)]
            for c, shm in enumerate(segs):
                cl = _Client(c, shm, self.lay)
                self.clients.append(cl)
                if self.register:
                    _register(cl)
            if self.rdv is not None:
                # the peers map the same segments and listen for the clients before they start
                self.rdv.publish_config({"layout": self.lay, "shm": [sh.name for sh in segs],
                                         "batch_max": self.batch_max, "max_bytes": max_bytes})
                self._published = True
                self.peer_sockets = self.rdv.sockets()
            base = {"layout": self.lay, "batch_max": self.batch_max, "max_latency_ms": max_latency_ms,
                    "depth": client_depth, "pool": pool_lay, "confluent": confluent, "n_clients": n_clients,
                    "peers": self.peer_sockets}
            self._saved_affinity = None
            plan = None
            if GROUP_PIN and confluent and hasattr(os, "sched_getaffinity"):
                plan, mine = client_cpu_plan(list(os.sched_getaffinity(0)), n_clients)
                if plan is not None:
                    self._saved_affinity = os.sched_getaffinity(0)
                    os.sched_setaffinity(0, mine)
            self.client_cpus = plan
            child_env = dict(os.environ, **(env or {}))
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            child_env["PYTHONPATH"] = root + os.pathsep + child_env.get("PYTHONPATH", "")
            for cl in self.clients:
                a, b = socket.socketpair()
                cfg = dict(base, index=cl.idx, shm=cl.shm.name, fd=b.fileno(),
                           cpus=plan[cl.idx] if plan is not None else None)
                # a fresh interpreter (never a fork of this GPU process); it touches no GPU
                cl.proc = subprocess.Popen([sys.executable, "-m", "fraud_detection_spark_kafka_llm_amd.stream.group",
                                            json.dumps(cfg)], pass_fds=(b.fileno(),), env=child_env)
                b.close()
                cl.conn = Connection(a.detach())
            for cl in self.clients:
                msg = self._control(cl)
                if msg[0] != "ready":
                    raise RuntimeError(f"client {cl.idx}: {msg}")
        except BaseException as e:
            self._abort_peers(f"{type(e).__name__}: {e}")
            self.close()
            raise
        self.loop = _ScoreLoop(scorer, postprocess, self.clients, self.batch_max, self.lay["max_bytes"])

    # ------------------------------------------------------------------ protocol
    def _control(self, cl: _Client, timeout: float = 300.0):
        if not cl.conn.poll(timeout):
            raise TimeoutError(f"client {cl.idx} did not answer")
        m = cl.conn.recv_bytes()
        if m[:1] != _CTL:
            raise RuntimeError(f"client {cl.idx}: expected a control message, got {m[:1]!r}")
        return pickle.loads(m[1:])

    def _send_ctl(self, cl: _Client, obj) -> None:
        cl.conn.send_bytes(_CTL + pickle.dumps(obj))

    def _abort_peers(self, why: str) -> None:
        """Release peers still waiting for a config or for their clients (a group that failed to
        start): an error config, or an abort hello on their sockets."""
        if self.rdv is None:
            return
        try:
            if not self._published:
                self.rdv.publish_config({"error": why})
                return
            # every peer that has published its socket so far (also when the wait for the others
            # is what failed); peers that publish later find the clients gone and time out
            for name in self.peer_sockets or self.rdv.published_sockets():
                try:
                    with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
                        s.settimeout(5.0)
                        s.connect("\0" + name)
                        s.sendall(_HELLO.pack(-1))
                except OSError:
                    pass
        except Exception:                          # noqa: BLE001 (best effort)
            pass

    def run(self, spec: dict, per_client: Optional[list] = None) -> list:
        """Send ``spec`` (merged with ``per_client[c]``) to every client, score their micro-batches
        until each has answered; returns the clients' result dicts in client order."""
        for cl in self.clients:
            cl.reply = None
            self._send_ctl(cl, ("run", dict(spec, **(per_client[cl.idx] if per_client else {}))))
        live = {cl.conn: cl for cl in self.clients}
        sc, loop = self.scorer, self.loop
        while live or sc.inflight:
            loop.pump()
            if not live:
                loop.finish()
                continue
            for conn in mp_wait(list(live), timeout=0.0002 if sc.inflight else 0.05):
                cl = live[conn]
                try:
                    m = conn.recv_bytes()
                except EOFError:
                    raise RuntimeError(f"client {cl.idx} exited (code {cl.proc.poll()})") from None
                if m[:1] == _SUB:
                    loop.submit(cl, m)
                else:
                    msg = pickle.loads(m[1:])
                    if msg[0] == "error":
                        raise RuntimeError(f"client {cl.idx} failed:\n{msg[1]}")
                    cl.reply = msg[1]
                    del live[conn]
            for cl in list(live.values()):
                if cl.proc.poll() is not None and not cl.conn.poll(0):
                    raise RuntimeError(f"client {cl.idx} exited (code {cl.proc.returncode})")
        return [cl.reply for cl in self.clients]

    @property
    def local_batches(self) -> int:
        return self.loop.batches if getattr(self, "loop", None) is not None else 0

    def close(self) -> None:
        saved = getattr(self, "_saved_affinity", None)
        if saved is not None:                     # (the scorer's CPUs back as they were)
            os.sched_setaffinity(0, saved)
            self._saved_affinity = None
        # no DMA may still read a segment when it is unregistered and unmapped (a run that raised
        # can leave micro-batches in the scorer's pipeline); a drain that fails (e.g. after the GPU
        # error that ended run()) is logged, and the clients are still stopped and the segments
        # still released below
        try:
            while self.scorer.inflight:
                self.scorer.collect(copy=False)
        except Exception as e:                    # noqa: BLE001
            print(f"[group] scorer drain failed during close: {type(e).__name__}: {e}", file=sys.stderr)
        try:
            if self.register and torch.cuda.is_available():
                torch.cuda.synchronize()
        except Exception as e:                    # noqa: BLE001
            print(f"[group] synchronize failed during close: {type(e).__name__}: {e}", file=sys.stderr)
        for cl in self.clients:
            if cl.conn is None:
                continue
            try:
                self._send_ctl(cl, ("exit", {}))
            except OSError:
                pass
        for cl in self.clients:
            if cl.proc is not None:
                try:
                    cl.proc.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    cl.proc.kill()
                    cl.proc.wait()
            _unregister(cl)
            if cl.conn is not None:
                cl.conn.close()
            cl.views = cl.slots = None
            try:
                cl.shm.close()
            except BufferError:      # a tensor view still alive somewhere: the unlink still frees it
                pass
            cl.shm.unlink()
        self.clients = []
        if self._pool_shm is not None:
            self._pool_shm.close()
            self._pool_shm.unlink()
            self._pool_shm = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class ScorerPeer:
    """A scoring process of a consumer group other than the coordinator (rank r > 0 of a torchrun
    job, on its own GPU): maps the clients' segments, page-locks them for its device, listens on
    a Unix socket (abstract namespace) that every client connects to, and scores the micro-batches
    the clients send it until all of them have closed their connections. ``serve()`` returns the
    number of batches and documents it scored."""

    def __init__(self, scorer, postprocess, rendezvous: GroupRendezvous, register: Optional[bool] = None,
                 accept_timeout_s: float = 600.0):
        import uuid

        self.scorer, self.postprocess, self.rdv = scorer, postprocess, rendezvous
        self.clients: list = []
        self.listener = None
        self.error = None
        cfg = rendezvous.config()
        if "error" in cfg:
            self.error = cfg["error"]
            return
        try:
            self.lay = cfg["layout"]
            dev = getattr(scorer, "dev", None)
            self.register = (dev is not None and dev.type == "cuda") if register is None else register
            for c, name in enumerate(cfg["shm"]):
                cl = _Client(c, _attach(name), self.lay)
                self.clients.append(cl)
                if self.register:
                    _register(cl)
            self.name = f"fdx-group-{os.getpid()}-{uuid.uuid4().hex[:12]}"
            self.listener = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            self.listener.bind("\0" + self.name)
            self.listener.listen(len(self.clients) + 4)
            self.listener.settimeout(accept_timeout_s)
        except BaseException as e:
            # the coordinator waits for this peer's socket key: answer with the error
            rendezvous.publish_socket_error(f"{type(e).__name__}: {e}")
            self.close()
            raise
        rendezvous.publish_socket(self.name)
        self.loop = _ScoreLoop(scorer, postprocess, self.clients, int(cfg["batch_max"]), int(cfg["max_bytes"]))

    def serve(self) -> dict:
        if self.error is not None:
            return {"batches": 0, "docs": 0, "error": self.error}
        pending = {cl.idx for cl in self.clients}
        while pending:
            s, _ = self.listener.accept()
            s.settimeout(60.0)
            hello = b""
            while len(hello) < _HELLO.size:
                chunk = s.recv(_HELLO.size - len(hello))
                if not chunk:
                    break
                hello += chunk
            idx = _HELLO.unpack(hello)[0] if len(hello) == _HELLO.size else -1
            if idx < 0 or idx not in pending:     # the coordinator aborted the group
                s.close()
                return {"batches": self.loop.batches, "docs": self.loop.docs, "error": "aborted"}
            s.settimeout(None)
            self.clients[idx].conn = Connection(s.detach())
            pending.discard(idx)
        live = {cl.conn: cl for cl in self.clients}
        sc, loop = self.scorer, self.loop
        while live or sc.inflight:
            loop.pump()
            if not live:
                loop.finish()
                continue
            for conn in mp_wait(list(live), timeout=0.0002 if sc.inflight else 0.05):
                cl = live[conn]
                try:
                    m = conn.recv_bytes()
                except (EOFError, ConnectionError):
                    del live[conn]                  # the client exited: the group is closing
                    continue
                if m[:1] != _SUB:
                    raise RuntimeError(f"client {cl.idx}: unexpected message {m[:1]!r} at a peer")
                loop.submit(cl, m)
        return {"batches": loop.batches, "docs": loop.docs}

    def close(self) -> None:
        try:
            while self.scorer.inflight:
                self.scorer.collect(copy=False)
        except Exception as e:                    # noqa: BLE001
            print(f"[group-peer] scorer drain failed during close: {type(e).__name__}: {e}", file=sys.stderr)
        try:
            if getattr(self, "register", False) and torch.cuda.is_available():
                torch.cuda.synchronize()
        except Exception as e:                    # noqa: BLE001
            print(f"[group-peer] synchronize failed during close: {type(e).__name__}: {e}", file=sys.stderr)
        for cl in self.clients:
            _unregister(cl)
            if cl.conn is not None:
                cl.conn.close()
            cl.views = cl.slots = None
            try:
                cl.shm.close()
            except BufferError:
                pass
        self.clients = []
        if self.listener is not None:
            self.listener.close()
            self.listener = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _share_pool(pool) -> tuple:
    arrs = {"vals": pool.vals, "voff": pool.voff, "keys": pool.keys, "koff": pool.koff}
    lay, pos = {}, 0
    for k, a in arrs.items():
        lay[k] = (pos, str(a.dtype), int(a.size))
        pos = _round(pos + a.nbytes)
    shm = shared_memory.SharedMemory(create=True, size=max(pos, 1))
    for k, a in arrs.items():
        o, dt, n = lay[k]
        np.ndarray(n, dtype=dt, buffer=shm.buf, offset=o)[:] = a
    lay["name"], lay["n"] = shm.name, pool.n
    return lay, shm


# ---------------------------------------------------------------------------------------------- aggregate runs
def merge_results(rs: list) -> dict:
    """Whole-group numbers: dialogues/s over the union of the clients' timed windows, exact
    latency percentiles from the summed histograms."""
    from .engine import LatencyHistogram

    h = LatencyHistogram()
    for r in rs:
        h.counts += np.asarray(r["lat_counts"], dtype=np.int64)
        h.n += int(r["lat_n"])
    t0, t1 = min(r["t0"] for r in rs), max(r["t1"] for r in rs)
    msgs = sum(r["messages"] for r in rs)
    return {"dialogues_per_s": msgs / max(t1 - t0, 1e-9), "sec": t1 - t0, "messages": msgs,
            "produced": sum(r["produced"] for r in rs), "committed": sum(r["committed"] for r in rs),
            "sent": sum(r.get("sent", 0) for r in rs), "batches": sum(r["batches"] for r in rs),
            "explanations": sum(r.get("explanations", 0) for r in rs),
            "scorer_batches": [int(x) for x in np.sum([r["scorer_batches"] for r in rs if "scorer_batches" in r],
                                                      axis=0)] if any("scorer_batches" in r for r in rs) else [],
            "p50_ms": h.percentile(50), "p95_ms": h.percentile(95), "p99_ms": h.percentile(99),
            "clients": len(rs), "client_dialogues_per_s": [r["messages"] / max(r["t1"] - r["t0"], 1e-9) for r in rs],
            # per client: CPU seconds over its window (1.0 = one core busy), its CPUs and NUMA node
            "client_cpu_util": [round(r.get("cpu_s", 0.0) / max(r["t1"] - r["t0"], 1e-9), 3) for r in rs],
            "client_cpus": [r.get("cpus", []) or r.get("n_cpus", 0) for r in rs],
            "client_numa": [r.get("numa", -1) for r in rs],
            "client_start_spread_ms": (max(r["t0"] for r in rs) - t0) * 1e3}


def group_throughput_run(group: ConsumerGroup, n: int, tag: str = "gtp", **extra) -> dict:
    """Each client drains a pre-filled partition of n / P records (partition c of a P-partition
    topic on its broker); rate over the whole group."""
    P = len(group.clients)
    share = [n // P + (1 if c < n % P else 0) for c in range(P)]
    rs = group.run(dict({"kind": "throughput", "tag": tag}, **extra), [{"n": k} for k in share])
    out = merge_results(rs)
    if extra.get("return_outputs"):
        out["outputs"] = [r["outputs"] for r in rs]
    return out


def group_latency_run(group: ConsumerGroup, rate: float, duration_s: float, warmup_s: float = 0.3,
                      tag: str = "glat", batch_max: int = 4096, max_latency_ms: float = 1.0, **extra) -> dict:
    """A paced producer per client appends rate / P records/s to its partition; per-message
    latency (append -> output delivered) over the whole group."""
    P = len(group.clients)
    r = merge_results(group.run({"kind": "latency", "rate": rate / P, "duration": duration_s, "warmup": warmup_s,
                                 "tag": tag, "batch_max": batch_max, "max_latency_ms": max_latency_ms, **extra}))
    r["offered_per_s"] = rate
    return r


# ---------------------------------------------------------------------------------------------- client process
def _client_pool(lay: dict):
    from .loadgen import MessagePool

    shm = _attach(lay["name"])
    pool = MessagePool.__new__(MessagePool)
    for k in ("vals", "voff", "keys", "koff"):
        o, dt, n = lay[k]
        setattr(pool, k, np.ndarray(n, dtype=dt, buffer=shm.buf, offset=o))
    pool.n = lay["n"]
    return pool, shm


def _client_run(cfg: dict, spec: dict, conn: Connection, ring: SharedRing, pool) -> dict:
    from . import fake_kafka, loadgen
    from .engine import StreamingEngine

    c, P = cfg["index"], cfg["n_clients"]
    lay = cfg["layout"]
    scorer = RemoteScorer([conn] + cfg.get("peer_conns", []), ring, lay["max_docs"], lay["max_bytes"], cfg["depth"],
                          first=c)
    if spec["kind"] == "serve":
        return _client_serve(cfg, spec, scorer, ring)
    url = f"memory://group-{os.getpid()}-{spec['tag']}"
    broker = fake_kafka.broker_for(url)
    broker.create_topic("in", P)
    broker.create_topic("out", P)
    inner = fake_kafka.Consumer({"bootstrap.servers": url, "group.id": "fdx-group", "auto.offset.reset": "earliest",
                                 "enable.auto.commit": False})
    inner.assign([fake_kafka.TopicPartition("in", c)])
    prod = fake_kafka.Producer({"bootstrap.servers": url})
    cons, producer = (fake_kafka.ConfluentConsumer(inner), fake_kafka.ConfluentProducer(prod)) if cfg["confluent"] \
        else (inner, prod)
    # per-run micro-batch policy (latency runs: small batches, short fill deadline)
    eng = StreamingEngine(scorer, remote_postprocess, cons, producer, "out",
                          batch_max=min(spec.get("batch_max", cfg["batch_max"]), cfg["batch_max"]),
                          max_latency_ms=spec.get("max_latency_ms", cfg["max_latency_ms"]), max_bytes=lay["max_bytes"],
                          ring=ring, **_explain_kw(spec))
    sent = 0
    import resource

    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    if spec["kind"] == "throughput":
        n = int(spec["n"])
        with broker.lock:
            for s in range(0, n, 8192):
                broker.topics["in"][c].append(pool.batch(c * 7919 + s, min(8192, n - s), "in", c))
            broker.cond.notify_all()
        t0 = time.perf_counter()
        st = eng.run(max_messages=n, idle_timeout_s=5.0)
        sent = n
    else:
        # this client's partition only: a paced producer appending to partition c
        gen = _PartitionPacer(broker, "in", c, pool, spec["rate"], spec["duration"] + spec["warmup"])
        import threading

        def reset():
            time.sleep(spec["warmup"])
            eng.stats.latency.reset()

        threading.Thread(target=reset, daemon=True).start()
        gen.start()
        t0 = time.perf_counter()
        st = eng.run(idle_timeout_s=0.5)
        gen.join()
        sent = gen.sent
    t1 = time.perf_counter()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    committed = sum(inner.committed_offsets().values())
    outputs = None
    if spec.get("return_outputs"):           # tests: the produced records, in partition order
        outputs = []
        for part in broker.topics["out"]:
            for it in part:       # columnar batches (produce_records) or Messages (per-record produce)
                outputs += [(it.key(i), it.value(i)) for i in range(it.n)] if hasattr(it, "n") \
                    else [(it.key(), it.value())]
    loadgen._drop(url)
    return {"outputs": outputs, "t0": t0, "t1": t1, "messages": st["messages"], "produced": st["produced"], "committed": committed,
            "batches": st["batches"], "sent": sent, "explanations": st["explanations"],
            "scorer_batches": list(scorer.sent), "cpu_s": cpu_s, "n_cpus": len(cpus),
            "cpus": cpu_list_str(cpus), "numa": numa_node_of(cpus[0]) if cpus else -1,
            "lat_counts": eng.stats.latency.counts.tolist(),
            "lat_n": eng.stats.latency.n, "p50_ms": st["p50_ms"]}


class _ClientExplainer:
    """What the engine needs of an agent for LLM explanations (serve/llm.py Analyzer), without the
    model: the GPU process classified the record already. No historical-case insight (that table
    lives with the agent)."""

    def __init__(self, llm):
        from ..serve.llm import Analyzer

        self.analyzer = Analyzer(llm)

    def classify_and_explain(self, dialogue: str, temperature: float = 0.7, prediction: Optional[dict] = None,
                             with_history: bool = True) -> dict:
        analysis = self.analyzer.analyze_prediction(dialogue, prediction["prediction"], prediction["confidence"],
                                                    temperature)
        return dict(prediction, analysis=analysis, historical_insight=None)


def _explain_kw(spec: dict) -> dict:
    """Engine arguments of a run's ``explain`` mode ("none" | "async" | "sync"); the LLM backend is
    ``spec["llm"]`` (serve/llm.py make_llm names; "stub" = the offline stub, optional latency)."""
    mode = spec.get("explain", "none")
    if mode == "none":
        return {}
    from ..serve.llm import StubLLM, make_llm

    backend = spec.get("llm", "stub")
    llm = StubLLM(latency_s=spec.get("llm_latency_s", 0.0)) if backend == "stub" else make_llm(backend)
    return {"explain": mode, "agent": _ClientExplainer(llm), "explain_every": int(spec.get("explain_every", 1))}


def _client_serve(cfg: dict, spec: dict, scorer: RemoteScorer, ring: SharedRing) -> dict:
    """A consumer-group member against the configured Kafka (stream/kafka.py factories, the
    reference's environment variables): subscribes with the group id, so the broker balances the
    topic's partitions over the group's clients; produces to KAFKA_OUTPUT_TOPIC, commits after
    delivery."""
    from . import kafka
    from .engine import StreamingEngine

    cons = kafka.get_kafka_consumer(group=spec.get("group"))
    try:
        eng = StreamingEngine(scorer, remote_postprocess, cons, kafka.get_kafka_producer(),
                              spec.get("output_topic") or os.getenv("KAFKA_OUTPUT_TOPIC", kafka.DEFAULT_OUTPUT),
                              batch_max=cfg["batch_max"], max_latency_ms=cfg["max_latency_ms"],
                              max_bytes=cfg["layout"]["max_bytes"], ring=ring, **_explain_kw(spec))
        t0 = time.perf_counter()
        st = eng.run(max_messages=spec.get("max_messages"), idle_timeout_s=spec.get("idle_timeout", float("inf")))
        t1 = time.perf_counter()
    finally:
        cons.close()
    return {"t0": t0, "t1": t1, "messages": st["messages"], "produced": st["produced"],
            "committed": st["committed"], "batches": st["batches"], "sent": 0,
            "lat_counts": eng.stats.latency.counts.tolist(), "lat_n": eng.stats.latency.n, "p50_ms": st["p50_ms"],
            "scorer_batches": list(scorer.sent), "summary": st}


class _PartitionPacer:
    """loadgen.PacedProducer restricted to one partition (one client of the group)."""

    def __init__(self, broker, topic: str, partition: int, pool, rate: float, duration_s: float, tick_ms: float = 1.0):
        import threading

        self.broker, self.topic, self.p, self.pool = broker, topic, partition, pool
        self.rate, self.duration, self.tick = rate, duration_s, tick_ms / 1000.0
        self.sent = 0
        self._t = threading.Thread(target=self._run, name="fdx-partition-pacer", daemon=True)

    def start(self) -> None:
        self._t.start()

    def join(self) -> None:
        self._t.join()

    def _run(self) -> None:
        t0 = time.perf_counter()
        nxt = t0
        while time.perf_counter() - t0 < self.duration:
            due = int((time.perf_counter() - t0) * self.rate) - self.sent
            if due > 0:
                with self.broker.lock:
                    rb = self.pool.batch(self.p * 7919 + self.sent, due, self.topic, self.p, ts=time.perf_counter())
                    self.broker.topics[self.topic][self.p].append(rb)
                    self.sent += due
                    self.broker.cond.notify_all()
            nxt += self.tick
            time.sleep(max(0.0, nxt - time.perf_counter()))


def _attach(name: str):
    """Attach a segment the GPU process owns (and unlinks): not this process's resource tracker's
    to remove at exit."""
    from multiprocessing import resource_tracker

    shm = shared_memory.SharedMemory(name=name)
    resource_tracker.unregister(shm._name, "shared_memory")
    return shm


def _connect_peers(cfg: dict) -> list:
    """This client's data connections to the group's peer scoring processes."""
    out = []
    for name in cfg.get("peers") or []:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.connect("\0" + name)
        s.sendall(_HELLO.pack(int(cfg["index"])))
        out.append(Connection(s.detach()))
    return out


def _client_main(cfg: dict) -> int:
    if cfg.get("cpus") and hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, cfg["cpus"])
    conn = Connection(cfg["fd"])
    shm = _attach(cfg["shm"])
    pool_shm = None
    peer_conns = []
    try:
        peer_conns = cfg["peer_conns"] = _connect_peers(cfg)
        ring = SharedRing(_views(shm.buf, cfg["layout"]))
        pool = None
        if cfg["pool"] is not None:
            pool, pool_shm = _client_pool(cfg["pool"])
        conn.send_bytes(_CTL + pickle.dumps(("ready", {})))
        while True:
            m = conn.recv_bytes()
            cmd, spec = pickle.loads(m[1:])
            if cmd == "exit":
                return 0
            try:
                prof_to = os.environ.get("FDX_CLIENT_PROFILE")      # (diagnostics: cProfile per run)
                if prof_to:
                    import cProfile

                    pr = cProfile.Profile()
                    r = pr.runcall(_client_run, cfg, spec, conn, ring, pool)
                    pr.dump_stats(f"{prof_to}.{cfg['index']}")
                else:
                    r = _client_run(cfg, spec, conn, ring, pool)
                conn.send_bytes(_CTL + pickle.dumps(("result", r)))
            except Exception:
                import traceback

                conn.send_bytes(_CTL + pickle.dumps(("error", traceback.format_exc())))
                return 1
    except (EOFError, ConnectionError):
        return 0
    finally:
        for c in peer_conns:
            c.close()
        cfg.pop("peer_conns", None)
        ring = pool = None
        import gc

        gc.collect()
        for s in (shm, pool_shm):
            if s is not None:
                try:
                    s.close()
                except BufferError:
                    pass


if __name__ == "__main__":
    sys.exit(_client_main(json.loads(sys.argv[1])))
