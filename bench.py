"""Headline benchmark (BASELINE.json): "dialogues/sec streaming inference + GBDT train sec on 10M rows,
1/2/4/8 GPU".

Per rank (one process per MI355X, RCCL over xGMI when N > 1):
  1. GBDT training — HashingTF(2^18) -> IDF -> GBDT (100 trees, depth 6, XGBoost binary:logistic)
     on 10M synthetic dialogues row-sharded across the N ranks. The corpus is generated first
     (untimed, reported as gbdt_datagen_sec_untimed) into pinned host memory; the timed phase
     ``gbdt_train_sec`` (max over ranks) is H2D of the raw text + fused featurization +
     all-reduced docFreq/IDF + quantization + boosting (per-level histogram reduce-scatter).
  2. Streaming inference (the timed K steps) — every step each rank takes one micro-batch of
     raw UTF-8 dialogues from a pinned host ring, copies it to HBM (copy stream), runs the fused
     clean/tokenize/stop-word/murmur3/IDF/100-tree-GBDT kernel (compute stream), which stores the
     scores straight into pinned host memory; the host then applies the sigmoid/threshold. The
     copy of step i+1 overlaps the kernel of step i. ``value`` = dialogues/s summed over all ranks
     (weak scaling: fixed micro-batch per GPU).
  3. RandomForest training (BASELINE config 3) — RandomForestClassifier(500 trees, depth 5,
     featureSubsetStrategy sqrt = ceil(sqrt(2^18)) features per node, Poisson(1) bootstrap, 32
     bins) on the SAME row-sharded 10M-row TF-IDF features (features are fitted once and shared, as
     train.py does; the reference refits them per model): ``rf_train_sec`` (max over ranks) =
     quantisation to 32 bins + 500 trees with per-level histogram reduce-scatter under DP.
  4. Kafka end-to-end (BASELINE config 5) — an in-memory broker topic with 3 partitions of
     ``{"text": ...}`` JSON records -> StreamingEngine (one reader thread per partition, native JSON
     extraction into the pinned ring, GPU scoring, native output encoding, async produce, commits
     gated on delivery callbacks). ``kafka_dialogues_per_s``: a pre-filled topic drained end to end
     (consume -> score -> produce -> commit); ``kafka_p50_ms`` / ``kafka_p95_ms``: per-message
     latency (broker append -> output delivered) under a paced producer at ``kafka_offered_per_s``.
     Per GPU (rank 0's engine on its own broker; not summed over ranks). ``kafka_confluent_*``: the
     same runs through clients restricted to the confluent_kafka surface (per-record Messages,
     produce + delivery callback per record). ``kafka_confluent_group_*``: the confluent surface as
     a consumer group over ONE 3-partition topic: one client process per partition around a
     scoring process PER RANK, each on its own GPU (stream/group.py: rank 0 coordinates, ranks
     1..N-1 are ScorerPeers; shared-memory slots page-locked by every scoring process for its
     device; no process opens another rank's GPU); ``..._explain_*``: the same latency run with
     the LLM-explain stub on every 10th record. ``kafka_multi_gpu_*``: the same N scoring
     processes fed by columnar clients (``..._scorer_procs`` = N, batches per scoring process).
     The throughput drains of the columnar engine and of both groups run three times and report
     the median (``..._runs_dialogues_per_s`` lists all three: a sub-second drain of Python clients
     on a shared host moves by +-15 % from run to run, profiles/r6/kafka/NOTES.md).
Phases 3 and 4 run after the headline (1, 2 and the single-dialogue latency) is measured, each
under a PhaseGuard: a failure is reported as ``rf_error`` / ``kafka_error`` in the record and a
hang is cut off after ``--phase-timeout`` s with the record printed as it stands.
Data is synthetic (the reference dataset is not available) with random-init-free trained trees.
Before the timed training, an untimed 2-tree fit on 65,536 rows loads the kernels' code objects
(lazily loaded on first launch by ROCm) and warms the allocators (``gbdt_warmup_sec_untimed``).
Compute dtype: the GBDT histograms are exact integer sums (gradients quantised to 2^-k with k
from the all-reduced max, accumulated as int64 by LDS atomics in the row-group kernel,
csrc/row_kernels.hip) — at least fp32-accurate and bitwise reproducible; gains, leaves and scores
are fp64; text is bytes. Reported as "fp32".

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 is launched by the driver via torch.distributed.run (RANK/WORLD_SIZE/MASTER_* in env).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
import traceback

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from fraud_detection_spark_kafka_llm_amd.data import synth  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.xgboost import SparkXGBClassifierModel  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops import text as T  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops.sparse import IncrementalFeatureOrder, feature_order  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.parallel import dist as D  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.parallel.affinity import bind_to_gpu  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.stream.gpu_worker import GpuScorer  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.stream.ring import PinnedRing  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.utils import memory  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.utils.config import Config  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.utils.profiling import run_profiled_if_requested  # noqa: E402

METRIC = "dialogues/sec streaming inference + GBDT train sec on 10M rows, 1/2/4/8 GPU"
F = 1 << 18
CHUNK_ROWS = 500_000       # rows per featurization chunk (pinned text, H2D overlapped with the kernel)
GROUP_TIMEOUT_S = 120.0    # consumer-group rendezvous waits (a peer that never starts fails the phase)


def sync_all(dev):
    torch.cuda.synchronize(dev)
    D.barrier()
    torch.cuda.synchronize(dev)


def max_over_ranks(x: float, dev) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    return float(D.all_reduce_max(t).item())


class PhaseGuard:
    """Runs the phases that follow the headline measurement so that none of them can lose the
    record. An exception lands in it as ``<phase>_error``, and the ranks agree on failure through
    a MAX all-reduce of an error flag (a phase that failed on one rank is reported by rank 0 too).
    A phase still running after ``timeout_s`` (a hang, e.g. a collective waiting for a rank that
    died) is cut off by a watchdog thread: it prints the record as it stands (rank 0) and ends the
    process with status 3 (a hang is a failure, not a clean run), on every rank, well inside the process group's own timeout (which
    would abort the job without a record)."""

    def __init__(self, record: dict, rank: int, timeout_s: float):
        self.record, self.rank, self.timeout_s = record, rank, float(timeout_s)

    def _expire(self, name: str) -> None:
        self.record[f"{name}_error"] = f"timeout: phase still running after {self.timeout_s:.0f} s"
        if self.rank == 0:
            print(json.dumps(self.record), flush=True)
        sys.stderr.flush()
        os._exit(3)

    def run(self, name: str, fn, dev) -> None:
        timer = threading.Timer(self.timeout_s, self._expire, args=(name,))
        timer.daemon = True
        timer.start()
        err = None
        try:
            try:
                self.record.update(fn() or {})
            except Exception as e:                 # noqa: BLE001 (reported in the record)
                traceback.print_exc()
                err = f"{type(e).__name__}: {e}"
            try:
                failed = max_over_ranks(1.0 if err else 0.0, dev) > 0
            except Exception as e:                 # noqa: BLE001
                failed, err = True, err or f"{type(e).__name__}: {e}"
        finally:
            timer.cancel()
        if failed:
            self.record[f"{name}_error"] = err or "failed on another rank"



def bench_fault(phase: str) -> None:
    """``FDX_BENCH_FAULT=<phase>[:hang]`` (tests): raise in, or hang, the named phase on every rank."""
    spec = os.environ.get("FDX_BENCH_FAULT", "")
    if not spec or spec.split(":")[0] != phase:
        return
    if spec.endswith(":hang"):
        time.sleep(1e9)
    raise RuntimeError(f"injected fault in the {phase} phase")


def generate_shard(lo: int, hi: int, dev, seed: int, chunk: int = 500_000) -> list:
    """Synthetic corpus of rows [lo, hi) as pinned host-resident UTF-8 chunks (the "dataset in
    memory" the timed training phase starts from; generation itself is not training)."""
    out = []
    for start in range(lo, hi, chunk):
        n = min(chunk, hi - start)
        pt, y = synth.generate(synth.SynthConfig(n=n, seed=seed), device=dev, start=start)
        host = T.PackedText(pt.data.cpu().pin_memory(), pt.offsets.cpu().pin_memory())
        out.append((host, y.cpu().pin_memory()))
        del pt
    return out


def featurize_shard(chunks: list, dev, spec, order: bool = False):
    """H2D + fused clean/tokenize/stop-words/murmur3 HashingTF of every chunk -> one CSR.

    The H2D of chunk i+1 runs on a copy stream (SDMA) while chunk i is featurized on the
    compute stream, so the PCIe transfer of the raw text hides behind the kernel. With
    ``order`` each chunk's entries are also sorted by feature right after its featurization
    (ops/sparse.py IncrementalFeatureOrder), still underneath the next chunk's H2D: the
    CSR -> CSC sort (docFreq for the IDF, the trainer's columns) is no longer a serial ~0.25 s
    pass after the transfer (profiles/r3s4/featurize_probe_10M.jsonl). Returns the CSR (+ the
    FeatureOrder when ``order``)."""
    rows = sum(int(h.offsets.numel()) - 1 for h, _ in chunks)
    indptr = torch.zeros(rows + 1, dtype=torch.int64, device=dev)
    labels = torch.empty(rows, dtype=torch.float64, device=dev)
    idx = counts = None
    off = r = 0
    inc = IncrementalFeatureOrder(F, dev) if order else None
    comp = torch.cuda.current_stream(dev)
    copy = comp if os.environ.get("FDX_BENCH_SERIAL_H2D") == "1" else torch.cuda.Stream(dev)
    # two device staging buffers, allocated once (a fresh ~1 GB allocation per chunk on the copy
    # stream left ~94 GB reserved and made the first pass 2x slower: profiles/r3s4/NOTES.md)
    mb = max((int(h.data.numel()) for h, _ in chunks), default=0)
    md = max((int(h.offsets.numel()) for h, _ in chunks), default=0)
    bufs = [(torch.empty(mb, dtype=torch.uint8, device=dev), torch.empty(md, dtype=torch.int64, device=dev),
             torch.empty(md, dtype=torch.float64, device=dev)) for _ in range(2 if chunks else 0)]
    freed = [None, None]                 # comp-stream event: staging buffer j consumed

    def stage(i):
        host, y = chunks[i]
        j = i % 2
        bd, bo, by = bufs[j]
        nb, no = int(host.data.numel()), int(host.offsets.numel())
        with torch.cuda.stream(copy):
            if freed[j] is not None:
                copy.wait_event(freed[j])
            bd[:nb].copy_(host.data, non_blocking=True)
            bo[:no].copy_(host.offsets, non_blocking=True)
            by[:no - 1].copy_(y, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(copy)
        return T.PackedText(bd[:nb], bo[:no]), by[:no - 1], ev

    nxt = stage(0) if chunks else None
    for i in range(len(chunks)):
        d, yd, ev = nxt
        comp.wait_event(ev)
        if i + 1 < len(chunks):
            nxt = stage(i + 1)
        res = T.featurize_score(d, spec, want_csr=True, device=dev)
        ip, ix, v = res.csr()
        del res, d
        # each chunk's entries go straight into buffers sized from the first chunk (grown if
        # needed), so the CSR is never held twice (HBM sizing, utils/memory.py)
        k, n = int(ip[-1]), int(ip.numel()) - 1
        if idx is None:
            cap = int(k / max(n, 1) * rows * 1.05) + k + 1024
            idx = torch.empty(cap, dtype=ix.dtype, device=dev)
            counts = torch.empty(cap, dtype=v.dtype, device=dev)
        if off + k > idx.numel():
            cap = int((off + k) * 1.25)
            idx = torch.cat([idx[:off], torch.empty(cap - off, dtype=idx.dtype, device=dev)])
            counts = torch.cat([counts[:off], torch.empty(cap - off, dtype=counts.dtype, device=dev)])
        idx[off:off + k] = ix
        counts[off:off + k] = v
        indptr[r + 1:r + n + 1] = ip[1:] + off
        labels[r:r + n] = yd
        if inc is not None:
            inc.add(ip, ix, v, r)
        freed[i % 2] = comp.record_event()   # staging buffer free for chunk i + 2
        off += k
        r += n
        del ip, ix, v, yd
    if idx is None:
        idx = torch.empty(0, dtype=torch.int32, device=dev)
        counts = torch.empty(0, dtype=torch.int32, device=dev)
    if inc is not None:
        return indptr, idx[:off], counts[:off], labels, inc.finish() if chunks else feature_order(indptr, idx, counts, F)
    return indptr, idx[:off], counts[:off], labels


def warmup_training(dev, spec, params: GBDTParams, rf_depth: int = 0) -> None:
    """Untimed: the pinned H2D copy path plus a small fit through the production path
    (models/warmup.py: lazily loaded kernel code objects, cold caching allocators). Every rank runs
    it on the same rows, so under data parallelism its collectives warm RCCL too."""
    # the timed phase's featurization path itself (chunked H2D + fused kernel + the per-chunk
    # feature-order sort and its merge) on a small pinned shard: its first run in a process cost
    # ~0.33 s extra (kernel code objects loaded on first launch; profiles/r4/cold_*.jsonl)
    small = generate_shard(3 * 10**9, 3 * 10**9 + (1 << 15), dev, seed=5, chunk=1 << 14)
    featurize_shard(small, dev, spec, order=True)
    del small
    warm_tree_kernels(dev, gbdt_depth=params.max_depth, gbdt_max_bin=params.max_bin, forest_depth=rf_depth,
                      forest_subset="sqrt")


def group_kafka(args, spec, idf_np, model, dev, pool) -> dict:
    """Config 5 as a consumer group whose scoring processes are the job's ranks (stream/group.py):
    rank 0 creates the shared-memory slots and starts one client process per partition of the
    3-partition topic; every rank scores on ITS OWN GPU (rank 0 with a ConsumerGroup, the others
    as ScorerPeers that page-lock the same slots for their device). Two groups run:
      * ``kafka_confluent_group_*``: clients restricted to the confluent_kafka surface
        (throughput, paced latency, latency with the LLM-explain stub on every 10th record);
      * ``kafka_multi_gpu_*``: columnar clients (the throughput the N scoring processes reach when
        the clients are cheap), with the micro-batches each scoring process took.
    A failure is reported in the record, not raised; no rank enters a device barrier before its
    scoring process has stopped."""
    from fraud_detection_spark_kafka_llm_amd.stream.group import single_host_group

    if not single_host_group():           # shared segments + Unix sockets: one host only
        return {"kafka_group_error": "ranks span hosts (LOCAL_WORLD_SIZE != WORLD_SIZE)"} if D.rank() == 0 else {}
    out = {}
    for name, fn in (("kafka_confluent_group", _group_confluent_runs), ("kafka_multi_gpu", _group_multi_runs)):
        if (name == "kafka_multi_gpu" and args.kafka_multi_msgs <= 0) or \
                (name == "kafka_confluent_group" and args.kafka_group_msgs <= 0):
            continue
        try:
            out.update(_group_session(name, fn, args, spec, idf_np, model, dev, pool))
        except Exception as e:     # the headline line must still be printed: report, do not abort
            import traceback

            traceback.print_exc()
            out[f"{name}_error"] = f"{type(e).__name__}: {e}"
        D.barrier()
    return out if D.rank() == 0 else {}


def _group_session(name, runs, args, spec, idf_np, model, dev, pool) -> dict:
    import gc

    from fraud_detection_spark_kafka_llm_amd.stream import group as G

    batch = 16384
    rdv = G.GroupRendezvous.from_process_group(name, timeout_s=GROUP_TIMEOUT_S) if D.world_size() > 1 else None
    try:
        sc = GpuScorer(spec, idf_np, model.scorer(), dev, max_docs=batch, max_bytes=batch * 4096, depth=3)
    except Exception as e:
        # the other side of the rendezvous waits for this rank: answer with the error
        if rdv is not None:
            why = f"{type(e).__name__}: {e}"
            rdv.publish_socket_error(why) if D.rank() > 0 else rdv.publish_config({"error": why})
        raise
    gc.collect()
    if D.rank() > 0:
        with G.ScorerPeer(sc, model.postprocess_numpy, rdv) as peer:
            try:
                st = peer.serve()
            except Exception as e:                 # noqa: BLE001 (reported by rank 0)
                st = {"batches": 0, "docs": 0, "error": f"{type(e).__name__}: {e}"}
        rdv.publish_stats(st)
        return {}
    with G.ConsumerGroup(sc, model.postprocess_numpy, args.kafka_group_clients, batch_max=batch,
                         max_latency_ms=5.0, max_bytes=batch * 4096, pool=pool,
                         confluent=(name == "kafka_confluent_group"), rendezvous=rdv) as grp:
        out = runs(args, grp)
        n_scorers = grp.n_scorers
        local = grp.local_batches
    peers = rdv.stats() if rdv is not None else []
    out.update({f"{name}_scorer_procs": n_scorers, f"{name}_batches_per_scorer": [local] + [p["batches"] for p in peers]})
    errs = [p["error"] for p in peers if "error" in p]
    if errs:
        out[f"{name}_peer_errors"] = errs
    del sc
    return out


def _group_confluent_runs(args, grp) -> dict:
    from fraud_detection_spark_kafka_llm_amd.stream import group as G

    G.group_throughput_run(grp, 60_000, tag="warm")
    cg0, h0, w0 = G.cgroup_cpu(), G.host_cpu_times(), time.perf_counter()
    # three drains of the same size, the median one reported: a ~1 s drain of Python clients on a
    # shared host moves by +-15 % from run to run (profiles/r6/kafka/NOTES.md)
    tps = sorted((G.group_throughput_run(grp, args.kafka_group_msgs, tag=f"tp{i}") for i in range(3)),
                 key=lambda r: r["dialogues_per_s"])
    tp = tps[1]
    cg1, h1, w1 = G.cgroup_cpu(), G.host_cpu_times(), time.perf_counter()
    host_busy = (h1[0] - h0[0]) / max(h1[1] - h0[1], 1) * (os.cpu_count() or 1)
    lat = G.group_latency_run(grp, args.kafka_group_rate, args.kafka_sec, tag="lat",
                              max_latency_ms=args.kafka_confluent_fill_ms)
    # the config's LLM-explain stub: every 10th classification explained asynchronously in the
    # clients (offline stub backend), its record produced after the classification
    ex = G.group_latency_run(grp, args.kafka_group_rate, args.kafka_sec, tag="lat-explain", explain="async",
                             max_latency_ms=args.kafka_confluent_fill_ms,
                             explain_every=10)
    place = {"kafka_confluent_group_client_dialogues_per_s": [round(v) for v in tp["client_dialogues_per_s"]],
             "kafka_confluent_group_client_cpu_util": tp["client_cpu_util"],
             "kafka_confluent_group_client_cpus": tp["client_cpus"],
             "kafka_confluent_group_client_numa": tp["client_numa"],
             "kafka_confluent_group_pinned": grp.client_cpus is not None,
             "kafka_confluent_group_cgroup_quota_cpus": cg1.get("quota_cpus"),
             "kafka_confluent_group_throttled_ms": round((cg1.get("throttled_usec", 0) - cg0.get("throttled_usec", 0))
                                                         / 1e3, 1),
             "kafka_confluent_group_cgroup_busy_cpus": round((cg1.get("usage_usec", 0) - cg0.get("usage_usec", 0))
                                                             / 1e6 / max(w1 - w0, 1e-9), 2),
             "kafka_confluent_group_host_busy_cpus": round(host_busy, 1),
             "kafka_confluent_group_runs_dialogues_per_s": [round(r["dialogues_per_s"]) for r in tps]}
    return {**place, "kafka_confluent_group_dialogues_per_s": tp["dialogues_per_s"],
            "kafka_confluent_group_clients": args.kafka_group_clients,
            "kafka_confluent_group_msgs": args.kafka_group_msgs,
            "kafka_confluent_group_p50_ms": lat["p50_ms"], "kafka_confluent_group_p95_ms": lat["p95_ms"],
            "kafka_confluent_group_offered_per_s": args.kafka_group_rate,
            "kafka_confluent_group_explain_p50_ms": ex["p50_ms"],
            "kafka_confluent_group_explain_p95_ms": ex["p95_ms"],
            "kafka_confluent_group_explanations": ex["explanations"],
            "kafka_confluent_group_all_committed": bool(
                tp["produced"] == tp["committed"] == args.kafka_group_msgs and
                lat["produced"] == lat["committed"] == lat["sent"] and
                ex["produced"] == ex["committed"] == ex["sent"] and ex["explanations"] > 0)}


def _group_multi_runs(args, grp) -> dict:
    from fraud_detection_spark_kafka_llm_amd.stream import group as G

    G.group_throughput_run(grp, 60_000, tag="mwarm")
    # (a ~0.1 s drain: the median of three, like the confluent group's)
    tps = sorted((G.group_throughput_run(grp, args.kafka_multi_msgs, tag=f"mtp{i}") for i in range(3)),
                 key=lambda r: r["dialogues_per_s"])
    tp = tps[1]
    return {"kafka_multi_gpu_dialogues_per_s": tp["dialogues_per_s"], "kafka_multi_gpu_msgs": args.kafka_multi_msgs,
            "kafka_multi_gpu_runs_dialogues_per_s": [round(r["dialogues_per_s"]) for r in tps],
            "kafka_multi_gpu_clients": args.kafka_group_clients,
            "kafka_multi_gpu_client_batches_per_scorer": tp["scorer_batches"],
            "kafka_multi_gpu_all_committed": bool(tp["produced"] == tp["committed"] == args.kafka_multi_msgs)}


def kafka_phase(args, spec, idf_np, model, dev, rank: int) -> dict:
    """BASELINE config 5 on this rank's GPU against its own in-memory broker (3 partitions)."""
    import gc

    from fraud_detection_spark_kafka_llm_amd.stream import loadgen
    from fraud_detection_spark_kafka_llm_amd.stream.engine import StreamingEngine

    pt, _ = synth.generate(synth.SynthConfig(n=65536, seed=77 + rank), device=dev, start=2 * 10**9)
    pool = loadgen.MessagePool(pt.strings())
    del pt

    def make(batch: int, latency_ms: float):
        def mk(consumers, producer, topic):
            sc = GpuScorer(spec, idf_np, model.scorer(), dev, max_docs=batch, max_bytes=batch * 4096, depth=2)
            return StreamingEngine(sc, model.postprocess_numpy, consumers, producer, topic, batch_max=batch,
                                   max_latency_ms=latency_ms, max_bytes=batch * 4096)
        return mk

    loadgen.throughput_run(make(16384, 5.0), pool, 100_000, url=f"memory://bench-warm-{rank}")   # warmup
    tps = []
    for i in range(3):                   # (a ~0.2 s drain: the median of three)
        gc.collect()
        tps.append(loadgen.throughput_run(make(16384, 5.0), pool, args.kafka_msgs, url=f"memory://bench-tp{i}-{rank}"))
    tps.sort(key=lambda r: r["dialogues_per_s"])
    tp = tps[1]
    gc.collect()
    lat = loadgen.latency_run(make(4096, args.kafka_fill_ms), pool, args.kafka_rate, args.kafka_sec,
                              url=f"memory://bench-lat-{rank}")
    ok = tp["produced"] == args.kafka_msgs and tp["committed"] == args.kafka_msgs and lat["produced"] == lat["sent"]
    conf = {}
    if args.kafka_confluent_msgs > 0:
        # the same engine through clients restricted to the confluent_kafka surface (per-record
        # Message objects on consume, one produce call + delivery callback per record): the path a
        # librdkafka client takes. The in-memory broker's own per-record Python work is inside
        # the timed region, as librdkafka's would be.
        gc.collect()
        ctp = loadgen.throughput_run(make(16384, 5.0), pool, args.kafka_confluent_msgs,
                                     url=f"memory://bench-ctp-{rank}", confluent=True)
        gc.collect()
        clat = loadgen.latency_run(make(4096, args.kafka_confluent_fill_ms), pool, args.kafka_confluent_rate,
                                   args.kafka_sec,
                                   url=f"memory://bench-clat-{rank}", confluent=True)
        ok = ok and ctp["produced"] == ctp["committed"] == args.kafka_confluent_msgs and \
            clat["produced"] == clat["sent"]
        conf = {"kafka_confluent_dialogues_per_s": ctp["dialogues_per_s"],
                "kafka_confluent_msgs": args.kafka_confluent_msgs,
                "kafka_confluent_p50_ms": clat["p50_ms"], "kafka_confluent_p95_ms": clat["p95_ms"],
                "kafka_confluent_offered_per_s": args.kafka_confluent_rate}
    conf.update(group_kafka(args, spec, idf_np, model, dev, pool))
    return {"kafka_dialogues_per_s": tp["dialogues_per_s"], "kafka_msgs": args.kafka_msgs,
            "kafka_runs_dialogues_per_s": [round(r["dialogues_per_s"]) for r in tps],
            "kafka_throughput_sec": tp["sec"], "kafka_p50_ms": lat["p50_ms"], "kafka_p95_ms": lat["p95_ms"],
            "kafka_p99_ms": lat["p99_ms"], "kafka_offered_per_s": args.kafka_rate,
            "kafka_latency_fill_ms": args.kafka_fill_ms, "kafka_confluent_latency_fill_ms": args.kafka_confluent_fill_ms,
            "kafka_latency_msgs": lat["sent"], "kafka_all_delivered_and_committed": bool(ok),
            "kafka_avg_record_bytes": round(pool.avg_bytes, 1), "kafka_api": "columnar (in-memory broker)", **conf}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rows", type=int, default=10_000_000, help="GBDT training rows (total over ranks)")
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--rf-trees", type=int, default=500, help="RandomForest trees (BASELINE config 3; 0: skip)")
    ap.add_argument("--rf-depth", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="dialogues per GPU per streaming step")
    ap.add_argument("--pool", type=int, default=6, help="distinct pinned micro-batches per GPU")
    ap.add_argument("--depth-pipeline", type=int, default=2)
    ap.add_argument("--kafka-msgs", type=int, default=1_000_000, help="records drained in the Kafka throughput run")
    ap.add_argument("--kafka-rate", type=float, default=300_000, help="paced producer rate of the latency run")
    ap.add_argument("--kafka-sec", type=float, default=2.0, help="duration of the latency run")
    ap.add_argument("--kafka-fill-ms", type=float, default=1.0,
                    help="micro-batch fill deadline of the columnar engine's latency run (throughput runs: 5 ms)")
    ap.add_argument("--kafka-confluent-fill-ms", type=float, default=0.5,
                    help="... of the confluent-surface latency runs (one process, the group): per-record client "
                         "work queues behind a longer fill (profiles/r6/kafka/fill_ab.jsonl)")
    ap.add_argument("--kafka-multi-msgs", type=int, default=1_000_000,
                    help="records of the shared 3-partition topic drained by rank 0 over every GPU (0: skip)")
    ap.add_argument("--kafka-confluent-msgs", type=int, default=300_000,
                    help="records drained through the confluent_kafka-surface clients (0: skip)")
    ap.add_argument("--kafka-group-msgs", type=int, default=1_200_000,
                    help="records drained by the confluent-surface consumer group (0: skip)")
    ap.add_argument("--kafka-group-clients", type=int, default=3, help="client processes of the consumer group")
    ap.add_argument("--kafka-group-rate", type=float, default=300_000,
                    help="paced producer rate (whole group) of the consumer-group latency run")
    ap.add_argument("--kafka-confluent-rate", type=float, default=100_000,
                    help="paced producer rate of the confluent-surface latency run")
    ap.add_argument("--phase-timeout", type=float, default=240.0,
                    help="seconds after which the RF / Kafka phase is cut off and the record printed as it stands")
    ap.add_argument("--pg-timeout", type=float, default=360.0,
                    help="process-group timeout of the bench (above --phase-timeout, inside the driver's limit)")
    Config.add_cli_args(ap)          # --gbdt-max-bin, --seed, --config, ... (utils/config.py)
    args = ap.parse_args()
    cfg = Config.from_cli(args)
    run_profiled_if_requested(cfg.profile)    # --profile: re-run under rocprofv3 (GPU untouched so far)

    # gloo: rehearse N ranks on one GPU
    D.init_from_env(os.environ.get("FDX_DIST_BACKEND", "nccl"), timeout_s=args.pg_timeout)
    rank, world = D.rank(), D.world_size()
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    dev = torch.device("cuda", D.local_rank() % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    numa = bind_to_gpu(dev.index)      # pinned rings on the GPU's NUMA node (before any pinned alloc)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=F)

    # ------------------------------------------------------------------ 1. GBDT training
    gparams = GBDTParams(n_estimators=args.trees, max_depth=args.depth, max_bin=cfg.gbdt_max_bin)
    t0 = time.perf_counter()
    warmup_training(dev, spec, gparams, args.rf_depth if args.rf_trees > 0 else 0)
    warm_sec = time.perf_counter() - t0
    lo, hi = D.shard_range(args.rows)
    t0 = time.perf_counter()
    chunks = generate_shard(lo, hi, dev, seed=11, chunk=CHUNK_ROWS)
    text_bytes = sum(int(h.data.numel()) for h, _ in chunks)
    gen_sec = max_over_ranks(time.perf_counter() - t0, dev)
    gen_peak = torch.cuda.max_memory_allocated(dev)
    sync_all(dev)
    # the HBM peak of the timed phase only (the untimed corpus generation runs on the device too)
    torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    # CSR + CSC by feature (docFreq now, the trainer's columns later), the sort overlapped with H2D
    indptr, idx, counts, y, fo = featurize_shard(chunks, dev, spec, order=True)
    df = D.all_reduce_sum(fo.df)
    idf = torch.log((args.rows + 1.0) / (df.double() + 1.0))
    vc = VectorColumn.tfidf(F, indptr, idx, counts, idf, fo)
    t_feat = time.perf_counter() - t0
    res = fit_gbdt(vc, y, gparams, device=dev)
    sync_all(dev)
    train_sec = max_over_ranks(time.perf_counter() - t0, dev)
    feat_sec = max_over_ranks(t_feat, dev)
    model = SparkXGBClassifierModel(res.trees, F, res.base_margin)
    idf_np = idf.cpu().numpy()
    gbdt_peak = torch.cuda.max_memory_allocated(dev)
    shard_rows, shard_nnz = len(vc), vc.nnz
    # HBM sizing rule (utils/memory.py): rows one GPU could train at this corpus' entries per row,
    # against the device's total memory (the bench's own allocations excluded)
    shape = dict(hot_features=res.shape.get("hot", memory.DEFAULT_HOT_FEATURES),
                 groups=res.shape.get("groups", memory.DEFAULT_GROUPS) or memory.DEFAULT_GROUPS,
                 sparse_frac=res.shape.get("sparse_frac", memory.DEFAULT_SPARSE_FRAC),
                 text_bytes_per_row=text_bytes / max(shard_rows, 1), chunk_rows=CHUNK_ROWS)
    modeled = memory.pipeline_bytes(shard_rows, shard_nnz, **shape)
    sizing = {"max_rows_per_gpu": memory.max_rows_per_gpu(
                  shard_nnz / max(shard_rows, 1), budget_bytes=int(torch.cuda.get_device_properties(dev).total_memory * 0.9),
                  **shape),
              "train_model_bytes_per_row": modeled / max(shard_rows, 1),
              "train_peak_bytes_per_row": gbdt_peak / max(shard_rows, 1),
              "train_peak_over_model": gbdt_peak / max(modeled, 1.0)}
    del chunks

    # ------------------------------------------------------------------ 2. streaming inference
    scorer = GpuScorer(spec, idf_np, model.scorer(), dev, max_docs=args.batch, max_bytes=args.batch * 4096,
                       depth=args.depth_pipeline)
    ring = PinnedRing(slots=args.pool, max_docs=args.batch, max_bytes=args.batch * 4096)
    pool_labels = []
    for i, slot in enumerate(ring.slots):
        pt, yb = synth.generate(synth.SynthConfig(n=args.batch, seed=1000 + rank), device=dev,
                                start=10**9 + i * args.batch)
        slot.fill_packed(pt.data.cpu().numpy(), pt.offsets.cpu().numpy())
        pool_labels.append(yb.cpu().numpy())
    avg_bytes = float(np.mean([s.n_bytes / max(s.n_docs, 1) for s in ring.slots]))

    def run(steps: int, check: bool):
        """Every step delivers (prediction, P(scam)) for a micro-batch to the host. Accuracy
        against the synthetic labels is only tallied in the (untimed) warmup pass."""
        correct = total = 0
        sink = 0.0

        def finish():
            nonlocal correct, total, sink
            a = time.perf_counter()
            slot, raw = scorer.collect(copy=False)
            b = time.perf_counter()
            pred, p = model.postprocess_numpy(raw)
            sink += float(p[0])
            if check:
                correct += int((pred == pool_labels[slot.index]).sum())
                total += len(pred)
            timing["collect"] += b - a
            timing["post"] += time.perf_counter() - b

        for i in range(steps):
            if scorer.inflight == scorer.depth:
                finish()
            a = time.perf_counter()
            scorer.submit(ring.slots[i % len(ring.slots)])
            timing["submit"] += time.perf_counter() - a
        while scorer.inflight:
            finish()
        return correct, total

    timing = {"collect": 0.0, "post": 0.0, "submit": 0.0}

    correct, total = run(max(args.warmup, len(ring.slots)), True)
    sync_all(dev)
    timing = {k: 0.0 for k in timing}
    t0 = time.perf_counter()
    run(args.steps, False)
    sync_all(dev)
    if os.environ.get("FDX_BENCH_TIMING") == "1":
        print(json.dumps({"rank": rank, **{k + "_ms_per_step": v / args.steps * 1e3 for k, v in timing.items()}}),
              file=sys.stderr, flush=True)
    dt = max_over_ranks(time.perf_counter() - t0, dev)
    acc = correct / max(total, 1)

    # single-dialogue end-to-end classify latency (unpipelined: H2D + kernel + D2H + postprocess)
    one = PinnedRing(slots=1, max_docs=1, max_bytes=8192)
    lat_scorer = GpuScorer(spec, idf_np, model.scorer(), dev, max_docs=1, max_bytes=8192, depth=1)
    text = ring.slots[0]
    first = bytes(text.data[: int(text.offsets[1])].numpy()).decode()
    one.slots[0].fill([first])
    lats = []
    for _ in range(60):
        t1 = time.perf_counter()
        raw = lat_scorer.score_packed(one.slots[0])
        model.postprocess_numpy(raw)
        lats.append((time.perf_counter() - t1) * 1e3)
    p50 = float(np.percentile(lats[10:], 50))
    del scorer, lat_scorer

    # the headline record is complete here: the phases below only add to it, each one isolated
    # (an error lands in the record as <phase>_error; a phase that hangs past --phase-timeout is
    # cut off by the watchdog, which prints the record as it stands)
    gbdt_peak_gb = max_over_ranks(gbdt_peak / 2 ** 30, dev)
    gen_peak_gb = max_over_ranks(gen_peak / 2 ** 30, dev)
    docs = args.steps * args.batch * world
    record = {
        "metric": METRIC,
        "value": docs / dt,
        "unit": "dialogues/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        "config": {"model": f"HashingTF(2^18)->IDF->GBDT({args.trees} trees, depth {args.depth})",
                   "global_batch": args.batch * world, "seq_len": round(avg_bytes),
                   "parallelism": f"dp{world}"},
        "gbdt_train_sec": train_sec,
        "gbdt_train_rows": args.rows,
        "gbdt_featurize_sec": feat_sec,
        "gbdt_datagen_sec_untimed": gen_sec,
        "gbdt_warmup_sec_untimed": warm_sec,
        "gbdt_nodes_tree0": res.trees[0].num_nodes,
        "gbdt_peak_hbm_gb": gbdt_peak_gb,
        "datagen_peak_hbm_gb_untimed": gen_peak_gb,
        **sizing,
        "stream_accuracy": acc,
        "p50_single_dialogue_ms": p50,
        "numa_bind_rank0": numa,
    }
    guard = PhaseGuard(record, rank, args.phase_timeout)

    if args.rf_trees > 0:
        # ------------------------------------------------------------------ 3. RandomForest
        def rf_phase():
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(dev)
            sync_all(dev)
            t0 = time.perf_counter()
            bench_fault("rf")
            forest = fit_forest(vc, y, num_trees=args.rf_trees, max_depth=args.rf_depth, max_bins=32, bootstrap=True,
                                feature_subset="sqrt", seed=42, device=dev)
            sync_all(dev)
            return {"rf_train_sec": max_over_ranks(time.perf_counter() - t0, dev), "rf_trees": len(forest.trees),
                    "rf_depth": args.rf_depth, "rf_nodes_tree0": int(forest.trees[0].num_nodes),
                    "rf_peak_hbm_gb": max_over_ranks(torch.cuda.max_memory_allocated(dev) / 2 ** 30, dev)}

        guard.run("rf", rf_phase, dev)
    del vc, indptr, idx, counts, y, fo
    torch.cuda.empty_cache()

    if args.kafka_msgs > 0:
        # ------------------------------------------------------------------ 4. Kafka end to end
        def kafka_run():
            kafka = kafka_phase(args, spec, idf_np, model, dev, rank)
            # every rank drains its own broker with one GPU: reported per GPU (rank 0's engine), not
            # summed -- the shared-topic -> N-GPU topology is kafka_multi_gpu_dialogues_per_s
            for k in ("kafka_p50_ms", "kafka_p95_ms", "kafka_p99_ms", "kafka_confluent_p50_ms",
                      "kafka_confluent_p95_ms"):
                if k in kafka:
                    kafka[k] = max_over_ranks(kafka[k], dev)
            return kafka

        guard.run("kafka", kafka_run, dev)
    if rank == 0:
        print(json.dumps(record), flush=True)
    try:
        D.barrier()
        if D.is_dist():
            torch.distributed.destroy_process_group()
    except Exception:                      # noqa: BLE001 (the record is out; a failed phase may leave the group broken)
        traceback.print_exc()


if __name__ == "__main__":
    main()
