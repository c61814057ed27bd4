"""Where the cold featurize pass of bench.py loses its time.

bench.py's timed GBDT phase starts with ``featurize_shard(order=True)`` over 20 pinned chunks.
The first such pass in a process took 0.71 s against 0.38 s for a second one over the same
chunks (profiles/r3s4/featurize_cold_vs_warm_final.jsonl). This probe separates the candidates,
one process per mode (all state is process-wide):

  base    bench's warm-up, then two passes over the same chunks (the r3 reproduction)
  sort    bench's warm-up + a 16K-row pass WITH order=True (sort path + its allocations warm),
          then the two passes
  fresh   as ``sort``, then one pass over the chunks and one over a second, freshly generated
          and pinned copy of them (first DMA of pinned pages vs everything else)

Per pass: wall seconds, caching-allocator device mallocs/frees during the pass (hipMalloc /
hipFree calls), and the reserved bytes. Usage: python bench/probes/cold_probe.py --mode sort
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench as B  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops import text as T  # noqa: E402


def _stats():
    s = torch.cuda.memory_stats()
    return {k: s.get(k, 0) for k in ("num_device_alloc", "num_device_free", "num_alloc_retries")}


def one_pass(tag, chunks, dev, spec):
    torch.cuda.synchronize()
    a = _stats()
    t0 = time.perf_counter()
    out = B.featurize_shard(chunks, dev, spec, order=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    b = _stats()
    rec = {"pass": tag, "sec": round(dt, 4), **{k: b[k] - a[k] for k in a},
           "reserved_gb": round(torch.cuda.memory_reserved() / 2 ** 30, 2),
           "allocated_gb": round(torch.cuda.memory_allocated() / 2 ** 30, 2)}
    print(json.dumps(rec), flush=True)
    del out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--mode", choices=("base", "sort", "fresh"), default="base")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    B.bind_to_gpu(0)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=1 << 18)
    B.warmup_training(dev, spec, GBDTParams(n_estimators=100, max_depth=6), 5)
    if a.mode != "base" and not getattr(B, "WARMS_ORDER", False):
        small = B.generate_shard(0, 1 << 14, dev, seed=5)
        B.featurize_shard(small, dev, spec, order=True)
        del small
    chunks = B.generate_shard(0, a.rows, dev, seed=11)
    print(json.dumps({"mode": a.mode, "rows": a.rows, "bench_warms_order": bool(getattr(B, "WARMS_ORDER", False)),
                      "alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF", ""), **_stats(),
                      "reserved_gb_after_datagen": round(torch.cuda.memory_reserved() / 2 ** 30, 2)}), flush=True)
    one_pass("first", chunks, dev, spec)
    if a.mode == "fresh":
        chunks2 = B.generate_shard(0, a.rows, dev, seed=11)
        one_pass("fresh_chunks", chunks2, dev, spec)
        one_pass("fresh_chunks_again", chunks2, dev, spec)
    else:
        one_pass("second", chunks, dev, spec)


if __name__ == "__main__":
    main()
