"""Streaming-path breakdown on one GPU: pinned H2D bandwidth, kernel time, pipelined step time.

Prints one JSON line per configuration so copy/compute overlap can be diagnosed.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from fraud_detection_spark_kafka_llm_amd.data import synth
from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH
from fraud_detection_spark_kafka_llm_amd.ops import text as T
from fraud_detection_spark_kafka_llm_amd.stream.gpu_worker import GpuScorer
from fraud_detection_spark_kafka_llm_amd.stream.ring import PinnedRing


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B = args.batch
    F = 1 << 18
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=F)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    from test_text_featurizer import random_forest_arrays

    trees = random_forest_arrays(100, F, 6, 1, seed=1)
    idf = np.random.default_rng(0).random(F)
    ring = PinnedRing(slots=4, max_docs=B, max_bytes=B * 4096)
    for i, s in enumerate(ring.slots):
        pt, _ = synth.generate(synth.SynthConfig(n=B, seed=3), device=dev, start=i * B)
        s.fill_packed(pt.data.cpu().numpy(), pt.offsets.cpu().numpy())
    nb = ring.slots[0].n_bytes
    # (a) raw pinned H2D
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(20):
        d.copy_(ring.slots[i % 4].data[:nb], non_blocking=True)
    torch.cuda.synchronize()
    h2d = (time.perf_counter() - t0) / 20
    print(json.dumps({"what": "h2d", "bytes": nb, "ms": h2d * 1e3, "GBps": nb / h2d / 1e9}), flush=True)
    for depth in (1, 2, 3):
        sc = GpuScorer(spec, idf, trees, dev, max_docs=B, max_bytes=B * 4096, depth=depth)
        for i in range(4):
            sc.submit(ring.slots[i % 4])
            if sc.inflight == depth:
                sc.collect()
        while sc.inflight:
            sc.collect()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            if sc.inflight == depth:
                sc.collect()
            sc.submit(ring.slots[i % 4])
        while sc.inflight:
            sc.collect()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        print(json.dumps({"what": "pipeline", "depth": depth, "ms_per_step": dt * 1e3, "docs_per_s": B / dt}),
              flush=True)
    # (b2) pipeline with host postprocess + per-phase host timing
    for depth in (2, 3):
        sc = GpuScorer(spec, idf, trees, dev, max_docs=B, max_bytes=B * 4096, depth=depth)
        ts = {"submit": 0.0, "collect_wait": 0.0, "post": 0.0}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            if sc.inflight == depth:
                a = time.perf_counter()
                _, raw = sc.collect(copy=False)
                b = time.perf_counter()
                m = raw[:, 0]
                p = np.reciprocal(np.exp(-m) + 1.0)
                c = time.perf_counter()
                ts["collect_wait"] += b - a
                ts["post"] += c - b
            a = time.perf_counter()
            sc.submit(ring.slots[i % 4])
            ts["submit"] += time.perf_counter() - a
        while sc.inflight:
            sc.collect(copy=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        print(json.dumps({"what": "pipeline+post", "depth": depth, "ms_per_step": dt * 1e3,
                          **{k + "_ms": v / args.steps * 1e3 for k, v in ts.items()}}), flush=True)
    # (c) kernel only (text resident)
    pt = T.PackedText(ring.slots[0].data[: nb + 16].to(dev), ring.slots[0].offsets[: B + 1].to(dev))
    for _ in range(3):
        T.featurize_score(pt, spec, idf=torch.from_numpy(idf), trees=trees, device=dev, fix_fallbacks=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        T.featurize_score(pt, spec, idf=torch.from_numpy(idf), trees=trees, device=dev, fix_fallbacks=False)
    torch.cuda.synchronize()
    k = (time.perf_counter() - t0) / 20
    print(json.dumps({"what": "kernel", "ms": k * 1e3, "docs_per_s": B / k}), flush=True)


if __name__ == "__main__":
    main()
