"""Micro-benchmark of the fused featurize+score kernel on one GPU.

Measures (a) device-resident throughput (text already in HBM) and (b) the streaming path
(pinned host text -> H2D -> kernel -> D2H scores), in dialogues/s and text GB/s.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--scorer", default="lr", choices=["none", "lr", "trees"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    pt, y = synth.generate(synth.SynthConfig(n=args.docs, seed=5), device=dev)
    F = 1 << 18
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=F)
    rng = np.random.default_rng(0)
    idf = torch.from_numpy(rng.random(F)).to(dev)
    lr = T.LinearScorer(rng.normal(size=F), -1.0) if args.scorer == "lr" else None
    trees = None
    if args.scorer == "trees":
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
        from test_text_featurizer import random_forest_arrays

        trees = random_forest_arrays(100, F, 6, 1, seed=1)
    for _ in range(3):
        T.featurize_score(pt, spec, idf=idf, lr=lr, trees=trees, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        r = T.featurize_score(pt, spec, idf=idf, lr=lr, trees=trees, device=dev, fix_fallbacks=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    out = {"docs": args.docs, "bytes_per_doc": pt.nbytes / args.docs, "scorer": args.scorer,
           "device_ms": dt * 1e3, "device_docs_per_s": args.docs / dt, "device_text_GBps": pt.nbytes / dt / 1e9}
    # streaming path: pinned host -> device -> score -> host
    host = pt.to("cpu")
    host = T.PackedText(host.data.pin_memory(), host.offsets.pin_memory())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        r = T.featurize_score(host, spec, idf=idf, lr=lr, trees=trees, device=dev, fix_fallbacks=False)
        s = r.raw.to("cpu")
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    out.update({"stream_ms": dt * 1e3, "stream_docs_per_s": args.docs / dt})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
