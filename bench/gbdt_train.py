"""GBDT training benchmark on synthetic dialogues (HashingTF(2^18) -> IDF -> GBDT) on one GPU.

Phases timed separately: corpus generation (on device), fused featurization, IDF fit, quantize
+ CSC build, boosting rounds. Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fraud_detection_spark_kafka_llm_amd.data import synth
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH
from fraud_detection_spark_kafka_llm_amd.models import grower
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
from fraud_detection_spark_kafka_llm_amd.ops import text as T
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order
from fraud_detection_spark_kafka_llm_amd.utils import tracing


def build_features(rows: int, dev, chunk: int = 500_000, num_features: int = 1 << 18, seed: int = 11,
                   first_row: int = 0, tail_words: int = 30000):
    """Synthetic dialogues -> fused featurization, chunk by chunk, into one CSR. Each chunk's
    entries are copied into buffers sized from the first chunk's entries per row (grown if a
    later chunk needs more) and freed at once, so the CSR is never held twice (a final
    concatenation of the chunks doubled the peak: HBM sizing, utils/memory.py)."""
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=num_features)
    indptr = torch.zeros(rows + 1, dtype=torch.int64, device=dev)
    y = torch.empty(rows, dtype=torch.float64, device=dev)
    idx = counts = None
    t_gen = t_feat = 0.0
    off = 0
    for start in range(0, rows, chunk):
        n = min(chunk, rows - start)
        t0 = time.perf_counter()
        pt, yc = synth.generate(synth.SynthConfig(n=n, seed=seed, tail_words=tail_words), device=dev,
                                start=first_row + start)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        res = T.featurize_score(pt, spec, want_csr=True, device=dev)
        ip, ix, v = res.csr()
        del pt, res
        k = int(ip[-1])
        if idx is None:
            cap = int(k / max(n, 1) * rows * 1.05) + k + 1024
            idx = torch.empty(cap, dtype=ix.dtype, device=dev)
            counts = torch.empty(cap, dtype=v.dtype, device=dev)
        if off + k > idx.numel():                 # rare: grow by 25 %
            cap = int((off + k) * 1.25)
            idx = torch.cat([idx[:off], torch.empty(cap - off, dtype=idx.dtype, device=dev)])
            counts = torch.cat([counts[:off], torch.empty(cap - off, dtype=counts.dtype, device=dev)])
        idx[off:off + k] = ix
        counts[off:off + k] = v
        indptr[start + 1:start + n + 1] = ip[1:] + off
        y[start:start + n] = yc
        off += k
        del ip, ix, v, yc
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        t_gen += t1 - t0
        t_feat += t2 - t1
    if idx is None:
        idx = torch.empty(0, dtype=torch.int32, device=dev)
        counts = torch.empty(0, dtype=torch.int32, device=dev)
    # views of the first nnz entries (the slack stays allocated; trimming would copy)
    return indptr, idx[:off], counts[:off], y, t_gen, t_feat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--trace", default="")
    ap.add_argument("--tail-words", type=int, default=30000,
                    help="synthetic long-tail vocabulary (1000000: >200K active features of 2^18)")
    ap.add_argument("--no-warmup", action="store_true", help="skip the untimed warm-up fit (models/warmup.py)")
    ap.add_argument("--rg-dbg", type=int, default=None, help="grower.RG_DBG (csrc/tree.h RgHistArgs::dbg) for A/Bs")
    args = ap.parse_args()
    if args.rg_dbg is not None:
        grower.RG_DBG = args.rg_dbg
    dev = torch.device("cuda:0")
    # CPUs of the GPU's NUMA node, as bench.py does (without it, the first quantize on the box
    # showed a ~0.1 s host stall: profiles/r2s4/NOTES.md)
    from fraud_detection_spark_kafka_llm_amd.parallel.affinity import bind_to_gpu
    bind_to_gpu(dev.index)
    if not args.no_warmup:     # lazily loaded code objects and cold allocators, as in bench.py
        from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels
        warm_tree_kernels(dev, gbdt_depth=args.depth)
    if args.trace:
        tracing.enable(args.trace)
    t0 = time.perf_counter()
    indptr, idx, counts, y, t_gen, t_feat = build_features(args.rows, dev, tail_words=args.tail_words)
    t1 = time.perf_counter()
    F = 1 << 18
    fo = feature_order(indptr, idx, counts, F)
    idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(F, indptr, idx, counts, idf, fo)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    feat_peak = torch.cuda.max_memory_allocated(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    grower.reset_level_stats()
    res = fit_gbdt(vc, y, GBDTParams(n_estimators=args.trees, max_depth=args.depth), device=dev)
    t3 = time.perf_counter()
    ls = grower.LEVEL_STATS
    print(json.dumps({"rows": args.rows, "nnz": int(idx.numel()), "trees": args.trees, "depth": args.depth,
                      "tail_words": args.tail_words, **res.shape,
                      "gen_s": t_gen, "featurize_s": t_feat, "idf_s": t2 - t1, "gbdt_total_s": res.train_seconds,
                      "per_tree_ms": (t3 - t2) / args.trees * 1e3, "wall_s": t3 - t0,
                      "peak_hbm_gb": torch.cuda.max_memory_allocated(dev) / 2 ** 30,
                      "featurize_peak_hbm_gb": feat_peak / 2 ** 30,
                      "built_nodes_per_level": ls["built_nodes"] / max(ls["levels"], 1),
                      "dp_hist_bytes_per_level": ls["hist_bytes"] / max(ls["levels"], 1),
                      "nodes_tree0": res.trees[0].num_nodes}))


if __name__ == "__main__":
    main()
