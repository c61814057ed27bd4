"""Shape of the 10M-row GBDT training matrix (feature density, bins, work items) on one GPU.

Prints one JSON line: nnz, active features, total bins, entries by feature-density class,
bins histogram, and work items per tile group (row-blocked vs whole-column) for the current
quantizer settings. Used to size the histogram engine.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

import numpy as np
import torch

from gbdt_train import build_features  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--max-bins", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    indptr, idx, counts, y, _, _ = build_features(args.rows, dev)
    F = 1 << 18
    fo = feature_order(indptr, idx, counts, F)
    idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(F, indptr, idx, counts, idf, fo)
    Q = quantize(vc, max_bins=args.max_bins, counts=counts, scale=idf)
    colptr = Q.colptr.cpu().numpy()
    n = np.diff(colptr)
    dens = n / args.rows
    nb = Q.nbins.cpu().numpy()
    out = {"rows": args.rows, "nnz": int(colptr[-1]), "Fa": int(Q.Fa), "TB": int(Q.TB)}
    edges = [0, 1e-4, 1e-3, 1e-2, 0.05, 0.1, 0.25, 0.5, 1.01]
    cls = []
    for a, b in zip(edges, edges[1:]):
        sel = (dens >= a) & (dens < b)
        cls.append({"density": [a, b], "features": int(sel.sum()), "entries": int(n[sel].sum()),
                    "bins": int(nb[sel].sum())})
    out["density_classes"] = cls
    out["nbins_hist"] = {str(k): int(v) for k, v in zip(*np.unique(nb, return_counts=True))}
    grp = []
    for g in Q.groups:
        st, en = g.item_start.cpu().numpy(), g.item_end.cpu().numpy()
        blk = g.item_blk.cpu().numpy()
        ln = en - st
        grp.append({"bt": g.bt, "items": int(g.num_items), "blocked_items": int((blk >= 0).sum()),
                    "blocked_entries": int(ln[blk >= 0].sum()), "whole_items": int((blk < 0).sum()),
                    "whole_entries": int(ln[blk < 0].sum()),
                    "items_lt_256": int((ln < 256).sum()), "items_lt_2048": int((ln < 2048).sum()),
                    "entries_in_items_lt_2048": int(ln[ln < 2048].sum())})
    out["groups"] = grp
    # entries per row (nnz per dialogue)
    rl = (indptr[1:] - indptr[:-1]).cpu().numpy()
    out["nnz_per_row"] = {"mean": float(rl.mean()), "p50": float(np.median(rl)), "max": int(rl.max())}
    top = np.argsort(-n)[:200]
    out["top200_entries"] = int(n[top].sum())
    out["top128_entries"] = int(n[top[:128]].sum())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
