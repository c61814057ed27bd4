"""Work-item statistics of the histogram CSC at a given row count (GPU box): items per group, entry
counts per item, wave slots, hot/dense sizes."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import torch

from gbdt_train import build_features  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
args = ap.parse_args()
dev = torch.device("cuda:0")
indptr, idx, counts, y, _, _ = build_features(args.rows, dev)
F = 1 << 18
fo = feature_order(indptr, idx, counts, F)
idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
vc = VectorColumn.tfidf(F, indptr, idx, counts, idf, fo)
Q = quantize(vc, max_bins=256, counts=counts, scale=idf)
nb = Q.nbins.cpu().numpy()
cnt = np.diff(Q.colptr.cpu().numpy())
print("rows", args.rows, "nnz", int(idx.numel()), "Fa", Q.Fa, "TB", int(Q.boff_host[-1]), "hot", len(Q.hot),
      "hot nnz frac", float(cnt[Q.hot].sum() / cnt.sum()), "super-blocks", Q.n_super)
for name, groups in (("cold", Q.groups), ("hot", Q.hot_groups)):
    for g in groups:
        n = (g.item_end - g.item_start).cpu().numpy()
        nf = ((g.item_meta.cpu().numpy() >> 8) & 0xFF)
        print(f"{name} bt={g.bt} items={g.num_items} entries={int(n.sum())} per-item p10/50/90/max="
              f"{np.percentile(n, [10, 50, 90]).astype(int).tolist()}/{int(n.max())} mean={n.mean():.0f} "
              f"packed={int((nf > 1).sum())} wave_slots={int(g.wave_order().numel())}")
