"""cProfile of the quantisation (prepare) phase of GBDT at --rows rows on one GPU, after the
untimed warm-up fit (host-side costs of building the histogram layout)."""
import argparse
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gbdt_train import build_features  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
args = ap.parse_args()
dev = torch.device("cuda:0")
warm_tree_kernels(dev)
indptr, idx, counts, y, _, _ = build_features(args.rows, dev)
F = 1 << 18
fo = feature_order(indptr, idx, counts, F)
idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
vc = VectorColumn.tfidf(F, indptr, idx, counts, idf, fo)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
Q = quantize(vc, max_bins=256, counts=counts, scale=idf)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
