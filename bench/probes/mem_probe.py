"""Per-stage HBM of bench.py's GBDT phase (VERDICT r3 missing #4: an honest sizing model).

Runs the bench's stages one by one on a --rows shard and records, per stage, the bytes allocated
before it, its peak (caching-allocator peak reset at the stage start) and what stays allocated
after it, next to utils/memory.py's model of the same stage. One JSON line per stage.
python bench/probes/mem_probe.py [--rows 10000000] [--trees 100]
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
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.tree import prepare  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops import text as T  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.utils import memory  # noqa: E402

GB = 2 ** 30


class Stage:
    def __init__(self, name, rows):
        self.name, self.rows = name, rows

    def __enter__(self):
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        self.before = torch.cuda.memory_allocated()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        torch.cuda.synchronize()
        peak, after = torch.cuda.max_memory_allocated(), torch.cuda.memory_allocated()
        rec = {"stage": self.name, "sec": round(time.perf_counter() - self.t0, 3),
               "before_gb": round(self.before / GB, 3), "peak_gb": round(peak / GB, 3),
               "after_gb": round(after / GB, 3), "peak_bytes_per_row": round(peak / self.rows, 1)}
        rec.update(getattr(self, "extra", {}))
        print(json.dumps(rec), flush=True)
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--trees", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=B.F)
    params = GBDTParams(n_estimators=a.trees, max_depth=6)
    B.warmup_training(dev, spec, params, 0)
    chunks = B.generate_shard(0, a.rows, dev, seed=11)
    torch.cuda.empty_cache()
    n = a.rows
    with Stage("featurize+order", n) as st:
        indptr, idx, counts, y, fo = B.featurize_shard(chunks, dev, spec, order=True)
        st.extra = {"nnz": int(idx.numel()), "nnz_per_row": round(idx.numel() / n, 2),
                    "idx_dtype": str(idx.dtype), "counts_dtype": str(counts.dtype)}
    nnz = int(idx.numel())
    text_bytes = sum(int(h.data.numel()) for h, _ in chunks)
    with Stage("idf+tfidf", n) as st:
        idf = torch.log((n + 1.0) / (fo.df.double() + 1.0))
        vc = VectorColumn.tfidf(B.F, indptr, idx, counts, idf, fo)
    with Stage("prepare(quantize)", n) as st:
        Q, yy, F, _ = prepare(vc, y, dev, params.max_bin)
    with Stage("rowgroups", n) as st:
        rg = Q.rowgroups()
        st.extra = {"groups": rg.G, "rg_gb": round(rg.nbytes / GB, 3),
                    "hot": int(Q.hot.size) if Q.hot is not None else 0}
    del Q, rg, yy
    torch.cuda.empty_cache()
    with Stage("fit_gbdt", n) as st:
        res = fit_gbdt(vc, y, params, device=dev)
        st.extra = {"trees": len(res.trees)}
    shape = dict(hot_features=res.shape["hot"], groups=res.shape["groups"] or memory.DEFAULT_GROUPS)
    print(json.dumps({"model_featurize_gb": round(memory.featurize_bytes(n, nnz, text_bytes / n) / GB, 3),
                      "model_training_gb": round(memory.training_bytes(n, nnz, **shape) / GB, 3), **shape,
                      "max_memory_reserved_gb": round(torch.cuda.max_memory_reserved() / GB, 3)}), flush=True)


if __name__ == "__main__":
    main()
