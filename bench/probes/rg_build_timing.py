"""Setup of a GBDT fit on one shard: quantisation (models/tree.prepare) and the row-group layout
build (models/quantize.RowGroups, FDX_RG_TIMING=1: synchronised time per build step), repeated.
Usage: FDX_RG_TIMING=1 ROWS=1250000 python bench/probes/rg_build_timing.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.quantize import RowGroups  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.tree import prepare  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    vc, y, _ = _tfidf(int(os.environ.get("ROWS", 1_250_000)), dev, seed=11, times={})
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Q, _, _, _ = prepare(vc, y, dev, 32)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rg = RowGroups(Q)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"prepare {(t1 - t0) * 1e3:.2f} ms, rowgroups {(t2 - t1) * 1e3:.2f} ms",
              {k: round(v * 1e3, 2) for k, v in rg.timing.items()}, flush=True)


if __name__ == "__main__":
    main()
