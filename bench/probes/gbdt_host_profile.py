"""Host-side profile of a GBDT fit at BASELINE config 2 (1M rows, depth 6): one warm fit, one timed
fit, then one fit under cProfile (top entries by own time and by cumulative time). Shows how much of
a ~1.2 ms boosting round the Python level loop and the per-tree table build take on the host."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    rows = int(os.environ.get("ROWS", 1_000_000))
    trees = int(os.environ.get("TREES", 100))
    warm_tree_kernels(dev)
    vc, y, _ = _tfidf(rows, dev, seed=11, times={})
    torch.cuda.synchronize()
    p = GBDTParams(n_estimators=trees, max_depth=6)
    for rep in range(2):
        t0 = time.perf_counter()
        fit_gbdt(vc, y, p, device=dev)
        torch.cuda.synchronize()
        print(f"fit {rep}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    fit_gbdt(vc, y, p, device=dev)
    torch.cuda.synchronize()
    pr.disable()
    print(f"fit under cProfile: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    for key in ("tottime", "cumulative"):
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats(key).print_stats(30)
        print(out.getvalue(), flush=True)


if __name__ == "__main__":
    main()
