"""In-process A/B of a grower switch on BASELINE config 2's GBDT fit (1M rows, 100 trees x depth 6):
the fits alternate between the settings REPS times on the same matrix, so process-to-process noise
drops out. Usage: python bench/probes/gbdt_ab.py FLAG [REPS]   (FLAG: a models.grower attribute,
e.g. GBDT_CXX_LEVELS; prints fit seconds per setting and the medians)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models import grower  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402


def main():
    flag = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda:0")
    warm_tree_kernels(dev)
    vc, y, _ = _tfidf(int(os.environ.get("ROWS", 1_000_000)), dev, seed=11, times={})
    torch.cuda.synchronize()
    p = GBDTParams(n_estimators=100, max_depth=6)
    fit_gbdt(vc, y, p, device=dev)                    # (warm: workspace shapes, allocator)
    times = {True: [], False: []}
    trees = {}
    for _ in range(reps):
        for v in (True, False):
            setattr(grower, flag, v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fit_gbdt(vc, y, p, device=dev)
            torch.cuda.synchronize()
            times[v].append(time.perf_counter() - t0)
            trees[v] = [(t.feature.tolist(), t.threshold.tolist()) for t in r.trees]
    for v in (True, False):
        print(f"{flag}={int(v)}: " + " ".join(f"{t:.4f}" for t in times[v]) +
              f"  median {statistics.median(times[v]):.4f} s", flush=True)
    print("same trees:", trees[True] == trees[False], flush=True)


if __name__ == "__main__":
    main()
