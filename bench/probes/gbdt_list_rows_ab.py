"""In-process A/B of the row-list wave size above 4M rows (csrc/tree.h rg_list_rows): 2048-row
waves with a counting list pass (default) against 512-row waves, which let the partition's row pass
write the list counts (partition_counts_ok) so the level's list pass 0 is skipped. The fits
alternate on the same matrix; same trees required.
Usage: ROWS=10000000 python bench/probes/gbdt_list_rows_ab.py [REPS]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops import native  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    C = native.lib()
    dev = torch.device("cuda:0")
    warm_tree_kernels(dev)
    rows = int(os.environ.get("ROWS", 10_000_000))
    vc, y, _ = _tfidf(rows, dev, seed=11, times={})
    p = GBDTParams(n_estimators=100, max_depth=6)
    default = C.tree_set_list_big_rows(4 << 20)
    settings = {"2048-row waves": default, "512-row waves": 1 << 40}
    times = {k: [] for k in settings}
    trees = {}
    fit_gbdt(vc, y, p, device=dev)                    # (warm)
    for _ in range(reps):
        for name, thr in settings.items():
            C.tree_set_list_big_rows(thr)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fit_gbdt(vc, y, p, device=dev)
            torch.cuda.synchronize()
            times[name].append(time.perf_counter() - t0)
            trees[name] = [(t.feature.tolist(), t.threshold.tolist()) for t in r.trees]
    C.tree_set_list_big_rows(default)
    for name in settings:
        print(f"{name}: " + " ".join(f"{t:.4f}" for t in times[name]) +
              f"  median {statistics.median(times[name]):.4f} s", flush=True)
    a, b = trees.values()
    print("same trees:", a == b, "partition counts at 512:", C.tree_partition_counts_ok(rows), flush=True)


if __name__ == "__main__":
    main()
