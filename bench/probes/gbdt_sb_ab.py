"""In-process A/B of the sparse groups' super-batches per step in the row-list histogram pass
(csrc/row_kernels.hip rg_range_sparse; tree_set_rg_sb): 3 spills 48 B per lane of
rg_hist_kernel<8192>, 2 does not. The fits alternate on the same matrix; same trees required.
Usage: ROWS=10000000 python bench/probes/gbdt_sb_ab.py [REPS]
It ran against a build with both variants and a tree_set_rg_sb hook; 2 won and is now the only
variant (profiles/r6/gbdt_late/NOTES.md §14), so the script is kept as the record of the A/B."""
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
    default = C.tree_set_rg_sb(3)
    times = {3: [], 2: []}
    trees = {}
    fit_gbdt(vc, y, p, device=dev)                    # (warm)
    for _ in range(reps):
        for sb in times:
            C.tree_set_rg_sb(sb)
            fit_gbdt(vc, y, p, device=dev) if not trees.get(sb) else None
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fit_gbdt(vc, y, p, device=dev)
            torch.cuda.synchronize()
            times[sb].append(time.perf_counter() - t0)
            trees[sb] = [(t.feature.tolist(), t.threshold.tolist()) for t in r.trees]
    C.tree_set_rg_sb(default)
    for sb in times:
        print(f"super-batches {sb}: " + " ".join(f"{t:.4f}" for t in times[sb]) +
              f"  median {statistics.median(times[sb]):.4f} s", flush=True)
    print("same trees:", trees[3] == trees[2], flush=True)


if __name__ == "__main__":
    main()
