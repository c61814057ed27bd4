"""RF 500 x depth 5 fitted twice in one process on the same 10M-row TF-IDF matrix (bench/suite.py
rf's data): the second fit runs with the caching allocator warm. The difference per span
(FDX_TRACE spans, synchronised) separates first-touch allocation cost from the work itself.
Prints one JSON line per fit."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.utils import tracing  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    rows = int(os.environ.get("ROWS", 10_000_000))
    trace = os.environ.get("FDX_TRACE")
    warm_tree_kernels(dev, gbdt_depth=0, forest_depth=5, forest_subset="sqrt")
    vc, y, _ = _tfidf(rows, dev, seed=21, times={})
    torch.cuda.synchronize()
    for rep in range(2):
        n0 = sum(1 for _ in open(trace)) if trace and os.path.exists(trace) else 0
        t0 = time.perf_counter()
        with tracing.span("fit", rep=rep):
            res = fit_forest(vc, y, num_trees=500, max_depth=5, max_bins=32, bootstrap=True, feature_subset="sqrt",
                             seed=42, device=dev)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        spans = {}
        if trace:
            with open(trace) as fh:
                for i, line in enumerate(fh):
                    if i < n0:
                        continue
                    r = json.loads(line)
                    if r["name"].startswith(("q.", "forest.prepare", "forest.lanes", "forest.workspace")):
                        spans[r["name"]] = round(spans.get(r["name"], 0.0) + r["dur_ms"], 2)
        print(json.dumps({"rep": rep, "rows": rows, "fit_s": round(dt, 4), "trees": len(res.trees), "spans_ms": spans}),
              flush=True)
        del res


if __name__ == "__main__":
    main()
