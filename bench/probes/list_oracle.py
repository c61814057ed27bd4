"""How many rows the listed row-group levels hold vs the fewest possible (the plan builds the
smaller-HESSIAN sibling; a fewest-rows rule would list min(rows) per sibling pair). GBDT 100 trees
x depth 6 on the bench corpus (ROWS, default 1M), generic level loop with FDX_LIST_ORACLE=1.
Prints the listed / fewest-possible rows per block of 20 rounds."""
import os
import sys

os.environ["FDX_LIST_ORACLE"] = "1"
os.environ["FDX_GBDT_CXX_LEVELS"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models import grower  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    rows = int(os.environ.get("ROWS", 1_000_000))
    vc, y, _ = _tfidf(rows, dev, seed=11, times={})
    fit_gbdt(vc, y, GBDTParams(n_estimators=100, max_depth=6), device=dev)
    log = grower.LIST_ORACLE_LOG
    print(f"rows {rows}, listed levels {len(log)}", flush=True)
    for b in range(0, 100, 20):
        sel = [r for r in log if b <= r[0] < b + 20]
        T = sum(r[2] for r in sel)
        m = sum(r[3] for r in sel)
        print(f"rounds {b:3d}-{b + 19:3d}: listed {T / 1e6:8.2f} M rows, fewest possible {m / 1e6:8.2f} M "
              f"({100.0 * (T - m) / max(T, 1):5.1f} % more)", flush=True)
    for d in range(1, 6):
        sel = [r for r in log if r[1] == d and r[0] >= 50]
        T = sum(r[2] for r in sel)
        m = sum(r[3] for r in sel)
        print(f"depth {d} (rounds 50-99): listed {T / 1e6:8.2f} M, fewest {m / 1e6:8.2f} M", flush=True)


if __name__ == "__main__":
    main()
