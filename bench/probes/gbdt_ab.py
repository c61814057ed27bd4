"""In-process A/B of a grower switch on BASELINE config 2's GBDT fit (1M rows, 100 trees x depth 6):
the fits alternate between the settings REPS times on the same matrix, so process-to-process noise
drops out. Usage: python bench/probes/gbdt_ab.py FLAG [REPS] [V1,V2]   (FLAG: a models.grower
attribute, e.g. GBDT_CXX_LEVELS, set to True / False or to the integers V1 / V2 (RG_DBG 0,8); ROWS
env: the rows; prints fit seconds per setting and the medians)."""
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


def _val(v: str):
    if v == "None":
        return None
    try:
        return int(v)
    except ValueError:
        return float(v)


def main():
    flag = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    vals = [_val(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [True, False]
    mod = grower
    if "." in flag:                                   # (another models module: quantize.RG_...)
        import importlib
        name, flag = flag.rsplit(".", 1)
        mod = importlib.import_module(f"fraud_detection_spark_kafka_llm_amd.models.{name}")
    dev = torch.device("cuda:0")
    warm_tree_kernels(dev)
    vc, y, _ = _tfidf(int(os.environ.get("ROWS", 1_000_000)), dev, seed=11, times={})
    torch.cuda.synchronize()
    p = GBDTParams(n_estimators=100, max_depth=6)
    fit_gbdt(vc, y, p, device=dev)                    # (warm: workspace shapes, allocator)
    times = {v: [] for v in vals}
    trees = {}
    for _ in range(reps):
        for v in vals:
            setattr(mod, flag, v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fit_gbdt(vc, y, p, device=dev)
            torch.cuda.synchronize()
            times[v].append(time.perf_counter() - t0)
            trees[v] = [(t.feature.tolist(), t.threshold.tolist()) for t in r.trees]
    for v in vals:
        print(f"{flag}={v}: " + " ".join(f"{t:.4f}" for t in times[v]) +
              f"  median {statistics.median(times[v]):.4f} s", flush=True)
    print("same trees:", trees[vals[0]] == trees[vals[1]], flush=True)


if __name__ == "__main__":
    main()
