"""Where the host spends a 500-tree forest (BASELINE config 3 shape): the features are built and
the forest warmed first, then ``fit_forest`` alone runs under cProfile. Prints the wall time, the
host's top functions by own time, and the share of the wall the host spent blocked on device
events (the forest driver waits for a lane's level counts before it launches the next level).

    python bench/probes/rf_host_probe.py --rows 10000000 --trees 500
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from suite import _tfidf
from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--trees", type=int, default=500)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--forced", action="store_true",
                    help="the data-parallel level path at world 1 over RCCL (FDX_FORCE_COLLECTIVES, compact levels)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.forced:
        os.environ["FDX_FORCE_COLLECTIVES"] = "1"
        os.environ["FDX_RF_COMPACT"] = "1"
        from fraud_detection_spark_kafka_llm_amd.models import grower
        from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

        grower.RF_COMPACT = "1"
        D.init_from_env("nccl")
    warm_tree_kernels(dev, gbdt_depth=0, forest_depth=5, forest_subset="sqrt")
    vc, y, _ = _tfidf(args.rows, dev, seed=21)
    torch.cuda.synchronize()

    def run():
        return fit_forest(vc, y, num_trees=args.trees, max_depth=5, max_bins=32, bootstrap=True,
                          feature_subset="sqrt", seed=42, device=dev)

    prof = cProfile.Profile()
    t0 = time.perf_counter()
    prof.enable()
    res = run()
    torch.cuda.synchronize()
    prof.disable()
    wall = time.perf_counter() - t0
    st = pstats.Stats(prof)
    blocked = sum(v[2] for k, v in st.stats.items() if "synchronize" in k[2] or "Event.wait" in k[2]
                  or "_cuda_synchronize" in k[2])
    out = io.StringIO()
    pstats.Stats(prof, stream=out).sort_stats("tottime").print_stats(args.top)
    print(json.dumps({"rows": args.rows, "trees": len(res.trees), "lanes": res.lanes, "wall_s": round(wall, 4),
                      "host_blocked_s": round(blocked, 4)}))
    print(out.getvalue())


if __name__ == "__main__":
    main()
