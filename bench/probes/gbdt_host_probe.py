"""Where the host spends a GBDT fit (BASELINE config 2 shape: 1M rows, 100 trees, depth 6): the
features are built and the kernels warmed first, then ``fit_gbdt`` alone runs under cProfile.
Prints the wall time, the time the host spent blocked on device events (the level loop waits for
each level's counts) and the host's top functions by own time.

    python bench/probes/gbdt_host_probe.py --rows 1000000 --trees 100
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
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--top", type=int, default=35)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    warm_tree_kernels(dev)
    vc, y, _ = _tfidf(args.rows, dev, seed=11)
    torch.cuda.synchronize()

    def run():
        return fit_gbdt(vc, y, GBDTParams(n_estimators=args.trees, max_depth=6), device=dev)

    run()                               # one untimed fit: the row-group layout's code paths warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    plain = time.perf_counter() - t0
    prof = cProfile.Profile()
    t0 = time.perf_counter()
    prof.enable()
    run()
    torch.cuda.synchronize()
    prof.disable()
    wall = time.perf_counter() - t0
    st = pstats.Stats(prof)
    blocked = sum(v[2] for k, v in st.stats.items() if "synchronize" in k[2] or "Event.wait" in k[2]
                  or "_cuda_synchronize" in k[2] or "tolist" in k[2])
    out = io.StringIO()
    pstats.Stats(prof, stream=out).sort_stats("tottime").print_stats(args.top)
    print(json.dumps({"rows": args.rows, "trees": args.trees, "wall_plain_s": round(plain, 4),
                      "wall_profiled_s": round(wall, 4), "host_blocked_s": round(blocked, 4)}))
    print(out.getvalue())


if __name__ == "__main__":
    main()
