"""A/B of RandomForest engine switches on one feature set (BASELINE config 3 shape): the forest is
fitted under each variant in turn, ``--reps`` rounds (interleaved, so drift hits every variant
alike), and the median / min train seconds per variant are printed as one JSON line each.

    python bench/probes/rf_variants.py --rows 10000000 --variants base,nopresel,nofuse --reps 3

A variant is a comma-free name bound to module switches in VARIANTS below.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from suite import _tfidf
from fraud_detection_spark_kafka_llm_amd.models import forest_batch, grower
from fraud_detection_spark_kafka_llm_amd.models import quantize as qmod
from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels

VARIANTS = {
    "base": {},
    "nopresel": {(grower, "PRESELECT"): False},
    "nofuse": {(grower, "FUSED_PACK"): False},
    "r4": {(grower, "PRESELECT"): False, (grower, "FUSED_PACK"): False},
    "lanes8": {(forest_batch, "TREES_IN_FLIGHT"): 8},
    "lanes24": {(forest_batch, "TREES_IN_FLIGHT"): 24},
    "lanes12": {(forest_batch, "TREES_IN_FLIGHT"): 12},
    "lanes6": {(forest_batch, "TREES_IN_FLIGHT"): 6},
    "l24g3": {(forest_batch, "TREES_IN_FLIGHT"): 24, (forest_batch, "LANE_GROUPS"): 3},
    "lanes32": {(forest_batch, "TREES_IN_FLIGHT"): 32},
    "l32g2": {(forest_batch, "TREES_IN_FLIGHT"): 32, (forest_batch, "LANE_GROUPS"): 2},
    "l32g4": {(forest_batch, "TREES_IN_FLIGHT"): 32, (forest_batch, "LANE_GROUPS"): 4},
    "g1": {(forest_batch, "LANE_GROUPS"): 1},
    "nonative": {(grower, "NATIVE_LEVELS"): False},
    "nolean": {(grower, "LEAN_RF"): False},
    "presel_all": {(grower, "PRESELECT_MIN_ROWS"): 0},
    "presel_4m": {(grower, "PRESELECT_MIN_ROWS"): 4_000_000},
    "chunk2k": {(qmod, "CHUNK"): 2048},
    "chunk4k": {(qmod, "CHUNK"): 4096},
    "chunk8k": {(qmod, "CHUNK"): 8192},
    "chunk16k": {(qmod, "CHUNK"): 16384},
    "mfma": {(grower, "RF_LDS"): False},
    "nonative_nopresel": {(grower, "NATIVE_LEVELS"): False, (grower, "PRESELECT"): False},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--trees", type=int, default=500)
    ap.add_argument("--variants", default="base,r4")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--forced", action="store_true",
                    help="the data-parallel level path at world 1 over RCCL (forced collectives, compact levels)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.forced:
        from fraud_detection_spark_kafka_llm_amd.parallel import dist as D

        os.environ["FDX_FORCE_COLLECTIVES"] = "1"
        grower.RF_COMPACT = "1"
        D.init_from_env("nccl")
    warm_tree_kernels(dev, gbdt_depth=0, forest_depth=5, forest_subset="sqrt")
    vc, y, _ = _tfidf(args.rows, dev, seed=21)
    torch.cuda.synchronize()
    names = args.variants.split(",")
    times = {n: [] for n in names}
    ref = None
    for _ in range(args.reps):
        for n in names:
            saved = {k: getattr(*k) for k in VARIANTS[n]}
            for (mod, attr), v in VARIANTS[n].items():
                setattr(mod, attr, v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = fit_forest(vc, y, num_trees=args.trees, max_depth=5, max_bins=32, bootstrap=True,
                             feature_subset="sqrt", seed=42, device=dev)
            torch.cuda.synchronize()
            times[n].append(time.perf_counter() - t0)
            for (mod, attr), v in saved.items():
                setattr(mod, attr, v)
            sig = [t.feature.tolist() for t in res.trees[:20]]
            assert ref is None or sig == ref, f"variant {n} changed the forest"
            ref = sig
    for n in names:
        print(json.dumps({"variant": n, "forced": args.forced, "rows": args.rows, "trees": args.trees, "median_s": statistics.median(times[n]),
                          "min_s": min(times[n]), "all_s": [round(t, 4) for t in times[n]]}), flush=True)


if __name__ == "__main__":
    main()
