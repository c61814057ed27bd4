"""LDS-instruction model of the row-group histogram pass (csrc/row_kernels.hip rg_hist_kernel) on
the real 10M-row layout, per group and per listed-row fraction, for the kernel's row-major modes
and the alternatives considered for VERDICT r5 #6 (the late rounds' listed multi-slot levels):

  dense  (rg_batch, gmode 1): per 64 listed rows, 16 x ceil(aligned 8-entry blocks / 64)
  sparse (rg_range_sparse):   per 64 listed rows, 16 x the longest row's aligned blocks
  entry  (entry-granular):    per 64 listed rows, 2 x ceil(entries / 64)
  em     (entry-major):       2 x ceil(group entries / 64) (all rows scanned; single slot only)

Prints one JSON line per (fraction, group class). Rows of a level are modelled as a uniform
random subset of the rows, in row order (the pass's list is sorted by (slot, row)).

    python bench/probes/rg_lds_model.py --rows 10000000
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

import torch  # noqa: E402

from gbdt_train import build_features  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order  # noqa: E402


def batch_sum(x: torch.Tensor, op: str) -> torch.Tensor:
    """Per 64 consecutive elements: sum or max (zero padded)."""
    n = x.numel()
    pad = (-n) % 64
    if pad:
        x = torch.cat([x, x.new_zeros(pad)])
    x = x.view(-1, 64)
    return x.sum(1) if op == "sum" else x.max(1).values


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--max-bins", type=int, default=64)
    ap.add_argument("--fractions", type=float, nargs="+", default=[1.0, 0.5, 0.3, 0.15, 0.05])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    indptr, idx, counts, y, _, _ = build_features(args.rows, dev)
    F = 1 << 18
    fo = feature_order(indptr, idx, counts, F)
    idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(F, indptr, idx, counts, idf, fo)
    Q = quantize(vc, max_bins=args.max_bins, counts=counts, scale=idf)
    del indptr, idx, counts, vc
    rg = Q.rowgroups()
    N, G = rg.n_rows, rg.G
    gmode = rg.gmode.cpu().tolist()
    print(json.dumps({"rows": N, "groups": G, "entries": rg.entries, "dense_groups": sum(gmode),
                      "group_entries": [int(e) for e in rg.group_entries]}), flush=True)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    for f in args.fractions:
        keep = torch.rand(N, generator=gen, device=dev) < f if f < 1.0 else torch.ones(N, dtype=torch.bool, device=dev)
        R = int(keep.sum())
        tot = {m: {"dense": 0, "sparse": 0} for m in ("row_major", "entry", "em", "entries")}
        for g in range(G):
            ptr = rg.ptr[g].long()
            st, en = ptr[:-1][keep], ptr[1:][keep]
            n = en - st
            blk = torch.where(n > 0, ((en - 1) >> 3) - (st >> 3) + 1, torch.zeros_like(n))
            cls = "dense" if gmode[g] else "sparse"
            if gmode[g]:
                rm = 16 * ((batch_sum(blk, "sum") + 63) // 64)
            else:
                rm = 16 * batch_sum(blk, "max")
            tot["row_major"][cls] += int(rm.sum())
            tot["entry"][cls] += int((2 * ((batch_sum(n, "sum") + 63) // 64)).sum())
            tot["em"][cls] += 2 * ((int(rg.group_entries[g]) + 63) // 64)
            tot["entries"][cls] += int(n.sum())
        print(json.dumps({"fraction": f, "listed_rows": R, **tot}), flush=True)


if __name__ == "__main__":
    main()
