"""Row-blocked histogram pass probe: the bench corpus (HashingTF(2^18) -> TF-IDF, 10M rows by
default), one root-level (and one 2-slot) launch of tree_hist_blk timed under the diagnostic
modes of FDX_BLK_DBG (csrc/tree.h BlkHistArgs::dbg: 1 = no K-steps, 2 = no step staging, 4 = no
row-state loads) and several workgroup targets, plus the shape of the work (groups, bands, chunk
visits, entries per segment). Prints JSON lines.

    python bench/probes/blk_probe.py --rows 10000000
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from gbdt_train import build_features
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.models import quantize as qmod
from fraud_detection_spark_kafka_llm_amd.models.grower import Workspace
from fraud_detection_spark_kafka_llm_amd.ops import native
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--wgs", default="768,1536,3072")
    ap.add_argument("--modes", default="0,1,2,3,4,7")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    C = native.lib()
    ip, ix, cn, y, _, _ = build_features(args.rows, dev)
    F = 1 << 18
    fo = feature_order(ip, ix, cn, F)
    idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(F, ip, ix, cn, idf, fo)
    Q = qmod.quantize(vc, max_bins=32, counts=vc.tf_counts, scale=vc.tf_scale)
    n = Q.n_rows
    ws = Workspace(Q)
    g = torch.linspace(-1, 1, n, device=dev, dtype=torch.float32)
    h = torch.linspace(0.01, 0.25, n, device=dev, dtype=torch.float32)
    C.tree_quant_max(g, h, None, None, 0, 0, False, 0, n, ws.maxabs, 0)
    C.tree_quant(g, h, None, None, 0, 0, False, 0, 4, ws.maxabs, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)
    t0 = time.perf_counter()
    blk = Q.blocked()
    torch.cuda.synchronize()
    build_ms = (time.perf_counter() - t0) * 1e3
    sc = blk.seg_counts
    w = np.sort(sc.sum(0))[::-1]
    nz = sc[sc > 0]
    shape = {"rows": n, "nnz": blk.nnz, "Fa": Q.Fa, "TB": Q.TB, "NG": blk.NG, "n_chunks": blk.n_chunks,
             "build_ms": build_ms, "nonempty_segments": int(nz.size), "mean_seg": float(nz.mean()),
             "median_seg": float(np.median(nz)),
             "entries_top_56_groups": float(w[:56].sum() / w.sum()),
             "entries_top_448_groups": float(w[:448].sum() / w.sum()),
             "groups_per_chunk_ge_64": int((w / blk.n_chunks >= 64).sum()),
             "groups_per_chunk_ge_8": int((w / blk.n_chunks >= 8).sum())}
    print(json.dumps(shape), flush=True)
    nslots_cases = [(1, True), (2, False)]
    node_slot = torch.full((4,), -1, dtype=torch.int32)
    node_slot[:2] = torch.arange(2, dtype=torch.int32)
    row_node = torch.from_numpy((np.arange(n) % 2).astype(np.int32)).to(dev)
    C.tree_slot8(row_node, node_slot.to(dev), 0, 2, ws.slot8, None, None)
    for target in [int(x) for x in args.wgs.split(",")]:
        for nslots, root in nslots_cases:
            ct = 1
            gw = int(C.tree_blk_gw(ct))
            plan = blk.plan(gw, target_wgs=target)
            c0 = plan[1].cpu().numpy()
            c1 = plan[2].cpu().numpy()
            s2n = torch.arange(nslots, dtype=torch.int32, device=dev)
            hist = torch.zeros((nslots, Q.TB, 2), dtype=torch.int64, device=dev)
            for mode in [int(x) for x in args.modes.split(",")]:
                os.environ["FDX_BLK_DBG"] = str(mode)

                def run():
                    hist.zero_()
                    C.tree_hist_blk(blk.ent_row, blk.ent_key, blk.seg, blk.NG, ws.rowdig,
                                    None if root else ws.slot8, *plan, gw, s2n, hist, Q.TB, ct, None, 0)
                ms = timed(run)
                print(json.dumps({"target_wgs": target, "n_wg": int(c0.size), "visits": int((c1 - c0).sum()),
                                  "root": root, "dbg": mode, "ms": round(ms, 3)}), flush=True)
    os.environ.pop("FDX_BLK_DBG", None)


if __name__ == "__main__":
    main()
