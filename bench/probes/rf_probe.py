"""Random-forest histogram pass probe (config 3 shape: sqrt-of-2^18 features sampled per node).

Per level d (2^d open nodes, every one built): the exact k-of-F sample of the level's nodes, the
CSC work items it activates, the entries those items hold against the entries of the sampled
features alone, and the time of the count-histogram passes (np = 1) the level loop launches.
Also the pass with no feature sampled (launch + early-exit cost) and with every feature.

    python bench/probes/rf_probe.py --rows 10000000
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
from fraud_detection_spark_kafka_llm_amd.models.grower import Workspace, pass_ct
from fraud_detection_spark_kafka_llm_amd.ops import native
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order


def timed(fn, reps=5):
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
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--trees", default="0,1,2")
    ap.add_argument("--device", default="cuda:0")
    args = ap.parse_args()
    dev = torch.device(args.device)
    C = native.lib()
    ip, ix, cn, y, _, _ = build_features(args.rows, dev)
    F = 1 << 18
    fo = feature_order(ip, ix, cn, F)
    idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(F, ip, ix, cn, idf, fo)
    Q = qmod.quantize(vc, max_bins=32, counts=vc.tf_counts, scale=vc.tf_scale)
    del ip, ix, cn, fo, vc
    n = Q.n_rows
    ws = Workspace(Q)
    label = y.to(torch.float32) if y.dtype != torch.float32 else y
    C.tree_quant(None, None, label, None, 7, 0, True, 1, 1, None, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)
    groups = Q.groups + Q.hot_groups
    colcnt = np.diff(Q.colptr.cpu().numpy())
    items = []
    for grp in groups:
        st, en = grp.item_start.cpu().numpy(), grp.item_end.cpu().numpy()
        f0, meta = grp.item_f0.cpu().numpy(), grp.item_meta.cpu().numpy()
        items.append((st, en, f0, (meta >> 8) & 0xFF))
    print(json.dumps({"rows": n, "nnz": int(Q.csc_row.numel()), "Fa": Q.Fa, "TB": Q.TB,
                      "groups": [int(g.num_items) for g in groups], "bt": [int(g.bt) for g in groups]}), flush=True)
    rng = np.random.default_rng(0)

    def passes(mask, slot8, ns, hist):
        s2n = torch.arange(ns, dtype=torch.int32, device=dev)
        ct = pass_ct(1, ns)
        for grp in groups:
            if grp.num_items:
                C.tree_hist_build(grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(), Q.h_row,
                                  Q.h_key, slot8, ws.rowdig, Q.boff, Q.nbins, s2n, hist, Q.TB, grp.bt, ct, 1, mask)

    def passes_sampled(mask, pack, ns, hist, listed=True, lds=False):
        s2n = torch.arange(ns, dtype=torch.int32, device=dev)
        ct = pass_ct(1, ns)
        for gi, grp in enumerate(groups):
            if grp.num_items:
                lst, cnt = ws.item_list(gi, grp) if listed else (None, None)
                C.tree_hist_sampled(grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(),
                                    Q.h_row, Q.h_key, pack, ws.rowdig, Q.boff, Q.nbins, s2n, hist, Q.TB, grp.bt, ct,
                                    mask, lst, cnt, lds)

    for tree in [int(t) for t in args.trees.split(",")]:
        for d in range(args.depth):
            ns = 1 << d
            open_d = torch.arange(ns - 1, 2 * ns - 1, dtype=torch.int32, device=dev)
            thr = torch.empty(ns, dtype=torch.float64, device=dev)
            mask = torch.empty(Q.Fa, dtype=torch.uint8, device=dev)
            C.tree_rf_sample(7, tree, open_d, F, args.k, Q.fid_orig, thr, mask, None)
            m = mask.cpu().numpy().astype(bool)
            act_items = act_entries = 0
            for st, en, f0, nf in items:
                act = np.array([m[a:a + b].any() for a, b in zip(f0, nf)], dtype=bool)
                act_items += int(act.sum())
                act_entries += int((en - st)[act].sum())
            slot8 = pack = None
            if d > 0:
                rn = torch.from_numpy(rng.integers(0, ns, n).astype(np.int32)).to(dev)
                node_slot = torch.arange(ns, dtype=torch.int32, device=dev)
                C.tree_slot8(rn, node_slot, 0, ns, ws.slot8, None, None)
                slot8 = ws.slot8
                pack = ws.rowpack()
                C.tree_slot_pack(rn, node_slot, ns, ws.rowdig, pack)
            hist = torch.zeros((ns, Q.TB, 2), dtype=torch.int64, device=dev)
            ms = timed(lambda: (hist.zero_(), passes(mask, slot8, ns, hist)))
            hist2 = torch.zeros_like(hist)
            ms_s = timed(lambda: (hist2.zero_(), passes_sampled(mask, pack, ns, hist2)))
            same = bool(torch.equal(hist, hist2))
            hist3 = torch.zeros_like(hist)
            ms_p = timed(lambda: (hist3.zero_(), passes_sampled(mask, pack, ns, hist3, False)))
            same = same and bool(torch.equal(hist, hist3))
            hist4 = torch.zeros_like(hist)
            ms_l = timed(lambda: (hist4.zero_(), passes_sampled(mask, pack, ns, hist4, False, True)))
            hist5 = torch.zeros_like(hist)
            ms_ll = timed(lambda: (hist5.zero_(), passes_sampled(mask, pack, ns, hist5, True, True)))
            same = same and bool(torch.equal(hist, hist4)) and bool(torch.equal(hist, hist5))
            none = torch.zeros_like(mask)
            ms0 = timed(lambda: passes(none, slot8, ns, hist))
            ms0_s = timed(lambda: passes_sampled(none, pack, ns, hist2))
            ms0_l = timed(lambda: passes_sampled(none, pack, ns, hist4, False, True))
            print(json.dumps({"tree": tree, "depth": d, "slots": ns, "sampled_feats": int(m.sum()),
                              "sampled_entries": int(colcnt[m].sum()), "active_items": act_items,
                              "active_item_entries": act_entries, "items_total": sum(len(i[0]) for i in items),
                              "pass_ms": round(ms, 3), "empty_mask_ms": round(ms0, 3),
                              "sampled_pass_ms": round(ms_s, 3), "sampled_empty_ms": round(ms0_s, 3),
                              "pack_only_ms": round(ms_p, 3), "lds_pass_ms": round(ms_l, 3),
                              "lds_listed_ms": round(ms_ll, 3), "lds_empty_ms": round(ms0_l, 3),
                              "equal": same}), flush=True)
            if not same:
                sys.exit("sampled pass differs from the build pass")
    for ns in (1, 16):
        slot8 = None
        if ns > 1:
            rn = torch.from_numpy(rng.integers(0, ns, n).astype(np.int32)).to(dev)
            C.tree_slot8(rn, torch.arange(ns, dtype=torch.int32, device=dev), 0, ns, ws.slot8, None, None)
            slot8 = ws.slot8
        hist = torch.zeros((ns, Q.TB, 2), dtype=torch.int64, device=dev)
        ms = timed(lambda: passes(None, slot8, ns, hist))
        print(json.dumps({"all_features": True, "slots": ns, "entries": int(Q.csc_row.numel()), "pass_ms": round(ms, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
