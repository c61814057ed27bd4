"""Row-group histogram engine probe: the bench corpus (HashingTF(2^18) -> TF-IDF, 10M rows by
default), the RowGroups build (time, groups, bytes), then the root pass and a few multi-slot
passes timed at several workgroup counts, each checked bitwise against the CSC + dense passes.
Prints JSON lines.

    python bench/probes/rg_probe.py --rows 10000000
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


def csc_passes(C, Q, ws, slot8, nslots, hist):
    """The default engine's passes (CSC items + dense hot block) into hist."""
    s2n = torch.arange(nslots, dtype=torch.int32, device=hist.device)
    ct = pass_ct(4, nslots)
    root = slot8 is None
    for grp in Q.groups + ([] if Q.dense is not None else Q.hot_groups):
        C.tree_hist_build(grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(), Q.h_row,
                          Q.h_key, slot8, ws.rowdig, Q.boff, Q.nbins, s2n, hist, Q.TB, grp.bt, ct, 4, None)
    if Q.dense is not None:
        for bt in (1, 2, 4):
            gfid, gden = ws.dense_groups(bt, C.tree_dense_fg(bt, 1 if root else ct))
            if gfid.numel():
                C.tree_hist_dense(Q.dense, ws.digp, ws.rowdig, None if root else ws.slot8_pad, gfid, gden,
                                  Q.boff, Q.nbins, s2n, hist, Q.TB, Q.n_rows, 32768, bt, ct, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--tail-words", type=int, default=30000)
    ap.add_argument("--wgs", default="512,1024,2048")
    ap.add_argument("--slots", default="1,2,8,16")
    ap.add_argument("--dbg", default="0", help="RgHistArgs::dbg modes (bits 1-2 give wrong sums)")
    ap.add_argument("--alphas", default="8")
    ap.add_argument("--bins", default="8192,4096")
    ap.add_argument("--split", action="store_true", help="also time the densest group and the rest apart")
    ap.add_argument("--only", default="", help="group0 / others: time only that part (PMC runs); no equality check")
    ap.add_argument("--modes", default="auto", help="group pass modes: auto (the layout's), 0 (lane per row), 1 (balanced)")
    ap.add_argument("--em", default="1", help="entry-major sparse pass at single-slot levels: 0, 1 or 0,1")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    C = native.lib()
    ip, ix, cn, y, _, _ = build_features(args.rows, dev, tail_words=args.tail_words)
    F = 1 << 18
    fo = feature_order(ip, ix, cn, F)
    idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(F, ip, ix, cn, idf, fo)
    Q = qmod.quantize(vc, max_bins=32, counts=vc.tf_counts, scale=vc.tf_scale)
    del ip, ix, cn, fo, vc
    n = Q.n_rows
    ws = Workspace(Q)
    g = torch.linspace(-1, 1, n, device=dev, dtype=torch.float32)
    h = torch.linspace(0.01, 0.25, n, device=dev, dtype=torch.float32)
    C.tree_quant_max(g, h, None, None, 0, 0, False, 0, n, ws.maxabs, 0)
    C.tree_quant(g, h, None, None, 0, 0, False, 0, 4, ws.maxabs, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)
    rgs = {}
    for B in [int(x) for x in args.bins.split(",")]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rg = rgs[B] = qmod.RowGroups(Q, bins=B)
        torch.cuda.synchronize()
        build_ms = (time.perf_counter() - t0) * 1e3
        ge = rg.group_entries
        print(json.dumps({"rows": n, "nnz": int(Q.csc_row.numel()), "Fa": Q.Fa, "TB": Q.TB, "bins": B, "G": rg.G,
                          "complete": rg.complete, "build_ms": round(build_ms, 1), "build_phases_ms": rg.timing,
                          "rg_bytes": rg.nbytes,
                          "group_entries": [int(x) for x in ge],
                          "entries_per_row_group0": float(ge[0] / n) if ge.size else 0.0}), flush=True)
    zb = None
    if Q.dense is not None:
        zb = torch.from_numpy((Q.boff_host[:-1] + Q.zbin_host)[Q.hot]).to(dev)
    rng = np.random.default_rng(0)
    lst = torch.empty(n, dtype=torch.int32, device=dev)
    start = torch.zeros(66, dtype=torch.int32, device=dev)
    work = torch.zeros(64 * (2 + n // native.lib().tree_rg_list_rows(n) + 1), dtype=torch.int32, device=dev)
    ldig = torch.empty((n, 2), dtype=torch.int32, device=dev)
    for ns_s in args.slots.split(","):
        # "1L": a listed level with one built slot (about half the rows)
        ns, root = int(ns_s.rstrip("L")), ns_s == "1"
        slot8 = None
        if not root:
            # about half the rows built (the smaller siblings), spread over ns slots
            rn = rng.integers(0, 2 * ns, n).astype(np.int32)
            node_slot = torch.full((2 * ns,), -1, dtype=torch.int32)
            node_slot[:ns] = torch.arange(ns, dtype=torch.int32)
            C.tree_slot8(torch.from_numpy(rn).to(dev), node_slot.to(dev), 0, ns, ws.slot8, None, None)
            slot8 = ws.slot8
        ref = torch.zeros((ns, Q.TB, 2), dtype=torch.int64, device=dev)
        csc_ms = timed(lambda: (ref.zero_(), csc_passes(C, Q, ws, slot8, ns, ref)))
        if zb is not None:
            ref[:, zb] = 0
        s2n = torch.arange(ns, dtype=torch.int32, device=dev)
        list_ms = 0.0
        rn_d = ns_d = emdig = None
        if not root:
            rn_d = torch.from_numpy(rn).to(dev)
            ns_d = node_slot.to(dev)
            # one slot: also every row's digit words masked to it (the entry-major listed pass)
            emdig = torch.empty((n, 2), dtype=torch.int32, device=dev) if ns == 1 else None
            list_ms = timed(lambda: C.tree_rg_list(rn_d, ns_d, None, n, ns, work, start, lst, ws.rowdig, ldig,
                                                   emdig))
        for B, wgs, alpha, dbg, mode, em in [(B, int(w), float(al), int(db), md, int(e)) for B in rgs
                                             for w in args.wgs.split(",") for al in args.alphas.split(",")
                                             for db in args.dbg.split(",") for md in args.modes.split(",")
                                             for e in args.em.split(",")]:
            if True:
                rg = rgs[B]
                kw = rg.em_args(emdig) if em else {}
                if kw and emdig is not None:
                    kw["em_min_rows"] = 1
                gm = rg.gmode if mode == "auto" else torch.full_like(rg.gmode, int(mode))
                hist = torch.zeros((ns, Q.TB, 2), dtype=torch.int64, device=dev)
                wt = rg.work(wgs, alpha)
                if args.only:
                    wt = wt[:, (wt[0] == 0) if args.only == "group0" else (wt[0] != 0)].contiguous()

                def run():
                    hist.zero_()
                    C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, ws.rowdig, 4, None if root else lst,
                                   None if root else start, None if root else ldig, ns, gm, wt, s2n, hist, Q.TB,
                                   None, 0, dbg, **kw)
                ms = timed(run)
                if zb is not None:
                    hist[:, zb] = 0
                eq = bool(torch.equal(hist, ref)) if not args.only else None
                print(json.dumps({"slots": ns_s, "em": em, "bins": B, "alpha": alpha, "mode": mode,
                                  "wgs": int(wt.shape[1]), "dbg": dbg,
                                  "rg_ms": round(ms, 3),
                                  "list_ms": round(list_ms, 3), "csc_ms": round(csc_ms, 3), "equal": eq}), flush=True)
                if eq is False and dbg < 2:
                    sys.exit("row-group histograms differ from the CSC passes")
                if args.split:
                    # the densest group alone, the other groups alone (which part bounds the pass)
                    for name, keep in (("group0", wt[0] == 0), ("others", wt[0] != 0)):
                        sub = wt[:, keep].contiguous()

                        def run_sub():
                            hist.zero_()
                            C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, ws.rowdig, 4, None if root else lst,
                                           None if root else start, None if root else ldig, ns, gm, sub, s2n, hist,
                                           Q.TB, None, 0, dbg, **kw)
                        print(json.dumps({"slots": ns_s, "em": em, "bins": B, "alpha": alpha, "mode": mode, "dbg": dbg, "part": name,
                                          "wgs": int(sub.shape[1]), "rg_ms": round(timed(run_sub), 3)}), flush=True)


if __name__ == "__main__":
    main()
