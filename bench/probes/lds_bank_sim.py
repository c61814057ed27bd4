"""Host simulation of the row-group histogram pass's LDS atomics (csrc/row_kernels.hip rg_batch,
dense groups): which bank pairs the 64 lanes of each ds_add_u64 wave instruction hit, for the
bench corpus' real row-group layout, under the current local-bin numbering and under candidate
renumberings. Cost model per wave instruction: the largest number of lanes on one of the 32
8-byte bank pairs (64 banks x 4 B); same-address lanes counted each (atomics serialise).

    python bench/probes/lds_bank_sim.py --rows 200000
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch


def wave_steps(ptr, ent, rows, bins, sink_base, perm=None):
    """Bins of every lane of every ds_add_u64 instruction of rg_batch over the listed rows (all
    rows here: the root pass), per 64-row batch: lane-balanced 8-entry blocks."""
    out = []
    for b0 in range(0, len(rows), 64):
        rs = rows[b0:b0 + 64]
        st, en = ptr[rs], ptr[rs + 1]
        nb = np.where(en > st, ((en - 1) >> 3) - (st >> 3) + 1, 0)
        total = int(nb.sum())
        if total == 0:
            continue
        K = (total + 63) // 64
        pb = np.concatenate([[0], np.cumsum(nb)[:-1]])
        # block t -> (row, j)
        blk_row = np.repeat(np.arange(len(rs)), nb)
        blk_j = np.arange(total) - pb[blk_row]
        lanes = np.arange(64)
        for step in range(K):
            t = lanes * K + step
            valid = t < np.minimum(lanes * K + K, total)
            tt = np.where(valid, t, 0)
            r = blk_row[tt]
            base = (st[r] & ~7) + 8 * blk_j[tt]
            for k in range(8):
                i = base + k
                inrun = valid & (i >= st[r]) & (i < en[r])
                bn = ent[np.minimum(i, len(ent) - 1)].astype(np.int64)
                if perm is not None:
                    bn = perm[bn]
                b = np.where(inrun, bn, sink_base + lanes)
                out.append(np.where(valid, b, -1))
    return np.array(out)


def cost(steps):
    pair = np.where(steps >= 0, steps % 32, -1)
    c = 0
    same = 0
    for row in pair:
        v = row[row >= 0]
        if v.size == 0:
            continue
        c += np.bincount(v, minlength=32).max()
    for row in steps:
        v = row[row >= 0]
        if v.size:
            same += np.bincount(v).max()
    n = len(steps)
    return {"instrs": n, "avg_max_lanes_per_pair": c / max(n, 1), "avg_max_same_addr": same / max(n, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--sample-rows", type=int, default=20_000)
    args = ap.parse_args()
    from fraud_detection_spark_kafka_llm_amd.data import synth
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH
    from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize
    from fraud_detection_spark_kafka_llm_amd.ops import text as T
    from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order

    F = 1 << 18
    pt, y = synth.generate(synth.SynthConfig(n=args.rows, seed=11), device="cpu")
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=F)
    ip, ix, cnt = T.featurize_score(pt, spec, want_csr=True, device="cpu").csr()
    fo = feature_order(ip, ix, cnt, F)
    idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(F, ip, ix, cnt, idf, fo)
    Q = quantize(vc, max_bins=256, counts=vc.tf_counts, scale=vc.tf_scale)
    rg = Q.rowgroups()
    g = 0
    N = Q.n_rows
    ptr = rg.ptr[g].numpy().astype(np.int64)
    gb = rg.gbase.numpy()
    ent = rg.ent.numpy()[gb[g]:gb[g + 1]].view(np.uint16)
    B = rg.bins
    freq = np.bincount(ent[:ptr[N]].astype(np.int64), minlength=B)
    rows = np.arange(min(N, args.sample_rows))
    res = {"rows": N, "group_entries": int(ptr[N]), "entries_per_row": float(ptr[N] / N),
           "top8_bin_share": float(np.sort(freq)[::-1][:8].sum() / freq.sum()),
           "top32_bin_share": float(np.sort(freq)[::-1][:32].sum() / freq.sum())}
    res["current"] = cost(wave_steps(ptr, ent, rows, B, B))
    # candidate: the most frequent bins dealt round-robin over the 32 bank pairs (a permutation
    # of the local bins: bank pair of slot s = s % 32)
    order = np.argsort(-freq, kind="stable")
    perm = np.empty(B, dtype=np.int64)
    slots = np.arange(B)
    # slot sequence visiting bank pairs round-robin: 0, 1, ..., 31, 32, ... is already round-robin
    # (s % 32), so rank r -> slot r puts the 32 hottest bins on 32 distinct pairs
    perm[order] = slots
    res["hot_round_robin"] = cost(wave_steps(ptr, ent, rows, B, B, perm))
    rng = np.random.default_rng(0)
    res["random"] = cost(wave_steps(ptr, ent, rows, B, B, rng.permutation(B)))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
