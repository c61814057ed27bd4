"""Tree engine: binning, histograms (MFMA vs host), split search vs brute force, DT/RF/GBDT."""
import itertools
import math

import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.ml.tree_model import ensemble_arrays
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
from fraud_detection_spark_kafka_llm_amd.models.grower import GrowParams, Workspace
from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize
from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
from fraud_detection_spark_kafka_llm_amd.ops import native
from fraud_detection_spark_kafka_llm_amd.ops.sparse import score_csr


def random_counts_matrix(n, F, density, seed, max_count=6):
    rng = np.random.default_rng(seed)
    dense = (rng.random((n, F)) < density) * rng.integers(1, max_count + 1, (n, F))
    y = ((dense[:, 0] > 0) | (dense[:, 1] >= 3)).astype(np.float32)
    flip = rng.random(n) < 0.05
    y[flip] = 1 - y[flip]
    return dense.astype(np.float64), y


def vc_from_dense(dense, device="cpu"):
    rows = []
    ptr, idx, val = [0], [], []
    for r in dense:
        nz = np.nonzero(r)[0]
        idx.extend(nz.tolist())
        val.extend(r[nz].tolist())
        ptr.append(len(idx))
    return VectorColumn(dense.shape[1], torch.tensor(ptr, dtype=torch.int64, device=device),
                        torch.tensor(idx, dtype=torch.int32, device=device),
                        torch.tensor(val, dtype=torch.float64, device=device))


def test_count_path_bins_and_thresholds():
    dense, _ = random_counts_matrix(200, 12, 0.3, 0)
    Q = quantize(vc_from_dense(dense), max_bins=4)
    assert Q.Fa == 12
    for f in range(Q.Fa):
        assert int(Q.nbins[f]) == min(int(dense[:, f].max()), 3) + 1
        assert Q.threshold(f, 0) == 0.5 and Q.threshold(f, 1) == 1.5
    # CSC holds every nonzero once, bins = min(count, 3), rows sorted within a column
    colptr = Q.colptr.numpy()
    for f in range(Q.Fa):
        rows = Q.csc_row[colptr[f]:colptr[f + 1]].numpy()
        assert np.all(np.diff(rows) > 0)
        np.testing.assert_array_equal(rows, np.nonzero(dense[:, f])[0])
        np.testing.assert_array_equal(Q.bins_of(f).numpy(), np.minimum(dense[rows, f], 3).astype(np.uint8))


def test_generic_path_with_negatives():
    rng = np.random.default_rng(1)
    dense = np.round(rng.normal(size=(300, 5)), 2) * (rng.random((300, 5)) < 0.5)
    Q = quantize(vc_from_dense(dense), max_bins=8)
    for f in range(Q.Fa):
        vals = np.unique(dense[:, f][dense[:, f] != 0])
        zb = int(Q.zbin[f])
        assert zb == int((vals < 0).sum()) or len(vals) > 7
        nb = int(Q.nbins[f])
        assert nb <= 8
        # thresholds are strictly increasing inside a feature
        th = [Q.threshold(f, b) for b in range(nb - 1)]
        assert all(a < b for a, b in zip(th, th[1:]))


def brute_best_gini(X, y, rows, min_inst=1):
    y = y.astype(np.float64)
    best = (0.0, None)
    n = len(rows)
    c1 = y[rows].sum()
    gp = 1 - (c1 / n) ** 2 - ((n - c1) / n) ** 2
    for f in range(X.shape[1]):
        vals = np.unique(X[rows, f])
        for a, b in zip(vals, vals[1:]):
            t = (a + b) / 2
            L = rows[X[rows, f] <= t]
            R = rows[X[rows, f] > t]
            if len(L) < min_inst or len(R) < min_inst:
                continue
            def imp(r):
                p = y[r].mean()
                return 1 - p * p - (1 - p) ** 2
            g = gp - len(L) / n * imp(L) - len(R) / n * imp(R)
            if g > best[0] + 1e-12:
                best = (g, (f, t))
    return best


def test_decision_tree_root_split_matches_brute_force():
    dense, y = random_counts_matrix(400, 10, 0.35, 3)
    res = fit_forest(vc_from_dense(dense), torch.from_numpy(y), num_trees=1, max_depth=3, device="cpu", prune=False)
    t = res.trees[0]
    g, (f, thr) = brute_best_gini(dense, y, np.arange(len(y)))
    assert t.feature[0] == f
    assert t.threshold[0] == pytest.approx(thr)
    assert t.gain[0] == pytest.approx(g, rel=1e-9)
    # training predictions = host traversal of the same tree
    arr = ensemble_arrays(res.trees, "counts")
    raw = score_csr(vc_from_dense(dense), arr).numpy()
    for i in range(0, len(y), 37):
        leaf = t.leaf_of({k: dense[i, k] for k in np.nonzero(dense[i])[0]})
        np.testing.assert_allclose(raw[i], t.stats[leaf])


def test_gbdt_learns_and_first_split_is_newton_optimal():
    dense, y = random_counts_matrix(600, 8, 0.4, 4)
    out = fit_gbdt(vc_from_dense(dense), torch.from_numpy(y), GBDTParams(n_estimators=1, max_depth=1, base_score=0.5))
    t = out.trees[0]
    g = 0.5 - y
    h = np.full(len(y), 0.25)
    best = (-1, None)
    for f in range(dense.shape[1]):
        for v in np.unique(dense[:, f])[:-1]:
            L = dense[:, f] <= v
            GL, HL, GR, HR = g[L].sum(), h[L].sum(), g[~L].sum(), h[~L].sum()
            gain = GL ** 2 / (HL + 1) + GR ** 2 / (HR + 1) - g.sum() ** 2 / (h.sum() + 1)
            if gain > best[0] + 1e-9:
                best = (gain, f)
    assert t.feature[0] == best[1]
    assert t.gain[0] == pytest.approx(best[0], rel=1e-5)
    out = fit_gbdt(vc_from_dense(dense), torch.from_numpy(y), GBDTParams(n_estimators=20, max_depth=3))
    m = out.base_margin + score_csr(vc_from_dense(dense), ensemble_arrays(out.trees, "value"))[:, 0].numpy()
    assert ((m > 0) == (y > 0.5)).mean() > 0.9


def test_random_forest_bootstrap_and_sampling_are_deterministic():
    dense, y = random_counts_matrix(300, 30, 0.3, 5)
    a = fit_forest(vc_from_dense(dense), torch.from_numpy(y), num_trees=5, bootstrap=True, feature_subset="sqrt", seed=7)
    b = fit_forest(vc_from_dense(dense), torch.from_numpy(y), num_trees=5, bootstrap=True, feature_subset="sqrt", seed=7)
    for ta, tb in zip(a.trees, b.trees):
        np.testing.assert_array_equal(ta.feature, tb.feature)
        np.testing.assert_array_equal(ta.stats, tb.stats)
    # bootstrap changes the root class counts away from the plain counts
    assert any(not np.allclose(t.stats[0], [len(y) - y.sum(), y.sum()]) for t in a.trees)


# --------------------------------------------------------------------------------------------- GPU
# odd chunks, row-blocked and packed items, dense hot features (>= 20% of rows)
QKW = dict(chunk=509, super_rows=1500, hot_density=0.2)


def _hist_on(dev, vc, max_bins, nslots, row_node_np, root=False, np_=4, g=None, h=None, qkw=QKW, dense_rows=640):
    """Histograms of node slots 0..nslots-1 (``row_node`` = slot) through tree_hist_build, plus
    the exponents used. g, h default to deterministic ramps."""
    from fraud_detection_spark_kafka_llm_amd.models.grower import pass_ct, slots_per_tile

    C = native.lib()
    n = row_node_np.shape[0]
    Q = quantize(vc.to(dev), max_bins=max_bins, **qkw)
    ws = Workspace(Q)
    row_node = torch.from_numpy(row_node_np).to(dev)
    node_slot = torch.full((nslots + 2,), -1, dtype=torch.int32)
    node_slot[:nslots] = torch.arange(nslots, dtype=torch.int32)
    node_slot = node_slot.to(dev)
    if np_ == 4:
        gg = torch.from_numpy(np.linspace(-1, 1, n).astype(np.float32) if g is None else g).to(dev)
        hh = torch.from_numpy(np.linspace(0.01, 0.25, n).astype(np.float32) if h is None else h).to(dev)
        C.tree_quant_max(gg, hh, None, None, 0, 0, False, 0, n, ws.maxabs, 0)
        C.tree_quant(gg, hh, None, None, 0, 0, False, 0, 4, ws.maxabs, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)
    else:   # class counts: Poisson(1) bootstrap weights, exact in one digit
        lab = torch.from_numpy((np.arange(n) % 3 == 0).astype(np.float32)).to(dev)
        C.tree_quant(None, None, lab, None, 5, 2, True, 1, 1, None, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)
    hist = torch.zeros((nslots, Q.TB, 2), dtype=torch.int64, device=dev)
    P = slots_per_tile(np_) * 8
    for s0 in range(0, nslots, P):
        cnt = min(P, nslots - s0)
        slot8 = None
        if not root:
            C.tree_slot8(row_node, node_slot, s0, cnt, ws.slot8, None, None)
            slot8 = ws.slot8
        s2n = torch.arange(s0, s0 + cnt, dtype=torch.int32).to(dev)
        ct = pass_ct(np_, cnt)
        for grp in Q.groups:
            C.tree_hist_build(grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(), Q.h_row,
                              Q.h_key, slot8, ws.rowdig, Q.boff, Q.nbins, s2n, hist, Q.TB, grp.bt, ct, np_, None)
        if Q.dense is not None:   # hot features: dense column-major kernel
            for bt in (1, 2, 4):
                gfid, gden = ws.dense_groups(bt, C.tree_dense_fg(bt, 1 if root else ct))
                if gfid.numel():
                    C.tree_hist_dense(Q.dense, ws.digp, ws.rowdig, None if root else ws.slot8_pad, gfid, gden,
                                      Q.boff, Q.nbins, s2n, hist, Q.TB, n, dense_rows, bt, ct, np_)
    if Q.dense is not None:       # the dense path stores the zero bin explicitly: the CSC never does
        zb = (Q.boff[:-1] + Q.zbin.to(torch.int64)).cpu().numpy()[Q.hot]
        hist[:, torch.from_numpy(zb).to(dev)] = 0
    return hist.cpu().numpy(), ws.kexp.cpu().numpy(), Q


def _hist_ref(Q, row_node, nslots, q0, q1):
    """numpy reference: exact int64 sums of the quantised statistics per (slot, bin)."""
    colptr, rows = Q.colptr.cpu().numpy(), Q.csc_row.cpu().numpy()
    boff = Q.boff.cpu().numpy()
    ref = np.zeros((nslots, Q.TB, 2), dtype=np.int64)
    for f in range(Q.Fa):
        e = np.arange(colptr[f], colptr[f + 1])
        r = rows[e]
        s = row_node[r]
        ok = (s >= 0) & (s < nslots)
        b = boff[f] + Q.bins_of(f).cpu().numpy().astype(np.int64)
        np.add.at(ref[:, :, 0], (s[ok], b[ok]), q0[r[ok]])
        np.add.at(ref[:, :, 1], (s[ok], b[ok]), q1[r[ok]])
    return ref


def _sampled_vs_build(dev, nslots, root, seed=3, lds=False):
    """RF count passes over a random feature sample: tree_hist_sampled (packed row state, listed
    active items; the i8 MFMA kernel, or with ``lds`` the LDS-atomic one) against tree_hist_build
    (slot bytes + digit words, every wave slot)."""
    from fraud_detection_spark_kafka_llm_amd.models.grower import pass_ct

    C = native.lib()
    rng = np.random.default_rng(seed)
    n, F = 3000, 700
    vc = vc_from_dense(random_counts_matrix(n, F, 0.03, seed)[0])
    Q = quantize(vc.to(dev), max_bins=32, **QKW)
    ws = Workspace(Q)
    lab = torch.from_numpy((np.arange(n) % 3 == 0).astype(np.float32)).to(dev)
    C.tree_quant(None, None, lab, None, 5, 2, True, 1, 1, None, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)
    row_node = torch.from_numpy(rng.integers(0, nslots + 2, n).astype(np.int32)).to(dev)
    node_slot = torch.full((nslots + 2,), -1, dtype=torch.int32)
    node_slot[:nslots] = torch.arange(nslots, dtype=torch.int32)
    node_slot = node_slot.to(dev)
    mask = torch.from_numpy((rng.random(Q.Fa) < 0.2).astype(np.uint8)).to(dev)
    s2n = torch.arange(nslots, dtype=torch.int32, device=dev)
    ct = pass_ct(1, nslots)
    ref = torch.zeros((nslots, Q.TB, 2), dtype=torch.int64, device=dev)
    got = torch.zeros_like(ref)
    slot8 = pack = None
    if not root:
        C.tree_slot8(row_node, node_slot, 0, nslots, ws.slot8, None, None)
        slot8 = ws.slot8
        pack = ws.rowpack()
        C.tree_slot_pack(row_node, node_slot, nslots, ws.rowdig, pack)
    for gi, grp in enumerate(Q.groups + Q.hot_groups):
        if grp.num_items == 0:
            continue
        C.tree_hist_build(grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(), Q.h_row,
                          Q.h_key, slot8, ws.rowdig, Q.boff, Q.nbins, s2n, ref, Q.TB, grp.bt, ct, 1, mask)
        lst, cnt = ws.item_list(gi, grp)
        C.tree_hist_sampled(grp.item_start, grp.item_end, grp.item_f0, grp.item_meta, grp.wave_order(), Q.h_row,
                            Q.h_key, pack, ws.rowdig, Q.boff, Q.nbins, s2n, got, Q.TB, grp.bt, ct, mask, lst, cnt, lds)
    assert int(ref.abs().sum()) > 0
    # only the sampled features' bins are defined: a pass may skip an active packed item's
    # unsampled features (hist_lds_kernel's key mask) -- nothing reads those bins
    nb = Q.nbins.cpu().numpy().astype(np.int64)
    keep = torch.from_numpy(np.repeat(mask.cpu().numpy().astype(bool), nb))
    return ref.cpu()[:, keep], got.cpu()[:, keep]


@pytest.mark.parametrize("nslots,root", [(1, True), (3, False), (16, False)])
def test_sampled_rf_pass_equals_build_pass(nslots, root):
    ref, got = _sampled_vs_build("cpu", nslots, root)
    assert torch.equal(ref, got)


@pytest.mark.gpu
@pytest.mark.parametrize("nslots,root", [(1, True), (3, False), (16, False), (40, False)])
@pytest.mark.parametrize("lds", [False, True])
def test_gpu_sampled_rf_pass_equals_build_pass_and_host(nslots, root, lds):
    ref, got = _sampled_vs_build("cuda:0", nslots, root, lds=lds)
    href, _ = _sampled_vs_build("cpu", nslots, root)
    assert torch.equal(ref, got) and torch.equal(got, href)


@pytest.mark.parametrize("light", [True, False])
def test_work_items_cover_histogram_csc_once_and_wave_order_is_xcd_grouped(monkeypatch, light):
    """The histogram CSC holds every entry of the non-dense features once, super-block-major;
    every entry belongs to exactly one item; packed items hold consecutive small features with
    distinct key ranges; an item stays inside its super-block, or (``light``: few-entry features)
    holds its whole column in row block 0 and is spread over the XCDs (row block -1)."""
    from fraud_detection_spark_kafka_llm_amd.models import quantize as qmod
    from fraud_detection_spark_kafka_llm_amd.models.quantize import wave_order

    monkeypatch.setattr(qmod, "LIGHT_ENTRIES", 60 if light else 0)
    rng = np.random.default_rng(2)
    n, F = 5000, 40
    dense = (rng.random((n, F)) < np.linspace(0.002, 0.6, F)) * rng.integers(1, 5, (n, F))
    Q = quantize(vc_from_dense(dense.astype(np.float64)), max_bins=8, chunk=100, super_rows=700, hot_density=0.0)
    assert Q.dense is None and Q.n_super == 8
    rows, keys = Q.h_row.numpy(), Q.h_key.numpy()
    assert rows.size == int(Q.colptr[-1])
    # (row, feature, bin) multiset of the histogram CSC == the feature-major CSC
    fid_of = {}
    cover = np.zeros(rows.size, dtype=np.int64)
    kinds = set()
    for grp in Q.groups:
        st, en = grp.item_start.numpy(), grp.item_end.numpy()
        f0, meta, blk = grp.item_f0.numpy(), grp.item_meta.numpy(), grp.item_blk.numpy()
        for i in range(grp.num_items):
            cover[st[i]:en[i]] += 1
            sl2, nf = meta[i] & 0xFF, (meta[i] >> 8) & 0xFF
            single = sl2 == 8                                          # one feature, key = bin
            assert en[i] - st[i] <= 100 or not single
            if blk[i] >= 0:
                assert np.all(rows[st[i]:en[i]] // 625 == blk[i])      # 5000 rows / 8 super-blocks
            else:
                kinds.add("column")
            kinds.add("single" if single else "packed")
            for e in range(st[i], en[i]):
                fl = (int(keys[e]) >> sl2) if not single else 0
                f = int(f0[i]) + fl
                assert fl < nf
                fid_of[e] = (f, int(keys[e]) - int(Q.kbase_host[f]))
        order = grp.wave_order().numpy()
        used = order[order >= 0]
        assert sorted(used.tolist()) == list(range(grp.num_items))   # every item exactly once
        slots = np.nonzero(order >= 0)[0]
        lab = (slots // 4) % 8                                     # workgroup % 8 = XCD group
        blocked = blk[order[slots]] >= 0
        assert np.all(blk[order[slots]][blocked] % 8 == lab[blocked])
    assert np.all(cover == 1)
    assert kinds == ({"packed", "single", "column"} if light else {"packed", "single"})
    got = sorted((int(rows[e]), f, b) for e, (f, b) in fid_of.items())
    colptr, crow, cbin = Q.colptr.numpy(), Q.csc_row.numpy(), Q.csc_bin.numpy()
    ref = sorted((int(crow[e]), f, int(cbin[e])) for f in range(Q.Fa) for e in range(colptr[f], colptr[f + 1]))
    assert got == ref
    # with a dense block: hot columns leave the histogram CSC, the dense block holds their bins
    Qh = quantize(vc_from_dense(dense.astype(np.float64)), max_bins=8, chunk=100, super_rows=700, hot_density=0.3)
    hot = set(Qh.hot.tolist())
    assert hot == {f for f in range(Qh.Fa) if (dense[:, Qh.fid_host[f]] > 0).mean() >= 0.3}
    assert Qh.h_row.numel() == int(Qh.colptr[-1])      # hot columns stay in the CSC (deep levels)
    for grp in Qh.groups:
        assert not any(int(f) in hot for f in grp.item_f0.numpy())
    assert {int(f) for grp in Qh.hot_groups for f in grp.item_f0.numpy()} == hot
    for d, f in enumerate(Qh.hot.tolist()):
        np.testing.assert_array_equal(Qh.dense[d, :n].numpy(), np.minimum(dense[:, Qh.fid_host[f]], 7))
    assert wave_order(None, 0, torch.device("cpu")).tolist() == [-1] * 4


def test_dense_and_csc_paths_give_identical_trees():
    """Hot features through the dense column-major kernel (at every level, at the shallow levels
    only) or through CSC work items: the same exact histograms, so the same DT / RF
    (feature-sampled, no sibling subtraction) / GBDT trees."""
    from fraud_detection_spark_kafka_llm_amd.models import grower as gr
    from fraud_detection_spark_kafka_llm_amd.models import quantize as qz

    dense, y = random_counts_matrix(500, 12, 0.35, 3)
    out = {}
    for hd, depth in ((0.0, 9), (0.1, 9), (0.1, 1)):
        old, qz.HOT_DENSITY = qz.HOT_DENSITY, hd
        old_d, gr.DENSE_MAX_DEPTH = gr.DENSE_MAX_DEPTH, depth
        try:
            vc, yy = vc_from_dense(dense), torch.from_numpy(y)
            dt = fit_forest(vc, yy, num_trees=1, max_depth=4, prune=False)
            rf = fit_forest(vc, yy, num_trees=3, max_depth=4, bootstrap=True, feature_subset="sqrt", seed=7)
            gb = fit_gbdt(vc, yy, GBDTParams(n_estimators=3, max_depth=3))
            out[(hd, depth)] = [(t.feature.tolist(), t.stats.tolist()) for t in dt.trees + rf.trees + gb.trees]
        finally:
            qz.HOT_DENSITY, gr.DENSE_MAX_DEPTH = old, old_d
    assert out[(0.0, 9)] == out[(0.1, 9)] == out[(0.1, 1)]


def test_host_histogram_is_exact():
    """Host tree_hist_build against a direct numpy int64 sum of the quantised statistics."""
    rng = np.random.default_rng(5)
    n, F = 3000, 40
    dense = (rng.random((n, F)) < np.linspace(0.01, 0.5, F)) * rng.integers(1, 9, (n, F))
    vc = vc_from_dense(dense.astype(np.float64))
    row_node = rng.integers(-1, 7, n).astype(np.int32)
    hist, k, Q = _hist_on("cpu", vc, 16, 5, row_node)
    g = np.linspace(-1, 1, n).astype(np.float32).astype(np.float64)
    h = np.linspace(0.01, 0.25, n).astype(np.float32).astype(np.float64)
    q0, q1 = np.rint(np.ldexp(g, int(k[0]))).astype(np.int64), np.rint(np.ldexp(h, int(k[1]))).astype(np.int64)
    np.testing.assert_array_equal(hist, _hist_ref(Q, row_node, 5, q0, q1))


@pytest.mark.gpu
@pytest.mark.parametrize("nslots,max_bins", [(3, 8), (13, 64), (16, 200), (1, 256)])
@pytest.mark.parametrize("np_", [4, 1])
def test_gpu_mfma_histograms_equal_host_bitwise(nslots, max_bins, np_):
    """i8 MFMA histograms (packed, row-blocked, windowed > 64-bin items; root and slot passes)
    equal the host's exact int64 sums bit for bit."""
    rng = np.random.default_rng(nslots * 100 + max_bins)
    n, F = 20000, 300
    dense = (rng.random((n, F)) < np.linspace(0.001, 0.3, F)) * rng.integers(1, 300, (n, F))
    vc = vc_from_dense(dense.astype(np.float64))
    ns = nslots if np_ == 4 else 4 * nslots
    row_node = rng.integers(-1, ns + 2, n).astype(np.int32)
    for root in (False, True):
        s = 1 if root else ns
        a, ka, _ = _hist_on("cpu", vc, max_bins, s, row_node, root, np_)
        b, kb, _ = _hist_on("cuda:0", vc, max_bins, s, row_node, root, np_)
        np.testing.assert_array_equal(ka, kb)
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_gpu_histogram_precision_vs_fp64_of_unsplit_fp32_stats():
    """Bound against an fp64 torch index_add_ of the unsplit fp32 g/h: every
    bin is within count * 2^-(k+1) of the fp64 sum (quantisation only, k from the round's max |g|
    so 2^-(k+1) <= max|g| * 2^-31), i.e. <= 1e-6 of the bin's sum of |g| wherever the bin's mean
    |g| is >= 1e-3 of the max (and far below fp32 accumulation error everywhere)."""
    rng = np.random.default_rng(11)
    n, F = 50000, 200
    dense = (rng.random((n, F)) < np.linspace(0.005, 0.5, F)) * rng.integers(1, 20, (n, F))
    vc = vc_from_dense(dense.astype(np.float64))
    p = 1.0 / (1.0 + np.exp(-rng.normal(0, 3, n)))
    y = (rng.random(n) < p).astype(np.float64)
    g = (p - y).astype(np.float32)                       # logistic gradients, heavy cancellation
    h = np.maximum(p * (1 - p), 1e-16).astype(np.float32)
    row_node = rng.integers(0, 4, n).astype(np.int32)
    hist, k, Q = _hist_on("cuda:0", vc, 64, 4, row_node, g=g, h=h)
    dev = torch.device("cuda:0")
    colptr, rows = Q.colptr.to(dev), Q.csc_row.to(dev).long()
    boff = Q.boff.to(dev)
    fe = torch.repeat_interleave(torch.arange(Q.Fa, device=dev), colptr[1:] - colptr[:-1])
    bins = Q.csc_bin.to(dev).long()
    slot = torch.from_numpy(row_node).to(dev).long()[rows]
    idx = slot * Q.TB + boff[fe] + bins
    gd, hd = torch.from_numpy(g).to(dev).double()[rows], torch.from_numpy(h).to(dev).double()[rows]
    ref = torch.zeros((4 * Q.TB, 2), dtype=torch.float64, device=dev)
    ref[:, 0].index_add_(0, idx, gd)
    ref[:, 1].index_add_(0, idx, hd)
    absg = torch.zeros(4 * Q.TB, dtype=torch.float64, device=dev).index_add_(0, idx, gd.abs())
    cnt = torch.zeros(4 * Q.TB, dtype=torch.float64, device=dev).index_add_(0, idx, torch.ones_like(gd))
    got = torch.from_numpy(hist.reshape(-1, 2)).to(dev).double() * torch.tensor(np.ldexp(1.0, -k), device=dev)
    err = (got - ref).abs()
    assert bool((err[:, 0] <= cnt * np.ldexp(1.0, -int(k[0]) - 1) + 1e-300).all())
    assert bool((err[:, 1] <= cnt * np.ldexp(1.0, -int(k[1]) - 1) + 1e-300).all())
    live = (cnt > 0) & (absg >= 1e-3 * float(np.abs(g).max()) * cnt)
    assert int(live.sum()) > 100
    assert float((err[:, 0][live] / absg[live]).max()) <= 1e-6


@pytest.mark.gpu
def test_gpu_trees_match_host_trees():
    dense, y = random_counts_matrix(3000, 60, 0.2, 9)
    vc = vc_from_dense(dense)
    for kw in (dict(num_trees=1, max_depth=5), dict(num_trees=4, max_depth=4, bootstrap=True, feature_subset="sqrt",
                                                    seed=3)):
        a = fit_forest(vc, torch.from_numpy(y), device="cpu", **kw)
        b = fit_forest(vc, torch.from_numpy(y), device="cuda:0", **kw)
        for ta, tb in zip(a.trees, b.trees):
            np.testing.assert_array_equal(ta.feature, tb.feature)
            np.testing.assert_array_equal(ta.stats, tb.stats)
    ga = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=5, max_depth=4), device="cpu")
    gb = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=5, max_depth=4), device="cuda:0")
    for ta, tb in zip(ga.trees, gb.trees):
        np.testing.assert_array_equal(ta.feature, tb.feature)
        np.testing.assert_array_equal(ta.stats, tb.stats)


@pytest.mark.gpu
def test_gpu_gbdt_bitwise_equals_host_and_repeats():
    """Every histogram sum is an exact integer, so the MFMA device path and the host path give
    bit-identical trees, and two device runs match bit for bit (race oracle)."""
    dense, y = random_counts_matrix(4000, 80, 0.2, 13)
    vc = vc_from_dense(dense)
    p = GBDTParams(n_estimators=6, max_depth=5)
    host = fit_gbdt(vc, torch.from_numpy(y), p, device="cpu")
    dev1 = fit_gbdt(vc, torch.from_numpy(y), p, device="cuda:0")
    dev2 = fit_gbdt(vc, torch.from_numpy(y), p, device="cuda:0")
    for a, b, c in zip(host.trees, dev1.trees, dev2.trees):
        np.testing.assert_array_equal(a.feature, b.feature)
        np.testing.assert_array_equal(a.stats, b.stats)
        np.testing.assert_array_equal(b.stats, c.stats)
        np.testing.assert_array_equal(b.threshold, c.threshold)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_feature_order_is_stable_csc_with_docfreq_and_max(dev):
    from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order

    rng = np.random.default_rng(4)
    n, F = 3000, 700
    dense = (rng.random((n, F)) < 0.03) * rng.integers(1, 400, (n, F))
    dense[:, 5] = 0                                    # empty column
    vc = vc_from_dense(dense.astype(np.float64))
    ip, ix, v = vc.csr()
    fo = feature_order(ip.to(dev), ix.to(dev), v.to(torch.float32).to(dev), F)
    colptr = fo.colptr.cpu().numpy()
    rows, cnt = fo.csc_row.cpu().numpy(), fo.csc_cnt.cpu().numpy()
    for f in range(F):
        r = np.nonzero(dense[:, f])[0]
        np.testing.assert_array_equal(rows[colptr[f]:colptr[f + 1]], r)        # stable: rows increasing
        np.testing.assert_array_equal(cnt[colptr[f]:colptr[f + 1]], np.minimum(dense[r, f], 255))
    np.testing.assert_array_equal(fo.df.cpu().numpy(), (dense > 0).sum(0))
    np.testing.assert_array_equal(fo.maxc.cpu().numpy(), np.minimum(dense.max(0), 255))


def _rf_sample(dev, F=5000, k=71, nodes=(0, 1, 2, 5, 9), seed=123456789, tree=7):
    from fraud_detection_spark_kafka_llm_amd.ops import native

    fid = torch.arange(0, F, 3, dtype=torch.int64, device=dev)     # a subset of active features
    nd = torch.tensor(nodes, dtype=torch.int32, device=dev)
    thr = torch.empty(len(nodes), dtype=torch.float64, device=dev)
    mask = torch.empty(fid.numel(), dtype=torch.uint8, device=dev)
    native.lib().tree_rf_sample(seed, tree, nd, F, k, fid, thr, mask, None)
    return thr.cpu(), mask.cpu(), fid.cpu()


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_rf_sampling_skips_padded_nodes(dev):
    """-1 entries (the padding of a capacity-sized open list: the next level's sample is drawn
    before its size reaches the host) sample nothing: threshold -1, no mask contribution."""
    a_thr, a_mask, _ = _rf_sample(dev, nodes=(3, 8))
    b_thr, b_mask, _ = _rf_sample(dev, nodes=(3, -1, 8, -1))
    assert torch.equal(a_mask, b_mask)
    assert b_thr[1] == -1.0 and b_thr[3] == -1.0
    assert b_thr[0] == a_thr[0] and b_thr[2] == a_thr[1]


def test_rf_sampling_native_equals_python_oracle():
    """Exactly k of F features per node: the native k-th smallest priority equals torch.kthvalue
    over the oracle priorities, and the union mask equals the oracle's."""
    from fraud_detection_spark_kafka_llm_amd.models.rf_sampling import _priorities, node_thresholds

    F, k, nodes, seed, tree = 5000, 71, [0, 1, 2, 5, 9], 123456789, 7
    thr, mask, fid = _rf_sample("cpu", F, k, tuple(nodes), seed, tree)
    ref = node_thresholds(F, seed, tree, nodes, k, torch.device("cpu"))
    assert torch.equal(thr, ref)
    for i, n in enumerate(nodes):
        assert int((_priorities(seed, tree, n, torch.arange(F)) <= thr[i]).sum()) == k
    want = torch.zeros(fid.numel(), dtype=torch.bool)
    for i, n in enumerate(nodes):
        want |= _priorities(seed, tree, n, fid) <= ref[i]
    assert torch.equal(mask.bool(), want)


@pytest.mark.gpu
def test_gpu_rf_sampling_equals_host():
    for F, k in ((5000, 71), (1 << 18, 512)):
        h = _rf_sample("cpu", F, k)
        g = _rf_sample("cuda:0", F, k)
        assert torch.equal(h[0], g[0]) and torch.equal(h[1], g[1])


@pytest.mark.parametrize("bootstrap,subset,n_trees,lanes", [(True, "sqrt", 11, 4), (False, "all", 3, 2),
                                                         (True, "onethird", 9, 3)])
def test_trees_in_flight_equal_single_tree_growth(monkeypatch, bootstrap, subset, n_trees, lanes):
    """PAR-05: trees grown several at a time (interleaved level loops, own workspaces) are exactly
    the trees of one-at-a-time growth."""
    from fraud_detection_spark_kafka_llm_amd.models import forest_batch
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest

    rng = np.random.default_rng(17)
    n, F = 1500, 90
    dense = (rng.random((n, F)) < 0.12) * rng.integers(1, 6, (n, F))
    y = ((dense[:, 3] > 0) ^ (dense[:, 11] >= 3)).astype(np.float32)
    vc = VectorColumn(F, dense=torch.from_numpy(dense.astype(np.float64)))
    kw = dict(num_trees=n_trees, max_depth=5, max_bins=16, bootstrap=bootstrap, feature_subset=subset, seed=7,
              device="cpu")
    monkeypatch.setattr(forest_batch, "TREES_IN_FLIGHT", 1)
    ref = fit_forest(vc, torch.from_numpy(y), **kw)
    monkeypatch.setattr(forest_batch, "TREES_IN_FLIGHT", lanes)
    got = fit_forest(vc, torch.from_numpy(y), **kw)
    sig = lambda r: [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in r.trees]  # noqa: E731
    assert sig(got) == sig(ref)


@pytest.mark.gpu
def test_gpu_trees_in_flight_equal_single_tree_and_host(monkeypatch):
    from fraud_detection_spark_kafka_llm_amd.models import forest_batch
    from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest

    rng = np.random.default_rng(23)
    n, F = 20000, 400
    dense = (rng.random((n, F)) < 0.05) * rng.integers(1, 6, (n, F))
    y = ((dense[:, 3] > 0) ^ (dense[:, 11] >= 3)).astype(np.float32)
    vc = VectorColumn(F, dense=torch.from_numpy(dense.astype(np.float64)))
    kw = dict(num_trees=13, max_depth=5, max_bins=32, bootstrap=True, feature_subset="sqrt", seed=5)
    sig = lambda r: [(t.feature.tolist(), t.threshold.tolist(), t.stats.tolist()) for t in r.trees]  # noqa: E731
    monkeypatch.setattr(forest_batch, "TREES_IN_FLIGHT", 4)
    g = sig(fit_forest(vc, torch.from_numpy(y), device="cuda:0", **kw))
    h = sig(fit_forest(vc, torch.from_numpy(y), device="cpu", **kw))
    monkeypatch.setattr(forest_batch, "TREES_IN_FLIGHT", 1)
    g1 = sig(fit_forest(vc, torch.from_numpy(y), device="cuda:0", **kw))
    assert g == g1 == h


def test_warm_tree_kernels_runs_the_production_path_on_the_host():
    """models/warmup.py (the untimed warm-up of bench.py / bench/suite.py) on the host path."""
    from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels

    warm_tree_kernels("cpu", rows=1500, gbdt_depth=3, forest_depth=3)


def _same_trees(ta_list, tb_list):
    assert len(ta_list) == len(tb_list)
    for ta, tb in zip(ta_list, tb_list):
        np.testing.assert_array_equal(ta.feature, tb.feature)
        np.testing.assert_array_equal(ta.threshold, tb.threshold)
        np.testing.assert_array_equal(ta.left, tb.left)
        np.testing.assert_array_equal(ta.right, tb.right)
        np.testing.assert_array_equal(ta.stats, tb.stats)
        np.testing.assert_array_equal(ta.gain, tb.gain)


@pytest.mark.parametrize("depth,hot", [(6, 0.2), (4, 0.0), (1, 0.2)])
def test_device_level_loop_grows_the_host_loop_trees(monkeypatch, depth, hot):
    """The device-resident level loop (tree.h level_plan + split-driven partition, run through its
    host twins here) grows the host loop's GBDT trees bit for bit: node numbering, smaller-sibling
    builds, subtraction, dense-block (hot feature) and column partitions, leaves at max depth."""
    from fraud_detection_spark_kafka_llm_amd.models import grower, quantize as qmod

    monkeypatch.setattr(qmod, "HOT_DENSITY", hot)
    dense, y = random_counts_matrix(3000, 80, 0.15, 21)
    dense[:, :6] = np.random.default_rng(1).integers(0, 5, (3000, 6))     # dense columns -> hot block
    vc = vc_from_dense(dense)
    params = GBDTParams(n_estimators=4, max_depth=depth, gamma=0.0)
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(grower, "DEVICE_LEVELS", flag)
        out[flag] = fit_gbdt(vc, torch.from_numpy(y), params, device="cpu")
    _same_trees(out[False].trees, out[True].trees)
    assert max(t.num_nodes for t in out[True].trees) == (3 if depth == 1 else max(t.num_nodes for t in out[True].trees))
    assert depth == 1 or max(t.num_nodes for t in out[True].trees) > 7


@pytest.mark.parametrize("kw", [dict(num_trees=1, max_depth=6),                                   # DT, subtraction
                                dict(num_trees=3, max_depth=5, bootstrap=True, feature_subset="sqrt", seed=7),
                                dict(num_trees=2, max_depth=4, impurity="entropy", feature_subset="onethird",
                                     bootstrap=True, seed=3),
                                dict(num_trees=1, max_depth=4, weights=True)])                    # 4-plane counts
def test_device_level_loop_grows_the_host_loop_forests(monkeypatch, kw):
    """DT / RF (per-node k-of-F sampling builds every open node, Poisson bootstrap, gini and
    entropy purity leaves) and weighted class counts: the device level loop's trees equal the host
    loop's bit for bit."""
    from fraud_detection_spark_kafka_llm_amd.models import grower

    dense, y = random_counts_matrix(2500, 70, 0.2, 33)
    vc = vc_from_dense(dense)
    kw = dict(kw)
    if kw.pop("weights", False):
        kw["weights"] = np.random.default_rng(2).uniform(0.2, 3.0, len(y))
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(grower, "DEVICE_LEVELS", flag)
        out[flag] = fit_forest(vc, torch.from_numpy(y), device="cpu", prune=False, **kw)
    _same_trees(out[False].trees, out[True].trees)
    assert max(t.num_nodes for t in out[True].trees) > 7


@pytest.mark.gpu
def test_gpu_device_level_loop_equals_gpu_host_loop(monkeypatch):
    """On the GPU, the device-resident level loop (level_plan / partition_cols kernels, masked
    single-slot passes) grows the same GBDT and RF trees as the host level loop."""
    from fraud_detection_spark_kafka_llm_amd.models import grower

    dense, y = random_counts_matrix(6000, 90, 0.2, 44)
    dense[:, :5] = np.random.default_rng(4).integers(0, 6, (6000, 5))
    vc = vc_from_dense(dense)
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(grower, "DEVICE_LEVELS", flag)
        g = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=4, max_depth=6), device="cuda:0")
        r = fit_forest(vc, torch.from_numpy(y), num_trees=3, max_depth=5, bootstrap=True, feature_subset="sqrt",
                       seed=5, device="cuda:0", prune=False)
        out[flag] = (g.trees, r.trees)
    _same_trees(out[False][0], out[True][0])
    _same_trees(out[False][1], out[True][1])


@pytest.mark.parametrize("max_delta_step", [0.0, 0.7])
def test_deferred_tree_build_equals_immediate(max_delta_step):
    """GBDT without per-round hooks builds tree t's host table during tree t + 1 and updates the
    margins with leaf values computed from the device node table (models/grower.py
    leaf_values_device); with an eval hook every tree is built immediately from host leaf values.
    Both give the same trees and the same final margins, bit for bit."""
    from fraud_detection_spark_kafka_llm_amd.models import grower

    dense, y = random_counts_matrix(2500, 60, 0.2, 57)
    vc = vc_from_dense(dense)
    params = GBDTParams(n_estimators=5, max_depth=5, max_delta_step=max_delta_step)
    margins = []
    immediate = fit_gbdt(vc, torch.from_numpy(y), params, device="cpu",
                         eval_fn=lambda t, trees, m: margins.append(m.clone()))
    deferred = fit_gbdt(vc, torch.from_numpy(y), params, device="cpu")
    _same_trees(immediate.trees, deferred.trees)
    base = torch.full((len(y),), deferred.base_margin, dtype=torch.float64)
    replay = base + score_csr(vc, ensemble_arrays(deferred.trees, "value", cmp_less=False))[:, 0]
    assert torch.allclose(replay, margins[-1], rtol=0, atol=1e-12)


def test_leaf_values_device_bitwise_equal_host_table():
    """The device leaf values are the host table's values bit for bit (exact 2^-k scaling)."""
    from fraud_detection_spark_kafka_llm_amd.models.grower import GrowParams, leaf_values_device

    rng = np.random.default_rng(3)
    stats = torch.from_numpy(np.stack([rng.integers(-2**50, 2**50, 64), rng.integers(0, 2**54, 64)], 1))
    kexp = torch.tensor([31, 29], dtype=torch.int32)
    for mds in (0.0, 0.5):
        p = GrowParams(mode=0, lambda_=1.0, eta=0.3, max_delta_step=mds)
        dev = leaf_values_device(stats, kexp, p).numpy()
        st = stats.numpy().astype(np.float64) * np.ldexp(1.0, -kexp.numpy().astype(np.int64))
        w = -st[:, 0] / (st[:, 1] + p.lambda_)
        if mds > 0:
            w = np.clip(w, -mds, mds)
        assert np.array_equal((p.eta * w).view(np.int64), dev.view(np.int64))


@pytest.mark.gpu
def test_gpu_leaf_values_device_bitwise_equal_host_table():
    """On the GPU (int64 -> fp64 conversion, fp64 division on the device): the same bits as the
    host table's leaf values."""
    from fraud_detection_spark_kafka_llm_amd.models.grower import GrowParams, leaf_values_device

    rng = np.random.default_rng(5)
    stats = torch.from_numpy(np.stack([rng.integers(-2**55, 2**55, 4096), rng.integers(0, 2**56, 4096)], 1))
    kexp = torch.tensor([33, 27], dtype=torch.int32)
    for mds in (0.0, 0.5):
        p = GrowParams(mode=0, lambda_=1.0, eta=0.3, max_delta_step=mds)
        dev = leaf_values_device(stats.cuda(), kexp.cuda(), p).cpu().numpy()
        st = stats.numpy().astype(np.float64) * np.ldexp(1.0, -kexp.numpy().astype(np.int64))
        w = -st[:, 0] / (st[:, 1] + p.lambda_)
        if mds > 0:
            w = np.clip(w, -mds, mds)
        assert np.array_equal((p.eta * w).view(np.int64), dev.view(np.int64))


@pytest.mark.gpu
def test_gpu_packed_item_cannot_overflow_int32_accumulators():
    """a packed run whose entries concentrate in one super-block used to form one work
    item of > 131,071 entries; with a plane digit of -128 on every row each entry adds 2^14 to one
    int32 MFMA accumulator, which overflowed. Items are now capped at ``chunk`` entries (and chunk
    at 131,071), so the device histogram still equals the host's exact int64 sums."""
    n, F = 280_000, 6
    rng = np.random.default_rng(5)
    cols = [np.arange(140_000)] + [np.sort(rng.choice(n, 3000, replace=False)) for _ in range(F - 1)]
    rows_of = np.concatenate(cols)
    feat_of = np.concatenate([np.full(c.size, f) for f, c in enumerate(cols)])
    order = np.lexsort((feat_of, rows_of))
    rows_of, feat_of = rows_of[order], feat_of[order]
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(indptr, rows_of + 1, 1)
    vc = VectorColumn(F, torch.from_numpy(np.cumsum(indptr)), torch.from_numpy(feat_of.astype(np.int32)),
                      torch.ones(rows_of.size, dtype=torch.float64))
    g = np.full(n, 1.0 + 2.0 ** -22, dtype=np.float32)        # q = 2^29 + 128: plane-0 digit -128
    h = np.full(n, 0.25, dtype=np.float32)
    row_node = np.zeros(n, dtype=np.int32)
    qkw = dict(chunk=131071, super_rows=140_000, hot_density=0.0)
    hist, k, Q = _hist_on("cuda:0", vc, 16, 1, row_node, root=True, g=g, h=h, qkw=qkw)
    q0 = np.rint(np.ldexp(g.astype(np.float64), int(k[0]))).astype(np.int64)
    q1 = np.rint(np.ldexp(h.astype(np.float64), int(k[1]))).astype(np.int64)
    assert int(q0[0]) % 256 == 128
    np.testing.assert_array_equal(hist, _hist_ref(Q, row_node, 1, q0, q1))


def _split_inputs(seed, nodes=5, Fa=300, mode=0):
    """Random exact histograms: features of 1..150 bins (wide ones span > 2 wave chunks), zero
    bins anywhere, node totals >= the stored sums."""
    rng = np.random.default_rng(seed)
    nb = rng.integers(1, 40, Fa).astype(np.int32)
    nb[rng.random(Fa) < 0.15] = rng.integers(17, 150, int((rng.random(Fa) < 0.15).sum()) or 1)[0]
    nb[:4] = [150, 64, 65, 17]
    zb = np.array([rng.integers(0, n) for n in nb], dtype=np.int32)
    boff = np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)
    TB = int(boff[-1])
    hist = np.zeros((nodes, TB + 3, 2), dtype=np.int64)                  # padded stride
    if mode == 0:
        hist[:, :TB, 0] = rng.integers(-(1 << 30), 1 << 30, (nodes, TB))
        hist[:, :TB, 1] = rng.integers(0, 1 << 28, (nodes, TB))
    else:
        hist[:, :TB, :] = rng.integers(0, 50, (nodes, TB, 2))
    for f in range(Fa):                                                   # zero bins hold nothing
        hist[:, boff[f] + zb[f], :] = 0
    totals = np.stack([hist[:, :TB, 0].sum(1) // 3 + (hist[:, :TB, 0].sum(1) if mode else 0),
                       hist[:, :TB, 1].sum(1) + rng.integers(0, 1 << 20, nodes)], 1).astype(np.int64)
    if mode:
        totals[:, 0] = hist[:, :TB, 0].sum(1) + rng.integers(0, 100, nodes)
    return hist, totals, boff, nb, zb


@pytest.mark.gpu
@pytest.mark.parametrize("mode,rf", [(0, False), (1, False), (2, False), (1, True)])
def test_gpu_wide_feature_split_search_equals_host(mode, rf):
    """split_wide_kernel (a wave per (node, wide feature): wave reductions / scans over 64-bin
    chunks) gives the serial scan's gain, bin and left sums bit for bit, ties to the lowest bin."""
    C = native.lib()
    hist, totals, boff, nb, zb = _split_inputs(7 + mode, mode=mode)
    nodes, Fa = totals.shape[0], nb.size
    # ties: a node whose feature 3 repeats one bin pattern (equal gains at several bins)
    hist[1, boff[3]:boff[4], :] = 0
    args_np = (hist, totals, boff, nb, zb, np.arange(Fa, dtype=np.int64) * 7, np.array([0, 3, 4, -1, 9], np.int32)[:nodes],
               np.array([20, 18] if mode == 0 else [0, 0], dtype=np.int32))
    out = {}
    for dev, use_wide in (("cpu", False), ("cuda:0", True), ("cuda:0", False)):
        t = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in args_np]
        thr = torch.full((nodes,), 0.6, dtype=torch.float64, device=dev) if rf else None
        og = torch.empty((nodes, Fa), dtype=torch.float64, device=dev)
        ob = torch.empty((nodes, Fa), dtype=torch.int32, device=dev)
        ol = torch.empty((nodes, Fa, 2), dtype=torch.int64, device=dev)
        wide = torch.nonzero(t[3] > 16).flatten().to(torch.int32) if use_wide else None
        C.tree_split_find(t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], mode, 1.0, 1.0 if mode == 0 else 2.0, thr,
                          11, 3, og, ob, ol, None, wide)
        out[(dev, use_wide)] = (og.cpu().numpy(), ob.cpu().numpy(), ol.cpu().numpy())
    assert (nb > 16).sum() >= 4

    def same(x, y):
        for a, b in zip(x, y):
            np.testing.assert_array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                                          b.view(np.int64) if b.dtype == np.float64 else b)

    # the wave search equals the device's serial scan bit for bit (every mode) ...
    same(out[("cuda:0", True)], out[("cuda:0", False)])
    # ... and the host's where no transcendental is involved (the device log of the entropy
    # gain is not the host's correctly rounded one: its gains may differ in the last bits)
    if mode != 2:
        same(out[("cpu", False)], out[("cuda:0", True)])
    assert (out[("cpu", False)][1] >= 0).any()


def test_histogram_csc_copy_pieces(monkeypatch):
    """The histogram CSC copy split into fixed-size pieces (quantize.COPY_PIECE) writes the same
    layout as one workgroup per segment."""
    from fraud_detection_spark_kafka_llm_amd.models import quantize as qmod

    dense, _ = random_counts_matrix(2000, 40, 0.3, 9)
    ref = quantize(vc_from_dense(dense), max_bins=32, **QKW)
    _ = ref.groups
    monkeypatch.setattr(qmod, "COPY_PIECE", 7)
    got = quantize(vc_from_dense(dense), max_bins=32, **QKW)
    _ = got.groups
    assert torch.equal(ref.h_row, got.h_row) and torch.equal(ref.h_key, got.h_key)
    for a, b in zip(ref.groups + ref.hot_groups, got.groups + got.hot_groups):
        assert torch.equal(a.item_start, b.item_start) and torch.equal(a.item_meta, b.item_meta)
