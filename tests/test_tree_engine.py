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
        np.testing.assert_array_equal(Q.csc_bin[colptr[f]:colptr[f + 1]].numpy(),
                                      np.minimum(dense[rows, f], 3).astype(np.uint8))


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
def _hist_on(dev, vc, max_bins, ct, nslots, row_node_np, root=False, src="stream"):
    """``src``: where the kernel reads row statistics (grower.stats_source): the per-tree
    entry-order copy or per-entry row gathers."""
    C = native.lib()
    n = row_node_np.shape[0]
    # odd chunk: unaligned item starts; small row blocks: dense columns split per block (XCD order)
    Q = quantize(vc.to(dev), max_bins=max_bins, chunk=509, row_block=1500, split_min=64)
    ws = Workspace(Q, 64, src=src)
    gather = src != "stream"
    row_node = torch.from_numpy(row_node_np).to(dev)
    node_slot = torch.full((nslots + 2,), -1, dtype=torch.int32)
    node_slot[:nslots] = torch.arange(nslots, dtype=torch.int32)
    node_slot = node_slot.to(dev)
    gg = torch.from_numpy(np.linspace(-1, 1, n).astype(np.float32)).to(dev)
    hh = torch.from_numpy(np.linspace(0.01, 0.25, n).astype(np.float32)).to(dev)
    C.tree_rowstats(gg, hh, None, None, 0, 0, False, 0, ws.rowstats)
    if not gather:
        for grp in Q.groups:
            C.tree_entry_stats_items(grp.item_start, grp.item_end, grp.wave_order(), Q.csc_row, ws.rowstats, ws.est)
    hist = torch.zeros((nslots, Q.TB, 2), dtype=torch.float64, device=dev)
    from fraud_detection_spark_kafka_llm_amd.models.grower import pass_ct, tile_shape

    P = 8 * ct      # node slots per pass; each tile shape picks its own column-tile count
    for s0 in range(0, nslots, P):
        cnt = min(P, nslots - s0)
        slot8 = None
        if not root:
            C.tree_slot8(row_node, node_slot, s0, cnt, ws.slot8)
            slot8 = ws.slot8
        for grp in Q.groups:
            c = pass_ct(grp.bt, cnt)
            s2n = torch.full((tile_shape(grp.bt, c)[0],), -1, dtype=torch.int32)
            s2n[:cnt] = torch.arange(s0, s0 + cnt, dtype=torch.int32)
            slab = ws.slab_for(grp.num_items, grp.bt, c)
            C.tree_hist_build(grp.item_start, grp.item_end, Q.csc_row, Q.csc_bin, slot8, ws.est, grp.bt, c,
                              slab, grp.feat, grp.feat_item0, grp.feat_nitems, Q.boff, Q.nbins, s2n.to(dev),
                              hist, Q.TB, grp.wave_order(), ws.rowstats if gather else None)
    return hist.cpu().numpy()


def test_row_blocked_items_cover_columns_and_wave_order_is_xcd_grouped():
    from fraud_detection_spark_kafka_llm_amd.models.quantize import wave_order

    rng = np.random.default_rng(2)
    n, F = 5000, 30
    dense = (rng.random((n, F)) < np.linspace(0.01, 0.6, F)) * rng.integers(1, 5, (n, F))
    Q = quantize(vc_from_dense(dense.astype(np.float64)), max_bins=8, chunk=100, row_block=700, split_min=200)
    colptr = Q.colptr.numpy()
    rows = Q.csc_row.numpy()
    for grp in Q.groups:
        st, en = grp.item_start.numpy(), grp.item_end.numpy()
        feat, blk = grp.item_feat.numpy(), grp.item_blk.numpy()
        # items tile every column exactly; a blocked item stays inside its row block
        for f in np.unique(feat):
            sel = np.nonzero(feat == f)[0]
            assert st[sel[0]] == colptr[f] and en[sel[-1]] == colptr[f + 1]
            assert np.all(st[sel[1:]] == en[sel[:-1]]) and np.all(en[sel] - st[sel] <= 100)
        for i in np.nonzero(blk >= 0)[0]:
            assert np.all(rows[st[i]:en[i]] // 700 == blk[i])
        assert (blk >= 0).any() and (blk < 0).any()
        order = grp.wave_order().numpy()
        used = order[order >= 0]
        assert sorted(used.tolist()) == list(range(grp.num_items))   # every item exactly once
        slots = np.nonzero(order >= 0)[0]
        lab = (slots // 4) % 8                                     # workgroup % 8 = XCD group
        b = blk[order[slots]]
        assert np.all((b < 0) | (b % 8 == lab))
        # within one XCD group, row blocks are visited in increasing order, whole columns last
        for x in range(8):
            bx = b[lab == x]
            key = np.where(bx < 0, 1 << 30, bx)
            assert np.all(np.diff(key) >= 0)
    assert wave_order(None, 0, torch.device("cpu")).tolist() == [-1] * 4


def test_host_histogram_matches_numpy():
    """Host tree_hist_build (slot table + entry-order statistics) against a direct numpy sum."""
    rng = np.random.default_rng(5)
    n, F = 3000, 40
    dense = (rng.random((n, F)) < 0.1) * rng.integers(1, 9, (n, F))
    vc = vc_from_dense(dense.astype(np.float64))
    row_node = rng.integers(-1, 7, n).astype(np.int32)
    hist = _hist_on("cpu", vc, 16, 1, 5, row_node)
    Q = quantize(vc, max_bins=16, chunk=509, row_block=1500, split_min=64)
    g = np.linspace(-1, 1, n).astype(np.float32).astype(np.float64)
    colptr, rows, bins = Q.colptr.numpy(), Q.csc_row.numpy(), Q.csc_bin.numpy()
    boff = Q.boff.numpy()
    ref = np.zeros((5, Q.TB))
    for f in range(Q.Fa):
        e = np.arange(colptr[f], colptr[f + 1])
        s = row_node[rows[e]]
        ok = (s >= 0) & (s < 5)
        np.add.at(ref, (s[ok], boff[f] + bins[e][ok]), g[rows[e][ok]])
    np.testing.assert_allclose(hist[:, :, 0], ref, rtol=1e-4, atol=1e-4)
    # row-gather mode reads the same statistics: identical sums
    np.testing.assert_array_equal(_hist_on("cpu", vc, 16, 1, 5, row_node, src="gather"), hist)


@pytest.mark.gpu
@pytest.mark.parametrize("ct,nslots", [(1, 3), (2, 13), (4, 29)])
@pytest.mark.parametrize("max_bins", [8, 64])
def test_gpu_mfma_histograms_match_host(ct, nslots, max_bins):
    rng = np.random.default_rng(ct * 100 + max_bins)
    n, F = 20000, 300
    dense = (rng.random((n, F)) < 0.05) * rng.integers(1, 80, (n, F))
    vc = vc_from_dense(dense.astype(np.float64))
    row_node = rng.integers(-1, nslots + 2, n).astype(np.int32)
    for root in (False, True):
        ns = 1 if root else nslots
        a = _hist_on("cpu", vc, max_bins, ct, ns, row_node, root)
        # device chunks accumulate in fp32 (MFMA), host in fp64: allow fp32 rounding of the partials
        scale = np.abs(a).max()
        for src in ("stream", "gather"):
            b = _hist_on("cuda:0", vc, max_bins, ct, ns, row_node, root, src)
            np.testing.assert_allclose(b, a, rtol=2e-6, atol=2e-7 * scale)


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
            np.testing.assert_allclose(ta.stats, tb.stats, rtol=1e-9)
    ga = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=5, max_depth=4), device="cpu")
    gb = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=5, max_depth=4), device="cuda:0")
    for ta, tb in zip(ga.trees, gb.trees):
        np.testing.assert_array_equal(ta.feature, tb.feature)
        np.testing.assert_allclose(ta.stats[:, 0], tb.stats[:, 0], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_gpu_deterministic_gbdt_bitwise_equals_host_and_repeats():
    """Deterministic mode: every histogram sum is exact, so the MFMA device path and the fp64 host
    path give bit-identical trees, and two device runs match bit for bit (race oracle)."""
    dense, y = random_counts_matrix(4000, 80, 0.2, 13)
    vc = vc_from_dense(dense)
    p = GBDTParams(n_estimators=6, max_depth=5, deterministic=True)
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
