"""Row-group histogram engine (csrc/row_kernels.hip, models/quantize.RowGroups): layout coverage,
exact histograms against the numpy int64 reference on the host and bitwise host == GPU, and the
level loop growing the CSC passes' trees."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
from fraud_detection_spark_kafka_llm_amd.models.grower import Workspace
from fraud_detection_spark_kafka_llm_amd.models.quantize import RowGroups, quantize
from fraud_detection_spark_kafka_llm_amd.ops import native

from test_tree_engine import QKW, _hist_ref, _same_trees, random_counts_matrix, vc_from_dense


def _wide(n, F, seed, hi=200, dmax=0.5):
    rng = np.random.default_rng(seed)
    dense = (rng.random((n, F)) < np.linspace(0.001, dmax, F)) * rng.integers(1, hi, (n, F))
    return vc_from_dense(dense.astype(np.float64))


def _quant(ws, n, dev, np_=4):
    C = native.lib()
    if np_ == 4:
        gg = torch.from_numpy(np.linspace(-1, 1, n).astype(np.float32)).to(dev)
        hh = torch.from_numpy(np.linspace(0.01, 0.25, n).astype(np.float32)).to(dev)
        C.tree_quant_max(gg, hh, None, None, 0, 0, False, 0, n, ws.maxabs, 0)
        C.tree_quant(gg, hh, None, None, 0, 0, False, 0, 4, ws.maxabs, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)
    else:
        lab = torch.from_numpy((np.arange(n) % 3 == 0).astype(np.float32)).to(dev)
        C.tree_quant(None, None, lab, None, 5, 2, True, 1, 1, None, ws.rowdig, ws.kexp, ws.totals, ws.digp, 0)


def _q_of(ws, np_):
    d = ws.rowdig.cpu().numpy().view(np.uint32).astype(np.int64)
    if np_ == 4:
        q = (d ^ 0x80808080) - 0x80808080
    else:
        q = ((d & 0xFF) ^ 0x80) - 0x80
    return q[:, 0], q[:, 1]


MODE = {"gmode": None}


def gmode(rg):
    """The groups' pass modes: the layout's own, or all balanced / all lane-per-row (MODE)."""
    m = MODE["gmode"]
    return rg.gmode if m is None else torch.full_like(rg.gmode, m)


def _rg_hist_on(dev, vc, max_bins, nslots, row_node_np, root=False, shards=None, np_=4, P=16, max_groups=None,
                dbg=0, bins=8192, em=False, part=False):
    """Histograms of node slots 0..nslots-1 through tree_rg_list + tree_rg_hist, plus q0, q1 and Q;
    ``shards`` = (S, bin_lo) writes the shard-major DP layout (returned unpacked); ``em`` passes
    the entry-major sparse pass's arguments (taken at single-slot levels, whatever the list size)."""
    C = native.lib()
    n = row_node_np.shape[0]
    Q = quantize(vc.to(dev), max_bins=max_bins, **QKW)
    ws = Workspace(Q)
    _quant(ws, n, dev, np_)
    rg = RowGroups(Q, max_groups=max_groups, bins=bins)
    list_ = start = ldig = None
    node_slot = torch.full((nslots + 2,), -1, dtype=torch.int32)
    node_slot[:nslots] = torch.arange(nslots, dtype=torch.int32)
    node_slot = node_slot.to(dev)
    row_node = torch.from_numpy(row_node_np).to(dev)
    emdig = torch.full((n, 2), 7, dtype=torch.int32, device=dev) if (em and not root and nslots == 1) else None
    if not root:
        list_ = torch.empty(n, dtype=torch.int32, device=dev)
        start = torch.zeros(nslots + 1, dtype=torch.int32, device=dev)
        work = torch.zeros(nslots * (2 + n // native.lib().tree_rg_list_rows(n) + 1), dtype=torch.int32, device=dev)
        ldig = torch.empty((n, 2), dtype=torch.int32, device=dev)
        C.tree_rg_list(row_node, node_slot, None, n, nslots, work, start, list_, ws.rowdig, ldig, emdig)
    s2n = torch.arange(nslots, dtype=torch.int32, device=dev)
    q0, q1 = _q_of(ws, np_)
    kw = {}
    if em:
        assert rg.erow is not None
        kw = rg.em_args(emdig)
        if emdig is not None:
            kw["em_min_rows"] = 1
            built = (row_node_np >= 0) & (row_node_np < nslots)
            want = np.where(built[:, None], ws.rowdig.cpu().numpy(), 0)
            np.testing.assert_array_equal(emdig.cpu().numpy(), want)       # every row written
    if part:        # per-workgroup partial tables + the reduction (straddling chunks: atomics)
        kw["part"] = torch.empty(rg.work(P).shape[1] * bins * 2, dtype=torch.int64, device=dev)
        kw["wg_first"] = rg.work_first(P)
    if shards is None:
        hist = torch.zeros((nslots, Q.TB, 2), dtype=torch.int64, device=dev)
        C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, ws.rowdig, np_, list_, start, ldig, nslots, gmode(rg),
                       rg.work(P), s2n, hist, Q.TB, None, 0, dbg, **kw)
        return hist.cpu().numpy(), q0, q1, Q, rg
    S, lo = shards
    Bs = int(np.diff(lo).max())
    buf = torch.zeros((S, nslots, Bs, 2), dtype=torch.int64, device=dev)
    C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, ws.rowdig, np_, list_, start, ldig, nslots, gmode(rg),
                   rg.work(P), s2n, buf.view(S * nslots, Bs, 2), Bs, torch.from_numpy(lo).to(dev), nslots * Bs, dbg,
                   **kw)
    b = buf.cpu().numpy()
    hist = np.concatenate([b[k, :, : lo[k + 1] - lo[k]] for k in range(S)], axis=1)
    return hist, q0, q1, Q, rg


def test_row_groups_cover_every_entry_once():
    """Every CSC entry appears once in its (group, row) run; local bins map back to the global
    column; a group holds <= RG_BINS bins, densest features first; group starts are 16-B aligned."""
    vc = _wide(4000, 300, 3)
    Q = quantize(vc, max_bins=100, **QKW)
    RG_BINS = 4096
    assert Q.TB > 2 * RG_BINS                              # several groups
    rg = RowGroups(Q, bins=RG_BINS)
    assert rg.complete and rg.G >= 2
    colptr, boff, rows = Q.colptr.numpy(), Q.boff.numpy(), Q.csc_row.numpy()
    want = sorted((int(r), int(boff[f] + b)) for f in range(Q.Fa)
                  for r, b in zip(rows[colptr[f]:colptr[f + 1]], Q.bins_of(f).numpy()))
    ptr, ent, gbase, gbin = rg.ptr.numpy(), rg.ent.numpy().view(np.uint16), rg.gbase.numpy(), rg.gbin.numpy()
    assert (gbase % 8 == 0).all()
    got = []
    for g in range(rg.G):
        assert (np.diff(ptr[g]) >= 0).all()
        for r in range(Q.n_rows):
            for i in range(ptr[g, r], ptr[g, r + 1]):
                col = int(gbin[g, ent[gbase[g] + i]])
                assert col >= 0
                got.append((r, col))
    assert sorted(got) == want
    cnt = np.diff(colptr)
    dens = [cnt[rg.fgroup_host == g].min() for g in range(rg.G)]
    assert all(dens[g] >= cnt[rg.fgroup_host == g + 1].max() for g in range(rg.G - 1))
    for g in range(rg.G):
        assert (gbin[g] >= 0).sum() <= RG_BINS


@pytest.mark.parametrize("dtype", [torch.float32, torch.int32, torch.float64])
def test_row_groups_from_csr_equal_csc_build(dtype):
    """The count-path CSR build (thread per row) gives the CSC build's layout: the same ptr and
    the same multiset of local bins in every (group, row) run (runs in CSR order)."""
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn

    rng = np.random.default_rng(5)
    n, F = 3000, 400
    dense = (rng.random((n, F)) < np.linspace(0.002, 0.6, F)) * rng.integers(1, 300, (n, F))
    dense[rng.random((n, F)) < 0.001] = 0
    nz = dense != 0
    indptr = torch.from_numpy(np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64))
    rr, cc = np.nonzero(nz)
    cnt = torch.from_numpy(dense[rr, cc]).to(dtype)
    scale = torch.from_numpy(rng.uniform(0.5, 2.0, F))
    scale[::17] = 0.0                                       # inactive features
    vc = VectorColumn.tfidf(F, indptr, torch.from_numpy(cc.astype(np.int32)), cnt, scale)
    Q = quantize(vc, max_bins=64, counts=vc.tf_counts, scale=vc.tf_scale)
    assert getattr(Q, "csr_src", None) is not None
    a = RowGroups(Q, bins=4096)
    csr = Q.csr_src
    del Q.csr_src
    b = RowGroups(Q, bins=4096)
    Q.csr_src = csr
    assert a.G == b.G >= 2
    np.testing.assert_array_equal(a.ptr.numpy(), b.ptr.numpy())
    # the entry-major rows: written inside the CSR build, by tree_rg_erow after the CSC build
    assert a.erow is not None and a.em_g0 == b.em_g0
    pa, ga = a.ptr.numpy(), a.gbase.numpy()
    for g in range(a.em_g0, a.G):          # the runs (the alignment padding is never written)
        s0 = ga[g] - a.ebase
        np.testing.assert_array_equal(a.erow.numpy()[s0: s0 + pa[g, -1]], b.erow.numpy()[s0: s0 + pa[g, -1]])
    ea, eb = a.ent.numpy(), b.ent.numpy()
    for g in range(a.G):
        for r in range(0, n, 7):
            s0, s1 = ga[g] + pa[g, r], ga[g] + pa[g, r + 1]
            np.testing.assert_array_equal(np.sort(ea[s0:s1]), np.sort(eb[s0:s1]))


def _csr_vc(dtype, n=3000, F=400, seed=5):
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn

    rng = np.random.default_rng(seed)
    dense = (rng.random((n, F)) < np.linspace(0.002, 0.6, F)) * rng.integers(1, 300, (n, F))
    nz = dense != 0
    indptr = torch.from_numpy(np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64))
    rr, cc = np.nonzero(nz)
    scale = torch.from_numpy(rng.uniform(0.5, 2.0, F))
    scale[::17] = 0.0
    return VectorColumn.tfidf(F, indptr, torch.from_numpy(cc.astype(np.int32)),
                              torch.from_numpy(dense[rr, cc]).to(dtype), scale)


def _csr_vc_wide(n=3000, F=7000, per_row=120, maxc=60, seed=4):
    """Sparse rows over many features with many count values: > 64 row groups of 4096 bins."""
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn

    rng = np.random.default_rng(seed)
    cols = np.sort(np.stack([rng.choice(F, per_row, replace=False) for _ in range(n)]), axis=1)
    cnt = rng.integers(1, maxc, (n, per_row))
    indptr = torch.from_numpy(np.arange(n + 1, dtype=np.int64) * per_row)
    return VectorColumn.tfidf(F, indptr, torch.from_numpy(cols.reshape(-1).astype(np.int32)),
                              torch.from_numpy(cnt.reshape(-1).astype(np.int32)), torch.ones(F, dtype=torch.float64))


def test_row_groups_from_csr_beyond_64_groups():
    """Lanes hold groups l and l + 64 in the CSR build: > 64 groups give the CSC build's layout."""
    vc = _csr_vc_wide()
    Q = quantize(vc, max_bins=64, counts=vc.tf_counts, scale=vc.tf_scale)
    a = RowGroups(Q, bins=4096)
    csr = Q.csr_src
    del Q.csr_src
    b = RowGroups(Q, bins=4096)
    Q.csr_src = csr
    assert a.complete and 64 < a.G == b.G <= 128
    np.testing.assert_array_equal(a.ptr.numpy(), b.ptr.numpy())
    pa, ga, ea, eb = a.ptr.numpy(), a.gbase.numpy(), a.ent.numpy(), b.ent.numpy()
    for g in range(0, a.G, 5):
        for r in range(0, Q.n_rows, 37):
            s0, s1 = ga[g] + pa[g, r], ga[g] + pa[g, r + 1]
            np.testing.assert_array_equal(np.sort(ea[s0:s1]), np.sort(eb[s0:s1]))


@pytest.mark.gpu
def test_gpu_row_groups_from_csr_beyond_64_groups():
    vc = _csr_vc_wide()
    out = []
    for dev in ("cpu", "cuda:0"):
        v = vc.to(dev)
        rg = RowGroups(quantize(v, max_bins=64, counts=v.tf_counts, scale=v.tf_scale), bins=4096)
        ptr, ent, gb = rg.ptr.cpu().numpy(), rg.ent.cpu().numpy(), rg.gbase.cpu().numpy()
        out.append((ptr, np.concatenate([ent[gb[g]: gb[g] + ptr[g, -1]] for g in range(rg.G)]), rg.G))
    assert 64 < out[0][2] == out[1][2]
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.int32])
def test_gpu_row_groups_from_csr_equal_host(dtype):
    """The wave-per-row ballot build on the GPU writes the host twin's layout bit for bit (runs
    in CSR order on both)."""
    vc = _csr_vc(dtype, n=20000, F=600, seed=8)
    out = []
    for dev in ("cpu", "cuda:0"):
        Q = quantize(vc.to(dev), max_bins=64, counts=vc.to(dev).tf_counts, scale=vc.to(dev).tf_scale)
        assert getattr(Q, "csr_src", None) is not None
        rg = RowGroups(Q, bins=4096)
        ptr, ent, gb = rg.ptr.cpu().numpy(), rg.ent.cpu().numpy(), rg.gbase.cpu().numpy()
        # the runs only (the 8-entry alignment padding between groups is never written)
        runs = np.concatenate([ent[gb[g]: gb[g] + ptr[g, -1]] for g in range(rg.G)])
        er = rg.erow.cpu().numpy()
        erow = np.concatenate([er[gb[g] - rg.ebase: gb[g] - rg.ebase + ptr[g, -1]] for g in range(rg.em_g0, rg.G)])
        out.append((ptr, runs, rg.G, erow))
    assert out[0][2] == out[1][2] >= 2
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    np.testing.assert_array_equal(out[0][3], out[1][3])


def test_row_groups_incomplete_beyond_max_groups():
    vc = _wide(2000, 300, 4)
    Q = quantize(vc, max_bins=100, **QKW)
    rg = RowGroups(Q, max_groups=1)
    assert not rg.complete and rg.G == 1


@pytest.mark.parametrize("nslots,root,np_,F,bins", [(1, True, 4, 250, 8192), (2, False, 4, 250, 4096),
                                                     (5, False, 4, 250, 8192), (33, False, 4, 250, 4096),
                                                     (3, False, 1, 250, 8192), (1, True, 4, 40, 8192),
                                                     (4, False, 4, 40, 8192)])
def test_row_group_histograms_equal_host_reference(nslots, root, np_, F, bins):
    """Several groups (F = 250) and a single group (F = 40: the cursor copy must not alias ptr)."""
    rng = np.random.default_rng(nslots)
    n = 5000
    vc = _wide(n, F, nslots)
    row_node = rng.integers(-1, nslots + 1, n).astype(np.int32) if not root else np.zeros(n, np.int32)
    hist, q0, q1, Q, rg = _rg_hist_on("cpu", vc, 100, nslots, row_node, root, np_=np_, bins=bins)
    assert (rg.G >= 2) == (F > 100)
    np.testing.assert_array_equal(hist, _hist_ref(Q, row_node, nslots, q0, q1))


def _list_check(dev, n, ns, seed):
    C = native.lib()
    rng = np.random.default_rng(seed)
    row_node = rng.integers(-1, 2 * ns + 2, n).astype(np.int32)
    node_slot = np.full(2 * ns + 1, -1, dtype=np.int32)
    node_slot[rng.permutation(2 * ns + 1)[:ns]] = np.arange(ns, dtype=np.int32)
    sl = np.where((row_node >= 0) & (row_node < node_slot.size), node_slot[np.clip(row_node, 0, node_slot.size - 1)], -1)
    lst = torch.full((n,), -7, dtype=torch.int32, device=dev)
    start = torch.zeros(ns + 1, dtype=torch.int32, device=dev)
    work = torch.full((ns * (2 + n // native.lib().tree_rg_list_rows(n) + 1),), 99, dtype=torch.int32, device=dev)
    dig = torch.from_numpy(rng.integers(0, 1 << 30, (n, 2)).astype(np.int32)).to(dev)
    ldig = torch.zeros((n, 2), dtype=torch.int32, device=dev)
    C.tree_rg_list(torch.from_numpy(row_node).to(dev), torch.from_numpy(node_slot).to(dev), None, n, ns, work,
                   start, lst, dig, ldig)
    st, lst, ldig = start.cpu().numpy(), lst.cpu().numpy(), ldig.cpu().numpy()
    for s in range(ns):                 # sorted by (slot, row)
        np.testing.assert_array_equal(lst[st[s]:st[s + 1]], np.nonzero(sl == s)[0])
    assert st[0] == 0 and st[-1] == (sl >= 0).sum()
    np.testing.assert_array_equal(ldig[:st[-1]], dig.cpu().numpy()[lst[:st[-1]]])
    # from slot bytes
    slot8 = np.where(sl >= 0, sl, 0xFF).astype(np.uint8)
    lst2 = torch.full((n,), -7, dtype=torch.int32, device=dev)
    C.tree_rg_list(None, None, torch.from_numpy(slot8).to(dev), n, ns, work, start, lst2, None, None)
    np.testing.assert_array_equal(lst2.cpu().numpy()[:st[-1]], lst[:st[-1]])
    return st


@pytest.mark.parametrize("root,np_,bins", [(True, 4, 8192), (False, 4, 8192), (False, 1, 4096), (True, 4, 4096)])
def test_row_group_entry_major_pass_equals_host_reference(root, np_, bins):
    """The entry-major pass of the sparse groups (a lane per entry, its row from erow, the row's
    slot from row_node at a listed level) gives the exact sums of the row-list pass."""
    rng = np.random.default_rng(31)
    n = 6000
    vc = _wide(n, 300, 31, dmax=0.6)
    row_node = np.zeros(n, np.int32) if root else rng.integers(-1, 3, n).astype(np.int32)
    hist, q0, q1, Q, rg = _rg_hist_on("cpu", vc, 100, 1, row_node, root, np_=np_, bins=bins, em=True)
    assert rg.erow is not None and rg.em_g0 < rg.G           # sparse groups take the pass
    np.testing.assert_array_equal(hist, _hist_ref(Q, row_node, 1, q0, q1))
    # erow: the row of every entry of the sparse tail
    ptr, gb, erow = rg.ptr.numpy(), rg.gbase.numpy(), rg.erow.numpy()
    for g in range(rg.em_g0, rg.G):
        want = np.repeat(np.arange(n), np.diff(ptr[g]))
        np.testing.assert_array_equal(erow[gb[g] - rg.ebase: gb[g] - rg.ebase + ptr[g, -1]], want)


def test_row_group_list_groups_built_rows_by_slot():
    _list_check("cpu", 20000, 7, 9)


@pytest.mark.gpu
@pytest.mark.parametrize("n,ns", [(20000, 7), (100003, 1), (300000, 16), (70001, 64)])
def test_gpu_row_group_list_equals_host(n, ns):
    """Ballot-placed lists: every built row once, grouped by slot, slot starts exact."""
    np.testing.assert_array_equal(_list_check("cuda:0", n, ns, n), _list_check("cpu", n, ns, n))


def test_row_group_sharded_layout_equals_plain():
    rng = np.random.default_rng(12)
    n = 4000
    vc = _wide(n, 200, 12)
    row_node = rng.integers(-1, 4, n).astype(np.int32)
    plain, *_ , Q, _ = _rg_hist_on("cpu", vc, 100, 3, row_node)
    lo = np.array([0, Q.TB // 3, (2 * Q.TB) // 3, Q.TB], dtype=np.int64)
    sh, *_ = _rg_hist_on("cpu", vc, 100, 3, row_node, shards=(3, lo))
    np.testing.assert_array_equal(plain, sh)


@pytest.mark.parametrize("depth,hot,bins,em_frac", [(6, 0.2, 8192, 2.0), (3, 0.0, 8192, 2.0), (6, 0.2, 4096, 2.0),
                                                    (6, 0.2, 8192, 0.0)])
def test_row_group_level_loop_grows_the_csc_trees(monkeypatch, depth, hot, bins, em_frac):
    """FDX_ROWHIST=1: every GBDT level's histograms come from the row-group engine; the trees
    equal the CSC / dense passes' trees bit for bit (device level loop, host twins). em_frac 0:
    every single-node level takes the entry-major pass with masked digit words."""
    from fraud_detection_spark_kafka_llm_amd.models import grower, quantize as qmod

    monkeypatch.setattr(qmod, "HOT_DENSITY", hot)
    monkeypatch.setattr(qmod, "RG_BINS", bins)
    monkeypatch.setattr(qmod, "RG_EM_MIN_FRAC", em_frac)
    dense, y = random_counts_matrix(3000, 300, 0.1, 21, max_count=40)
    dense[:, :6] = np.random.default_rng(1).integers(0, 5, (3000, 6))
    vc = vc_from_dense(dense)
    params = GBDTParams(n_estimators=4, max_depth=depth, gamma=0.0, max_bin=64)
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(grower, "ROWHIST", flag)
        out[flag] = fit_gbdt(vc, torch.from_numpy(y), params, device="cpu")
    _same_trees(out[False].trees, out[True].trees)
    assert max(t.num_nodes for t in out[True].trees) > 7


@pytest.mark.gpu
@pytest.mark.parametrize("nslots,root,bins,em", [(1, True, 8192, False), (2, False, 4096, False),
                                                 (5, False, 8192, False), (32, False, 4096, False),
                                                 (1, True, 8192, True), (1, False, 8192, True),
                                                 (1, False, 4096, True)])
@pytest.mark.parametrize("sharded", [False, True])
# (the partial tables run with the layout's own pass modes only: no forced-mode combination)
@pytest.mark.parametrize("mode,part", [(None, False), (0, False), (1, False), (None, True)])
def test_gpu_row_group_histograms_equal_host_bitwise(nslots, root, bins, em, sharded, mode, part, monkeypatch):
    """The row-group pass (LDS int64 atomics, 16-B row-run loads, per-slot flushes; the
    entry-major pass of the sparse groups with ``em``; with ``part`` the workgroups' partial
    tables and their reduction) equals the host's exact int64 sums bit for bit, plain and in the
    shard-major DP layout."""
    rng = np.random.default_rng(20 + nslots)
    n = 30000
    vc = _wide(n, 400, 20 + nslots, hi=300)
    row_node = rng.integers(-1, nslots + 1, n).astype(np.int32) if not root else np.zeros(n, np.int32)
    shards = None
    if sharded:
        Q0 = quantize(vc, max_bins=200, **QKW)
        lo = np.array([0, Q0.TB // 3, (2 * Q0.TB) // 3, Q0.TB], dtype=np.int64)
        shards = (3, lo)
    monkeypatch.setitem(MODE, "gmode", mode)
    a, *_ = _rg_hist_on("cpu", vc, 200, nslots, row_node, root, shards, P=24, bins=bins)
    b, *_ , Q, rg = _rg_hist_on("cuda:0", vc, 200, nslots, row_node, root, shards, P=24, bins=bins, em=em, part=part)
    assert rg.G >= 2
    np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("bins,em_frac", [(8192, 2.0), (4096, 2.0), (8192, 0.0)])
def test_gpu_row_group_level_loop_grows_the_same_trees(monkeypatch, bins, em_frac):
    from fraud_detection_spark_kafka_llm_amd.models import grower, quantize as qmod

    monkeypatch.setattr(qmod, "RG_BINS", bins)
    monkeypatch.setattr(qmod, "RG_EM_MIN_FRAC", em_frac)

    dense, y = random_counts_matrix(9000, 300, 0.1, 61, max_count=40)
    dense[:, :4] = np.random.default_rng(6).integers(0, 9, (9000, 4))
    vc = vc_from_dense(dense)
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(grower, "ROWHIST", flag)
        out[flag] = fit_gbdt(vc, torch.from_numpy(y), GBDTParams(n_estimators=4, max_depth=6, max_bin=64),
                             device="cuda:0").trees
    _same_trees(out[False], out[True])


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_row_group_entry_cap_splits_groups_same_trees(monkeypatch, device):
    """a row group closes before RG_GROUP_MAX_ENTRIES entries (its uint32
    offsets), so a large shard gets more groups instead of raising at 2^31 entries. Forced here to
    a small cap: more groups, the same trees bit for bit."""
    from fraud_detection_spark_kafka_llm_amd.models import quantize as qmod

    dense, y = random_counts_matrix(4000, 300, 0.1, 23, max_count=40)
    dense[:, :6] = np.random.default_rng(3).integers(0, 5, (4000, 6))
    vc = vc_from_dense(dense)
    params = GBDTParams(n_estimators=3, max_depth=5, gamma=0.0, max_bin=64)
    ref = fit_gbdt(vc, torch.from_numpy(y), params, device=device)
    monkeypatch.setattr(qmod, "RG_GROUP_MAX_ENTRIES", 6000)
    capped = fit_gbdt(vc, torch.from_numpy(y), params, device=device)
    _same_trees(ref.trees, capped.trees)
    assert capped.shape["groups"] > ref.shape["groups"] >= 1
    Q = quantize(vc_from_dense(dense), max_bins=64, **QKW)
    rg = RowGroups(Q)
    assert int(rg.group_entries.max()) <= 6000 and rg.G == capped.shape["groups"]
