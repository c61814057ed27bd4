"""Independent oracles for the three trainers (VERDICT r3 "missing" #3).

The engine's other tests compare the device kernels with their C++ host twins, which proves
determinism but not semantics: a wrong gain formula, child rule or leaf formula shared by both
twins would pass them. These tests check whole trees against implementations that share no code
with the engine:

* DecisionTree (reference: /root/reference/fraud_detection_spark.py:59-65, gini, depth 5) against
  ``sklearn.tree.DecisionTreeClassifier(max_depth=5)``: integer features with at most 24
  distinct values (so 32 bins are lossless and every threshold sklearn can pick is one we can),
  predictions equal on a held-out set. Exact gain ties between different partitions are ruled out
  by the data (wide continuous-ish value ranges, thousands of rows per node); a tie would show as
  an arbitrary sklearn choice, and the test checks the training partition first.
* RandomForest (reference :67-74, 100 trees, depth 5, sqrt features, bootstrap) against
  ``sklearn.ensemble.RandomForestClassifier``: held-out accuracy within one point on the same
  TF-IDF features of synthetic dialogues (the random draws differ, so only statistics can agree).
* GBDT (reference :76-83, XGBoost binary:logistic hist) against a NumPy exact-histogram booster
  written here from the XGBoost definitions: Newton gain GL^2/(HL+l) + GR^2/(HR+l) - G^2/(H+l),
  split iff gain > max(gamma, 1e-6) with both children's hessian >= min_child_weight, leaf value
  -eta * G / (H + lambda), ties to the lowest feature then the lowest threshold. The one
  engine-specific rule it shares is the documented fixed-point statistic (fp32 g, h quantised to
  rint(v * 2^k), k = 30 - exponent(max |v|), csrc/tree.h quant_exponent), so that sums are exact
  on both sides; leaf values must then agree to 1e-12 and margins after every round likewise.
"""
import math

import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
from fraud_detection_spark_kafka_llm_amd.ml.tree_model import ensemble_arrays
from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
from fraud_detection_spark_kafka_llm_amd.models.tree import fit_forest
from fraud_detection_spark_kafka_llm_amd.ops.sparse import score_csr

sklearn = pytest.importorskip("sklearn")


def _csr_vc(X: np.ndarray) -> VectorColumn:
    nz = X != 0
    indptr = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64)
    r, c = np.nonzero(nz)
    return VectorColumn(X.shape[1], torch.from_numpy(indptr), torch.from_numpy(c.astype(np.int32)),
                        torch.from_numpy(X[r, c].astype(np.float64)))


def _int_features(n: int, seed: int) -> tuple:
    """Integer features, value ranges of 9..24 distinct values (zero included, some negative so
    that the zero bin sits inside the range), and a noisy non-linear label."""
    rng = np.random.default_rng(seed)
    F = 10
    X = np.zeros((n, F))
    for f in range(F):
        lo = -(f % 4)
        hi = 8 + 2 * f if f < 8 else 12
        vals = rng.integers(lo, hi, n)
        keep = rng.random(n) < (0.55 + 0.04 * f)
        X[:, f] = np.where(keep, vals, 0)
    score = (1.3 * (X[:, 0] > 3) + 0.9 * (X[:, 2] * X[:, 5] > 20) - 0.8 * (X[:, 7] < 2) + 0.05 * X[:, 9]
             + 0.4 * np.sin(X[:, 4]))
    y = (score + rng.normal(0, 0.6, n) > 0.6).astype(np.float32)
    return X, y


DEVICES = ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", DEVICES)
def test_decision_tree_equals_sklearn_on_lossless_integer_features(device):
    """(cuda:0: the default device engines, checked against sklearn directly, not only through the
    bitwise host twin)"""
    from sklearn.tree import DecisionTreeClassifier

    X, y = _int_features(24000, 5)
    tr, te = slice(0, 18000), slice(18000, None)
    assert max(len(np.unique(X[:, f])) for f in range(X.shape[1])) <= 32
    ours = fit_forest(_csr_vc(X[tr]), torch.from_numpy(y[tr]), num_trees=1, max_depth=5, max_bins=32,
                      feature_subset="all", device=device)
    arr = ensemble_arrays(ours.trees, "counts")
    sk = DecisionTreeClassifier(max_depth=5, criterion="gini", random_state=0).fit(X[tr], y[tr])
    for part in (tr, te):
        raw = score_csr(_csr_vc(X[part]), arr).numpy()
        pred = np.argmax(raw, axis=1).astype(np.float32)
        np.testing.assert_array_equal(pred, sk.predict(X[part]))
    # the root split is the same (feature, threshold) too: sklearn's threshold is the midpoint
    t = ours.trees[0]
    assert t.feature[t.root] == sk.tree_.feature[0]
    lo = t.threshold[t.root]
    assert lo <= sk.tree_.threshold[0] < lo + 1


def _tfidf_corpus(n: int, seed: int, F: int = 1 << 14):
    from fraud_detection_spark_kafka_llm_amd.data import synth
    from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH
    from fraud_detection_spark_kafka_llm_amd.ops import text as T

    pt, y = synth.generate(synth.SynthConfig(n=n, seed=seed), device="cpu")
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=F)
    ip, ix, cnt = T.featurize_score(pt, spec, want_csr=True, device="cpu").csr()
    return ip, ix, cnt.to(torch.int32), y.to(torch.float32), F


@pytest.mark.parametrize("device", DEVICES)
def test_random_forest_accuracy_matches_sklearn_within_one_point(device):
    import scipy.sparse as sp
    from sklearn.ensemble import RandomForestClassifier

    ip, ix, cnt, y, F = _tfidf_corpus(4000, 9)
    n = len(y)
    df = np.bincount(ix.numpy(), minlength=F)
    ntr = 2800
    df_tr = np.bincount(ix[: int(ip[ntr])].numpy(), minlength=F)
    idf = torch.from_numpy(np.log((ntr + 1.0) / (df_tr + 1.0)))
    assert df.sum() == ix.numel()

    def part(a, b):
        p = ip[a:b + 1] - ip[a]
        return p, ix[int(ip[a]):int(ip[b])], cnt[int(ip[a]):int(ip[b])]

    p_tr, x_tr, c_tr = part(0, ntr)
    p_te, x_te, c_te = part(ntr, n)
    vtr = VectorColumn.tfidf(F, p_tr, x_tr, c_tr, idf)
    vte = VectorColumn.tfidf(F, p_te, x_te, c_te, idf)
    ours = fit_forest(vtr, y[:ntr], num_trees=100, max_depth=5, max_bins=32, bootstrap=True, feature_subset="sqrt",
                      seed=42, device=device)
    raw = score_csr(vte, ensemble_arrays(ours.trees, "normalized")).numpy()
    acc_ours = float(((raw[:, 1] > raw[:, 0]).astype(np.float32) == y[ntr:].numpy()).mean())

    def csr(p, x, c):
        vals = c.numpy().astype(np.float64) * idf.numpy()[x.numpy()]
        return sp.csr_matrix((vals, x.numpy(), p.numpy()), shape=(len(p) - 1, F))

    sk = RandomForestClassifier(n_estimators=100, max_depth=5, max_features="sqrt", random_state=42, n_jobs=4)
    sk.fit(csr(p_tr, x_tr, c_tr), y[:ntr].numpy())
    acc_sk = float((sk.predict(csr(p_te, x_te, c_te)) == y[ntr:].numpy()).mean())
    assert acc_sk > 0.9
    assert abs(acc_ours - acc_sk) <= 0.01, (acc_ours, acc_sk)


# ----------------------------------------------------------------------------- GBDT oracle
def _quant_exponent(m: float) -> int:
    if not m > 0:
        return 0
    return 30 - math.frexp(m)[1]


def _oracle_tree(Xb, thr_vals, g, h, params, depth_max):
    """One depth-wise tree on exact integer sums; returns (per-row leaf value, list of leaves)."""
    k0 = _quant_exponent(float(np.abs(g.astype(np.float64)).max()))
    k1 = _quant_exponent(float(np.abs(h.astype(np.float64)).max()))
    q0 = np.rint(np.ldexp(g.astype(np.float64), k0)).astype(np.int64)
    q1 = np.rint(np.ldexp(h.astype(np.float64), k1)).astype(np.int64)
    s0, s1 = math.ldexp(1.0, -k0), math.ldexp(1.0, -k1)
    lam, mcw = params.reg_lambda, params.min_child_weight
    n, F = Xb.shape
    node_of = np.zeros(n, dtype=np.int64)
    leaf_value = np.zeros(n)
    nodes = [(0, 0)]        # (node id, depth)
    next_id = 1
    leaves = []
    while nodes:
        nid, d = nodes.pop(0)
        rows = np.nonzero(node_of == nid)[0]
        T0, T1 = int(q0[rows].sum()), int(q1[rows].sum())
        G, H = T0 * s0, T1 * s1
        best = None
        if d < depth_max:
            parent = G * G / (H + lam)
            for f in range(F):
                nb = len(thr_vals[f])
                a0 = np.zeros(nb, dtype=np.int64)
                a1 = np.zeros(nb, dtype=np.int64)
                np.add.at(a0, Xb[rows, f], q0[rows])
                np.add.at(a1, Xb[rows, f], q1[rows])
                l0 = l1 = 0
                for b in range(nb - 1):
                    l0 += int(a0[b])
                    l1 += int(a1[b])
                    L0, L1 = l0 * s0, l1 * s1
                    R0, R1 = (T0 - l0) * s0, (T1 - l1) * s1
                    if L1 < mcw or R1 < mcw:
                        continue
                    gain = L0 * L0 / (L1 + lam) + R0 * R0 / (R1 + lam) - parent
                    if best is None or gain > best[0]:
                        best = (gain, f, b)
        if best is not None and best[0] > max(params.gamma, 1e-6):
            _, f, b = best
            left = rows[Xb[rows, f] <= b]
            right = rows[Xb[rows, f] > b]
            node_of[left], node_of[right] = next_id, next_id + 1
            nodes += [(next_id, d + 1), (next_id + 1, d + 1)]
            next_id += 2
            continue
        w = -G / (H + lam)
        v = params.learning_rate * w
        leaf_value[rows] = v
        leaves.append(v)
    return leaf_value, leaves


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("gamma,mcw", [(0.5, 2.0), (30.0, 40.0)])
def test_gbdt_equals_numpy_exact_histogram_oracle(gamma, mcw, device):
    X, y = _int_features(6000, 11)
    # value -> bin index per feature (sorted distinct values: bin b <=> x <= thr_vals[f][b])
    thr_vals = [np.unique(X[:, f]) for f in range(X.shape[1])]
    Xb = np.stack([np.searchsorted(thr_vals[f], X[:, f]) for f in range(X.shape[1])], 1)
    params = GBDTParams(n_estimators=4, max_depth=3, learning_rate=0.3, reg_lambda=1.0, gamma=gamma,
                        min_child_weight=mcw, max_bin=64)
    ours = fit_gbdt(_csr_vc(X), torch.from_numpy(y), params, device=device)
    if device != "cpu":
        from fraud_detection_spark_kafka_llm_amd.models import grower

        assert grower.ROWHIST           # the default row-group engine ran (not the CSC passes)
    ybar = float(y.astype(np.float64).mean())
    base = math.log(ybar / (1 - ybar))
    assert ours.base_margin == pytest.approx(base, abs=1e-12)
    margin = np.full(len(y), base)
    vc = _csr_vc(X)
    for t, tree in enumerate(ours.trees):
        p = 1.0 / (1.0 + np.exp(-margin))
        g = (p - y.astype(np.float64)).astype(np.float32)
        h = np.maximum(p * (1.0 - p), 1e-16).astype(np.float32)
        ov, leaves = _oracle_tree(Xb, thr_vals, g, h, params, params.max_depth)
        got = score_csr(vc, ensemble_arrays([tree], "value", cmp_less=False))[:, 0].numpy()
        np.testing.assert_allclose(got, ov, rtol=0, atol=1e-12, err_msg=f"tree {t}")
        ours_leaves = sorted(float(tree.stats[i, 0]) for i in range(tree.num_nodes) if tree.feature[i] < 0)
        np.testing.assert_allclose(ours_leaves, sorted(leaves), rtol=0, atol=1e-12)
        margin = margin + ov
    assert len(ours.trees) == params.n_estimators
