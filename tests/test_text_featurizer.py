"""Featurizer numerics: pure-Python oracle vs native host path vs gfx950 kernel."""
import random

import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.data import fixtures
from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH
from fraud_detection_spark_kafka_llm_amd.ops import oracle as O
from fraud_detection_spark_kafka_llm_amd.ops import text as T

EDGE = ["", " ", "   ", "a", " a", "a ", "  a  b  ", "a\tb\nc", "don't stop", "İstanbul KELVIN K x",
        "UPPER lower MiXeD", "123 456 !!! ...", "été café \U0001F600 emoji", "the and of a an",
        "x" * 40, ("word " * 300).strip(), "ab  " * 50, fixtures.SCAM_SAMPLE, fixtures.BENIGN_SAMPLE]


def random_docs(n, seed=0, max_words=80):
    rng = random.Random(seed)
    vocab = ["hello", "the", "Suspect:", "Innocent:", "verify", "your", "social", "security", "number", "I'm",
             "please", "account", "Bank", "prize", "don't", "it's", "a", "and", "", "OK.", "x1", "café"]
    seps = [" ", " ", " ", "  ", "\n", "\t", ". ", ", "]
    out = []
    for _ in range(n):
        k = rng.randint(0, max_words)
        s = "".join(rng.choice(vocab) + rng.choice(seps) for _ in range(k))
        if rng.random() < 0.3:
            s = s.strip()
        out.append(s)
    return out


def csr_rows(res):
    ip, ix, v = res.csr()
    ip, ix, v = ip.cpu().numpy(), ix.cpu().numpy(), v.cpu().numpy()
    return [{int(a): float(b) for a, b in zip(ix[ip[i]:ip[i + 1]], v[ip[i]:ip[i + 1]])} for i in range(len(ip) - 1)]


def test_murmur_buckets():
    for w, b in fixtures.BUCKETS_10000.items():
        assert O.term_index(w, 10000) == b
    assert O.term_index("", 1 << 18) == 249180


def test_java_split_semantics():
    assert O.java_split_ws("") == [""]
    assert O.java_split_ws(" ") == []
    assert O.java_split_ws(" a") == ["", "a"]
    assert O.java_split_ws("a  b ") == ["a", "", "b"]
    assert O.java_split_ws("a\tb") == ["a", "b"]


def test_clean_text_rules():
    assert O.clean_text("Don't STOP-now 42\n!") == "dont stopnow "
    assert O.clean_text("İx K") == "ix k"


@pytest.mark.parametrize("clean", [True, False])
@pytest.mark.parametrize("stop", [True, False])
def test_native_cpu_matches_oracle(clean, stop):
    docs = EDGE + random_docs(300, seed=1)
    sw = list(ENGLISH) if stop else None
    spec = T.FeatureSpec(clean=clean, stopwords=sw, num_features=10007)
    res = T.featurize_score(T.PackedText.from_strings(docs), spec, want_csr=True, device="cpu")
    got = csr_rows(res)
    for d, g in zip(docs, got):
        s = O.clean_text(d) if clean else d
        toks = O.tokenize(s)
        if sw:
            toks = O.remove_stopwords(toks, sw)
        assert g == O.hashing_tf(toks, 10007), repr(d)[:80]


# the densest possible documents for the CSR scratch bound (csrc/scoring.h csr_slot: at most
# L / 2 + 2 distinct terms per L-byte document): distinct one-character tokens, a leading empty
# token, every parity of start offset
DENSE = ["".join(chr(c) + " " for c in range(33, 127)), " " + " ".join(chr(c) for c in range(33, 127)),
         "x", "", "a b", " " * 7 + "q", "\u00e9 \u00e8 \u00ea \u00eb \u00e0 " * 3]


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_densest_documents_fit_the_csr_scratch(device):
    docs = [d for k in range(3) for d in (DENSE[k % len(DENSE):] + DENSE[:k % len(DENSE)] + ["y" * (k + 1)])]
    spec = T.FeatureSpec(clean=False, stopwords=None, num_features=1 << 18)
    res = T.featurize_score(T.PackedText.from_strings(docs), spec, want_csr=True, device=device)
    got = csr_rows(res)
    for d, g in zip(docs, got):
        want = O.hashing_tf(O.tokenize(d), 1 << 18)
        assert g == want, repr(d)[:60]
        assert len(want) <= len(d.encode()) // 2 + 2


def test_vocab_mode_and_min_tf():
    docs = random_docs(200, seed=2)
    vocab = ["hello", "verify", "social", "security", "im", "dont", "please", "bank"]
    for min_tf in (1.0, 2.0, 0.1):
        spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), vocab=vocab, min_tf=min_tf)
        got = csr_rows(T.featurize_score(T.PackedText.from_strings(docs), spec, want_csr=True, device="cpu"))
        for d, g in zip(docs, got):
            toks = O.remove_stopwords(O.tokenize(O.clean_text(d)), ENGLISH)
            assert g == O.count_vectorize(toks, vocab, min_tf), d


def test_binary_and_idf_scaling():
    docs = random_docs(50, seed=3)
    idf = np.random.default_rng(0).random(997)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=997, binary=True)
    got = csr_rows(T.featurize_score(T.PackedText.from_strings(docs), spec, idf=torch.from_numpy(idf),
                                     want_csr=True, device="cpu"))
    for d, g in zip(docs, got):
        toks = O.remove_stopwords(O.tokenize(O.clean_text(d)), ENGLISH)
        ref = {k: np.float32(v * idf[k]) for k, v in O.hashing_tf(toks, 997, binary=True).items()}
        assert g == pytest.approx({k: float(v) for k, v in ref.items()})


def test_lr_margin_matches_oracle():
    docs = random_docs(100, seed=4)
    rng = np.random.default_rng(1)
    w = rng.normal(size=1000)
    idf = rng.random(1000)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=1000)
    res = T.featurize_score(T.PackedText.from_strings(docs), spec, idf=torch.from_numpy(idf),
                            lr=T.LinearScorer(w, 0.25), device="cpu")
    for d, m in zip(docs, res.raw[:, 0].numpy()):
        x = O.pipeline_vector(d, ENGLISH, 1000, idf)
        assert m == pytest.approx(O.lr_margin(x, w, 0.25), rel=1e-12, abs=1e-12)


def random_forest_arrays(num_trees, num_features, depth, K, seed=0, cmp_less=False):
    rng = np.random.default_rng(seed)
    feat, thr, left, right, leaf, roots = [], [], [], [], [], []

    def build(d):
        i = len(feat)
        feat.append(-1); thr.append(0.0); left.append(-1); right.append(-1)
        leaf.append(rng.random(K).tolist())
        if d < depth and rng.random() < 0.85:
            feat[i] = int(rng.integers(0, num_features))
            thr[i] = float(rng.choice([0.0, 0.5, 1.5, 2.5, 3.7]))
            left[i] = build(d + 1)
            right[i] = build(d + 1)
        return i

    for _ in range(num_trees):
        roots.append(build(0))
    return T.TreeArrays(feat, thr, left, right, np.asarray(leaf), roots, rng.random(num_trees), K, cmp_less)


def host_tree_score(arrs, x, cmp_less):
    out = np.zeros(arrs.K)
    for t, r in enumerate(arrs.roots):
        i = r
        while arrs.feat[i] >= 0:
            v = x.get(int(arrs.feat[i]), 0.0)
            i = arrs.left[i] if (v < arrs.thr[i] if cmp_less else v <= arrs.thr[i]) else arrs.right[i]
        out += arrs.tree_weights[t] * arrs.leaf[i * arrs.K:(i + 1) * arrs.K]
    return out


@pytest.mark.parametrize("cmp_less", [False, True])
def test_tree_scoring_matches_oracle(cmp_less):
    docs = random_docs(60, seed=5)
    arrs = random_forest_arrays(70, 64, 5, 2, seed=2, cmp_less=cmp_less)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=64)
    res = T.featurize_score(T.PackedText.from_strings(docs), spec, trees=arrs, device="cpu")
    for d, r in zip(docs, res.raw.numpy()):
        x = O.pipeline_vector(d, ENGLISH, 64)
        np.testing.assert_allclose(r, host_tree_score(arrs, x, cmp_less), rtol=1e-12)


# ------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("clean", [True, False])
def test_gpu_kernel_bitwise_equals_host(clean):
    docs = EDGE + random_docs(3000, seed=7, max_words=400)
    spec = T.FeatureSpec(clean=clean, stopwords=list(ENGLISH), num_features=1 << 18)
    pt = T.PackedText.from_strings(docs)
    idf = torch.rand(1 << 18, dtype=torch.float64)
    w = torch.randn(1 << 18, dtype=torch.float64)
    lr = T.LinearScorer(w.numpy(), -0.5)
    cpu = T.featurize_score(pt, spec, idf=idf, lr=lr, want_csr=True, device="cpu")
    gpu = T.featurize_score(pt, spec, idf=idf, lr=lr, want_csr=True, device="cuda:0")
    assert torch.equal(cpu.status, gpu.status.cpu())
    assert torch.equal(cpu.nnz, gpu.nnz.cpu())
    for a, b in zip(cpu.csr(), gpu.csr()):
        assert torch.equal(a, b.cpu())
    assert torch.equal(cpu.raw, gpu.raw.cpu())   # same fp64 summation order, no FMA


@pytest.mark.gpu
def test_gpu_tree_scoring_bitwise():
    docs = random_docs(2000, seed=8, max_words=200)
    arrs = random_forest_arrays(130, 4096, 6, 2, seed=3)
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=4096)
    pt = T.PackedText.from_strings(docs)
    cpu = T.featurize_score(pt, spec, trees=arrs, device="cpu")
    gpu = T.featurize_score(pt, spec, trees=arrs, device="cuda:0")
    assert torch.equal(cpu.raw, gpu.raw.cpu())


@pytest.mark.gpu
def test_gpu_vocab_mode():
    docs = random_docs(500, seed=9)
    vocab = ["hello", "verify", "social", "security", "im", "dont", "please", "bank", "prize"]
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), vocab=vocab, min_tf=2.0)
    pt = T.PackedText.from_strings(docs)
    cpu = T.featurize_score(pt, spec, want_csr=True, device="cpu")
    gpu = T.featurize_score(pt, spec, want_csr=True, device="cuda:0")
    for a, b in zip(cpu.csr(), gpu.csr()):
        assert torch.equal(a, b.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("scorer", ["lr", "trees"])
def test_gpu_long_dialogues_stay_on_device_and_match_host(scorer):
    """Dialogues over the streaming kernel's 4 KB capacity run on the long-dialogue kernel (64 KB,
    16K tokens); only larger ones reach the host path. Results are bitwise equal to the host."""
    rng = np.random.default_rng(3)
    words = ["bank", "verify", "account", "please", "the", "hello", "prize", "ssn", "x", "zebra"]
    docs = ["word " * 2000,                                   # 10 KB
            "a " * 3000,                                      # 1 token x 3000 (token cap, short text)
            " ".join(rng.choice(words, 6000)),                # ~33 KB
            " ".join(f"w{i}" for i in range(9000)),           # 9000 distinct tokens
            "z" * 70000,                                      # > 64 KB -> host
            fixtures.SCAM_SAMPLE] + random_docs(300, seed=4)
    pt = T.PackedText.from_strings(docs)
    F = 1 << 14
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=F)
    idf = torch.rand(F, dtype=torch.float64)
    kw = dict(idf=idf)
    if scorer == "lr":
        kw["lr"] = T.LinearScorer(torch.randn(F, dtype=torch.float64).numpy(), 0.25)
    else:
        kw["trees"] = random_forest_arrays(40, F, 6, 2, seed=5)
    cpu = T.featurize_score(pt, spec, want_csr=True, device="cpu", **kw)
    gpu = T.featurize_score(pt, spec, want_csr=True, device="cuda:0", fix_fallbacks=False, **kw)
    st = gpu.status.cpu()
    assert st[:4].eq(T.STATUS_OK).all() and st[4] == T.STATUS_TOO_LONG   # only the 70 KB one left
    gpu = T.featurize_score(pt, spec, want_csr=True, device="cuda:0", **kw)
    assert torch.equal(cpu.nnz, gpu.nnz.cpu())
    for a, b in zip(cpu.csr(), gpu.csr()):
        assert torch.equal(a, b.cpu())
    assert torch.equal(cpu.raw, gpu.raw.cpu())
