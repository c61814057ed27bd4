"""Dialogues over 64 KB stay on the device: cut into segments at "<letter><space>", featurized per
segment, merged and scored (ops/longdoc.py). Host-side checks of the cut rule; on the GPU a 1 MB
dialogue must score bitwise equal to the host featurizer."""
import numpy as np
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ops.longdoc import split_points
from fraud_detection_spark_kafka_llm_amd.ops.text import FeatureSpec, LinearScorer, PackedText, featurize_score


def _doc(n_words, seed=0):
    rng = np.random.default_rng(seed)
    words = ["Bank", "verify", "ACCOUNT", "please", "hello", "prize!", "meeting", "doctor.", "a", "the", "123",
             "call-me", "", "  ", "ssn:", "\n", "Innocent:", "Suspect:", "wire", "transfer"]
    return " ".join(rng.choice(words, n_words))


def _counts(texts, spec):
    res = featurize_score(PackedText.from_strings(texts), spec, want_csr=True, device="cpu")
    ip, ix, v = res.csr()
    out = []
    for i in range(len(texts)):
        a, b = int(ip[i]), int(ip[i + 1])
        out.append(dict(zip(ix[a:b].tolist(), v[a:b].tolist())))
    return out


@pytest.mark.parametrize("clean", [True, False])
def test_segment_counts_sum_to_whole_document(clean):
    spec = FeatureSpec(clean=clean, stopwords=["the", "a"], num_features=1 << 12)
    doc = _doc(3000, seed=1) + "   "
    raw = doc.encode()
    buf = np.frombuffer(raw, dtype=np.uint8)
    b = split_points(buf, 0, len(raw), seg=300)
    assert b is not None and b[0] == 0 and b[-1] == len(raw) and np.all(np.diff(b) <= 300)
    for c in b[1:-1]:                 # every cut follows "<letter><space>"
        assert raw[c - 1] == 0x20 and chr(raw[c - 2]).isalpha()
    segs = [raw[b[i]:b[i + 1]].decode() for i in range(len(b) - 1)]
    whole = _counts([doc], spec)[0]
    merged: dict = {}
    for c in _counts(segs, spec):
        for k, v in c.items():
            merged[k] = merged.get(k, 0.0) + v
    assert merged == whole


def test_no_cut_inside_a_giant_word():
    buf = np.frombuffer(b"x" * 5000, dtype=np.uint8)
    assert split_points(buf, 0, 5000, seg=1000) is None
    assert split_points(buf, 0, 800, seg=1000).tolist() == [0, 800]


@pytest.mark.gpu
@pytest.mark.parametrize("clean", [True, False])
def test_gpu_one_megabyte_dialogue_bitwise_equals_host(clean):
    from fraud_detection_spark_kafka_llm_amd.ml.tree_model import Tree, ensemble_arrays
    from fraud_detection_spark_kafka_llm_amd.stream.gpu_worker import GpuScorer, HostScorer
    from fraud_detection_spark_kafka_llm_amd.stream.ring import PinnedRing

    F = 1 << 14
    rng = np.random.default_rng(5)
    spec = FeatureSpec(clean=clean, stopwords=["the", "a"], num_features=F)
    big = _doc(160000, seed=3)                        # ~1 MB
    assert len(big.encode()) > 900_000
    docs = [big, "short dialogue here", _doc(9000, seed=4), _doc(20000, seed=6)]   # 1 MB, tiny, ~50 KB, ~110 KB
    idf = rng.random(F)
    lr = LinearScorer(rng.standard_normal(F), -0.25)
    # featurize_score on the device (LR) equals the host featurizer bitwise
    g = featurize_score(PackedText.from_strings(docs), spec, idf=torch.from_numpy(idf), lr=lr, want_csr=True,
                        device="cuda:0", fix_fallbacks=False)
    assert torch.all(g.status.cpu() == 0), "every dialogue scored on the device"
    h = featurize_score(PackedText.from_strings(docs), spec, idf=torch.from_numpy(idf), lr=lr, want_csr=True,
                        device="cpu")
    assert torch.equal(g.raw.cpu(), h.raw)
    gi, gx, gv = (t.cpu() for t in g.csr())
    hi, hx, hv = h.csr()
    assert torch.equal(gi, hi) and torch.equal(gx, hx) and torch.equal(gv, hv)
    # streaming scorer (trees) on a pinned slot
    feat = rng.integers(0, F, 15).astype(np.int32)
    tree = Tree(np.concatenate([feat[:7], -np.ones(8, np.int32)]), np.concatenate([rng.random(7) * 3, np.zeros(8)]),
                np.concatenate([np.arange(1, 15, 2), -np.ones(8, np.int64)]).astype(np.int32),
                np.concatenate([np.arange(2, 16, 2), -np.ones(8, np.int64)]).astype(np.int32),
                np.stack([rng.standard_normal(15), np.ones(15)], 1), np.zeros(15), np.zeros(15),
                np.zeros(15, np.int64), rng.standard_normal(15), 0)
    trees = ensemble_arrays([tree] * 3, "value")
    ring = PinnedRing(slots=1, max_docs=8, max_bytes=2 << 20)
    ring.slots[0].fill(docs)
    gpu = GpuScorer(spec, idf, trees, "cuda:0", max_docs=8, max_bytes=2 << 20)
    host = HostScorer(spec, idf, trees, max_docs=8, max_bytes=2 << 20)
    gpu.submit(ring.slots[0])
    assert gpu._inflight[0].very_long is not None and gpu._inflight[0].very_long[0].tolist() == [0, 3]
    _, graw = gpu.collect()
    np.testing.assert_array_equal(graw, host.score_packed(ring.slots[0]))
