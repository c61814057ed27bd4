"""Consumer-group streaming (stream/group.py): client processes with shared-memory slot rings
around one scoring process. Every record of every partition is classified exactly like the
single-process engine, produced once and committed (reference loop: /root/reference/app_ui.py:196-226)."""
import json

import numpy as np
import pytest

from fraud_detection_spark_kafka_llm_amd.data import synth
from fraud_detection_spark_kafka_llm_amd.ops.text import PackedText, featurize_score
from fraud_detection_spark_kafka_llm_amd.serve.agent import ClassificationAgent
from fraud_detection_spark_kafka_llm_amd.serve.llm import StubLLM
from fraud_detection_spark_kafka_llm_amd.stream import group as G
from fraud_detection_spark_kafka_llm_amd.stream.gpu_worker import make_scorer
from fraud_detection_spark_kafka_llm_amd.stream.loadgen import MessagePool


@pytest.fixture(scope="module")
def agent(tmp_path_factory):
    """A small HashingTF -> IDF -> LogisticRegression pipeline trained on synthetic dialogues
    (self-contained: the GPU box has no /root/reference)."""
    from fraud_detection_spark_kafka_llm_amd.ml import (IDF, Frame, HashingTF, LogisticRegression, Pipeline,
                                                         StopWordsRemover, TextColumn, Tokenizer)

    pt, y = synth.generate(synth.SynthConfig(n=600, seed=21))
    raw = TextColumn(pt.strings())
    df = Frame({"dialogue": raw, "clean_text": TextColumn.cleaned_from(raw), "labels": y.numpy()})
    model = Pipeline(stages=[Tokenizer(inputCol="clean_text", outputCol="words"),
                             StopWordsRemover(inputCol="words", outputCol="filtered_words"),
                             HashingTF(inputCol="filtered_words", outputCol="raw_features", numFeatures=1 << 18),
                             IDF(inputCol="raw_features", outputCol="features"),
                             LogisticRegression(featuresCol="features", labelCol="labels", maxIter=10)]).fit(df)
    path = tmp_path_factory.mktemp("group") / "model"
    model.save(str(path))
    return ClassificationAgent(str(path), llm=StubLLM(), device="cpu")


def _expected(agent, texts):
    fp = agent.fused
    idf = fp.idf.idf if fp.idf is not None else None
    import torch
    res = featurize_score(PackedText.from_strings(texts), fp.spec(True),
                          idf=torch.as_tensor(np.asarray(idf)) if idf is not None else None,
                          lr=fp.model.scorer(), device="cpu")
    return fp.model.postprocess_numpy(res.raw.numpy())


@pytest.mark.parametrize("confluent", [True, False])
def test_group_throughput_all_records_scored_once(agent, confluent):
    pt, _ = synth.generate(synth.SynthConfig(n=500, seed=5), device="cpu")
    texts = pt.strings()
    pool = MessagePool(texts)
    fp = agent.fused
    sc = make_scorer(fp.spec(True), fp.idf.idf if fp.idf is not None else None, fp.model.scorer(), "cpu",
                     max_docs=256, max_bytes=256 * 4096, depth=2)
    n = 1700                       # wraps the pool; 3 partitions of uneven size
    with G.ConsumerGroup(sc, fp.model.postprocess_numpy, 3, batch_max=256, max_latency_ms=2.0,
                         max_bytes=256 * 4096, pool=pool, confluent=confluent) as grp:
        r = G.group_throughput_run(grp, n, return_outputs=True)
        r2 = G.group_throughput_run(grp, 300)          # the clients serve several runs
    assert r["messages"] == r["produced"] == r["committed"] == n
    assert r2["produced"] == r2["committed"] == 300
    pred, p1 = _expected(agent, texts)
    from collections import Counter
    want, got = Counter(), Counter()
    for c in range(3):
        share = n // 3 + (1 if c < n % 3 else 0)
        want.update((c * 7919 + j) % pool.n for j in range(share))
    for outs in r["outputs"]:
        for key, val in outs:       # output partitions come from the producer's partitioner
            i = int(key.decode()[3:])
            rec = json.loads(val)
            assert rec["original_text"] == texts[i]
            assert rec["prediction"] == float(pred[i]) and rec["confidence"] == float(p1[i])
            got[i] += 1
    assert got == want
    assert r["p50_ms"] > 0


def test_group_latency_run(agent):
    pt, _ = synth.generate(synth.SynthConfig(n=200, seed=6), device="cpu")
    pool = MessagePool(pt.strings())
    fp = agent.fused
    sc = make_scorer(fp.spec(True), fp.idf.idf, fp.model.scorer(), "cpu", max_docs=128, max_bytes=128 * 4096)
    with G.ConsumerGroup(sc, fp.model.postprocess_numpy, 2, batch_max=128, max_latency_ms=1.0,
                         max_bytes=128 * 4096, pool=pool) as grp:
        r = G.group_latency_run(grp, rate=4000, duration_s=0.5, warmup_s=0.1)
    assert r["sent"] > 0 and r["produced"] == r["sent"] == r["committed"]
    assert 0 < r["p50_ms"] <= r["p95_ms"]


def test_group_async_explanations(agent):
    """Config 5's LLM-explain stub in the client processes: every 5th classification gets an
    explanation record; classifications are produced and committed as without it."""
    pt, _ = synth.generate(synth.SynthConfig(n=200, seed=7), device="cpu")
    pool = MessagePool(pt.strings())
    fp = agent.fused
    sc = make_scorer(fp.spec(True), fp.idf.idf, fp.model.scorer(), "cpu", max_docs=128, max_bytes=128 * 4096)
    with G.ConsumerGroup(sc, fp.model.postprocess_numpy, 2, batch_max=128, max_latency_ms=1.0,
                         max_bytes=128 * 4096, pool=pool) as grp:
        r = G.group_throughput_run(grp, 1000, explain="async", explain_every=5, return_outputs=True)
    assert r["produced"] == r["committed"] == 1000
    assert r["explanations"] == 200
    recs = [json.loads(v) for outs in r["outputs"] for _, v in outs]
    expl = [x for x in recs if x.get("type") == "explanation"]
    assert len(expl) == 200 and all("stub-llm" in x["analysis"] for x in expl)
    assert len(recs) - len(expl) == 1000


def test_client_failure_surfaces(agent):
    fp = agent.fused
    sc = make_scorer(fp.spec(True), fp.idf.idf, fp.model.scorer(), "cpu", max_docs=64, max_bytes=64 * 4096)
    with G.ConsumerGroup(sc, fp.model.postprocess_numpy, 1, batch_max=64, max_bytes=64 * 4096) as grp:
        with pytest.raises(RuntimeError, match="client 0 failed"):
            grp.run({"kind": "throughput", "tag": "x", "n": 10})      # no pool shared: the client raises


def test_slot_layout_page_aligned():
    lay = G.slot_layout(5, 1000, 1 << 20)
    assert lay["stride"] % 4096 == 0 and lay["size"] == 5 * lay["stride"]
    assert lay["data"] >= (1 << 20) and lay["res"] >= 1000 * 16


@pytest.mark.gpu
def test_group_gpu_scorer_registered_slots(agent):
    """The GPU process page-locks the clients' segments and DMAs from them: same records as the host."""
    import torch
    pt, _ = synth.generate(synth.SynthConfig(n=400, seed=8), device="cpu")
    texts = pt.strings()
    pool = MessagePool(texts)
    fp = agent.fused
    sc = make_scorer(fp.spec(True), fp.idf.idf, fp.model.scorer(), torch.device("cuda", 0), max_docs=512,
                     max_bytes=512 * 4096, depth=3)
    with G.ConsumerGroup(sc, fp.model.postprocess_numpy, 3, batch_max=512, max_latency_ms=2.0,
                         max_bytes=512 * 4096, pool=pool) as grp:
        assert grp.register
        r = G.group_throughput_run(grp, 3000, return_outputs=True)
    assert r["produced"] == r["committed"] == 3000
    pred, p1 = _expected(agent, texts)
    n = 0
    for outs in r["outputs"]:
        for key, val in outs:
            i = int(key.decode()[3:])
            rec = json.loads(val)
            assert rec["prediction"] == float(pred[i])
            assert abs(rec["confidence"] - float(p1[i])) <= 1e-12
            n += 1
    assert n == 3000


def _group_rank(rank, world, model_path, n, device="cpu"):
    """One rank of a multi-process scoring group: rank 0 coordinates (segments, clients, its own
    scorer), every other rank is a ScorerPeer on its own device."""
    import torch

    agent = ClassificationAgent(model_path, llm=StubLLM(), device="cpu")
    fp = agent.fused
    dev = torch.device(device)
    sc = make_scorer(fp.spec(True), fp.idf.idf, fp.model.scorer(), dev, max_docs=256, max_bytes=256 * 4096,
                     depth=2)
    rdv = G.GroupRendezvous.from_process_group("test-multi")
    if rank == 0:
        pt, _ = synth.generate(synth.SynthConfig(n=400, seed=12), device="cpu")
        pool = MessagePool(pt.strings())
        with G.ConsumerGroup(sc, fp.model.postprocess_numpy, 3, batch_max=256, max_latency_ms=2.0,
                             max_bytes=256 * 4096, pool=pool, confluent=False, rendezvous=rdv) as grp:
            assert grp.n_scorers == world
            r = G.group_throughput_run(grp, n, return_outputs=True)
            local = grp.local_batches
        outs = [(k, v) for o in r.pop("outputs") for k, v in o]
        return {"run": r, "local_batches": local, "outputs": outs, "texts": pt.strings()}
    with G.ScorerPeer(sc, fp.model.postprocess_numpy, rdv) as peer:
        return {"peer": peer.serve()}


def test_group_scores_on_every_rank_process(agent, tmp_path):
    """BASELINE config 5 topology: one 3-partition topic, a scoring process per rank (rank 0 the
    coordinator, rank 1 a ScorerPeer), each with its own scorer; every record scored once,
    produced and committed, and both processes scored micro-batches."""
    from fraud_detection_spark_kafka_llm_amd.parallel.launch import spawn

    path = tmp_path / "model"
    agent.model.save(str(path))
    n = 6000
    r0, r1 = spawn(_group_rank, 2, str(path), n, backend="gloo")
    run = r0["run"]
    assert run["messages"] == run["produced"] == run["committed"] == n
    assert len(run["scorer_batches"]) == 2 and min(run["scorer_batches"]) > 0
    assert r1["peer"]["batches"] == run["scorer_batches"][1] > 0
    assert r0["local_batches"] == run["scorer_batches"][0]
    texts = r0["texts"]
    pred, p1 = _expected(agent, texts)
    for key, val in r0["outputs"]:
        i = int(key.decode()[3:])
        rec = json.loads(val)
        assert rec["prediction"] == float(pred[i]) and rec["confidence"] == float(p1[i])
    assert len(r0["outputs"]) == n


@pytest.mark.gpu
def test_gpu_group_two_rank_processes_share_the_topic(agent, tmp_path):
    """Two rank processes scoring one shared topic on the GPU (both on cuda:0 on a 1-GPU box: each
    page-locks the clients' segments for its own context)."""
    from fraud_detection_spark_kafka_llm_amd.parallel.launch import spawn

    path = tmp_path / "model"
    agent.model.save(str(path))
    n = 20000
    r0, r1 = spawn(_group_rank, 2, str(path), n, "cuda:0", backend="gloo")
    run = r0["run"]
    assert run["messages"] == run["produced"] == run["committed"] == n
    assert min(run["scorer_batches"]) > 0 and r1["peer"]["batches"] == run["scorer_batches"][1]
    pred, p1 = _expected(agent, r0["texts"])
    for key, val in r0["outputs"]:
        i = int(key.decode()[3:])
        rec = json.loads(val)
        assert rec["prediction"] == float(pred[i]) and abs(rec["confidence"] - float(p1[i])) <= 1e-12


def _group_rank_peer_fails(rank, world, model_path):
    """Rank 1's ScorerPeer fails while mapping the segments: it publishes the error, so rank 0's
    ConsumerGroup fails at once (not at the rendezvous timeout) and releases everything."""
    import time

    import torch

    agent = ClassificationAgent(model_path, llm=StubLLM(), device="cpu")
    fp = agent.fused
    sc = make_scorer(fp.spec(True), fp.idf.idf, fp.model.scorer(), torch.device("cpu"), max_docs=64,
                     max_bytes=64 * 4096, depth=2)
    rdv = G.GroupRendezvous.from_process_group("test-fail", timeout_s=300.0)
    t0 = time.perf_counter()
    if rank == 0:
        try:
            with G.ConsumerGroup(sc, fp.model.postprocess_numpy, 2, batch_max=64, max_bytes=64 * 4096,
                                 confluent=False, rendezvous=rdv):
                return {"error": None}
        except RuntimeError as e:
            return {"error": str(e), "sec": time.perf_counter() - t0}

    def boom(name):
        raise OSError("injected attach failure")

    G._attach = boom
    try:
        G.ScorerPeer(sc, fp.model.postprocess_numpy, rdv)
    except OSError as e:
        return {"peer_error": str(e)}
    return {"peer_error": None}


def test_group_peer_start_failure_fails_fast(agent, tmp_path):
    """a peer that fails before publishing its socket no longer stalls the coordinator
    for the whole rendezvous timeout."""
    from fraud_detection_spark_kafka_llm_amd.parallel.launch import spawn

    path = tmp_path / "model"
    agent.model.save(str(path))
    r0, r1 = spawn(_group_rank_peer_fails, 2, str(path), backend="gloo")
    assert r1["peer_error"] == "injected attach failure"
    assert "failed to start" in r0["error"] and "injected attach failure" in r0["error"]
    assert r0["sec"] < 60


def test_single_host_group_check(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert G.single_host_group()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert not G.single_host_group()


def test_client_cpu_plan_gives_each_client_its_own_cpus():
    """client processes get CPUs of their own, disjoint from the scoring
    process's (which keeps at least as many); too few CPUs: no pinning."""
    from fraud_detection_spark_kafka_llm_amd.stream.group import client_cpu_plan

    alone = lambda c: (c,)                      # noqa: E731 (no SMT)
    plan, mine = client_cpu_plan(list(range(16)), 3, per_client=2, siblings=alone, shared=False)
    assert plan == [[10, 11], [12, 13], [14, 15]] and mine == list(range(10))
    flat = [c for p in plan for c in p]
    assert not set(flat) & set(mine) and len(set(flat)) == 6
    assert client_cpu_plan(list(range(8)), 3, per_client=2, siblings=alone, shared=False) == (None, None)
    # SMT: cpu c and c + 16 share a core; a client takes whole cores, the scorer none of them
    smt = lambda c: (c % 16, c % 16 + 16)       # noqa: E731
    plan, mine = client_cpu_plan(list(range(32)), 3, per_client=2, siblings=smt, shared=False)
    assert plan == [[10, 11, 26, 27], [12, 13, 28, 29], [14, 15, 30, 31]]
    assert mine == list(range(10)) + list(range(16, 26))
    # siblings outside the allowed set are ignored
    plan, mine = client_cpu_plan(list(range(16)), 3, per_client=2, siblings=smt, shared=False)
    assert plan == [[10, 11], [12, 13], [14, 15]]
    # shared: every client on the pooled cores
    plan, mine = client_cpu_plan(list(range(16)), 3, per_client=2, siblings=alone, shared=True)
    assert plan == [list(range(10, 16))] * 3 and mine == list(range(10))
    # shared on a machine too small for per_client cores each: fewer each, the scorer keeps half
    plan, mine = client_cpu_plan(list(range(16)), 3, per_client=8, siblings=alone, shared=True)
    assert plan == [list(range(10, 16))] * 3 and mine == list(range(10))
    assert client_cpu_plan(list(range(4)), 3, per_client=8, siblings=alone, shared=True) == (None, None)
    from fraud_detection_spark_kafka_llm_amd.stream.group import cpu_list_str
    assert cpu_list_str([129, 0, 1, 2, 5, 128]) == "0-2,5,128-129" and cpu_list_str([]) == ""
