"""bench.py output contract (one JSON line from rank 0 with the driver's required keys), at N=1 and
at N=2 ranks sharing one GPU over gloo (rehearses the multi-rank path: reduce-scatter histograms,
all-gathered splits, per-rank streaming, max-over-ranks timing)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
TINY = ["--steps", "4", "--warmup", "2", "--rows", "100000", "--trees", "3", "--batch", "4096", "--pool", "2",
        "--rf-trees", "4", "--kafka-msgs", "20000", "--kafka-sec", "0.5", "--kafka-multi-msgs", "20000",
        "--kafka-confluent-msgs", "5000", "--kafka-confluent-rate", "5000", "--kafka-group-msgs", "20000",
        "--kafka-group-rate", "6000"]


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _check(rec: dict, n: int):
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == n and rec["steps"] == 4 and rec["warmup"] == 2
    assert rec["value"] > 0 and rec["ms_per_step"] > 0 and rec["higher_is_better"] is True
    assert rec["config"]["parallelism"] == f"dp{n}" and rec["config"]["global_batch"] == 4096 * n
    assert rec["stream_accuracy"] > 0.9
    assert rec["rf_train_sec"] > 0 and rec["rf_trees"] == 4
    assert rec["kafka_confluent_dialogues_per_s"] > 0 and rec["kafka_multi_gpu_dialogues_per_s"] > 0
    assert rec["kafka_all_delivered_and_committed"] and rec["kafka_multi_gpu_all_committed"]
    assert rec["kafka_confluent_group_dialogues_per_s"] > 0 and rec["kafka_confluent_group_clients"] == 3
    assert rec["kafka_confluent_group_all_committed"]
    # config 5: a scoring process per rank, each on its own GPU, every one of them fed
    assert rec["kafka_multi_gpu_scorer_procs"] == n and rec["kafka_confluent_group_scorer_procs"] == n
    assert len(rec["kafka_multi_gpu_batches_per_scorer"]) == n and min(rec["kafka_multi_gpu_batches_per_scorer"]) > 0


@pytest.mark.gpu
def test_bench_single_gpu_contract():
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "1", *TINY], cwd=REPO, capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    _check(_json_line(out.stdout), 1)


@pytest.mark.gpu
def test_bench_two_ranks_contract_gloo_rehearsal():
    env = {**os.environ, "FDX_DIST_BACKEND": "gloo"}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29547", "bench.py", "--gpus", "2", *TINY],
                         cwd=REPO, capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    _check(_json_line(out.stdout), 2)


@pytest.mark.gpu
def test_bench_rf_fault_two_ranks_still_prints_the_headline():
    """the headline phases (GBDT train, streaming, single-dialogue latency)
    run first; an RF-phase fault on every rank (FDX_FAULT: a tree of the forest raises) lands in
    the record as rf_error and the Kafka phase still runs."""
    env = {**os.environ, "FDX_DIST_BACKEND": "gloo", "FDX_FAULT": "model:rf,tree:1"}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29553", "bench.py", "--gpus", "2", *TINY],
                         cwd=REPO, capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert KEYS <= set(rec) and rec["n_gpus"] == 2 and rec["value"] > 0 and rec["gbdt_train_sec"] > 0
    assert "injected" in rec["rf_error"] and "rf_train_sec" not in rec
    assert rec["kafka_dialogues_per_s"] > 0 and rec["kafka_multi_gpu_scorer_procs"] == 2


@pytest.mark.gpu
def test_bench_phase_watchdog_prints_the_record_of_a_hung_phase():
    """A phase that hangs (FDX_BENCH_FAULT=rf:hang) is cut off after --phase-timeout: the record
    is printed as it stands with rf_error, and the process exits 3 (a hang is not a clean run)."""
    env = {**os.environ, "FDX_BENCH_FAULT": "rf:hang"}
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "1", *TINY, "--phase-timeout", "20"], cwd=REPO,
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 3, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert KEYS <= set(rec) and rec["value"] > 0 and rec["p50_single_dialogue_ms"] > 0
    assert rec["rf_error"].startswith("timeout") and "kafka_dialogues_per_s" not in rec


@pytest.mark.gpu
def test_suite_xgb_and_rf_two_ranks_gloo_rehearsal():
    """bench/suite.py xgb / rf under torchrun: --rows is global, row-sharded, one JSON line."""
    env = {**os.environ, "FDX_DIST_BACKEND": "gloo"}
    for which, port in (("xgb", "29549"), ("rf", "29551")):
        out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                              "--master-addr", "127.0.0.1", "--master-port", port, "bench/suite.py", which,
                              "--rows", "60000", "--trees", "3"], cwd=REPO, capture_output=True, text=True,
                             timeout=900, env=env)
        assert out.returncode == 0, out.stderr[-3000:]
        lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, out.stdout[-2000:]
        rec = json.loads(lines[0])
        assert rec["bench"] == which and rec["world"] == 2 and rec["rows"] == 60000
        assert rec["rows_per_rank"] == 30000 and rec["train_s"] > 0 and rec["trees"] == 3


@pytest.mark.gpu
def test_bench_gbdt_phase_peak_matches_the_hbm_model():
    """bench.py's timed GBDT phase (chunked featurization with the per-chunk feature order, IDF,
    100-tree fit) on a 2M-row shard: the caching allocator's peak is within 15 % of
    utils/memory.py's pipeline model (the full 10M-row bench reports it as train_peak_over_model:
    0.955 in profiles/r4/bench_full_session_f.json)."""
    import torch

    sys.path.insert(0, REPO)
    import bench as B
    from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn
    from fraud_detection_spark_kafka_llm_amd.ml.stopwords import ENGLISH
    from fraud_detection_spark_kafka_llm_amd.models.gbdt import GBDTParams, fit_gbdt
    from fraud_detection_spark_kafka_llm_amd.ops import text as T
    from fraud_detection_spark_kafka_llm_amd.utils import memory

    dev = torch.device("cuda:0")
    rows, chunk = 2_000_000, 250_000
    spec = T.FeatureSpec(clean=True, stopwords=list(ENGLISH), num_features=B.F)
    chunks = B.generate_shard(0, rows, dev, seed=11, chunk=chunk)
    text_bytes = sum(int(h.data.numel()) for h, _ in chunks)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    indptr, idx, counts, y, fo = B.featurize_shard(chunks, dev, spec, order=True)
    idf = torch.log((rows + 1.0) / (fo.df.double() + 1.0))
    vc = VectorColumn.tfidf(B.F, indptr, idx, counts, idf, fo)
    res = fit_gbdt(vc, y, GBDTParams(n_estimators=20, max_depth=6), device=dev)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(dev) - base
    model = memory.pipeline_bytes(rows, int(idx.numel()), hot_features=res.shape["hot"],
                                  groups=res.shape["groups"] or memory.DEFAULT_GROUPS,
                                  sparse_frac=res.shape["sparse_frac"],
                                  text_bytes_per_row=text_bytes / rows, chunk_rows=chunk)
    assert 0.85 <= peak / model <= 1.15, (peak / 2 ** 30, model / 2 ** 30)
