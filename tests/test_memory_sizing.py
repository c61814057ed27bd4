"""HBM sizing rule (utils/memory.py): the modelled peak is monotone, the row cap
inverts it, and the estimators' launcher asks for enough ranks that each shard fits."""
import torch

from fraud_detection_spark_kafka_llm_amd.parallel import estimator_dp
from fraud_detection_spark_kafka_llm_amd.utils import memory


def test_max_rows_inverts_the_training_bytes_model():
    budget = 288 * 2 ** 30 * 0.9
    cap = memory.max_rows_per_gpu(100.0, budget_bytes=budget)
    assert cap > 50_000_000                    # a 288 GB GPU holds far more than a 12.5M-row shard
    assert memory.pipeline_bytes(cap, cap * 100) <= budget < memory.pipeline_bytes(cap + 1000, (cap + 1000) * 100)
    # featurization's last chunk dominates small shards, training's per-entry state large ones
    assert memory.featurize_bytes(10_000_000, 10 ** 9) > memory.training_bytes(10_000_000, 10 ** 9)
    assert memory.max_rows_per_gpu(200.0, budget_bytes=budget) < cap
    assert memory.max_rows_per_gpu(100.0) == 0 or torch.cuda.is_available()   # no budget on the CPU
    assert memory.min_workers(10 * cap, 10 * cap * 100, budget_bytes=budget) == 10
    assert memory.min_workers(cap // 2, cap // 2 * 100, budget_bytes=budget) == 1


def test_effective_workers_raises_ranks_when_a_shard_would_not_fit(monkeypatch):
    monkeypatch.setattr(estimator_dp, "_resolve_device", lambda d: torch.device("cuda", 0))
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("FDX_HBM_BUDGET_GB", "20")
    cap = memory.max_rows_per_gpu(100.0)
    rows = 3 * cap + 10
    assert estimator_dp.effective_workers(1, rows, "cuda:0", nnz=rows * 100) == 4
    assert estimator_dp.effective_workers(2, rows, "cuda:0") == 2        # without nnz: as requested
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    assert estimator_dp.effective_workers(1, rows, "cuda:0", nnz=rows * 100) == 2   # capped at the GPUs



def test_rf_lanes_enter_the_sizing_rule():
    """RF trains with several trees in flight, each with its own ~27 B/row workspace: a shard that
    fits the GBDT rule can need more ranks as a 16-lane forest, and fit_forest caps
    its lanes to half the free memory."""
    from fraud_detection_spark_kafka_llm_amd.utils import memory as M

    rows, nnz = 100_000_000, 110 * 100_000_000
    g = M.training_bytes(rows, nnz)
    r = M.training_bytes(rows, nnz, rf_lanes=16)
    assert r - g >= 16 * M.RF_LANE_ROW_BYTES * rows
    budget = int(g * 1.05)
    assert M.min_workers(rows, nnz, budget_bytes=budget) == 1
    assert M.min_workers(rows, nnz, budget_bytes=budget, rf_lanes=16) >= 2
    assert M.rf_lanes_that_fit(10_000_000, 16, 200 * 2 ** 30) == 16
    assert M.rf_lanes_that_fit(10_000_000, 16, 2 * 2 ** 30) == 3
    assert M.rf_lanes_that_fit(10_000_000, 16, 0) == 16          # no budget known (CPU)


def test_max_rows_never_exceeds_the_engine_index_limits():
    """whatever the HBM budget, the row cap stays within the engine's index
    widths (int32 row ids); the row groups' uint32 entry offsets are no row limit because the
    groups split (RowGroups), and the model charges the extra groups' run starts per row."""
    huge = 64 * 2 ** 40                       # 64 TB: far beyond any device
    cap = memory.max_rows_per_gpu(97.0, budget_bytes=huge)
    assert 0 < cap <= memory.ENGINE_MAX_ROWS
    assert memory.min_workers(3 * memory.ENGINE_MAX_ROWS, 0, budget_bytes=huge) >= 3
    # 100M rows x 97 entries: the dense group's ~7.7G entries need 4 groups of < 2^31 entries
    assert memory.row_groups_for(100_000_000 * 97) == memory.DEFAULT_GROUPS + 3
    assert memory.row_groups_for(10_000_000 * 97) == memory.DEFAULT_GROUPS
    small = memory.training_bytes(10_000_000, 10_000_000 * 97)
    big = memory.training_bytes(100_000_000, 100_000_000 * 97)
    assert big > 10 * small                   # (the extra groups' per-row run starts)
