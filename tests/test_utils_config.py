"""Runtime configuration precedence: CLI > YAML > FDX_* environment > defaults (utils/config.py)."""
import argparse

from fraud_detection_spark_kafka_llm_amd.utils.config import Config


def _parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=None)       # a flag the tool defines itself is left alone
    Config.add_cli_args(ap)
    return ap.parse_args(argv)


def test_config_precedence(tmp_path, monkeypatch):
    monkeypatch.setenv("FDX_NUM_TREES", "7")
    assert Config.from_cli(_parse([])).num_trees == 7
    y = tmp_path / "c.yaml"
    y.write_text("num_trees: 9\nstream_batch: 512\nmy_extra: 3\n")
    c = Config.from_cli(_parse(["--config", str(y)]))
    assert c.num_trees == 9 and c.stream_batch == 512 and c.extra == {"my_extra": 3}
    c = Config.from_cli(_parse(["--config", str(y), "--num-trees", "11", "--no-deterministic", "--seed", "5"]))
    assert c.num_trees == 11 and c.deterministic is False and c.seed == 5
    assert Config().gbdt_max_bin == 256


def test_train_cli_reads_config(tmp_path, monkeypatch):
    from fraud_detection_spark_kafka_llm_amd import train

    seen = {}

    def fake_classifiers(num_trees, max_depth, seed):
        seen.update(num_trees=num_trees, max_depth=max_depth, seed=seed)
        raise SystemExit(0)

    monkeypatch.setattr(train, "make_classifiers", fake_classifiers)
    y = tmp_path / "c.yaml"
    y.write_text("num_trees: 3\nmax_depth: 2\n")
    try:
        train.main(["--data", "", "--synthetic", "60", "--no-plots", "--out-dir", str(tmp_path), "--config", str(y),
                    "--seed", "4"])
    except SystemExit:
        pass
    assert seen == {"num_trees": 3, "max_depth": 2, "seed": 4}
