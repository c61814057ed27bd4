"""Typed runtime configuration.

Defaults equal the reference's hard-coded values; every field can be overridden from the
environment (``FDX_*``), a YAML file, or CLI flags (``add_cli_args``/``from_cli``). The Kafka and
LLM environment variables of the reference (``KAFKA_*``, ``DEEPSEEK_API_KEY``) are read unchanged
by the drop-in modules under ``utils/``.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field
from typing import Optional

import torch


@dataclass
class Config:
    device: str = ""                      # "" -> cuda:LOCAL_RANK if available else cpu
    world_size: int = 1
    num_features: int = 1 << 18           # HashingTF default
    vocab_size: int = 20000               # fraud_detection_spark.py:52
    max_depth: int = 5                    # fraud_detection_spark.py:62,71,81
    num_trees: int = 100                  # fraud_detection_spark.py:70,82
    max_bins: int = 32                    # Spark DecisionTree default
    gbdt_max_bin: int = 256               # XGBoost hist default; histograms are exact at any width
    seed: int = 42                        # fraud_detection_spark.py:72,338-339
    deterministic: bool = True            # training is always bitwise reproducible (exact histograms)
    llm_backend: str = "deepseek"         # deepseek | openai | stub
    llm_base_url: str = "https://api.deepseek.com/v1"   # agent_api.py:36
    llm_model: str = "deepseek-chat"      # agent_api.py:35
    llm_timeout: float = 90.0             # agent_api.py:42
    llm_max_tokens: int = 1000            # agent_api.py:62
    stream_batch: int = 4096
    stream_max_latency_ms: float = 5.0
    profile: bool = False
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_env(cls) -> "Config":
        c = cls()
        for f in dataclasses.fields(cls):
            key = "FDX_" + f.name.upper()
            if key in os.environ and f.name != "extra":
                setattr(c, f.name, _coerce(f.type, os.environ[key]))
        return c

    @classmethod
    def from_yaml(cls, path: str) -> "Config":
        import yaml

        with open(path) as fh:
            data = yaml.safe_load(fh) or {}
        c = cls.from_env()
        for k, v in data.items():
            if hasattr(c, k):
                setattr(c, k, v)
            else:
                c.extra[k] = v
        return c

    @staticmethod
    def add_cli_args(ap: argparse.ArgumentParser) -> None:
        """``--config FILE.yaml`` plus one ``--<field>`` flag per field (``--num-trees``,
        ``--stream-batch``, ...) in a "runtime configuration" group; flags the parser already
        defines are left to it. Precedence: CLI > YAML > ``FDX_*`` environment > defaults."""
        grp = ap.add_argument_group("runtime configuration (utils/config.py)")
        if "--config" not in ap._option_string_actions:
            grp.add_argument("--config", default=None, help="YAML file of Config fields")
        for f in dataclasses.fields(Config):
            if f.name == "extra":
                continue
            flag = "--" + f.name.replace("_", "-")
            if flag in ap._option_string_actions:
                continue
            if f.type in ("bool", bool):
                grp.add_argument(flag, action=argparse.BooleanOptionalAction, default=None)
            else:
                grp.add_argument(flag, default=None, help=f"default {f.default!r}")

    @classmethod
    def from_cli(cls, ns: argparse.Namespace, base: Optional["Config"] = None) -> "Config":
        path = getattr(ns, "config", None)
        c = base or (cls.from_yaml(path) if path else cls.from_env())
        for f in dataclasses.fields(cls):
            v = getattr(ns, f.name, None)
            if v is not None and f.name != "extra":
                setattr(c, f.name, _coerce(f.type, v))
        if c.device:
            os.environ["FDX_DEVICE"] = c.device
        return c

    def torch_device(self) -> torch.device:
        if self.device:
            return torch.device(self.device)
        return default_device()


def _coerce(typ, v):
    t = typ if isinstance(typ, str) else getattr(typ, "__name__", str(typ))
    if isinstance(v, str):
        if t == "bool":
            return v.lower() in ("1", "true", "yes", "on")
        if t == "int":
            return int(v)
        if t == "float":
            return float(v)
    return v


def load_dotenv(path=None, override: bool = False) -> bool:
    """Minimal ``python-dotenv`` replacement: ``KEY=VALUE`` lines (``export`` prefix, quotes and
    ``#`` comments allowed) are copied into ``os.environ``. Without ``path`` the nearest ``.env``
    from the current directory upwards is used. Returns whether a file was read."""
    from pathlib import Path

    if path is None:
        cur = Path.cwd()
        for d in [cur, *cur.parents]:
            if (d / ".env").is_file():
                path = d / ".env"
                break
        if path is None:
            return False
    p = Path(path)
    if not p.is_file():
        return False
    for line in p.read_text(encoding="utf-8", errors="replace").splitlines():
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        if line.startswith("export "):
            line = line[7:]
        k, v = line.split("=", 1)
        k, v = k.strip(), v.strip()
        if len(v) >= 2 and v[0] == v[-1] and v[0] in "\"'":
            v = v[1:-1]
        elif " #" in v:
            v = v.split(" #", 1)[0].rstrip()
        if override or k not in os.environ:
            os.environ[k] = v
    return True


def default_device() -> torch.device:
    env = os.environ.get("FDX_DEVICE")
    if env:
        return torch.device(env)
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    return torch.device("cpu")
