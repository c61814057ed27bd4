import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

REFERENCE = Path("/root/reference")
SHIPPED_MODEL = REFERENCE / "dialogue_classification_model"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def shipped_model_path():
    if not SHIPPED_MODEL.exists():
        pytest.skip("reference model not mounted")
    return SHIPPED_MODEL


@pytest.fixture(scope="session")
def scam_sample():
    """The commented-out usage-example dialogue (/root/reference/utils/agent_api.py:224)."""
    from fraud_detection_spark_kafka_llm_amd.data.fixtures import SCAM_SAMPLE

    return SCAM_SAMPLE


@pytest.fixture(scope="session")
def device():
    import torch

    return torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")
