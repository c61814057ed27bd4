"""Dashboard logic + a headless run of app_ui.py against a recording fake of the streamlit API."""
import json
import runpy
import sys
import types

import pandas as pd
import pytest

from fraud_detection_spark_kafka_llm_amd.data import fixtures
from fraud_detection_spark_kafka_llm_amd.serve import ui_logic
from fraud_detection_spark_kafka_llm_amd.serve.agent import ClassificationAgent
from fraud_detection_spark_kafka_llm_amd.serve.llm import StubLLM
from fraud_detection_spark_kafka_llm_amd.stream import fake_kafka
from utils.st_functions import styled_badge


@pytest.fixture(scope="module")
def agent(shipped_model_path):
    return ClassificationAgent(str(shipped_model_path), llm=StubLLM(), device="cpu")


def test_badge_and_confidence_format():
    assert "Potentially Fraudulent" in ui_logic.badge_for(1.0)[0]
    assert ui_logic.format_confidence(0.0) == "0.00%"      # the reference drops 0.0 as falsy
    assert ui_logic.format_confidence(None) is None
    html = styled_badge("<b>x</b>", "#fff")
    assert "&lt;b&gt;" in html and "border-radius:12px" in html


def test_single_and_batch(agent):
    r = ui_logic.analyze_single(agent, fixtures.SCAM_SAMPLE, temperature=0.3)
    assert r["prediction"] == 1.0 and r["analysis"] and r["error"] is None
    df = pd.DataFrame({"dialogue": [fixtures.SCAM_SAMPLE, fixtures.BENIGN_SAMPLE, None]})
    table, csv = ui_logic.predict_dataframe(agent, df)
    assert table["predicted_label"].tolist() == ["Potentially Scam", "Non-Scam (Safe)", "Non-Scam (Safe)"]
    assert csv.startswith("dialogue,predicted_label,confidence")
    with pytest.raises(ValueError):
        ui_logic.predict_dataframe(agent, pd.DataFrame({"text": ["x"]}))


def test_kafka_monitor_step(agent):
    b = fake_kafka.broker_for("memory://ui")
    b.create_topic("in", 3)
    p = fake_kafka.Producer({"bootstrap.servers": "memory://ui"})
    p.produce("in", key="a", value=json.dumps({"text": fixtures.SCAM_SAMPLE}))
    p.produce("in", key="b", value="not json")
    c = fake_kafka.Consumer({"bootstrap.servers": "memory://ui", "group.id": "ui", "auto.offset.reset": "earliest",
                             "enable.auto.commit": False})
    c.subscribe(["in"])
    mon = ui_logic.KafkaMonitor(agent, c, p, "out")
    assert mon.step(timeout=0.1) == 1
    assert len(mon.errors) == 1
    out = json.loads(b.messages("out")[0].value())
    assert out["prediction"] == 1.0 and out["analysis"] and out["original_text"] == fixtures.SCAM_SAMPLE
    assert "prediction-badge scam" in ui_logic.render_message_card(mon.last(1)[0])


class _Ctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __getattr__(self, name):
        return getattr(_FAKE, name)


def _make_fake_streamlit(calls):
    st = types.ModuleType("streamlit")

    def rec(name, ret=None):
        def f(*a, **k):
            calls.append(name)
            return ret() if callable(ret) else ret
        return f

    for n in ("set_page_config", "markdown", "title", "header", "divider", "info", "success", "error", "write",
              "subheader", "text", "metric", "dataframe", "download_button", "warning", "rerun"):
        setattr(st, n, rec(n))
    st.slider = lambda *a, **k: 0.7
    st.checkbox = lambda label, default=False, **k: default
    st.file_uploader = lambda *a, **k: None
    st.text_area = lambda *a, **k: fixtures.SCAM_SAMPLE
    st.button = lambda label, **k: label == "Analyze"
    st.cache_resource = lambda f: f
    st.session_state = types.SimpleNamespace()
    st.session_state.__contains__ = lambda k: hasattr(st.session_state, k)
    ctx = _Ctx()
    st.sidebar = ctx
    st.spinner = lambda *a, **k: _Ctx()
    st.expander = lambda *a, **k: _Ctx()
    st.tabs = lambda names: [_Ctx() for _ in names]
    st.columns = lambda n: [_Ctx() for _ in range(n)]
    st.empty = lambda: _Ctx()
    return st


class _SessionState(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


_FAKE = None


def test_app_ui_headless(shipped_model_path, monkeypatch):
    global _FAKE
    calls = []
    st = _make_fake_streamlit(calls)
    st.session_state = _SessionState()
    _FAKE = st
    monkeypatch.setitem(sys.modules, "streamlit", st)
    monkeypatch.setenv("FDX_LLM_BACKEND", "stub")
    monkeypatch.setenv("MODEL_PATH", str(shipped_model_path))
    monkeypatch.setenv("FDX_DEVICE", "cpu")
    sys.modules.pop("utils.agent_api", None)
    runpy.run_path("app_ui.py", run_name="__main__")
    assert "set_page_config" in calls and "metric" in calls and "write" in calls   # analysed + explained
    assert "error" not in calls
