"""Streamlit-independent logic of the dashboard (R-21..R-25), unit-testable without streamlit.

Fixes the reference's UI quirks: the single-dialogue tab reuses its first
prediction for the explanation (no second inference), the historical expander checks the right
result, the temperature slider is passed to the LLM, batch confidence 0.0 is not dropped as falsy,
the batch tab is one batched kernel launch, and the Kafka monitor commits after producing and
skips bad messages instead of dying.
"""
from __future__ import annotations

import html
import json
from typing import Optional

LABEL_MAPPING = {0: "Non-Scam (Safe)", 1: "Potentially Scam"}
BADGES = {0: ("✅ Non-Fraudulent (Safe)", "#4CAF50"), 1: ("⚠️ Potentially Fraudulent", "#F44336")}


def badge_for(prediction) -> tuple:
    return BADGES.get(int(prediction), (str(prediction), "#607D8B"))


def format_confidence(conf: Optional[float], digits: int = 2) -> Optional[str]:
    return None if conf is None else f"{conf * 100:.{digits}f}%"


def analyze_single(agent, text: str, temperature: float = 0.7, with_history: bool = False) -> dict:
    pred = agent.predict_and_get_label(text)
    out = {"prediction": pred["prediction"], "confidence": pred["confidence"], "analysis": None,
           "historical_insight": None, "error": None}
    try:
        res = agent.classify_and_explain(text, temperature=temperature, prediction=pred, with_history=with_history)
        out["analysis"] = res["analysis"]
        out["historical_insight"] = res["historical_insight"]
    except Exception as e:   # the prediction is still shown
        out["error"] = f"Cannot get AI explanation: {e}"
    return out


def predict_dataframe(agent, df):
    """Batch tab: one fused launch for the whole uploaded CSV -> result table + CSV text."""
    import pandas as pd

    if "dialogue" not in df.columns:
        raise ValueError("CSV must contain a 'dialogue' column.")
    texts = ["" if (v is None or (isinstance(v, float) and v != v)) else str(v) for v in df["dialogue"].tolist()]
    res = agent.predict_batch(texts)
    out = pd.DataFrame({"dialogue": texts,
                        "predicted_label": [LABEL_MAPPING.get(int(r["prediction"]), r["prediction"]) for r in res],
                        "confidence": [format_confidence(r["confidence"]) for r in res]})
    return out, out.to_csv(index=False)


def render_message_card(msg: dict) -> str:
    label = LABEL_MAPPING.get(int(msg["prediction"]), "Unknown")
    conf = format_confidence(msg.get("confidence"), 1) or "N/A"
    preview = html.escape((msg.get("dialogue") or "")[:100])
    css = "scam" if int(msg["prediction"]) == 1 else "safe"
    return (f'<div class="kafka-message"><span class="prediction-badge {css}">{html.escape(label)}</span>'
            f'<span class="confidence">{conf}</span><div class="dialogue-preview">{preview}...</div></div>')


class KafkaMonitor:
    """One iteration = consume a small batch, classify it in one launch, produce, commit."""

    def __init__(self, agent, consumer, producer, output_topic: Optional[str], explain: bool = True,
                 temperature: float = 0.7, batch: int = 64):
        self.agent, self.consumer, self.producer = agent, consumer, producer
        self.topic, self.explain, self.temperature, self.batch = output_topic, explain, temperature, batch
        self.messages: list = []
        self.errors: list = []

    def step(self, timeout: float = 1.0) -> int:
        msgs = self.consumer.consume(num_messages=self.batch, timeout=timeout)
        good, texts = [], []
        for m in msgs:
            if m.error() is not None:
                self.errors.append(str(m.error()))
                continue
            try:
                texts.append(json.loads(m.value().decode("utf-8"))["text"])
                good.append(m)
            except (ValueError, KeyError, TypeError, AttributeError) as e:
                self.errors.append(f"bad message: {e}")
        if not good:
            return 0
        preds = self.agent.predict_batch(texts)
        for m, t, p in zip(good, texts, preds):
            rec = {"prediction": p["prediction"], "confidence": p["confidence"], "analysis": None,
                   "historical_insight": None}
            if self.explain:
                r = self.agent.classify_and_explain(t, temperature=self.temperature, prediction=p, with_history=False)
                rec["analysis"] = r["analysis"]
            self.messages.append({"id": m.key(), "dialogue": t, **p})
            if self.topic:
                self.producer.produce(self.topic, key=m.key(), value=json.dumps({**rec, "original_text": t}))
        self.producer.flush()
        for m in good:
            self.consumer.commit(message=m)
        return len(good)

    def last(self, n: int = 5) -> list:
        return self.messages[-n:]
