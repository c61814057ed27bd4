"""LLM explanation clients (R-14, R-15, R-26).

``ChatClient`` speaks the OpenAI-style ``POST {base_url}/chat/completions`` contract used by the
reference for DeepSeek (/root/reference/utils/agent_api.py:33-77) and LM Studio
(deepseek_chat_ui.py:7-12), with a *working* retry (the reference re-raises every
``RequestException`` as a bare ``Exception`` so its tenacity policy never fires): connection
errors, timeouts, HTTP 429 and 5xx are retried with exponential backoff (3 attempts, 2..10 s by
default); other failures raise ``LLMError`` immediately. ``StubLLM`` is the in-process backend for
tests and benchmarks. ``Analyzer`` builds the reference's prompt verbatim in structure.
"""
from __future__ import annotations

import hashlib
import json
import os
import time
from dataclasses import dataclass
from typing import Optional, Sequence

SYSTEM_PROMPT = "You are an expert AI assistant specialized in analyzing customer service interactions."
LABELS = {0: "Non-Fraudulent (Safe)", 1: "Potentially Fraudulent"}


class LLMError(Exception):
    pass


class RetryableLLMError(LLMError):
    pass


@dataclass
class RetryPolicy:
    attempts: int = 3
    multiplier: float = 1.0
    min_wait: float = 2.0
    max_wait: float = 10.0

    def wait(self, attempt: int) -> float:
        return min(self.max_wait, max(self.min_wait, self.multiplier * (2 ** attempt)))


class ChatClient:
    """OpenAI-compatible chat-completions client (DeepSeek by default)."""

    def __init__(self, api_key: Optional[str] = None, model: str = "deepseek-chat",
                 base_url: str = "https://api.deepseek.com/v1", timeout: float = 90.0, max_tokens: int = 1000,
                 retry: RetryPolicy = RetryPolicy(), sleep=time.sleep):
        self.api_key = api_key
        self.model = model
        self.base_url = base_url.rstrip("/")
        self.timeout = timeout
        self.max_tokens = max_tokens
        self.retry = retry
        self._sleep = sleep
        self.headers = {"Content-Type": "application/json"}
        if api_key:
            self.headers["Authorization"] = f"Bearer {api_key}"

    def chat(self, messages: Sequence[dict], temperature: float = 0.7, max_tokens: Optional[int] = None) -> str:
        import requests

        payload = {"model": self.model, "messages": list(messages), "temperature": temperature,
                   "max_tokens": self.max_tokens if max_tokens is None else max_tokens}
        last: Optional[Exception] = None
        for attempt in range(self.retry.attempts):
            try:
                r = requests.post(f"{self.base_url}/chat/completions", headers=self.headers, json=payload,
                                  timeout=self.timeout)
                if r.status_code == 429 or r.status_code >= 500:
                    raise RetryableLLMError(f"HTTP {r.status_code}: {r.text[:200]}")
                if r.status_code >= 400:
                    raise LLMError(f"LLM request failed: HTTP {r.status_code}: {r.text[:200]}")
                try:
                    return r.json()["choices"][0]["message"]["content"]
                except (KeyError, IndexError, ValueError) as e:
                    raise LLMError(f"Failed to parse API response: {e}") from e
            except (requests.exceptions.Timeout, requests.exceptions.ConnectionError, RetryableLLMError) as e:
                last = e
                if attempt + 1 < self.retry.attempts:
                    self._sleep(self.retry.wait(attempt))
        raise LLMError(f"LLM request failed after {self.retry.attempts} attempts: {last}") from last

    def generate(self, prompt: str, temperature: float = 0.7) -> str:
        return self.chat([{"role": "system", "content": SYSTEM_PROMPT}, {"role": "user", "content": prompt}],
                         temperature)


class StubLLM:
    """Deterministic offline backend: a canned structured analysis derived from the prompt."""

    def __init__(self, latency_s: float = 0.0):
        self.latency_s = latency_s
        self.calls = 0

    def chat(self, messages: Sequence[dict], temperature: float = 0.7, max_tokens: Optional[int] = None) -> str:
        self.calls += 1
        if self.latency_s:
            time.sleep(self.latency_s)
        text = messages[-1]["content"] if messages else ""
        return stub_completion(text)

    def generate(self, prompt: str, temperature: float = 0.7) -> str:
        return self.chat([{"role": "user", "content": prompt}], temperature)


def stub_completion(prompt: str) -> str:
    digest = hashlib.sha256(prompt.encode()).hexdigest()[:8]
    fraud = "Potentially Fraudulent" in prompt
    flags = [w for w in ("verify", "social security", "urgent", "gift card", "wire", "password", "suspended",
                         "arrest", "prize") if w in prompt.lower()]
    return (f"- Summary of Key Findings: {'red flags: ' + ', '.join(flags) if flags else 'no explicit red flags'}\n"
            f"- Classification Evaluation: {'agree — fraud indicators present' if fraud else 'agree — benign'}\n"
            f"- Recommended Actions: {'do not share personal data; verify through official channels' if fraud else 'no action needed'}\n"
            f"[stub-llm {digest}]")


def make_llm(backend: Optional[str] = None, api_key: Optional[str] = None, **kw):
    backend = (backend or os.environ.get("FDX_LLM_BACKEND") or "deepseek").lower()
    if backend == "stub":
        return StubLLM()
    if backend == "openai":
        return ChatClient(api_key=api_key or os.environ.get("OPENAI_API_KEY", "not-needed"),
                          model=kw.pop("model", os.environ.get("FDX_LLM_MODEL", "deepseek-r1-0528-qwen3-8b")),
                          base_url=kw.pop("base_url", os.environ.get("FDX_LLM_BASE_URL", "http://192.168.56.1:1234/v1")),
                          **kw)
    return ChatClient(api_key=api_key, **kw)


class Analyzer:
    """Prompt construction + call (R-15; agent_api.py:83-122)."""

    def __init__(self, llm):
        self.llm = llm

    @staticmethod
    def create_prompt(dialogue: str, predicted_label, confidence: Optional[float] = None) -> str:
        try:
            key = int(predicted_label)
        except (TypeError, ValueError):
            key = predicted_label
        label = LABELS.get(key, str(predicted_label))
        conf = "" if confidence is None else f"(Confidence Score: {confidence:.2f})"
        return f"""Perform a detailed analysis of this customer service interaction:

        **Dialogue**:
        {dialogue}

        **Current Classification**:
        {label}
        {conf}

        **Analysis Instructions**:
        1. Content Examination:
          - Extract key phrases indicating intent
          - Identify emotional tone markers
          - Highlight potential red flags

        2. Classification Assessment:
          - Evaluate if the label matches content
          - Suggest alternative classifications
          - Assess confidence level validity

        3. Actionable Recommendations:
          - Agree/Disagree with classification
          - Suggest next steps if fraudulent
          - Provide specific evidence from text

        **Required Output Format**:
        - Summary of Key Findings
        - Classification Evaluation
        - Recommended Actions"""

    def analyze_prediction(self, dialogue: str, predicted_label, confidence: Optional[float] = None,
                           temperature: float = 0.7) -> str:
        return self.llm.generate(self.create_prompt(dialogue, predicted_label, confidence), temperature)
