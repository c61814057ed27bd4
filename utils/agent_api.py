"""Drop-in for the reference's ``utils/agent_api.py`` (R-14..R-17) on the gfx950 engine.

``DeepSeekAPI``, ``DeepSeekAnalyzer`` and ``DeepSeekClassificationAgent`` keep their constructor
signatures and methods; predictions come from the fused featurize+score kernel over the saved
Spark-layout pipeline instead of Spark jobs. Environment: ``utils/.env`` then the process
environment; ``DEEPSEEK_API_KEY`` is required (as in the reference) unless the LLM backend is the
offline stub (``FDX_LLM_BACKEND=stub``) or an OpenAI-compatible local server
(``FDX_LLM_BACKEND=openai``, ``FDX_LLM_BASE_URL``).
"""
from __future__ import annotations

import os
from pathlib import Path

from fraud_detection_spark_kafka_llm_amd.serve.agent import ClassificationAgent
from fraud_detection_spark_kafka_llm_amd.serve.llm import Analyzer, ChatClient, RetryPolicy, StubLLM, make_llm
from fraud_detection_spark_kafka_llm_amd.utils.config import load_dotenv

current_dir = Path(__file__).parent
env_path = current_dir / ".env"
load_dotenv(env_path)

BACKEND = os.getenv("FDX_LLM_BACKEND", "deepseek").lower()
DEEPSEEK_API_KEY = os.getenv("DEEPSEEK_API_KEY")
if not DEEPSEEK_API_KEY and BACKEND == "deepseek":
    raise ValueError(f"""
    Missing DEEPSEEK_API_KEY (looked in {env_path} and the environment).
    Set DEEPSEEK_API_KEY, or run offline with FDX_LLM_BACKEND=stub.
    """)


class DeepSeekAPI(ChatClient):
    def __init__(self, api_key, model: str = "deepseek-chat"):
        super().__init__(api_key=api_key, model=model, base_url="https://api.deepseek.com/v1", timeout=90,
                         max_tokens=1000, retry=RetryPolicy(attempts=3, multiplier=1, min_wait=2, max_wait=10))


def _llm_for(api_key):
    if BACKEND == "deepseek":
        return DeepSeekAPI(api_key)
    return make_llm(BACKEND, api_key)


class DeepSeekAnalyzer(Analyzer):
    def __init__(self, api_key):
        super().__init__(_llm_for(api_key))

    def _create_prompt(self, dialogue, predicted_label, confidence=None):
        return self.create_prompt(dialogue, predicted_label, confidence)


class DeepSeekClassificationAgent(ClassificationAgent):
    def __init__(self, model_path, historical_data_path=None, device=None):
        super().__init__(model_path, historical_data_path, analyzer=DeepSeekAnalyzer(DEEPSEEK_API_KEY), device=device)
