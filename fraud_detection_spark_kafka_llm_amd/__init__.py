"""MI355X-native streaming scam-dialogue classification framework.

A brand-new gfx950 implementation of the capabilities of
``wangwang2111/fraud-detection-spark-kafka-llm``: Spark-ML-compatible pipelines and on-disk models,
hand-written HIP kernels for the text featurizer and tree/LR engines, RCCL data parallelism, a
Kafka -> pinned-ring -> multi-GPU streaming engine and the LLM-explanation agent.

Layout: ``ops`` (native op wrappers), ``models`` (GPU trainers), ``ml`` (Spark-ML API), ``io``
(Spark/XGBoost persistence), ``parallel`` (RCCL data parallelism), ``stream`` (Kafka + micro-batch
ring), ``serve`` (agent + LLM clients), ``data`` (synthetic corpus), ``viz`` (plots), ``utils``.
"""
__version__ = "0.1.0"


def native_core():
    """Load (building if necessary) the native ``_C`` extension and return it."""
    from .ops import native

    return native.lib()
