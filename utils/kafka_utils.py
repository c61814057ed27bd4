"""Drop-in for the reference's ``utils/kafka_utils.py`` (R-18, R-19).

``get_kafka_consumer()`` / ``get_kafka_producer()`` read the same environment variables
(``KAFKA_BOOTSTRAP_SERVERS``, ``KAFKA_CONSUMER_GROUP``, ``KAFKA_INPUT_TOPIC``,
``KAFKA_SECURITY_PROTOCOL``, ``KAFKA_USERNAME``, ``KAFKA_PASSWORD``; ``.env`` in the working
directory is honoured). librdkafka (confluent_kafka) is used when installed; a ``memory://``
bootstrap or ``FDX_KAFKA=memory`` selects the in-process broker.
"""
from fraud_detection_spark_kafka_llm_amd.stream.kafka import get_kafka_consumer, get_kafka_producer  # noqa: F401
from fraud_detection_spark_kafka_llm_amd.utils.config import load_dotenv

load_dotenv()
