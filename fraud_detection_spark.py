"""Drop-in for the reference's training entry point (`python fraud_detection_spark.py`).

Runs the gfx950-native training application (fraud_detection_spark_kafka_llm_amd.train): same
flow, outputs and saved ``fraud_detection_model`` directory, no Spark JVM. All functions of the
reference module are re-exported under their original names.
"""
from fraud_detection_spark_kafka_llm_amd.train import (  # noqa: F401
    analyze_word_associations, build_feature_pipeline, evaluate_model, initialize_spark, load_and_clean_data, main,
    train_models)
from fraud_detection_spark_kafka_llm_amd.viz.plots import (  # noqa: F401
    plot_with_annotations, plot_word_associations, visualize_results)

if __name__ == "__main__":
    main()
