"""Offline training application (R-01..R-13): the reference's ``main()`` flow on the gfx950 engine.

/root/reference/fraud_detection_spark.py:326-402: load + clean -> randomSplit 70/30 then 1/3:2/3
(= 70/10/20, seed 42) -> Tokenizer -> StopWordsRemover -> CountVectorizer(20000) -> IDF ->
{DecisionTree(depth 5), RandomForest(100 trees, depth 5, seed 42), XGBoost(100 rounds, depth 5)}
-> metrics on Validation/Test -> plots -> RF/DT word associations -> save the DT pipeline to
``fraud_detection_model``. Deliberate differences: the feature stages are
fitted once and shared by the three classifiers (the reference refits them 3x), word statistics
for all top-N words come from one device pass, and the dataset falls back to the synthetic corpus
when the Hugging Face CSV is unreachable (no network here).

    python -m fraud_detection_spark_kafka_llm_amd.train [--data CSV] [--synthetic N] [--out-dir D]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time
from typing import Optional

import numpy as np
import torch

from .data import synth
from .ml import (IDF, CountVectorizer, DecisionTreeClassifier, Frame, Pipeline, PipelineModel, RandomForestClassifier,
                 StopWordsRemover, TextColumn, Tokenizer)
from .ml.evaluation import evaluate_all
from .ml.xgboost import SparkXGBClassifier
from .ops.sparse import term_presence_by_label
from .session import SparkSession
from .utils.config import Config
from .utils.profiling import run_profiled_if_requested
from .utils.logging import get_logger

DATA_URL = ("https://huggingface.co/datasets/BothBosu/multi-agent-scam-conversation/raw/main/"
            "agent_conversation_all.csv")
log = get_logger("train")


def initialize_spark() -> SparkSession:
    return SparkSession.builder.config("spark.jars.packages", "ml.dmlc:xgboost4j-spark_2.12:1.7.1") \
        .appName("FraudDetection").getOrCreate()


def load_and_clean_data(spark: SparkSession, url: Optional[str] = DATA_URL, synthetic: int = 1600,
                        seed: int = 42) -> Frame:
    """CSV (dialogue, personality, type, labels) -> keep labels in {"0","1"} -> labels as double ->
    clean_text = regexp_replace(lower(dialogue), "[^a-zA-Z ]", "") -> drop empty clean_text."""
    import pandas as pd

    pdf = None
    if url:
        try:
            pdf = pd.read_csv(url, dtype=str)
        except Exception as e:   # no network / missing file -> synthetic stand-in
            log.warning("could not read %s (%s); using %d synthetic dialogues", url, type(e).__name__, synthetic)
    if pdf is None:
        pdf = synth.generate_frame(synth.SynthConfig(n=synthetic, seed=seed)).toPandas()
    df = spark.createDataFrame(pdf, ["dialogue", "personality", "type", "labels"])
    lab = [(v or "").strip() for v in df.column("labels").strings]
    keep = np.array([v in ("0", "1") for v in lab])
    df = df.take_rows(np.nonzero(keep)[0])
    df = df.withColumn("labels", np.array([float(v.strip()) for v in df.column("labels").strings]))
    raw = df.column("dialogue")
    clean = TextColumn.cleaned_from(raw)
    df = df.withColumn("clean_text", clean)
    nonempty = np.array([len(s) > 0 for s in clean.strings])
    return df.take_rows(np.nonzero(nonempty)[0])


def build_feature_pipeline(vocab_size: int = 20000) -> list:
    return [Tokenizer(inputCol="clean_text", outputCol="words"),
            StopWordsRemover(inputCol="words", outputCol="filtered_words"),
            CountVectorizer(inputCol="filtered_words", outputCol="raw_features", vocabSize=vocab_size),
            IDF(inputCol="raw_features", outputCol="features")]


def make_classifiers(num_trees: int = 100, max_depth: int = 5, seed: int = 42) -> dict:
    return {
        "DecisionTree": DecisionTreeClassifier(featuresCol="features", labelCol="labels", maxDepth=max_depth,
                                               probabilityCol="probability", rawPredictionCol="rawPrediction"),
        "RandomForest": RandomForestClassifier(featuresCol="features", labelCol="labels", numTrees=num_trees,
                                               maxDepth=max_depth, seed=seed, featureSubsetStrategy="auto"),
        "XGBoost": SparkXGBClassifier(features_col="features", label_col="labels", num_workers=4,
                                      max_depth=max_depth, n_estimators=num_trees, eval_metric="auc"),
    }


def train_models(train_df: Frame, feature_stages: list, classifiers: Optional[dict] = None,
                 concurrent: Optional[bool] = None) -> dict:
    """Fit the feature stages once, then every classifier on the shared feature matrix.

    On a GPU the classifiers train concurrently (PAR-07): one host thread and one HIP stream per
    fit, so the small per-level kernels of DT, RF and GBDT fill each other's gaps (the reference
    fits them one after another, fraud_detection_spark.py:86-97). ``FDX_CONCURRENT_FITS=0`` or
    ``concurrent=False`` fits sequentially; the models are identical either way."""
    from .utils.config import default_device

    classifiers = classifiers or make_classifiers()
    feat_model = Pipeline(stages=feature_stages).fit(train_df)
    feats = feat_model.transform(train_df)
    dev = default_device()
    if concurrent is None:
        concurrent = dev.type == "cuda" and os.environ.get("FDX_CONCURRENT_FITS", "1") == "1"

    def fit_one(name, clf):
        t0 = time.perf_counter()
        if concurrent:
            stream = torch.cuda.Stream(dev)
            with torch.cuda.stream(stream):
                m = clf.fit(feats)
            stream.synchronize()
        else:
            m = clf.fit(feats)
        log.info("trained %s in %.3fs", name, time.perf_counter() - t0)
        return m

    if concurrent and len(classifiers) > 1:
        import concurrent.futures as cf

        torch.cuda.synchronize(dev)            # features ready before the side streams read them
        with cf.ThreadPoolExecutor(max_workers=len(classifiers)) as pool:
            futs = {name: pool.submit(fit_one, name, clf) for name, clf in classifiers.items()}
            fitted = {name: f.result() for name, f in futs.items()}
    else:
        fitted = {name: fit_one(name, clf) for name, clf in classifiers.items()}
    return {name: PipelineModel(list(feat_model.stages) + [fitted[name]]) for name in classifiers}


def evaluate_model(model: PipelineModel, datasets: dict) -> dict:
    out = {}
    for name, data in datasets.items():
        res = evaluate_all(model.transform(data), "labels")
        out[name] = {"metrics": res["metrics"], "confusion_matrix": res["confusion_matrix"]}
    return out


def analyze_word_associations(spark, model: PipelineModel, df: Frame, vocab: list, top_n: int = 10) -> Optional[Frame]:
    """Top-N features by importance -> docs containing the word by label (full dataset, like the
    reference) -> [word, scam_count, non_scam_count, scam_ratio, importance] by importance desc."""
    clf = model.stages[-1]
    if not hasattr(clf, "featureImportances"):
        log.warning("Model type not supported for feature importance analysis")
        return None
    imp = clf.featureImportances.toArray()
    top = np.argsort(imp, kind="stable")[-top_n:][::-1]
    tf = model.stages[0:3]
    cur = df
    for s in tf:
        cur = s.transform(cur)
    counts = term_presence_by_label(cur.column(tf[-1].getOutputCol()), top.copy(),
                                    torch.as_tensor(np.asarray(df.column("labels"), dtype=np.float64))).cpu().numpy()
    rows = []
    for k, idx in enumerate(top):
        scam, non = int(counts[k, 1]), int(counts[k, 0])
        ratio = scam / (scam + non) if scam + non > 0 else 0.0
        rows.append((vocab[int(idx)], scam, non, round(float(ratio), 3), round(float(imp[idx]), 3)))
    rows.sort(key=lambda r: -r[4])
    return Frame.from_records(rows, ["word", "scam_count", "non_scam_count", "scam_ratio", "importance"])


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data", default=DATA_URL, help="CSV path or URL ('' = synthetic only)")
    ap.add_argument("--synthetic", type=int, default=1600, help="synthetic dialogues when the CSV is unavailable")
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--model-path", default="fraud_detection_model")
    ap.add_argument("--no-plots", action="store_true")
    Config.add_cli_args(ap)          # --num-trees, --max-depth, --vocab-size, --seed, --device, --config ...
    args = ap.parse_args(argv)
    cfg = Config.from_cli(args)
    run_profiled_if_requested(cfg.profile, argv, module="fraud_detection_spark_kafka_llm_amd.train")
    args.num_trees, args.max_depth, args.vocab_size, args.seed = cfg.num_trees, cfg.max_depth, cfg.vocab_size, cfg.seed

    spark = initialize_spark()
    try:
        df = load_and_clean_data(spark, args.data or None, args.synthetic, args.seed)
        train_df, temp_df = df.randomSplit([0.7, 0.3], seed=args.seed)
        val_df, test_df = temp_df.randomSplit([1 / 3, 2 / 3], seed=args.seed)
        print("\nData Split Counts:")
        print(f"Training: {train_df.count()}")
        print(f"Validation: {val_df.count()}")
        print(f"Test: {test_df.count()}")
        models = train_models(train_df, build_feature_pipeline(args.vocab_size),
                              make_classifiers(args.num_trees, args.max_depth, args.seed))
        results = {name: evaluate_model(m, {"Validation": val_df, "Test": test_df}) for name, m in models.items()}
        print("\nModel Evaluation Results:")
        for name, res in results.items():
            print(f"\n{name}:")
            for ds, vals in res.items():
                print(f"\n{ds} Set:")
                for metric, score in vals["metrics"].items():
                    print(f"{metric}: {score:.4f}")
        os.makedirs(args.out_dir, exist_ok=True)
        if not args.no_plots:
            from .viz.plots import plot_word_associations, visualize_results

            visualize_results(results, args.out_dir)
        word_stats = {}
        for name in ("RandomForest", "DecisionTree"):
            if name not in models:
                continue
            m = models[name]
            vocab = m.stages[2].vocabulary
            if name == "DecisionTree":
                path = os.path.join(args.out_dir, args.model_path)
                if os.path.exists(path):
                    shutil.rmtree(path)
                m.save(path)
            ws = analyze_word_associations(spark, m, df, vocab)
            if ws is not None:
                print(f"\n{'Random Forest' if name == 'RandomForest' else 'Decision Tree'} - Top Words and Associations:")
                ws.show()
                word_stats[name] = [dict(r) for r in ws.collect()]
                if not args.no_plots:
                    plot_word_associations(ws, name, args.out_dir)
        summary = {n: {ds: v["metrics"] for ds, v in r.items()} for n, r in results.items()}
        with open(os.path.join(args.out_dir, "results.json"), "w") as fh:
            json.dump({"metrics": summary, "word_stats": word_stats,
                       "split": [train_df.count(), val_df.count(), test_df.count()]}, fh, indent=2)
        return summary
    finally:
        spark.stop()


if __name__ == "__main__":
    main()
    sys.exit(0)
