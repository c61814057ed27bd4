"""Result plots (R-09, R-10, R-12) with matplotlib only (seaborn is optional in the reference's
environment and absent here).

Artefacts and names match the reference (/root/reference/fraud_detection_spark.py:140-324):
``metrics_comparison.png`` (one panel per metric, bars per model grouped by dataset, value labels),
``confusion_matrices_{model}.png`` (one annotated heatmap per dataset, accuracy caption, dpi 300),
``word_associations_{model}.png`` (counts by class | scam ratio bars + importance line).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

_COLORS = ["#4C72B0", "#DD8452", "#55A868", "#C44E52", "#8172B3"]


def _label_bars(ax, bars, fmt="{:.3f}", dy=0.01):
    for b in bars:
        h = b.get_height()
        ax.text(b.get_x() + b.get_width() / 2.0, h + dy, fmt.format(h), ha="center", va="bottom", fontsize=7)


def plot_with_annotations(ax, labels, values, xlabel: str, ylabel: str, title: str, rotation: int = 45):
    """Bar plot with value labels (the reference's unused helper, R-09)."""
    bars = ax.bar(range(len(values)), values, color=_COLORS[0])
    ax.set_xticks(range(len(values)))
    ax.set_xticklabels(labels, rotation=rotation)
    ax.set_title(title)
    ax.set_xlabel(xlabel)
    ax.set_ylabel(ylabel)
    _label_bars(ax, bars)
    return bars


def visualize_results(results: dict, out_dir: str = ".") -> list:
    """``results[model][dataset] = {"metrics": {...}, "confusion_matrix": 2x2}``."""
    os.makedirs(out_dir, exist_ok=True)
    written = []
    models = list(results)
    datasets = list(next(iter(results.values())).keys()) if results else []
    metrics = list(next(iter(next(iter(results.values())).values()))["metrics"].keys()) if results else []
    ncol = 3
    nrow = max(1, int(np.ceil(len(metrics) / ncol)))
    fig, axes = plt.subplots(nrow, ncol, figsize=(15, 4 * nrow), squeeze=False)
    width = 0.8 / max(1, len(datasets))
    for k, metric in enumerate(metrics):
        ax = axes[k // ncol][k % ncol]
        for j, ds in enumerate(datasets):
            vals = [results[m][ds]["metrics"][metric] for m in models]
            bars = ax.bar(np.arange(len(models)) + j * width, vals, width, label=ds, color=_COLORS[j % len(_COLORS)])
            _label_bars(ax, bars)
        ax.set_xticks(np.arange(len(models)) + width * (len(datasets) - 1) / 2)
        ax.set_xticklabels(models)
        ax.set_title(f"Metric = {metric}")
        ax.set_ylabel("Score")
        lo = min(results[m][d]["metrics"][metric] for m in models for d in datasets)
        ax.set_ylim(max(0.0, lo - 0.05), 1.05)
    for k in range(len(metrics), nrow * ncol):
        axes[k // ncol][k % ncol].axis("off")
    if metrics:
        axes[0][0].legend(title="Dataset")
    fig.suptitle("Model Performance Comparison Across Datasets", y=1.02)
    fig.tight_layout()
    p = os.path.join(out_dir, "metrics_comparison.png")
    fig.savefig(p, bbox_inches="tight")
    plt.close(fig)
    written.append(p)

    for m in models:
        res = results[m]
        fig, axes = plt.subplots(1, len(res), figsize=(15, 6), squeeze=False)
        fig.suptitle(f"{m} - Confusion Matrices", y=1.05, fontsize=16, fontweight="bold")
        for i, (ds, vals) in enumerate(res.items()):
            ax = axes[0][i]
            cm = np.asarray(vals["confusion_matrix"], dtype=float)
            ax.imshow(cm, cmap="Blues")
            for (r, c), v in np.ndenumerate(cm):
                ax.text(c, r, f"{int(v)}", ha="center", va="center", fontsize=15,
                        color="white" if v > cm.max() / 2 else "black")
            ax.set_xticks(range(cm.shape[1]))
            ax.set_yticks(range(cm.shape[0]))
            ax.set_title(ds, fontsize=15, pad=12)
            ax.set_xlabel("Predicted", fontsize=15)
            ax.set_ylabel("Actual", fontsize=15)
            ax.text(0.5, -0.2, f"Accuracy: {vals['metrics']['Accuracy']:.4f}", ha="center", va="center",
                    transform=ax.transAxes, fontsize=14)
        fig.tight_layout()
        p = os.path.join(out_dir, f"confusion_matrices_{m.lower()}.png")
        fig.savefig(p, dpi=300, bbox_inches="tight")
        plt.close(fig)
        written.append(p)
    return written


def plot_word_associations(stats, model_name: str, out_dir: str = ".") -> Optional[str]:
    """``stats``: rows with word, scam_count, non_scam_count, scam_ratio, importance."""
    rows = [dict(r) for r in (stats.collect() if hasattr(stats, "collect") else stats)]
    if not rows:
        return None
    os.makedirs(out_dir, exist_ok=True)
    fig = plt.figure(figsize=(16, 6))
    ax = fig.add_subplot(1, 2, 1)
    words = [r["word"] for r in rows]
    x = np.arange(len(words))
    b1 = ax.bar(x - 0.2, [r["scam_count"] for r in rows], 0.4, label="scam_count", color=_COLORS[3])
    b2 = ax.bar(x + 0.2, [r["non_scam_count"] for r in rows], 0.4, label="non_scam_count", color=_COLORS[0])
    for b in list(b1) + list(b2):
        if b.get_height() > 0:
            ax.text(b.get_x() + b.get_width() / 2, b.get_height() + 5, f"{int(b.get_height())}", ha="center",
                    va="bottom", fontsize=7)
    ax.set_xticks(x)
    ax.set_xticklabels(words, rotation=45, ha="right")
    ax.set_title(f"Word Frequency - {model_name}")
    ax.set_xlabel("Words")
    ax.set_ylabel("Count")
    ax.legend()
    srt = sorted(rows, key=lambda r: -r["scam_ratio"])
    ax = fig.add_subplot(1, 2, 2)
    ax.bar(range(len(srt)), [r["scam_ratio"] for r in srt], color="salmon")
    ax2 = ax.twinx()
    ax2.plot(range(len(srt)), [r["importance"] for r in srt], color="blue", marker="o")
    for i, r in enumerate(srt):
        ax.text(i, r["scam_ratio"] + 0.02, f"{r['scam_ratio']:.2f}", ha="center", va="bottom", fontsize=7)
        ax2.text(i, r["importance"] + 0.01, f"{r['importance']:.3f}", ha="center", va="bottom", color="blue", fontsize=7)
    ax.set_xticks(range(len(srt)))
    ax.set_xticklabels([r["word"] for r in srt], rotation=45, ha="right")
    ax.set_title(f"Scam Ratio vs Importance - {model_name}")
    ax.set_xlabel("Words")
    ax.set_ylabel("Scam Ratio")
    ax2.set_ylabel("Feature Importance", color="blue")
    fig.tight_layout()
    p = os.path.join(out_dir, f"word_associations_{model_name.lower()}.png")
    fig.savefig(p)
    plt.close(fig)
    return p
