"""Pure-Python reference semantics (test oracles).

Straight-line, obviously-correct implementations of what the reference pipeline computes through
Spark 3.5.5. They are slow on purpose and are used only to check the
native CPU path and the gfx950 kernels:

* ``clean_text``      — ``regexp_replace(lower(dialogue), "[^a-zA-Z ]", "")``
                        (/root/reference/fraud_detection_spark.py:42-45, utils/agent_api.py:139-145)
* ``java_split_ws``   — ``Tokenizer``: ``lower().split("\\\\s")`` with Java split semantics
* ``murmur3_x86_32``  — Spark ``Murmur3_x86_32.hashUnsafeBytes2`` (HashingTF, seed 42)
* ``hashing_tf``      — ``nonNegativeMod(hash, numFeatures)`` term counts
* ``idf_fit``         — ``ln((N + 1) / (df + 1))``, zeroed below ``minDocFreq``
* ``lr_margin``       — ``w . x + b`` (LogisticRegressionModel, binary)
"""
from __future__ import annotations

import math
import re
from collections import Counter
from typing import Iterable, Sequence

_STRIP = re.compile(r"[^a-zA-Z ]")
JAVA_WS = " \t\n\x0b\x0c\r"


def clean_text(s: str) -> str:
    return _STRIP.sub("", s.lower())


def java_split_ws(s: str) -> list[str]:
    """``s.split("\\\\s")`` in Java: single-char delimiters, leading/middle empties kept,
    trailing empties dropped; no delimiter at all -> ``[s]``."""
    if not any(c in JAVA_WS for c in s):
        return [s]
    parts: list[str] = []
    cur = []
    for c in s:
        if c in JAVA_WS:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(c)
    parts.append("".join(cur))
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def tokenize(s: str) -> list[str]:
    return java_split_ws(s.lower())


def remove_stopwords(tokens: Sequence[str], stopwords: Iterable[str], case_sensitive: bool = False) -> list[str]:
    if case_sensitive:
        sw = set(stopwords)
        return [t for t in tokens if t not in sw]
    sw = {w.lower() for w in stopwords}
    return [t for t in tokens if t.lower() not in sw]


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF


def murmur3_x86_32(data: bytes, seed: int = 42) -> int:
    """Unsigned 32-bit MurmurHash3_x86_32."""
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h = seed & 0xFFFFFFFF
    n = len(data)
    nb = n - n % 4
    for i in range(0, nb, 4):
        k = int.from_bytes(data[i:i + 4], "little")
        k = (k * c1) & 0xFFFFFFFF
        k = _rotl(k, 15)
        k = (k * c2) & 0xFFFFFFFF
        h ^= k
        h = _rotl(h, 13)
        h = (h * 5 + 0xE6546B64) & 0xFFFFFFFF
    k = 0
    for j, b in enumerate(data[nb:]):
        k ^= b << (8 * j)
    k = (k * c1) & 0xFFFFFFFF
    k = _rotl(k, 15)
    k = (k * c2) & 0xFFFFFFFF
    h ^= k
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def non_negative_mod(h: int, n: int) -> int:
    s = h - (1 << 32) if h >= (1 << 31) else h
    r = int(math.fmod(s, n))   # Java % truncates toward zero
    return r + n if r < 0 else r


def term_index(term: str, num_features: int) -> int:
    return non_negative_mod(murmur3_x86_32(term.encode("utf-8"), 42), num_features)


def hashing_tf(tokens: Sequence[str], num_features: int, binary: bool = False) -> dict[int, float]:
    c = Counter(term_index(t, num_features) for t in tokens)
    return {k: (1.0 if binary else float(v)) for k, v in sorted(c.items())}


def count_vectorize(tokens: Sequence[str], vocab: Sequence[str], min_tf: float = 1.0,
                    binary: bool = False) -> dict[int, float]:
    index = {w: i for i, w in enumerate(vocab)}
    c = Counter(index[t] for t in tokens if t in index)
    thr = min_tf if min_tf >= 1.0 else min_tf * len(tokens)
    return {k: (1.0 if binary else float(v)) for k, v in sorted(c.items()) if v >= thr}


def idf_fit(docs: Iterable[dict[int, float]], num_features: int, min_doc_freq: int = 0):
    df = [0] * num_features
    n = 0
    for d in docs:
        n += 1
        for k, v in d.items():
            if v != 0:
                df[k] += 1
    idf = [math.log((n + 1.0) / (x + 1.0)) if x >= min_doc_freq else 0.0 for x in df]
    return idf, df, n


def lr_margin(x: dict[int, float], w: Sequence[float], b: float) -> float:
    return sum(v * w[k] for k, v in x.items()) + b


def sigmoid(m: float) -> float:
    return 1.0 / (1.0 + math.exp(-m))


def pipeline_vector(text: str, stopwords: Iterable[str], num_features: int, idf: Sequence[float] | None = None,
                    clean: bool = True, binary: bool = False) -> dict[int, float]:
    """clean -> Tokenizer -> StopWordsRemover -> HashingTF (-> IDF) for one document."""
    s = clean_text(text) if clean else text
    toks = remove_stopwords(tokenize(s), stopwords)
    tf = hashing_tf(toks, num_features, binary)
    if idf is not None:
        tf = {k: v * idf[k] for k, v in tf.items()}
    return tf
