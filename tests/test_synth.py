"""Synthetic corpus (data/synth.py): deterministic, and the wide-vocabulary option (tail_words)
widens the active feature space while leaving the default corpus byte-identical."""
import hashlib

from fraud_detection_spark_kafka_llm_amd.data import synth


def _tokens(pt) -> set:
    return {w for s in pt.strings() for w in s.lower().replace(".", " ").replace(",", " ").split()}


def test_default_corpus_is_unchanged_and_wide_vocab_extends_it():
    pt, _ = synth.generate(synth.SynthConfig(n=50, seed=42))
    assert hashlib.md5(bytes(pt.data.numpy())).hexdigest() == hashlib.md5(
        bytes(synth.generate(synth.SynthConfig(n=50, seed=42, tail_words=30000))[0].data.numpy())).hexdigest()
    assert synth._tail_words(200_000)[:30000] == synth.TAIL
    narrow, _ = synth.generate(synth.SynthConfig(n=3000, seed=5))
    wide, _ = synth.generate(synth.SynthConfig(n=3000, seed=5, tail_words=200_000))
    assert len(_tokens(wide)) > 1.5 * len(_tokens(narrow))
    again, _ = synth.generate(synth.SynthConfig(n=3000, seed=5, tail_words=200_000))
    assert bytes(again.data.numpy()) == bytes(wide.data.numpy())
