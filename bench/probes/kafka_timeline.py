"""Wall time per engine component (per thread) of a confluent-surface Kafka run with an instant
scorer: where the host time of config 5 goes. python bench/probes/kafka_timeline.py"""
import os, sys, time, threading, collections, functools
sys.argv = ["x"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from fraud_detection_spark_kafka_llm_amd.stream import engine as E, loadgen, fake_kafka
from fraud_detection_spark_kafka_llm_amd.data import synth
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kafka_host_probe as K
acc = collections.defaultdict(float); cnt = collections.Counter()
def wrap(obj, name, label):
    f = getattr(obj, name)
    @functools.wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        try: return f(*a, **k)
        finally:
            acc[(threading.current_thread().name[:10], label)] += time.perf_counter() - t; cnt[(threading.current_thread().name[:10], label)] += 1
    setattr(obj, name, g)
wrap(E.StreamingEngine, "_finish_one", "finish")
wrap(E.StreamingEngine, "_encode", "encode")
wrap(E.StreamingEngine, "_produce_each", "produce_each")
wrap(E._Reader, "_fill", "fill")
wrap(E._Reader, "_poll", "poll")
wrap(E, "_to_pieces", "to_pieces")
wrap(E, "extract_into", "extract")
wrap(fake_kafka.Consumer, "consume", "consume")
wrap(fake_kafka.RecordBatch, "messages", "build_messages")
wrap(fake_kafka.Producer, "poll", "prod_poll")
wrap(E.StreamingEngine, "_on_delivery", "on_delivery")
pt, _ = synth.generate(synth.SynthConfig(n=65536, seed=77), device="cpu", start=2 * 10**9)
pool = loadgen.MessagePool(pt.strings())
def mk(consumers, producer, topic):
    return E.StreamingEngine(K.InstantScorer(16384), K.post, consumers, producer, topic, batch_max=16384, max_latency_ms=5.0, max_bytes=16384 * 4096)
loadgen.throughput_run(mk, pool, 50_000, url="memory://warm", confluent=True)
acc.clear(); cnt.clear()
r = loadgen.throughput_run(mk, pool, 300000, url="memory://probe", confluent=True)
print(round(r["dialogues_per_s"]), round(r["sec"], 3))
for k in sorted(acc): print(k, round(acc[k], 3), cnt[k])
