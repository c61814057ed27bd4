"""Host-side ceiling of the streaming engine: the Kafka config-5 runs (columnar and confluent-surface
clients) with a scorer that returns at once, so only the client / broker / engine host work is
timed (the GPU scorer overlaps with it in the real runs). Optional cProfile of the engine thread.

    python bench/probes/kafka_host_probe.py --msgs 300000 [--confluent] [--profile]
"""
import argparse
import cProfile
import json
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np

from fraud_detection_spark_kafka_llm_amd.data import synth
from fraud_detection_spark_kafka_llm_amd.stream import loadgen
from fraud_detection_spark_kafka_llm_amd.stream.engine import StreamingEngine


class InstantScorer:
    """The GpuScorer surface (submit / ready / collect), scoring nothing."""

    def __init__(self, max_docs: int, depth: int = 2):
        self.max_docs, self.max_bytes, self.depth = max_docs, max_docs * 4096, depth
        self._q = []

    @property
    def inflight(self) -> int:
        return len(self._q)

    def submit(self, slot) -> None:
        self._q.append(slot)

    def ready(self) -> bool:
        return bool(self._q)

    def collect(self, copy: bool = True):
        slot = self._q.pop(0)
        return slot, slot.n_docs


def post(n):
    z = np.zeros(n)
    return z, z


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=300_000)
    ap.add_argument("--confluent", action="store_true")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--batch", type=int, default=16384)
    args = ap.parse_args()
    pt, _ = synth.generate(synth.SynthConfig(n=65536, seed=77), device="cpu", start=2 * 10**9)
    pool = loadgen.MessagePool(pt.strings())

    def mk(consumers, producer, topic):
        return StreamingEngine(InstantScorer(args.batch), post, consumers, producer, topic, batch_max=args.batch,
                               max_latency_ms=5.0, max_bytes=args.batch * 4096)

    loadgen.throughput_run(mk, pool, 50_000, url="memory://warm", confluent=args.confluent)
    prof = cProfile.Profile() if args.profile else None
    if prof:
        prof.enable()
    r = loadgen.throughput_run(mk, pool, args.msgs, url="memory://probe", confluent=args.confluent)
    if prof:
        prof.disable()
        pstats.Stats(prof).sort_stats("tottime").print_stats(25)
    print(json.dumps({"confluent": args.confluent, "msgs": args.msgs, "dialogues_per_s": round(r["dialogues_per_s"]),
                      "sec": round(r["sec"], 3), "committed": r["committed"]}))


if __name__ == "__main__":
    main()
