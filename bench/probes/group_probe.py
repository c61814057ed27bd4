"""Host ceiling of the consumer-group layout (stream/group.py): P confluent-surface client
processes around one scoring process whose scorer returns at once (kafka_host_probe.InstantScorer),
so only client / broker / engine / IPC host work is timed.

    python bench/probes/group_probe.py --msgs 600000 --clients 1 2 3 4
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fraud_detection_spark_kafka_llm_amd.data import synth  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.stream import group as G, loadgen  # noqa: E402
import kafka_host_probe as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=600_000)
    ap.add_argument("--clients", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--batch", type=int, default=16384)
    args = ap.parse_args()
    pt, _ = synth.generate(synth.SynthConfig(n=65536, seed=77), device="cpu", start=2 * 10**9)
    pool = loadgen.MessagePool(pt.strings())
    for P in args.clients:
        with G.ConsumerGroup(K.InstantScorer(args.batch, depth=4), K.post, P, batch_max=args.batch,
                             max_bytes=args.batch * 4096, pool=pool) as grp:
            G.group_throughput_run(grp, 60_000, tag="warm")
            r = G.group_throughput_run(grp, args.msgs)
        print(json.dumps({"clients": P, "dialogues_per_s": round(r["dialogues_per_s"]), "sec": round(r["sec"], 3),
                          "produced": r["produced"], "committed": r["committed"], "batches": r["batches"],
                          "per_client": [round(x) for x in r["client_dialogues_per_s"]],
                          "start_spread_ms": round(r["client_start_spread_ms"], 1)}), flush=True)


if __name__ == "__main__":
    main()
