"""Streaming classification service (the reference's Streamlit tab-3 loop as a headless process,
/root/reference/app_ui.py:168-248, without its per-message Spark job and without losing offsets).

  python -m fraud_detection_spark_kafka_llm_amd.stream.serve --model dialogue_classification_model \
      [--gpus N] [--explain none|sync|async] [--batch 4096] [--max-messages M] [--metrics-port 9108]

Kafka settings come from the reference's environment variables (utils/kafka_utils.py; `.env` in the
working directory is honoured): the consumer group reads KAFKA_INPUT_TOPIC, classifications go to
KAFKA_OUTPUT_TOPIC as JSON {prediction, confidence, analysis, historical_insight, original_text}
keyed like the input; offsets are committed after the outputs are produced (at-least-once).
With --gpus N the micro-batches of the consumer are spread over N devices of this process.
With --group-clients P the Kafka clients run as P consumer-group member processes (one GIL each,
stream/group.py) around this process's GPU scorer; the broker balances the topic's partitions over
them (a real bootstrap only: a memory:// broker lives inside one process). Explanations run in
the client processes (no historical-case insight there).
Under torchrun (WORLD_SIZE > 1) with --group-clients, every rank is one scoring process on its
own GPU (LOCAL_RANK): rank 0 starts the client processes, ranks 1..N-1 join as ScorerPeers that
page-lock the same slots for their device (BASELINE config 5, "3-partition topic -> 8-GPU
batched inference"); the rendezvous uses the process group's store (gloo, no device collective).
``/metrics`` serves the Prometheus text format of the metrics registry when --metrics-port is set.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import torch

from ..utils.config import Config, load_dotenv
from ..utils.profiling import run_profiled_if_requested
from ..utils.metrics import REGISTRY
from .kafka import DEFAULT_OUTPUT, get_kafka_consumer, get_kafka_producer, get_partition_consumers

log = logging.getLogger("fdx.serve")


def start_metrics_server(port: int) -> HTTPServer:
    class Handler(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            if self.path.rstrip("/") not in ("/metrics", ""):
                self.send_response(404)
                self.end_headers()
                return
            body = REGISTRY.to_prometheus().encode()
            self.send_response(200)
            self.send_header("Content-Type", "text/plain; version=0.0.4")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = HTTPServer(("0.0.0.0", port), Handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv=None) -> int:
    from ..serve.agent import ClassificationAgent
    from ..serve.llm import StubLLM, make_llm
    from .engine import StreamingEngine

    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="dialogue_classification_model")
    ap.add_argument("--gpus", type=int, default=1, help="devices of this process (0 = CPU host path)")
    ap.add_argument("--explain", choices=["none", "sync", "async"], default="none")
    ap.add_argument("--batch", type=int, default=None, help="micro-batch size (default: Config.stream_batch)")
    ap.add_argument("--max-latency-ms", type=float, default=None, help="default: Config.stream_max_latency_ms")
    ap.add_argument("--max-messages", type=int, default=None)
    ap.add_argument("--idle-timeout", type=float, default=float("inf"), help="exit after this many idle seconds")
    ap.add_argument("--metrics-port", type=int, default=0)
    ap.add_argument("--partition-readers", action="store_true",
                    help="one consumer (and reader thread) per input partition instead of one subscriber")
    ap.add_argument("--group-clients", type=int, default=0,
                    help="run the Kafka clients as this many consumer-group processes around this GPU process")
    Config.add_cli_args(ap)
    args = ap.parse_args(argv)
    load_dotenv()
    cfg = Config.from_cli(args)
    run_profiled_if_requested(cfg.profile, argv, module="fraud_detection_spark_kafka_llm_amd.stream.serve")
    args.batch = args.batch if args.batch is not None else cfg.stream_batch
    args.max_latency_ms = args.max_latency_ms if args.max_latency_ms is not None else cfg.stream_max_latency_ms
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    from ..parallel import dist as D

    ranks = int(os.environ.get("WORLD_SIZE", "1"))
    if ranks > 1 and args.group_clients > 0:
        from .group import single_host_group

        if not single_host_group():
            raise SystemExit("--group-clients under torchrun needs every rank on one host "
                             "(LOCAL_WORLD_SIZE != WORLD_SIZE): the group shares memory segments and Unix sockets")
        D.init_from_env("gloo")                 # the group's rendezvous store; no device collective
        devices = [torch.device("cuda", D.local_rank() % torch.cuda.device_count())] \
            if torch.cuda.is_available() else [torch.device("cpu")]
    elif args.gpus > 0 and torch.cuda.is_available():
        devices = [torch.device("cuda", i) for i in range(min(args.gpus, torch.cuda.device_count()))]
    else:
        devices = [torch.device("cpu")]
    llm = make_llm() if args.explain != "none" else StubLLM()   # no LLM calls without --explain
    agent = ClassificationAgent(args.model, llm=llm, device=devices[0])
    if args.group_clients > 0:
        return _serve_group(args, agent, devices, out_topic=os.getenv("KAFKA_OUTPUT_TOPIC", DEFAULT_OUTPUT))
    consumer = get_partition_consumers() if args.partition_readers else get_kafka_consumer()
    producer = get_kafka_producer()
    out_topic = os.getenv("KAFKA_OUTPUT_TOPIC", DEFAULT_OUTPUT)
    if args.metrics_port:
        start_metrics_server(args.metrics_port)
    eng = StreamingEngine.from_agent(agent, consumer, producer, out_topic, devices=devices, batch_max=args.batch,
                                     max_latency_ms=args.max_latency_ms, explain=args.explain)
    log.info("serving %s on %s -> %s", args.model, [str(d) for d in devices], out_topic)
    try:
        stats = eng.run(max_messages=args.max_messages, idle_timeout_s=args.idle_timeout)
    finally:
        for c in (consumer if isinstance(consumer, list) else [consumer]):
            c.close()
    print(json.dumps(stats), flush=True)
    return 0


def _serve_group(args, agent, devices, out_topic: str) -> int:
    from ..parallel import dist as D
    from .gpu_worker import make_multi_scorer
    from .group import ConsumerGroup, GroupRendezvous, ScorerPeer, merge_results

    if os.getenv("KAFKA_BOOTSTRAP_SERVERS", "").startswith("memory://") or os.getenv("FDX_KAFKA", "") == "memory":
        raise SystemExit("--group-clients needs a real Kafka bootstrap (an in-memory broker is per process)")
    fp = agent.fused
    scorer = make_multi_scorer(fp.spec(True), fp.idf.idf if fp.idf is not None else None, fp.model.scorer(),
                               devices, max_docs=args.batch, max_bytes=args.batch * 4096, depth=3)
    rdv = GroupRendezvous.from_process_group("serve") if D.world_size() > 1 else None
    if rdv is not None and D.rank() > 0:
        log.info("rank %d: scoring process of the group on %s", D.rank(), devices[0])
        with ScorerPeer(scorer, fp.model.postprocess_numpy, rdv) as peer:
            st = peer.serve()
        print(json.dumps({"rank": D.rank(), **st}), flush=True)
        return 0
    if args.metrics_port:
        start_metrics_server(args.metrics_port)
    log.info("serving %s on %s with %d client processes (%d scoring processes) -> %s", args.model,
             [str(d) for d in devices], args.group_clients, D.world_size(), out_topic)
    with ConsumerGroup(scorer, fp.model.postprocess_numpy, args.group_clients, batch_max=args.batch,
                       max_latency_ms=args.max_latency_ms, max_bytes=args.batch * 4096, rendezvous=rdv) as grp:
        P, m = args.group_clients, args.max_messages
        share = None if m is None else [{"max_messages": m // P + (1 if c < m % P else 0)} for c in range(P)]
        rs = grp.run({"kind": "serve", "max_messages": m, "idle_timeout": args.idle_timeout,
                      "output_topic": out_topic, "explain": args.explain,
                      "llm": os.environ.get("FDX_LLM_BACKEND") or "deepseek"}, share)
    print(json.dumps({k: v for k, v in merge_results(rs).items() if k != "client_dialogues_per_s"}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
