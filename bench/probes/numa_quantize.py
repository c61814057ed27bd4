"""Probe: is the quantize-phase host stall NUMA-balancing page migration? Times quantize() at
--rows rows after the warm-up and prints /proc/vmstat numa_* and page-migration deltas plus the
process's minor faults; ``--local-policy`` first sets an MPOL_LOCAL task memory policy (no
migrate-on-fault flag, so automatic NUMA balancing skips the process's memory)."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def vmstat():
    out = {}
    for line in open("/proc/vmstat"):
        k, v = line.split()
        if k.startswith("numa_") or k.startswith("pgmigrate") or k.startswith("thp_"):
            out[k] = int(v)
    return out


def minflt():
    return int(open("/proc/self/stat").read().rsplit(")", 1)[1].split()[7])


ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--local-policy", action="store_true")
ap.add_argument("--no-bind", action="store_true")
args = ap.parse_args()
if args.local_policy:
    libc = ctypes.CDLL(None, use_errno=True)
    rc = libc.syscall(238, 4, None, 0)          # set_mempolicy(MPOL_LOCAL, NULL, 0)
    print("set_mempolicy rc", rc, ctypes.get_errno(), file=sys.stderr)
import torch  # noqa: E402

from gbdt_train import build_features  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ml.linalg import VectorColumn  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.quantize import quantize  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops.sparse import feature_order  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.parallel.affinity import bind_to_gpu  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.utils import tracing  # noqa: E402

try:
    nb = open("/proc/sys/kernel/numa_balancing").read().strip()
except OSError:
    nb = "?"
dev = torch.device("cuda:0")
numa = None if args.no_bind else bind_to_gpu(0)
warm_tree_kernels(dev)
indptr, idx, counts, y, _, _ = build_features(args.rows, dev)
F = 1 << 18
fo = feature_order(indptr, idx, counts, F)
idf = torch.log((args.rows + 1.0) / (fo.df.double() + 1.0))
vc = VectorColumn.tfidf(F, indptr, idx, counts, idf, fo)
torch.cuda.synchronize()
res = []
for rep in range(2):
    v0, f0, r0 = vmstat(), minflt(), os.times()
    t0 = time.perf_counter()
    if os.path.exists(f"/tmp/q_spans_{rep}.jsonl"):
        os.remove(f"/tmp/q_spans_{rep}.jsonl")
    tracing.enable(f"/tmp/q_spans_{rep}.jsonl")
    Q = quantize(vc, max_bins=256, counts=counts, scale=idf)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    v1, f1, r1 = vmstat(), minflt(), os.times()
    d = {k: v1[k] - v0[k] for k in v1 if v1[k] != v0.get(k)}
    spans = {}
    for line in open(f"/tmp/q_spans_{rep}.jsonl"):
        r = json.loads(line)
        spans[r["name"]] = round(spans.get(r["name"], 0.0) + r.get("dur_ms", r.get("ms", 0.0)), 2)
    res.append({"rep": rep, "quantize_s": dt, "minflt": f1 - f0, "user_s": r1.user - r0.user, "sys_s": r1.system - r0.system,
                "vmstat_delta": d, "spans_ms": spans})
    del Q
print(json.dumps({"numa_balancing": nb, "local_policy": args.local_policy, "numa": numa, "runs": res}))
