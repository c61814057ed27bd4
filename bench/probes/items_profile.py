"""Host profile of the RF work-item build (quantize._build_items, the sampled passes' histogram
CSC and item tables) on the 10M-row bench matrix: cProfile of the first use of Q.groups after the
quantisation, twice (the second with warm allocators). Prints the wall times and the top entries."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.tree import prepare  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.warmup import warm_tree_kernels  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    rows = int(os.environ.get("ROWS", 10_000_000))
    warm_tree_kernels(dev, gbdt_depth=0, forest_depth=5, forest_subset="sqrt")
    vc, y, _ = _tfidf(rows, dev, seed=21, times={})
    torch.cuda.synchronize()
    if os.environ.get("WARM_BIG_OPS") == "1":     # (large-size torch kernels loaded: A/B)
        n = torch.ones(3_000_000, dtype=torch.int64, device=dev)
        c = torch.cumsum(n, 0)
        r = torch.repeat_interleave(torch.arange(3_000_000, device=dev), n, output_size=3_000_000)
        torch.minimum(c[r] - r, torch.full_like(r, 8192))
        torch.cuda.synchronize()
    pre = float(os.environ.get("PREALLOC_GB", 0))
    if pre > 0:       # (a cached-allocator segment of this size made and freed: fresh-memory A/B)
        x = torch.empty(int(pre * 2 ** 30), dtype=torch.uint8, device=dev)
        x.fill_(0)
        del x
        torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        Q, _, _, _ = prepare(vc, y, dev, 32)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        pr = cProfile.Profile()
        pr.enable()
        Q.groups
        torch.cuda.synchronize()
        pr.disable()
        t2 = time.perf_counter()
        print(f"rep {rep}: prepare {1e3 * (t1 - t0):.1f} ms, items {1e3 * (t2 - t1):.1f} ms", flush=True)
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(22)
        print(out.getvalue(), flush=True)
        del Q


if __name__ == "__main__":
    main()
