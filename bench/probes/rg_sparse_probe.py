"""Listed row-group pass (csrc/row_kernels.hip rg_hist_kernel) split by group class, with and without
its LDS atomics (RgHistArgs dbg value 2: a register sum instead, sums invalid): how much of a
listed level is LDS issue. (Round 6 ran it with an entry-granular sparse variant as well:
profiles/r6/gbdt_late/listed_pass_by_class_eg_vs_row.txt.) Synthetic level on the bench matrix: rows spread over 2 * nslots nodes, every
other node built, the listed levels' work table (RowGroups.list_work) restricted to the dense or to
the sparse groups' workgroups. Event-timed medians over REPS launches.
Usage: ROWS=10000000 python bench/probes/rg_sparse_probe.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops import native  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.tree import prepare  # noqa: E402

REPS = int(os.environ.get("REPS", 10))


def main():
    C = native.lib()
    dev = torch.device("cuda:0")
    rows = int(os.environ.get("ROWS", 10_000_000))
    vc, y, _ = _tfidf(rows, dev, seed=11, times={})
    Q, _, _, _ = prepare(vc, y, dev, 32)
    rg = Q.rowgroups()
    N, TB = Q.n_rows, Q.TB
    g = torch.Generator(device="cpu").manual_seed(5)
    rowdig = torch.randint(1, 1 << 20, (N, 2), dtype=torch.int32, generator=g).to(dev)
    nw = -(-N // C.tree_rg_list_rows(N))
    work = torch.zeros(64 * (2 + nw), dtype=torch.int32, device=dev)
    start = torch.zeros(66, dtype=torch.int32, device=dev)
    lst = torch.empty(N, dtype=torch.int32, device=dev)
    listdig = torch.empty((N, 2), dtype=torch.int32, device=dev)
    wl = rg.list_work()
    dense = rg.gmode.to(torch.bool)[wl[0].long()]
    tables = {"all": wl, "dense": wl[:, dense].contiguous(), "sparse": wl[:, ~dense].contiguous()}
    print(f"rows {N} groups {rg.G} list workgroups {wl.shape[1]} (dense {int(dense.sum())})", flush=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for nslots in (2, 8, 32):
        for frac in (0.5, 0.2):
            nodes = 2 * nslots
            u = torch.rand(N, generator=g)
            pick = torch.randint(0, nslots, (N,), generator=g)
            row_node = torch.where(u < frac, 2 * pick, 2 * pick + 1).to(torch.int32).to(dev)
            node_slot = torch.tensor([n // 2 if n % 2 == 0 else -1 for n in range(nodes)], dtype=torch.int32,
                                     device=dev)
            s2n = torch.arange(nslots, dtype=torch.int32, device=dev)
            hist = torch.zeros((nslots, TB, 2), dtype=torch.int64, device=dev)
            C.tree_rg_list(row_node, node_slot, None, N, nslots, work, start, lst, rowdig, listdig)
            out = []
            for tname, tab in tables.items():
                for mode, dbg in (("atomics", 0), ("no-atomics", 2)):
                    ts = []
                    for _ in range(REPS):
                        ev0.record()
                        C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, rowdig, 4, lst, start, listdig, nslots,
                                       rg.gmode, tab, s2n, hist, TB, None, 0, dbg)
                        ev1.record()
                        ev1.synchronize()
                        ts.append(ev0.elapsed_time(ev1) * 1e3)
                    out.append(f"{tname}/{mode} {statistics.median(ts):7.1f}")
            print(f"nslots {nslots:2d} listed {frac:.2f} (us): " + ", ".join(out), flush=True)


if __name__ == "__main__":
    main()
