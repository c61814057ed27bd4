"""Single-slot listed level of the dense groups (csrc/row_kernels.hip rg_hist_kernel): the row-list
pass (listed rows' ptr pairs and runs read scattered) against the masked all-rows pass
(tree.h rg_use_dm: every row in order, digit words zeroed outside the slot), and the all-rows root
pass for scale. Synthetic level on the bench matrix: a random fraction of the rows is built.
Event-timed medians over REPS launches; the two listed variants must give the same sums.
Usage: ROWS=10000000 python bench/probes/rg_dm_probe.py
The masked pass (tree_rg_hist dm_min_rows) was removed after this measurement
(profiles/r6/gbdt_late/NOTES.md §3); the script is kept as the record of how it was timed."""
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
    emdig = torch.empty((N, 2), dtype=torch.int32, device=dev)
    wl, wr = rg.list_work(), rg.work()
    dl = rg.gmode.to(torch.bool)[wl[0].long()]
    dr = rg.gmode.to(torch.bool)[wr[0].long()]
    tab, rtab = wl[:, dl].contiguous(), wr[:, dr].contiguous()
    print(f"rows {N} groups {rg.G} dense list workgroups {tab.shape[1]} root {rtab.shape[1]}", flush=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s2n = torch.zeros(1, dtype=torch.int32, device=dev)

    def timed(fn):
        ts = []
        for _ in range(REPS):
            ev0.record()
            fn()
            ev1.record()
            ev1.synchronize()
            ts.append(ev0.elapsed_time(ev1) * 1e3)
        return statistics.median(ts)

    hist = torch.zeros((1, TB, 2), dtype=torch.int64, device=dev)
    root = timed(lambda: C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, rowdig, 4, None, None, None, 1,
                                        rg.gmode, rtab, s2n, hist, TB, None, 0, 0))
    print(f"root all-rows pass, dense groups: {root:7.1f} us", flush=True)
    for frac in (0.5, 0.4, 0.3, 0.2, 0.1):
        u = torch.rand(N, generator=g)
        row_node = torch.where(u < frac, 0, 1).to(torch.int32).to(dev)
        node_slot = torch.tensor([0, -1], dtype=torch.int32, device=dev)
        C.tree_rg_list(row_node, node_slot, None, N, 1, work, start, lst, rowdig, listdig, emdig)
        out, sums = [], []
        for name, dm in (("listed", 0), ("masked", 1)):
            h = torch.zeros((1, TB, 2), dtype=torch.int64, device=dev)
            C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, rowdig, 4, lst, start, listdig, 1, rg.gmode, tab,
                           s2n, h, TB, None, 0, 0, emdig=emdig, dm_min_rows=dm)
            sums.append(h)
            t = timed(lambda: C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, rowdig, 4, lst, start, listdig, 1,
                                             rg.gmode, tab, s2n, hist, TB, None, 0, 0, emdig=emdig, dm_min_rows=dm))
            out.append(f"{name} {t:7.1f}")
        print(f"listed {frac:.2f} (us): " + ", ".join(out) + f"  same sums: {bool(torch.equal(*sums))}",
              flush=True)


if __name__ == "__main__":
    main()
