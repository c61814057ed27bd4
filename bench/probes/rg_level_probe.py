"""Cost of a listed row-group histogram level (csrc/row_kernels.hip rg_hist_kernel) by number of
built slots and listed fraction, with and without the flush of the workgroups' LDS tables
(RgHistArgs dbg bit 2: timing only, sums invalid), and with per-workgroup partial tables + their
reduction (RgHistArgs part). Synthetic level on the bench matrix: rows spread
over 2 * nslots nodes, every other node built. Times are event-timed medians over REPS launches.
Usage: ROWS=1000000 python bench/probes/rg_level_probe.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from suite import _tfidf  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.ops import native  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.models.tree import prepare  # noqa: E402

REPS = int(os.environ.get("REPS", 20))


def main():
    C = native.lib()
    dev = torch.device("cuda:0")
    rows = int(os.environ.get("ROWS", 1_000_000))
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
    wg = rg.work()
    part_kw = dict(part=torch.empty(wg.shape[1] * rg.gbin.shape[1] * 2, dtype=torch.int64, device=dev),
                   wg_first=rg.work_first())
    print(f"rows {N} TB {TB} groups {rg.G} workgroups {wg.shape[1]}", flush=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for nslots in (1, 4, 16, 32):
        for frac in (0.5, 0.25):
            nodes = 2 * nslots
            # built nodes (even ids) hold frac of the rows
            u = torch.rand(N, generator=g)
            pick = torch.randint(0, nslots, (N,), generator=g)
            row_node = torch.where(u < frac, 2 * pick, 2 * pick + 1).to(torch.int32).to(dev)
            node_slot = torch.tensor([n // 2 if n % 2 == 0 else -1 for n in range(nodes)], dtype=torch.int32,
                                     device=dev)
            s2n = torch.arange(nslots, dtype=torch.int32, device=dev)
            hist = torch.zeros((nslots, TB, 2), dtype=torch.int64, device=dev)
            C.tree_rg_list(row_node, node_slot, None, N, nslots, work, start, lst, rowdig, listdig)
            res = {}
            for mode, dbg, kw in (("atomics", 0, {}), ("partials", 0, part_kw), ("no flush", 4, {})):
                ts = []
                for _ in range(REPS):
                    ev0.record()
                    C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, rowdig, 4, lst, start, listdig, nslots, rg.gmode,
                                   wg, s2n, hist, TB, None, 0, dbg, **kw)
                    ev1.record()
                    ev1.synchronize()
                    ts.append(ev0.elapsed_time(ev1) * 1e3)
                res[mode] = statistics.median(ts)
            print(f"nslots {nslots:2d} listed {frac:.2f}: atomics {res['atomics']:7.1f} us, partial tables + "
                  f"reduction {res['partials']:7.1f} us, no flush {res['no flush']:7.1f} us", flush=True)
    # the all-rows pass (the root) for scale
    hist = torch.zeros((1, TB, 2), dtype=torch.int64, device=dev)
    z = torch.zeros(1, dtype=torch.int32, device=dev)
    for dbg in (0, 4):
        ts = []
        for _ in range(REPS):
            ev0.record()
            C.tree_rg_hist(rg.ptr, rg.ent, rg.gbase, rg.gbin, rowdig, 4, None, None, None, 1, rg.gmode, wg, z, hist, TB,
                           None, 0, dbg)
            ev1.record()
            ev1.synchronize()
            ts.append(ev0.elapsed_time(ev1) * 1e3)
        print(f"all rows (atomics) dbg {dbg}: {statistics.median(ts):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
