"""Summarise rocprofv3 ``*_counter_collection.csv`` files per kernel (summed over dispatches).

Usage: python bench/pmc_summary.py DIR [DIR ...] [--match hist_mfma] [--md]
Each DIR is a ``-d`` output directory of one ``rocprofv3 --pmc`` pass; counters of all passes are
joined by kernel name. Also prints derived per-kernel ratios when their inputs are present.
"""
import argparse
import collections
import csv
import glob
import os


def load(dirs, match):
    val = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k = r["Kernel_Name"]
                if match and match not in k:
                    continue
                key = k[:120]
                val[key][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[key].add((d, r["Dispatch_Id"]))
                dur[key][(d, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return val, disp, dur


def per_dispatch(dirs, match, n):
    """Counters of the first ``n`` dispatches of each matching kernel, per pass directory (e.g.
    the root vs the deeper levels of a tree: one histogram dispatch per level)."""
    for d in dirs:
        rows = collections.defaultdict(lambda: collections.defaultdict(dict))
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                if match and match not in r["Kernel_Name"]:
                    continue
                k = (r["Kernel_Name"][:60], int(r["Dispatch_Id"]))
                rows[k[0]][k[1]][r["Counter_Name"]] = float(r["Counter_Value"])
                rows[k[0]][k[1]]["_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for kern, ds in rows.items():
            print(f"\n[{os.path.basename(d)}] {kern}")
            for i, did in enumerate(sorted(ds)[:n]):
                c = ds[did]
                extra = ""
                if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
                    extra = f"  lds_conflict/active {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}"
                cs = "  ".join(f"{k}={v:.4g}" for k, v in sorted(c.items()) if k != "_us")
                print(f"  #{i:3d} {c['_us']:9.1f} us{extra}  {cs}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--per-dispatch", type=int, default=0,
                    help="also list the first N dispatches of each kernel (duration + conflict ratio), by pass")
    args = ap.parse_args()
    val, disp, dur = load(args.dirs, args.match)
    if args.per_dispatch:
        per_dispatch(args.dirs, args.match, args.per_dispatch)
    for k in sorted(val, key=lambda k: -sum(dur[k].values())):
        c = val[k]
        n_pass = len({d for d, _ in disp[k]})
        ms = sum(dur[k].values()) / 1e6 / max(n_pass, 1)
        print(f"\n{k}\n  dispatches/pass {len(disp[k]) // max(n_pass, 1)}  time/pass {ms:.3f} ms")
        for name in sorted(c):
            print(f"  {name:28s} {c[name]:.4g}")
        waves = c.get("SQ_WAVES")
        if waves:
            for name in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
                if name in c:
                    print(f"  {name + '/wave':28s} {c[name] / waves:.1f}")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
            print(f"  {'lds conflict/active':28s} {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
            print(f"  {'wait_inst/wave_cycles':28s} {c['SQ_WAIT_INST_ANY'] / max(c['SQ_WAVE_CYCLES'], 1):.3f}")
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
            print(f"  {'valu_active/wave_cycles':28s} {c['SQ_ACTIVE_INST_VALU'] / max(c['SQ_WAVE_CYCLES'], 1):.3f}")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            print(f"  {'L2 hit rate':28s} {c['TCC_HIT_sum'] / max(c['TCC_HIT_sum'] + c['TCC_MISS_sum'], 1):.3f}")


if __name__ == "__main__":
    main()
