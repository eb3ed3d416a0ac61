#!/usr/bin/env python3
"""Per-kernel PMC counter table from rocprofv3 sqlite output (run_results.db; the pmc_events view): for every
kernel name matching --match, the median over its dispatches of each counter (summed over the counter's instances
per dispatch), plus the median duration and the resources (VGPR / AGPR / LDS) of the dispatch.
Usage: python tools/pmc_db.py <run_results.db> [--match gemm_glds] [--top 8]"""
import argparse
import collections
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    c = sqlite3.connect(a.db).cursor()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for did, name, cn, cv in c.execute("select dispatch_id, name, counter_name, counter_value from pmc_events"):
        if a.match and a.match not in name:
            continue
        per[did][cn] += cv
        names[did] = name
    info = {r[0]: r[1:] for r in c.execute("select dispatch_id, duration, vgpr_count, accum_vgpr_count, lds_size, "
                                          "grid_x, workgroup_x from kernels")}
    byk = collections.defaultdict(list)
    for did, cnt in per.items():
        byk[names[did]].append((did, cnt))
    rows = sorted(byk.items(), key=lambda kv: -sum(info.get(d, (0,))[0] for d, _ in kv[1]))[:a.top]
    for name, lst in rows:
        durs = [info[d][0] for d, _ in lst if d in info]
        d0 = info.get(lst[0][0], (0, 0, 0, 0, 0, 0))
        print(f"{name[:110]}")
        print(f"  dispatches {len(lst)}  median {statistics.median(durs) / 1e3 if durs else 0:.1f} us  "
              f"vgpr {d0[1]} agpr {d0[2]} lds {d0[3]} grid {d0[4]} wg {d0[5]}")
        keys = sorted({k for _, cnt in lst for k in cnt})
        for k in keys:
            v = statistics.median(cnt.get(k, 0.0) for _, cnt in lst)
            print(f"    {k:28s} {v:16.0f}")


if __name__ == "__main__":
    main()
