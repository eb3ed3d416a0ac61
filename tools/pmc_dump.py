#!/usr/bin/env python3
"""Print per-kernel durations (rocprofv3 --kernel-trace db) and summed PMC counters (csv dirs) matching a name filter.
Usage: python tools/pmc_dump.py FILTER gpurun_out/<kt dir> [gpurun_out/<pmc dir> ...]"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def main():
    filt = sys.argv[1]
    for d in sys.argv[2:]:
        dbs = glob.glob(os.path.join(d, "*.db"))
        if dbs:
            cur = sqlite3.connect(dbs[0]).cursor()
            t = [r[0] for r in cur.execute("select name from sqlite_master where type='table' and name like "
                                           "'rocpd_kernel_dispatch%'")][0]
            sfx = t.split("rocpd_kernel_dispatch_")[1]
            agg = collections.defaultdict(list)
            for name, gx, dur in cur.execute(f"select s.kernel_name, d.grid_size_x, d.end-d.start from {t} d join "
                                             f"rocpd_info_kernel_symbol_{sfx} s on d.kernel_id=s.id"):
                if filt in name:
                    agg[(name[:70], gx)].append(dur / 1e3)
            for k, v in agg.items():
                print(f"{d}: {k[0]} grid {k[1]}: {sum(v) / len(v):.1f} us x{len(v)}")
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            agg = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if filt in r["Kernel_Name"]:
                    agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
            for k, v in agg.items():
                print(f"{d}: {k}: " + ", ".join(f"{a}={b:.3g}" for a, b in sorted(v.items())))


if __name__ == "__main__":
    main()
