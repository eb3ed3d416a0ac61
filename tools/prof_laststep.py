#!/usr/bin/env python3
"""Per-kernel table of ONE training step (the dispatches between the last two fused-updater launches) from a
rocprofv3 --kernel-trace db: steady-state cost without the first-step kernel tuning.
Usage: python tools/prof_laststep.py <run_results.db> [--top N] [--marker fused_update]"""
import argparse
import collections
import glob
import os
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--marker", default="fused_update")
    a = ap.parse_args()
    path = a.db if a.db.endswith(".db") else glob.glob(os.path.join(a.db, "*.db"))[0]
    cur = sqlite3.connect(path).cursor()
    t = [r[0] for r in cur.execute("select name from sqlite_master where type='table' and name like "
                                   "'rocpd_kernel_dispatch%'")][0]
    sfx = t.split("rocpd_kernel_dispatch_")[1]
    rows = list(cur.execute(f"select s.kernel_name, d.end-d.start, d.start, d.end from {t} d join "
                            f"rocpd_info_kernel_symbol_{sfx} s on d.kernel_id=s.id order by d.start"))
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    lo, hi = idx[-2] + 1, idx[-1] + 1
    step = rows[lo:hi]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, dur, _, _ in step:
        n = re.sub(r"\(anonymous namespace\)::|void ", "", name).split("(")[0][:70]
        agg[n][0] += 1
        agg[n][1] += dur / 1e6
    tot = sum(v[1] for v in agg.values())
    wall = (step[-1][3] - step[0][2]) / 1e6
    print(f"one step: {len(step)} dispatches, GPU time {tot:.2f} ms, first-start..last-end {wall:.2f} ms")
    print("      ms  share calls  kernel")
    for n, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{ms:8.3f} {100 * ms / tot:5.1f}% {c:5d}  {n}")


if __name__ == "__main__":
    main()
