#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace SQLite db (or kernel_trace.csv) into a per-kernel table.

Usage: tools/prof_summary.py <run_results.db|kernel_trace.csv> [--steps N] [--top K]
Groups kernels by (truncated) name, reports calls, total ms, ms per step and share of GPU time."""
import argparse
import collections
import csv
import sqlite3


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
        q = f"select {name_col}, start, end from kernels"
        for n, s, e in c.execute(q + " order by start"):
            rows.append((n, (e - s) / 1e6))
    else:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    return rows


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0]
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--last", type=int, default=0,
                    help="keep only the dispatches after the last N+1-th --marker kernel (steady-state steps)")
    ap.add_argument("--marker", default="fused_update_kernel")
    ap.add_argument("--steady", type=int, default=0,
                    help="only the last N complete training steps (split at the fused-updater kernel), so "
                         "initialisation and warm-up dispatches do not dilute per-step numbers")
    a = ap.parse_args()
    rows = load(a.path)
    if a.last:
        idx = [i for i, (n, _) in enumerate(rows) if a.marker in n]
        if len(idx) > a.last:
            rows = rows[idx[-a.last - 1] + 1:]
    if a.steady:
        steps = [[]]
        for r in rows:
            steps[-1].append(r)
            if "fused_update" in r[0]:
                steps.append([])
        full = steps[:-1]
        sel = full[-a.steady:]
        rows = [r for st in sel for r in st]
        a.steps = len(sel)
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, ms in rows:
        k = short(n)
        agg[k][0] += 1
        agg[k][1] += ms
    total = sum(v[1] for v in agg.values())
    print(f"kernels: {len(rows)} dispatches, total GPU time {total:.2f} ms ({total / a.steps:.2f} ms/step over "
          f"{a.steps} steps)")
    print(f"{'ms/step':>9} {'share':>6} {'calls':>7}  kernel")
    for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{ms / a.steps:9.3f} {100 * ms / total:5.1f}% {c:7d}  {k}")


if __name__ == "__main__":
    main()
