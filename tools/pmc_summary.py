#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 PMC passes (scripts/gpu_pmc.sh): MFMA busy %, achieved bf16 MFMA TFLOP/s,
LDS bank conflicts per LDS instruction, HBM bytes (FETCH_SIZE+WRITE_SIZE, KiB units; gfx950 FETCH_SIZE reads
about half of a wide coalesced stream, so read bytes are a lower bound) and L2 hit rate.

Usage: tools/pmc_summary.py gpurun_out/pmc/<workload> [--top 15]"""
import argparse
import collections
import csv
import glob
import os


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:70]


def last_step_ids(d, marker="fused_update"):
    """Dispatch ids of ONE steady-state step: between the last two ``marker`` dispatches of the kernel trace (the
    first-call kernel tuning of earlier steps is excluded)."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), r.get("Dispatch_Id"), r["Kernel_Name"]))
    rows.sort()
    idx = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(idx) < 2 or rows[0][1] is None:
        return None
    return {r[1] for r in rows[idx[-2] + 1:idx[-1] + 1]}


def load_pass(d, last_step=False):
    """{kernel: {counter: sum}}, {kernel: total_ns}, {kernel: calls} for one pass directory."""
    keep = last_step_ids(d) if last_step else None
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if keep is not None and r.get("Dispatch_Id") not in keep:
                    continue
                vals[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    times = collections.defaultdict(float)
    calls = collections.Counter()
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if keep is not None and r.get("Dispatch_Id") not in keep:
                    continue
                k = short(r["Kernel_Name"])
                times[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                calls[k] += 1
    return vals, times, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--last-step", action="store_true", help="only the dispatches of the last training step")
    a = ap.parse_args()
    merged = collections.defaultdict(dict)
    times, calls = collections.defaultdict(float), collections.Counter()
    passes = sorted(glob.glob(os.path.join(a.root, "p*"))) or [a.root]    # one pass directory, or p1/p2/p3
    for p in passes:
        v, t, c = load_pass(p, a.last_step)
        for k, d in v.items():
            merged[k].update(d)
        if p.endswith("p1") or p == a.root:
            times, calls = t, c
    total = sum(times.values()) or 1.0
    # MIOpen's find-mode benchmarking kernels (first call of a new shape) are not part of the steady state
    rows = [kv for kv in sorted(times.items(), key=lambda kv: -kv[1]) if not kv[0].startswith(("naive_conv", "_ZN2ck"))]
    rows = rows[:a.top]
    print(f"{'kernel':<70} {'calls':>5} {'ms':>8} {'bf16 TF':>8} {'%peak':>6} {'LDSconf/inst':>12} "
          f"{'HBM GB/s':>9} {'L2hit%':>6}")
    for k, ns in rows:
        d = merged.get(k, {})
        busy = d.get("SQ_BUSY_CYCLES", 0.0)
        gui = d.get("GRBM_GUI_ACTIVE", 0.0)
        mfma = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in d:
            tf = d["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / ns / 1e3 if ns else 0.0
        else:   # MFMA busy cycles (all SIMDs) x 1024 dense bf16 FLOP per SIMD-cycle (32x32x16 and 16x16x32 alike)
            tf = mfma * 1024 / ns / 1e3 if ns else 0.0
        peak = 100.0 * tf / 2500.0                       # dense bf16 MFMA peak of an MI355X (no sparsity)
        lds_c = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, d.get("SQ_INSTS_LDS", 0.0))
        hbm = (d.get("FETCH_SIZE", 0.0) + d.get("WRITE_SIZE", 0.0)) * 1024 / ns if ns else 0.0
        hit, miss = d.get("TCC_HIT_sum", 0.0), d.get("TCC_MISS_sum", 0.0)
        l2 = 100.0 * hit / (hit + miss) if hit + miss else float("nan")
        _ = (gui, total, mfma, busy)
        print(f"{k:<70} {calls[k]:5d} {ns / 1e6:8.3f} {tf:8.1f} {peak:6.1f} {lds_c:12.3f} {hbm:9.1f} "
              f"{l2:6.1f}")


if __name__ == "__main__":
    main()
