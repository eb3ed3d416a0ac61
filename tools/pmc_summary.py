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

PEAK_TF = 2500.0     # dense bf16 MFMA peak of an MI355X (no sparsity)


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
    ap.add_argument("--hbm-tbs", type=float, default=8.0, help="HBM peak for the roofline (spec 8.0)")
    ap.add_argument("--raw-fetch", action="store_true", help="do not double FETCH_SIZE")
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
    print(f"{'kernel':<60} {'calls':>5} {'ms':>7} {'bf16 TF':>7} {'%peak':>5} {'LDSc/i':>6} {'rdMB':>8} {'wrMB':>8} "
          f"{'GB/s':>7} {'L2hit%':>6} {'bound':>5} {'%roof':>5}")
    tot_ns = tot_roof = 0.0
    for k, ns in rows:
        d = merged.get(k, {})
        mfma = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in d:
            flop = d["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512
        else:   # MFMA busy cycles (all SIMDs) x 1024 dense bf16 FLOP per SIMD-cycle (32x32x16 and 16x16x32 alike)
            flop = mfma * 1024
        tf = flop / ns / 1e3 if ns else 0.0
        peak = 100.0 * tf / PEAK_TF
        lds_c = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, d.get("SQ_INSTS_LDS", 0.0))
        # FETCH_SIZE / WRITE_SIZE are KiB. gfx950 FETCH_SIZE tallies a wide coalesced stream at half its bytes
        # (MI355X_MICROARCH.md, HBM): the read column is FETCH_SIZE x 2 (x1 with --raw-fetch)
        rd = d.get("FETCH_SIZE", 0.0) * 1024 * (1 if a.raw_fetch else 2)
        wr = d.get("WRITE_SIZE", 0.0) * 1024
        gbs = (rd + wr) / ns if ns else 0.0
        hit, miss = d.get("TCC_HIT_sum", 0.0), d.get("TCC_MISS_sum", 0.0)
        l2 = 100.0 * hit / (hit + miss) if hit + miss else float("nan")
        # roofline: the kernel's own lower bound max(FLOP / MFMA peak, bytes / HBM peak)
        t_mfma = flop / (PEAK_TF * 1e12) * 1e9
        t_mem = (rd + wr) / (a.hbm_tbs * 1e12) * 1e9
        t_roof = max(t_mfma, t_mem)
        bound = "mfma" if t_mfma >= t_mem else "hbm"
        roof = 100.0 * t_roof / ns if ns else 0.0
        tot_ns += ns
        tot_roof += t_roof
        print(f"{k[:60]:<60} {calls[k]:5d} {ns / 1e6:7.3f} {tf:7.1f} {peak:5.1f} {lds_c:6.2f} {rd / 1e6:8.1f} "
              f"{wr / 1e6:8.1f} {gbs:7.0f} {l2:6.1f} {bound:>5} {roof:5.1f}")
    print(f"listed kernels: {tot_ns / 1e6:.3f} ms, roofline bound {tot_roof / 1e6:.3f} ms "
          f"({100.0 * tot_roof / max(tot_ns, 1.0):.1f} %); all kernels {total / 1e6:.3f} ms; "
          f"peaks {PEAK_TF:.0f} TF/s bf16 dense, {a.hbm_tbs:.1f} TB/s HBM")

if __name__ == "__main__":
    main()
