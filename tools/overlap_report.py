#!/usr/bin/env python3
"""Collective / compute overlap of ONE training step from a rocprofv3 --kernel-trace db (the dispatches between the
last two fused-updater launches): every RCCL kernel (name matching nccl / rccl) with its stream, duration and the
fraction of its duration during which a non-collective kernel of the step was also running (i.e. overlapped by
backward compute), plus per-stream busy time.
Usage: python tools/overlap_report.py <run_results.db|dir> [--marker fused_update]"""
import argparse
import glob
import os
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="fused_update")
    a = ap.parse_args()
    path = a.db if a.db.endswith(".db") else glob.glob(os.path.join(a.db, "*.db"))[0]
    cur = sqlite3.connect(path).cursor()
    t = [r[0] for r in cur.execute("select name from sqlite_master where type='table' and name like "
                                   "'rocpd_kernel_dispatch%'")][0]
    sfx = t.split("rocpd_kernel_dispatch_")[1]
    cols = [r[1] for r in cur.execute(f"pragma table_info({t})")]
    sq = "d.stream_id" if "stream_id" in cols else ("d.queue_id" if "queue_id" in cols else "0")
    rows = list(cur.execute(f"select s.kernel_name, d.start, d.end, {sq} from {t} d join "
                            f"rocpd_info_kernel_symbol_{sfx} s on d.kernel_id=s.id order by d.start"))
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(idx) < 2:
        print("fewer than two marker dispatches")
        return
    step = rows[idx[-2] + 1:idx[-1] + 1]
    is_coll = [bool(re.search(r"nccl|rccl", n, re.I)) for n, *_ in step]
    comp = [(s, e) for (n, s, e, _), c in zip(step, is_coll) if not c]
    busy = {}
    print(f"{'start_us':>9s} {'dur_us':>8s} {'stream':>6s} {'overlap':>8s}  kernel")
    t0 = step[0][1]
    tot = ovl = 0.0
    for (n, s, e, sid), c in zip(step, is_coll):
        busy[sid] = busy.get(sid, 0) + (e - s)
        if not c:
            continue
        # union of compute intervals intersected with [s, e]
        cov, last = 0, s
        for cs, ce in comp:
            if ce <= last or cs >= e:
                continue
            a0, a1 = max(cs, last), min(ce, e)
            if a1 > a0:
                cov += a1 - a0
                last = a1
        dur = e - s
        tot += dur
        ovl += cov
        short = re.sub(r"\(.*", "", n)[:70]
        print(f"{(s - t0) / 1e3:9.1f} {dur / 1e3:8.1f} {sid:>6} {100.0 * cov / max(dur, 1):7.1f}%  {short}")
    span = (max(r[2] for r in step) - t0) / 1e3
    print(f"collectives: {sum(is_coll)} kernels, {tot / 1e3:.1f} us, {100.0 * ovl / max(tot, 1):.1f}% overlapped by "
          f"compute; step span {span:.1f} us")
    print("busy per stream: " + ", ".join(f"s{k} {v / 1e3:.1f} us" for k, v in sorted(busy.items(), key=str)))


if __name__ == "__main__":
    main()
