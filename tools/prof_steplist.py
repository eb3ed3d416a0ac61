#!/usr/bin/env python3
"""Ordered dispatch list (duration, gap to the previous kernel, grid) of ONE training step — the dispatches between
the last two fused-updater launches — from a rocprofv3 --kernel-trace db.
Usage: python tools/prof_steplist.py <run_results.db>"""
import sqlite3, glob, re, sys
path = sys.argv[1]
cur = sqlite3.connect(path).cursor()
t = [r[0] for r in cur.execute("select name from sqlite_master where type='table' and name like 'rocpd_kernel_dispatch%'")][0]
sfx = t.split("rocpd_kernel_dispatch_")[1]
cols = [r[1] for r in cur.execute(f"pragma table_info({t})")]
sq = "d.stream_id" if "stream_id" in cols else ("d.queue_id" if "queue_id" in cols else "0")
rows = list(cur.execute(f"select s.kernel_name, d.end-d.start, d.start, d.end, d.grid_size_x, d.workgroup_size_x, {sq} "
                        f"from {t} d join rocpd_info_kernel_symbol_{sfx} s on d.kernel_id=s.id order by d.start"))
idx = [i for i, r in enumerate(rows) if "fused_update" in r[0]]
lo, hi = idx[-2] + 1, idx[-1] + 1
prev = None
busy = {}
t0 = rows[lo][2]
for name, dur, st, en, gx, wx, sid in rows[lo:hi]:
    n = re.sub(r"\(anonymous namespace\)::|void ", "", name).split("(")[0][:90]
    gap = (st - prev) / 1e3 if prev else 0
    busy[sid] = busy.get(sid, 0) + dur
    print(f"{(st - t0)/1e3:8.1f} {dur/1e3:7.1f}us gap {gap:6.1f} s{sid} grid {gx:7d} {n}")
    prev = en if prev is None else max(prev, en)
span = (max(r[3] for r in rows[lo:hi]) - t0) / 1e3
print(f"span {span:.1f} us; busy per stream: " + ", ".join(f"s{k} {v/1e3:.1f} us" for k, v in sorted(busy.items())))
