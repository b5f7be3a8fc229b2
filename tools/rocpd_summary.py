#!/usr/bin/env python3
"""Summarize a rocprofv3 SQLite (rocpd) database: per-kernel stats restricted to the query phase
(everything dispatched after the first scan kernel), plus memory-copy totals.

usage: rocpd_summary.py run_results.db [--all] [--top N]
"""
import argparse
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    if name.startswith("void at::native::"):
        n = name[len("void at::native::"):]
        return "at::" + n.split("<")[0] + ("<" + n.split("<")[1].split(",")[0][:60] + ">" if "<" in n else "")
    return name[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--tail-ms", type=float, default=0.0,
                    help="only kernels starting in the last T ms of the trace (the timed steps)")
    ap.add_argument("--timeline-ms", type=float, default=0.0,
                    help="also print every kernel of the last T ms in order (start offset, duration, gap)")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    t0 = None
    if not a.all:
        for n, s, e in rows:
            if n.startswith("sdo_jit") or n.startswith("sdo::olap_scan"):
                t0 = s
                break
    if a.tail_ms > 0 and rows:
        t0 = max(e for _, _, e in rows) - int(a.tail_ms * 1e6)
    agg = defaultdict(lambda: [0, 0.0, 1e30, 0.0])
    total = 0.0
    for n, s, e in rows:
        if t0 is not None and s < t0:
            continue
        d = (e - s) / 1e3  # us
        x = agg[short(n)]
        x[0] += 1
        x[1] += d
        x[2] = min(x[2], d)
        x[3] = max(x[3], d)
        total += d
    print(f"{'kernel':110s} {'calls':>6s} {'total_us':>11s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'%':>6s}")
    for n, (c, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{n:110s} {c:6d} {t:11.1f} {t / c:9.1f} {mn:9.1f} {mx:9.1f} {100 * t / max(total, 1e-9):6.2f}")
    print(f"{'TOTAL':110s} {sum(v[0] for v in agg.values()):6d} {total:11.1f}")
    if a.timeline_ms > 0 and rows:
        end = max(e for _, _, e in rows)
        tl = [(n, s, e) for n, s, e in rows if s >= end - int(a.timeline_ms * 1e6)]
        print(f"--- timeline of the last {a.timeline_ms} ms ({len(tl)} kernels)")
        prev = None
        for n, s, e in tl:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"{(s - tl[0][1]) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:8.1f}  {short(n)[:90]}")
            prev = e
    try:
        mc = con.execute("select start, end, size from memory_copies").fetchall()
        if t0 is not None:
            mc = [m for m in mc if m[0] >= t0]
        tb = sum(m[2] or 0 for m in mc)
        tt = sum((m[1] - m[0]) / 1e3 for m in mc)
        print(f"memory copies: {len(mc)} copies, {tb / 1e6:.1f} MB, {tt:.1f} us")
    except sqlite3.Error as e:
        print("memory copies: n/a", e)


if __name__ == "__main__":
    main()
