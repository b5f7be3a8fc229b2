#!/usr/bin/env python3
"""Summarize a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv) per kernel name."""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
    ks = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = c.execute("select kernel_id, start, end from rocpd_kernel_dispatch").fetchall()
    out = defaultdict(list)
    for kid, s, e in rows:
        out[ks.get(kid, str(kid))].append((e - s) / 1e3)
    return out


def from_csv(path):
    out = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            out[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return out


def main(p):
    files = glob.glob(os.path.join(p, "**", "*.db"), recursive=True) if os.path.isdir(p) else [p]
    if not files:
        files = glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
    data = defaultdict(list)
    for f in files:
        d = from_db(f) if f.endswith(".db") else from_csv(f)
        for k, v in d.items():
            data[k].extend(v)
    tot = sum(sum(v) for v in data.values())
    print(f"{'kernel':70s} {'calls':>7s} {'total_us':>12s} {'avg_us':>10s} {'max_us':>10s} {'pct':>6s}")
    for k, v in sorted(data.items(), key=lambda kv: -sum(kv[1])):
        name = k if len(k) <= 70 else k[:67] + "..."
        print(f"{name:70s} {len(v):7d} {sum(v):12.1f} {sum(v)/len(v):10.2f} {max(v):10.2f} {100*sum(v)/tot:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
