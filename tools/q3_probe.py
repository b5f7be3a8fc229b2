#!/usr/bin/env python3
"""Where the headline TPC-H Q3's host time goes (verdict r5 #7): the engine's finalize of the
~1.2M-group result at SF100 -- the native decode + one D2H (partials._native_sparse: rows, bytes
shipped, wall) against the rest of the statement, then a cProfile of repeated runs.

  python tools/q3_probe.py [--sf 100] [--iters 30] [--query 'TPCH Q3']"""
import argparse
import cProfile
import io
import os
import pstats
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--query", default="TPCH Q3")
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine import executor as EX
    from spark_druid_olap_amd.engine import partials as PT
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.session import Session

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session()
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    q = dict(tpch.BENCH_QUERIES)[a.query]
    stats = []
    real_ns, real_fin = PT._native_sparse, PT.finalize

    def ns(prog, parts, out_types, want_gid):
        t0 = time.perf_counter()
        r = real_ns(prog, parts, out_types, want_gid)
        stats.append(("native_sparse", (time.perf_counter() - t0) * 1e3, int(parts.keys.numel()),
                      None if r is None else sum(x.nbytes for x in list(r[1]) + list(r[4].values())
                                                  if hasattr(x, "nbytes"))))
        return r

    def fin(*args, **kw):
        t0 = time.perf_counter()
        r = real_fin(*args, **kw)
        stats.append(("finalize", (time.perf_counter() - t0) * 1e3, None, None))
        return r

    PT._native_sparse, EX.finalize = ns, fin
    pq = s.sql(q).prepared()  # (as bench.py times it: the prepared statement's run)
    for _ in range(3):
        pq.run()
    stats.clear()
    walls = []
    for _ in range(a.iters):
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        b = pq.run()
        walls.append((time.perf_counter() - t0) * 1e3)
    print(f"{a.query}: {b.n} rows, wall median {statistics.median(walls):.3f} ms (min {min(walls):.3f})")
    for name in ("native_sparse", "finalize"):
        xs = [x for x in stats if x[0] == name]
        if xs:
            print(f"  {name:14s} median {statistics.median(x[1] for x in xs):.3f} ms  rows {xs[-1][2]}  "
                  f"host bytes {xs[-1][3]}")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.iters):
        pq.run()
    pr.disable()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(25)
    print(out.getvalue()[:6000])


if __name__ == "__main__":
    main()
