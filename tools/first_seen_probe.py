#!/usr/bin/env python3
"""Host cost of a first-seen BI statement text (BASELINE config 5's cold start).

The cold serving run prewarms one text per template; every other literal binding of a template is
planned on first sight inside the measured window.  This runs the same thing in one thread: prewarm
one text per template, then plan (and run) every other text once, reporting per-template wall time
of the first sight and, with ``--profile``, the top host frames of those first sights.

  python tools/first_seen_probe.py --sf 0.05 [--profile 25]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=0.05)
    ap.add_argument("--profile", type=int, default=0, help="print the top N cumulative frames")
    ap.add_argument("--bind", default="years")
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.models import bi, tpch
    from spark_druid_olap_amd.session import Session

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    bi.register(s)
    qs = [(n, q) for n, _, q in bi.statements(25, a.bind)]
    seen, rest = set(), []
    for n, q in qs:
        if n in seen:
            rest.append((n, q))
            continue
        seen.add(n)
        s.sql(q).collect()
    if dev == "cuda":
        from spark_druid_olap_amd.engine.device_exec import wait_background_compiles

        wait_background_compiles()
    per = {}
    prof = cProfile.Profile() if a.profile else None
    plan_t = run_t = 0.0
    for n, q in rest:
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        df = s.sql(q)
        t1 = time.perf_counter()
        df.collect()
        if prof:
            prof.disable()
        t2 = time.perf_counter()
        plan_t += t1 - t0
        run_t += t2 - t1
        per.setdefault(n, []).append((t1 - t0, t2 - t1))
    print(f"{len(rest)} first-seen texts on {dev}: sql() {1e3 * plan_t / max(1, len(rest)):.2f} ms, "
          f"collect() {1e3 * run_t / max(1, len(rest)):.2f} ms per text")
    for n, xs in sorted(per.items(), key=lambda kv: -sum(p + r for p, r in kv[1])):
        print(f"  {n[:48]:48s} n={len(xs):3d} sql {1e3 * sum(p for p, _ in xs) / len(xs):7.2f} ms"
              f"  collect {1e3 * sum(r for _, r in xs) / len(xs):7.2f} ms")
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(a.profile)
        pstats.Stats(prof).sort_stats("tottime").print_stats(a.profile)


if __name__ == "__main__":
    main()
