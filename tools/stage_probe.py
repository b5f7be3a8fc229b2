#!/usr/bin/env python3
"""Per-stage host/GPU latency of the headline queries (where the end-to-end time goes).

For each of the 8 benchmark queries (SQL path, prepared once) this reports, as medians over
``--reps`` runs:

* ``e2e``     -- ``DataFrame.run()`` (what bench.py times);
* ``kernel``  -- the prepared scan alone (``PreparedScan.run`` + synchronize);
* ``scan/merge/finalize/post`` -- the engine's own stage clocks (``QueryResult.stats``);
* ``sql``     -- e2e minus the engine's ``exec_ms`` (the SQL operators above the Druid query).

usage: python tools/stage_probe.py --sf 100 [--reps 30]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--query", default=None, help="only queries whose name contains this")
    ap.add_argument("--wrap", default="", help="comma-separated module:function names to time (per-call ms)")
    a = ap.parse_args()
    timers = _wrap(a.wrap.split(",")) if a.wrap else {}
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.session import Session

    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(engine=Engine(), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    sync = torch.cuda.synchronize if dev != "cpu" else (lambda: None)
    print(f"{'query':52s} {'e2e':>7s} {'kernel':>7s} {'scan':>7s} {'merge':>7s} {'final':>7s} {'post':>7s} {'sql':>7s}")
    for name, q in tpch.BENCH_QUERIES:
        if a.query and a.query.lower() not in name.lower():
            continue
        df = s.sql(q)
        for _ in range(3):
            df.run()
        sync()
        prep = df.druid_queries()[0]._prepared
        scan = prep.scans[0][2]
        e2e, ker, st = [], [], {k: [] for k in ("scan_ms", "merge_ms", "finalize_ms", "post_ms", "sql")}
        for _ in range(a.reps):
            t = time.perf_counter()
            df.run()
            e2e.append((time.perf_counter() - t) * 1e3)
            hist = df.last_stats.get("druid") or []
            res_stats = getattr(prep, "last_stats", None) or {}
            for k in ("scan_ms", "merge_ms", "finalize_ms", "post_ms"):
                st[k].append(res_stats.get(k, float("nan")))
            st["sql"].append(e2e[-1] - res_stats.get("exec_ms", float("nan")))
            if scan is not None:
                sync()
                t = time.perf_counter()
                scan.run()
                sync()
                ker.append((time.perf_counter() - t) * 1e3)
        for k in timers:
            timers[k].clear()
        for _ in range(a.reps):
            df.run()
        med = statistics.median
        for k, v in timers.items():
            if v:
                print(f"    {k:60s} calls/run {len(v) / a.reps:5.1f}  median {med(v):8.3f} ms  total/run {sum(v) / a.reps:8.3f} ms")
        print(f"{name[:52]:52s} {med(e2e):7.3f} {med(ker) if ker else float('nan'):7.3f} "
              + " ".join(f"{med(st[k]):7.3f}" for k in ("scan_ms", "merge_ms", "finalize_ms", "post_ms", "sql")))


def _wrap(names):
    """Replace module-level functions / class methods by timing wrappers."""
    import functools
    import importlib

    out = {}
    for spec in names:
        mod, _, attr = spec.partition(":")
        m = importlib.import_module(mod)
        owner, fname = m, attr
        if "." in attr:
            cls, fname = attr.split(".", 1)
            owner = getattr(m, cls)
        f = getattr(owner, fname)
        rec = out.setdefault(spec, [])

        def mk(f, rec):
            @functools.wraps(f)
            def w(*args, **kw):
                t = time.perf_counter()
                try:
                    return f(*args, **kw)
                finally:
                    rec.append((time.perf_counter() - t) * 1e3)
            return w
        setattr(owner, fname, mk(f, rec))
        # modules that imported the function by name
        for mm in list(sys.modules.values()):
            if mm is not None and getattr(mm, "__name__", "").startswith("spark_druid_olap_amd") and \
                    getattr(mm, fname, None) is f and owner is m:
                setattr(mm, fname, getattr(owner, fname))
    return out


if __name__ == "__main__":
    main()
