#!/usr/bin/env python3
"""Where the host time of a headline query goes, layer by layer (SQL path, one GPU).

For every statement, medians over --reps interleaved runs of:

* ``sql``     -- ``DataFrame.run()`` (what bench.py times);
* ``engine``  -- the pushed query's ``PreparedQuery.run()`` alone (no SQL operators);
* ``partials``-- ``PreparedQuery.run_partials`` + a stream sync (scan + merge, no finalize);
* ``kernel``  -- the scan's native launch + a stream sync (the GPU floor plus one launch/sync);
* ``sql_outside`` -- within each ``sql`` run, the time outside the engine's ``PreparedQuery.run``.

``sql - engine`` is the SQL layer's cost, ``engine - partials`` finalize + post, ``partials - kernel``
the engine's launch path.

usage: python tools/host_floor.py --sf 100 [--reps 100]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    os.environ.setdefault("SDO_JIT_SPECIALIZE", "sync")
    os.environ.setdefault("SDO_JIT_SPECIALIZE_AFTER", "1")
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.ops import native
    from spark_druid_olap_amd.session import Session
    from spark_druid_olap_amd.sql import plan as P

    dev = torch.device("cuda:0")
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(engine=Engine(), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    qs = [(n, s.sql(q)) for n, q in tpch.BENCH_QUERIES]
    for _ in range(3):
        for _, df in qs:
            df.run()
    torch.cuda.synchronize()
    layers = {}
    for n, df in qs:
        dqs = P.find_all_deep(df.plan, P.DruidQuery)
        pqs = [s.prepare_druid(d) for d in dqs]
        pq = pqs[0] if len(pqs) == 1 else None
        fns = {"sql": df.run}
        if pq is not None:
            fns["engine"] = pq.run

            def partials(pq=pq):
                pq.run_partials(time.perf_counter())
                native.stream_sync(dev)

            fns["partials"] = partials
            prep = pq.scans[0][2]
            if prep is not None and getattr(prep, "jit", None) is not None:
                def kernel(prep=prep):
                    prep.run()
                    native.stream_sync(dev)

                fns["kernel"] = kernel
        layers[n] = fns
    # inside each sql run: the time spent in the engine's PreparedQuery.run itself (same call)
    from spark_druid_olap_amd.engine import executor as E

    inner = []
    orig_run = E.PreparedQuery.run

    def timed_run(self):
        t = time.perf_counter()
        try:
            return orig_run(self)
        finally:
            inner.append(time.perf_counter() - t)

    E.PreparedQuery.run = timed_run
    res = {n: {k: [] for k in list(fns) + ["sql_outside"]} for n, fns in layers.items()}
    for _ in range(a.reps):
        for n, fns in layers.items():
            for k, f in fns.items():
                inner.clear()
                t0 = time.perf_counter()
                f()
                dt = time.perf_counter() - t0
                res[n][k].append(dt * 1e6)
                if k == "sql":
                    res[n]["sql_outside"].append((dt - sum(inner)) * 1e6)
    med = statistics.median
    cols = ("sql", "sql_outside", "engine", "partials", "kernel")
    print(f"{'query':52s} " + " ".join(f"{c:>11s}" for c in cols) + f"   (us, median of {a.reps})")
    for n, r in res.items():
        cells = [f"{med(r[k]):11.1f}" if r.get(k) else f"{'-':>11s}" for k in cols]
        print(f"{n[:52]:52s} " + " ".join(cells))


if __name__ == "__main__":
    main()
