#!/usr/bin/env python3
"""Host time before the launch and after the result wait of each headline query (SQL path).

For every statement: ``pre`` = DataFrame.run() entry -> the native launch call (SQL operators,
prepared-query dispatch, buffer lookup), ``gpu`` = launch call -> the end of the result wait
(native.run_scan + native.fetch_small / stream_sync), ``post`` = wait end -> run() return
(decode, Druid post-processing, SQL projections, result wrapping).  Medians over --reps runs.

usage: python tools/host_phases.py --sf 100 [--reps 200]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.ops import native
    from spark_druid_olap_amd.session import Session

    m = native.load()
    marks = {}

    class Wrap:  # the extension module's functions, timestamped
        def __init__(self, mod):
            self._m = mod

        def __getattr__(self, k):
            f = getattr(self._m, k)
            if k in ("run_scan", "module_launch", "scan"):
                def g(*x, **y):
                    marks.setdefault("launch", time.perf_counter())
                    return f(*x, **y)
                return g
            if k in ("fetch_small", "stream_sync"):
                def h(*x, **y):
                    r = f(*x, **y)
                    marks["wait_end"] = time.perf_counter()
                    return r
                return h
            return f

    native._mod = Wrap(m)
    dev = "cuda:0"
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
    res = {n: {"pre": [], "gpu": [], "post": [], "e2e": []} for n, _ in qs}
    for _ in range(a.reps):
        for n, df in qs:
            marks.clear()
            t0 = time.perf_counter()
            df.run()
            t1 = time.perf_counter()
            if "launch" in marks and "wait_end" in marks:
                res[n]["pre"].append(marks["launch"] - t0)
                res[n]["gpu"].append(marks["wait_end"] - marks["launch"])
                res[n]["post"].append(t1 - marks["wait_end"])
            res[n]["e2e"].append(t1 - t0)
    med = statistics.median
    print(f"{'query':52s} {'e2e':>8s} {'pre':>8s} {'gpu+wait':>9s} {'post':>8s}   (us, median)")
    for n, r in res.items():
        f = lambda k: med(r[k]) * 1e6 if r[k] else float("nan")  # noqa: E731
        print(f"{n[:52]:52s} {f('e2e'):8.1f} {f('pre'):8.1f} {f('gpu'):9.1f} {f('post'):8.1f}")


if __name__ == "__main__":
    main()
