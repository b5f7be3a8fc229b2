#!/usr/bin/env python3
"""cProfile the host side of the benchmark loop (per-query Python/launch/merge/finalize cost).

usage: python tools/host_profile.py --sf 100 --mode sql|spec --steps 3 [--query NAME]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--mode", default="sql")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--query", default=None)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import bench_specs
    from spark_druid_olap_amd.session import Session

    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    eng = Engine()
    if a.mode == "sql":
        s = Session(engine=eng, conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
        s.register_datasource(ds)
        s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
        s.sql(tpch.druid_ddl(with_column_mapping=False))
        qs = [(n, s.sql(q)) for n, q in tpch.BENCH_QUERIES]
    else:
        qs = [(n, eng.prepare(q, ds)) for n, q in bench_specs()]
    if a.query:  # comma-separated name substrings
        want = [w.strip().lower() for w in a.query.split(",")]
        qs = [(n, q) for n, q in qs if any(w in n.lower() for w in want)]
    for _ in range(2):
        for n, q in qs:
            q.run()
    torch.cuda.synchronize() if dev != "cpu" else None
    for n, q in qs:
        t = time.perf_counter()
        for _ in range(5):
            q.run()
        print(f"{n:55s} {(time.perf_counter() - t) / 5 * 1e3:8.3f} ms")
    # interleaved (bench) order, with and without the cyclic GC
    import gc

    for gc_on in (True, False):
        if not gc_on:
            gc.disable()
        lat = {n: [] for n, _ in qs}
        for _ in range(5):
            for n, q in qs:
                t = time.perf_counter()
                q.run()
                lat[n].append((time.perf_counter() - t) * 1e3)
        gc.enable()
        print(f"--- interleaved, gc={'on' if gc_on else 'off'}")
        for n, v in lat.items():
            print(f"{n:55s} avg {sum(v) / len(v):8.3f}  min {min(v):8.3f}  max {max(v):8.3f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        for n, q in qs:
            q.run()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(a.top)
    st.sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
