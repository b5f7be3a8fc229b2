"""cProfile one TPC-H 22 SQL query end to end on the GPU box (where the host time goes).

usage: python tools/tpch22_host_profile.py --sf 100 --query Q17 [--reps 3] [--top 30]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--query", action="append", default=[])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--sort", default="tottime", help="pstats order: tottime | cumulative")
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch, tpch22
    from spark_druid_olap_amd.session import Session

    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(engine=Engine())
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    for name in a.query or ["Q17"]:
        df = s.sql(dict(tpch22.QUERIES)[name])
        df.run()
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        for _ in range(a.reps):
            df.run()
        pr.disable()
        print(f"== {name}: {(time.perf_counter() - t0) / a.reps * 1e3:.2f} ms per run (profiled)", flush=True)
        pstats.Stats(pr).sort_stats(a.sort).print_stats(a.top)


if __name__ == "__main__":
    main()
