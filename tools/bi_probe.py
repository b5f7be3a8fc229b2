#!/usr/bin/env python3
"""Per-template cost of the reference's BI workload (models/bi) on one GPU: for each template and
a few CSV bindings, the plan / prepare (lowering + kernel) / first-run / repeat-run wall times and
the result size -- first-seen statements are what a BI dashboard sends.

  python tools/bi_probe.py --sf 100 [--iters 2] [--bind years] [--profile TEMPLATE]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--iters", type=int, default=2, help="bindings per template")
    ap.add_argument("--bind", default="years")
    ap.add_argument("--profile", default=None, help="cProfile this template's first binding (plan + run)")
    ap.add_argument("--only", default=None)
    ap.add_argument("--profile-repeat", default=None, help="cProfile the repeat runs of this template's last binding")
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import bi, tpch
    from spark_druid_olap_amd.session import Session

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    t0 = time.time()
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(engine=Engine(use_native=dev.type == "cuda"))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    bi.register(s)
    print(f"data ready sf={a.sf} rows={ds.num_rows} in {time.time() - t0:.1f}s", flush=True)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    rows = []
    for t in bi.templates():
        if a.only and a.only.lower() not in t["name"].lower():
            continue
        for k in range(a.iters):
            q = bi.render(t["sql"], bi.binding(k, a.bind))
            prof = None
            if a.profile and a.profile.lower() in t["name"].lower() and k == 0:
                import cProfile

                prof = cProfile.Profile()
                prof.enable()
            t1 = time.perf_counter()
            df = s.sql(q)
            t2 = time.perf_counter()
            df.prepare()
            sync()
            t3 = time.perf_counter()
            r = df.run()
            sync()
            t4 = time.perf_counter()
            if prof is not None:
                prof.disable()
                import pstats

                pstats.Stats(prof, stream=sys.stdout).sort_stats("cumulative").print_stats(45)
            reps = []
            rprof = None
            if a.profile_repeat and a.profile_repeat.lower() in t["name"].lower() and k == a.iters - 1:
                import cProfile

                rprof = cProfile.Profile()
                rprof.enable()
            for _ in range(3):
                t5 = time.perf_counter()
                df.run()
                sync()
                reps.append((time.perf_counter() - t5) * 1e3)
            if rprof is not None:
                rprof.disable()
                import pstats

                print(f"== repeat runs of {t['name']} (b{k}), cumulative", flush=True)
                pstats.Stats(rprof, stream=sys.stdout).sort_stats("cumulative").print_stats(40)
                pstats.Stats(rprof, stream=sys.stdout).sort_stats("tottime").print_stats(25)
            rows.append((t["name"], k, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, statistics.median(reps), r.n,
                         len(df.druid_queries())))
            print(f"{t['name'][:44]:44s} b{k} plan {rows[-1][2]:8.1f} prep {rows[-1][3]:8.1f} first {rows[-1][4]:8.1f} "
                  f"repeat {rows[-1][5]:8.2f} ms rows={r.n} druid={rows[-1][7]}", flush=True)
    tot = [sum(x[i] for x in rows) for i in (2, 3, 4, 5)]
    print(f"TOTAL plan {tot[0]:.0f} prep {tot[1]:.0f} first {tot[2]:.0f} repeat {tot[3]:.1f} ms over {len(rows)} statements")


if __name__ == "__main__":
    main()
