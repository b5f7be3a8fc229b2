#!/usr/bin/env python3
"""cProfile of the server-side work of one HiveServer2 statement (native gateway): planning-cache
lookup, execution, result conversion and column encoding, for the 8 benchmark texts issued by one
client against one executor thread -- the per-execution host cost that bounds concurrent
executions/s.

usage: python tools/server_profile.py --sf 10 --iters 50 [--top 50]"""
import argparse
import cProfile
import os
import pstats
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--top", type=int, default=50)
    a = ap.parse_args()
    os.environ["SDO_GATEWAY_EXECUTORS"] = "1"
    os.environ["SDO_COALESCE"] = "0"
    import torch

    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.server import gateway as GW
    from spark_druid_olap_amd.server.hive_client import connect
    from spark_druid_olap_amd.session import Session

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    srv = GW.NativeHiveServer(s, port=0)
    prof = cProfile.Profile()
    on = threading.Event()
    cost = []
    real_exec = srv._execute
    real_enc = GW.encode_columns

    def exec_(bid, sid, stmt):
        if not on.is_set():
            return real_exec(bid, sid, stmt)
        c0, w0 = time.thread_time(), time.perf_counter()
        prof.enable()
        try:
            return real_exec(bid, sid, stmt)
        finally:
            prof.disable()
            cost.append((time.thread_time() - c0, time.perf_counter() - w0))

    def enc(types, pdf):
        if not on.is_set():
            return real_enc(types, pdf)
        prof.enable()
        try:
            return real_enc(types, pdf)
        finally:
            prof.disable()

    srv._execute = exec_
    GW.encode_columns = enc
    srv.start()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import concurrency_bench as CB

    qs = [q for _, q in CB.queries()]  # the concurrency benchmark's texts (TPC-H Q3 with its LIMIT 10)
    with connect(port=srv.port) as c:
        for q in qs * 3:
            c.cursor().execute(q).fetchall()
        on.set()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            for q in qs:
                c.cursor().execute(q).fetchall()
        dt = time.perf_counter() - t0
        on.clear()
    srv.stop()
    n = len(cost)
    print(f"statements {n}: client-observed {dt / n * 1e3:.3f} ms each; server _execute thread CPU "
          f"{sum(x for x, _ in cost) / n * 1e3:.3f} ms, wall {sum(y for _, y in cost) / n * 1e3:.3f} ms")
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumulative").print_stats(a.top)


if __name__ == "__main__":
    main()
