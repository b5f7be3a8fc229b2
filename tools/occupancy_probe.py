#!/usr/bin/env python3
"""Grid / occupancy of every headline query's scan kernel on the GPU: kernel name, registers,
resident workgroups per CU (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor) and the grid the
engine launches.  python tools/occupancy_probe.py [--sf 1]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.ops import native
    from spark_druid_olap_amd.session import Session

    ds = tpch.to_datasource(tpch.generate_flat(a.sf, "cuda"), profile="bench")
    s = Session(engine=Engine(), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    nat = native.load()
    for name, q in tpch.BENCH_QUERIES:
        df = s.sql(q)
        df.run()
        df.run()
        for dq in df.druid_queries():
            pq = getattr(dq, "_prepared", None)
            for _, prog, prep in (pq.scans if pq is not None else []):
                js = getattr(prep, "jit", None)
                if js is None:
                    continue
                print(f"{name[:40]:40s} {js.name}{' lit' if js.literals else ''} U={js.U} lds={js.lay.total} "
                      f"attrs={nat.module_attrs(js.handle)} occ={js.occupancy()} grid={prep.grid}", flush=True)


if __name__ == "__main__":
    main()
