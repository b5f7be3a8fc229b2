#!/usr/bin/env python3
"""In-process A/B of partitioned group-by layout choices: record packing (engine/device_exec.py
PACK_RECORDS, default) or the sub-bucket LDS table size (``--table 32768,65536``: PART_TABLE_BYTES)
-- the same statements re-prepared under each variant, best-of-two median wall times.

  python tools/pack_ab.py [--sf 100] [--queries Q18,Q13] [--iters 15] [--table 32768,65536]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--queries", default="Q18")
    ap.add_argument("--bi", default="TopVolumeCustomers")
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--only", type=int, default=None, help="1 / 0: run one variant only (profiling)")
    ap.add_argument("--table", default=None, help="PART_TABLE_BYTES variants instead of packing on / off")
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.models import bi, tpch, tpch22
    from spark_druid_olap_amd.session import Session

    dev = torch.device("cuda", 0)
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session()
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    bi.register(s)
    stmts = [(q, dict(tpch22.QUERIES)[q]) for q in a.queries.split(",") if q]
    if a.bi:
        stmts += [(n, q) for n, _, q in bi.statements(1, "years") if n == a.bi][:1]
    for name, sql in stmts:
        res = {}
        if a.table:
            variants = [("table", int(x)) for x in a.table.split(",")]
        else:
            variants = [("pack", p) for p in ((True, False) if a.only is None else (bool(a.only),))]
        for rnd in range(2):
            for kind, val in variants:
                if kind == "table":
                    DE.PART_TABLE_BYTES = val
                else:
                    DE.PACK_RECORDS = val
                s._plan_cache.clear()
                d = s.sql(sql).prepared()
                for _ in range(3):
                    d.run()
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.iters):
                    t0 = time.perf_counter()
                    d.run()
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) * 1e3)
                res.setdefault((kind, val), []).append(statistics.median(ts))
        print(f"{name:24s} " + "  ".join(f"{k}={v} {min(t):7.3f} ms" for (k, v), t in res.items()), flush=True)
    DE.PACK_RECORDS = True


if __name__ == "__main__":
    main()
