"""Per-Druid-query breakdown of SQL benchmark queries on the GPU.

  python tools/sql_probe.py SF Q17 Q2 ...     (TPC-H 22 query names)

For every DruidQuery leaf of each statement: accumulator mode (0 LDS, 1 HBM dense, 2 hash),
key space G, slots, hash capacity, and the median scan / merge / finalize / post times, plus the
whole statement's median wall time."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch, tpch22
    from spark_druid_olap_amd.session import Session

    sf = float(sys.argv[1])
    names = sys.argv[2:]
    dev = torch.device("cuda", 0)
    ds = tpch.to_datasource(tpch.generate_flat(sf, dev), profile="bench")
    torch.cuda.synchronize()
    s = Session(engine=Engine())
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    print(f"data ready sf={sf} rows={ds.num_rows}", flush=True)
    for name in names:
        print(f"{name}: planning", flush=True)
        d = s.sql(dict(tpch22.QUERIES)[name])
        print(f"{name}: running", flush=True)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            d.run()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        print(f"{name}: median {statistics.median(ts[1:]):.2f} ms (first {ts[0]:.1f})", flush=True)
        for st in d.last_stats.get("druid", []):
            print(f"   druid {st['ms']:8.2f} ms rows={st['rows']} {type(st['spec']).__name__}", flush=True)
        for dq in d.druid_queries():
            pq = getattr(dq, "_prepared", None)
            for q in (getattr(dq, "_resolved", {}) or {}).values():
                pq = getattr(q, "_prepared", pq)
            inner = getattr(pq, "inner", None)
            for p in (pq, inner):
                if p is None or not getattr(p, "scans", None):
                    continue
                prog, prep = p.scans[0][1], p.scans[0][2]
                print(f"   scan mode={getattr(prep, 'mode', None)} G={prog.G} slots={prog.nslots} "
                      f"cap={getattr(prep, 'cap', None)} keys={[k.name for k in prog.keys]} "
                      f"derived={[k.name for k, _, _ in prog.derived]} est_rows={prog.est_rows:.0f}", flush=True)
                torch.cuda.synchronize()
                t = time.perf_counter()
                part = prep.run() if prep is not None else None
                torch.cuda.synchronize()
                print(f"   raw scan {(time.perf_counter() - t) * 1e3:.2f} ms groups={getattr(part, 'rows', '?')}",
                      flush=True)


if __name__ == "__main__":
    main()
