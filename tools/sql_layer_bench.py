import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, statistics
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.session import Session
from spark_druid_olap_amd.engine.executor import Engine
ds = tpch.to_datasource(tpch.generate_flat(0.05, "cpu"), profile="bench")
s = Session(engine=Engine(use_native=False), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
s.register_datasource(ds)
s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
s.sql(tpch.druid_ddl(with_column_mapping=False))
for name in ["Basic Aggregation", "SubQuery + nation,Type predicates + ShipDate Range", "TPCH Q8", "TPCH Q7"]:
    df = s.sql(dict(tpch.BENCH_QUERIES)[name])
    real = s.run_druid; cache = {}
    def fake(dq, real=real):
        k = id(dq)
        if k not in cache: cache[k] = real(dq)
        return cache[k]
    s.run_druid = fake
    df.run()
    ts=[]
    for _ in range(500):
        t=time.perf_counter(); df.run(); ts.append((time.perf_counter()-t)*1e3)
    print(name[:30], "sql layer median ms", round(statistics.median(ts), 3))
    s.run_druid = real
