"""roctx tracing + host timeline."""
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.session import Session
from spark_druid_olap_amd.utils import trace as T


def test_stage_timeline(ds_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    T.enable(True)
    try:
        T.reset()
        s.sql(tpch.BENCH_QUERIES[0][1]).collect()
        names = [n.strip() for n, _ in T.timeline().summary()]
        for st in ("sdo.parse", "sdo.plan", "sdo.lower", "sdo.scan", "sdo.merge", "sdo.finalize", "sdo.post",
                   "sdo.druid.groupBy"):
            assert st in names, names
        assert all(ms >= 0 for _, ms in T.timeline().summary())
    finally:
        T.enable(False)
    T.reset()
    s.sql(tpch.BENCH_QUERIES[1][1]).collect()
    assert T.timeline().events == []


def test_roctx_library_loads():
    # the ROCm image ships the roctx library; ranges must be callable without a profiler attached
    assert T.available()
    T.enable(True)
    try:
        with T.span("sdo.test"):
            T.mark("inside")
    finally:
        T.enable(False)
