"""CUBE / ROLLUP / GROUPING SETS from one scan (SURVEY C5, 2.5 query-level fan-out).

The planner keeps the reference's plan shape -- one Druid groupBy per grouping set under a UNION
(``asd/DruidStrategy.scala:74-75``, 2-dim cube = 4 queries, ``tc/DruidRewriteCubeTest.scala:28-36``)
-- and the executor answers all of them from ONE scan of the widest set, re-aggregating the merged
partials per set on the device.  Results must equal per-set execution exactly."""
import pytest

from spark_druid_olap_amd.engine.executor import Engine, execute_grouping_sets, fusable_sets
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.session import Session

QUERIES = [
    "select l_returnflag, l_linestatus, count(*), sum(l_extendedprice), max(l_quantity), min(l_discount) "
    "from orderLineItemPartSupplier group by l_returnflag, l_linestatus with cube",
    "select s_region, s_nation, count(*), approx_count_distinct(o_orderkey) from orderLineItemPartSupplier "
    "where l_shipdate >= '1995-01-01' group by s_region, s_nation with rollup",
    "select l_shipmode, p_brand, sum(l_quantity) from orderLineItemPartSupplier where c_region = 'ASIA' "
    "group by grouping sets ((l_shipmode), (p_brand), ())",
]


def _session(ds, df, fuse):
    s = Session(engine=Engine(use_native=False),
                conf={"spark.sparklinedata.druid.fuse.groupingsets": str(fuse).lower(),
                      "spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", df, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    return s


def _norm(rows):
    return sorted((tuple("<null>" if x is None else (round(x, 6) if isinstance(x, float) else x) for x in r)
                   for r in rows), key=repr)


@pytest.mark.parametrize("q", QUERIES)
def test_fused_sets_equal_per_set_queries(ds_small, df_small, q):
    fused, single = _session(ds_small, df_small, True), _session(ds_small, df_small, False)
    d = fused.sql(q)
    specs = d.druid_query_specs()
    assert len(specs) >= 3 and fusable_sets(specs)  # plan shape unchanged: one Druid query per set
    assert _norm(d.collect()) == _norm(single.sql(q).collect())
    # the engine answered every set from one fine scan
    res = execute_grouping_sets(fused.engine, specs, ds_small)
    assert res is not None and all(r.stats["fused_sets"] == len(specs) for r in res)


def test_not_fusable_falls_back(ds_small, df_small):
    from spark_druid_olap_amd.query import spec as S

    a = S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("l_returnflag")],
                           aggregations=[S.FunctionAggregationSpec("count", "n")], intervals=["1992-01-01/1999-01-01"])
    b = a.copy(filter=S.SelectorFilterSpec("l_linestatus", "F"))
    assert not fusable_sets([a, b])
    assert Engine(use_native=False).execute_sets([a, b], ds_small) is None


@pytest.mark.gpu
def test_gpu_fused_sets_equal_per_set_queries():
    """Fine scan + device re-aggregation on the HIP path (dense LDS table -> compacted partials)."""
    from spark_druid_olap_amd.engine.columns import materialize

    flat = tpch.generate_flat(0.05, "cuda")
    ds = tpch.to_datasource(flat, profile="bench")
    df = tpch.to_pandas(flat)
    for q in QUERIES:
        a = _session_native(ds, df, True).sql(q).collect()
        b = _session_native(ds, df, False).sql(q).collect()
        assert _norm(a) == _norm(b), q
    del materialize


def _session_native(ds, df, fuse):
    s = Session(engine=Engine(use_native=True),
                conf={"spark.sparklinedata.druid.fuse.groupingsets": str(fuse).lower(),
                      "spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", df, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    return s
