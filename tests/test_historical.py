"""Broker vs historical execution equivalence (tc/HistoricalServerTest.scala:177-350).

"Historical" here = the query runs as one partial scan per batch of ``numSegmentsPerHistoricalQuery``
segments and the engine merges the partials (the reference's historical partitions + Spark-side
PostAggregate); "broker" = one fused scan over all segments.  Each case runs the same SQL against
the broker-backed table and its ``_historical`` twin with the cost model off (as ``testCompare``
does), checks the physical plan runs in the requested mode, and compares the results."""
import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
from spark_druid_olap_amd.query.spec import query_from_json
from spark_druid_olap_amd.session import Session

T = "orderLineItemPartSupplier"

CASES = {
    "projFilterAgg": ("""select s_nation, round(count(*),2) as count_order, round(sum(l_extendedprice),2) as s,
        round(max(ps_supplycost),2) as m, round(avg(ps_availqty),2) as a, count(distinct o_orderkey)
        from (select l_returnflag as f, l_linestatus as s, l_shipdate, s_region, s_nation, c_nation, p_type,
                     l_extendedprice, ps_supplycost, ps_availqty, o_orderkey from %s
              where p_type = 'ECONOMY ANODIZED STEEL') t
        where dateIsBeforeOrEqual(dateTime(l_shipdate), dateMinus(dateTime('1997-12-01'), period('P90D')))
          and dateIsAfter(dateTime(l_shipdate), dateTime('1995-12-01'))
          and ((s_nation = 'FRANCE' and c_nation = 'GERMANY') or (c_nation = 'FRANCE' and s_nation = 'GERMANY'))
        group by s_nation order by s_nation""", 2),
    "basicCube": ("select l_returnflag, l_linestatus, count(*), round(sum(l_extendedprice),2) as s "
                  "from %s group by l_returnflag, l_linestatus with cube", 4),
    "gbexprtest1": ("select sum(c_acctbal) as bal from %s group by (substr(CAST(Date_Add(TO_DATE(CAST(CONCAT("
                    "TO_DATE(o_orderdate), 'T00:00:00.000') AS TIMESTAMP)), 5) AS TIMESTAMP), 0, 10)) order by bal", 1),
    "timeseries": ("""SELECT min(cast(cast(l_shipdate AS timestamp) AS timestamp)) AS x0,
        max(cast(cast(l_shipdate AS timestamp) AS timestamp)) AS x3, count(1) AS c
        FROM %s WHERE (NOT (cast(l_shipdate AS timestamp) IS NULL)) HAVING count(1) > 0""", 1),
    "noMetricsCName": ("select c_name from %s group by c_name", 1),
    "noMetricsCNameCountDistinct": ("select count(distinct c_name) from %s", 1),
    "avgHistorical": ("select avg((CASE WHEN 1000 = 0 THEN NULL ELSE CAST(l_suppkey AS DOUBLE) / 1000 END)) as x1 "
                      "from %s group by s_region order by x1", 1),
}


@pytest.fixture(scope="module")
def sess(ds_small, df_small):
    s = Session(engine=Engine(use_native=False),
                conf={"spark.sparklinedata.druid.querycostmodel.enabled": "false"})
    s.register_datasource(ds_small)
    s.register_table(T + "Base", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    s.sql(tpch.druid_ddl(table=T + "_historical", with_column_mapping=False,
                         star_schema=f'{{"factTable" : "{T}_historical", "relations" : []}}',
                         extra_options=', queryHistoricalServers "true", numSegmentsPerHistoricalQuery "7"'))
    return s


def _rows(df):
    out = []
    for r in df.collect():
        out.append(tuple(round(v, 4) if isinstance(v, float) else v for v in r))
    return sorted(out, key=lambda r: tuple((x is None, str(x)) for x in r))


@pytest.mark.parametrize("name", sorted(CASES))
def test_broker_vs_historical(sess, name):
    sql, nq = CASES[name]
    d1 = sess.sql(sql % T)
    d2 = sess.sql(sql % (T + "_historical"))
    q1, q2 = d1.druid_queries(), d2.druid_queries()
    assert len(q1) == len(q2) == nq
    assert all(not q.info.get("historical") for q in q1)
    assert all(q.info.get("historical") == 7 for q in q2 if q.info.get("groupby"))
    assert "queryHistorical=true" in d2.explain()
    r1, r2 = _rows(d1), _rows(d2)
    assert len(r1) == len(r2)
    for a, b in zip(r1, r2):
        for x, y in zip(a, b):
            if isinstance(x, float):
                assert x == pytest.approx(y, rel=1e-9, abs=1e-6)
            else:
                assert x == y


@pytest.mark.parametrize("nseg", [1, 3, 100])
def test_engine_segment_batches_match_broker(ds_small, nseg):
    eng = Engine(use_native=False)
    for name in ("TPCH Q1", "TPCH Q3", "TPCH Q7"):
        q = query_from_json(DRUID_JSON[name])
        a, b = eng.execute(q, ds_small), eng.execute(q, ds_small, segments_per_query=nseg)
        assert a.sorted_rows() == b.sorted_rows() or all(
            x == pytest.approx(y, rel=1e-6) for ra, rb in zip(a.sorted_rows(), b.sorted_rows()) for x, y in zip(ra, rb))
        p = eng.prepare(q, ds_small, segments_per_query=nseg)
        assert len(p.scans) >= (1 if nseg == 100 else 2)


def test_execute_query_using_historical(sess):
    import json

    j = json.dumps(DRUID_JSON["TPCH Q1"])
    a = sess.sql(f"ON DRUIDDATASOURCE {T} EXECUTE QUERY {j}").collect()
    b = sess.sql(f"ON DRUIDDATASOURCE {T}_historical USING HISTORICAL EXECUTE QUERY {j}").collect()
    assert sorted(map(str, a)) == sorted(map(str, b))


def test_cost_model_prefers_broker(ds_small):
    from spark_druid_olap_amd.planner.cost import choose_method

    for name in ("TPCH Q1", "TPCH Q3"):
        assert choose_method(ds_small, query_from_json(DRUID_JSON[name])) is None
