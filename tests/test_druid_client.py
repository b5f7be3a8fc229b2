"""The reference's DruidClientTest (``tc/DruidClientTest.scala:43-131``), case by case, against the
Druid-compatible HTTP API of this engine: broker / coordinator time boundary, segment metadata,
the TPC-H QuerySpecs (day and month grain), a streamed result, server and datasource inventory,
and the basicAgg / tpchQ3 SQL that the suite also runs through the planner."""
import pytest

from spark_druid_olap_amd.client.druid_client import DruidCoordinatorClient, DruidQueryServerClient
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
from spark_druid_olap_amd.server.druid_http import DruidHTTPServer
from spark_druid_olap_amd.session import Session


@pytest.fixture(scope="module")
def env(ds_small, df_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    h = DruidHTTPServer(s, port=0).start()
    yield s, DruidQueryServerClient("127.0.0.1", h.port), DruidCoordinatorClient("127.0.0.1", h.port)
    h.stop()


def test_time_boundary(env):
    _, broker, _ = env
    tb = broker.time_boundary("tpch")
    assert tb["minTime"] < tb["maxTime"] and tb["minTime"].startswith("1992")


def test_coord_time_boundary(env):
    _, _, coord = env
    info = coord.datasource_info("tpch")
    assert info  # the coordinator's datasource interval / segment summary


def test_metadata(env, ds_small):
    _, broker, _ = env
    md = broker.metadata("tpch")
    text = str(md)
    assert "l_returnflag" in text and "o_orderkey" in text


@pytest.mark.parametrize("name", ["TPCH Q1", "TPCH Q3"])
def test_tpch_queries(env, name):
    _, broker, _ = env
    r = broker.execute_query(DRUID_JSON[name])
    assert r and {"version", "timestamp", "event"} <= set(r[0])


def test_tpch_q1_month_grain(env):
    _, broker, _ = env
    q = dict(DRUID_JSON["TPCH Q1"], granularity="month")
    r = broker.execute_query(q)
    months = {e["timestamp"][:7] for e in r}
    assert len(months) > 12  # one row group per month bucket


def test_stream_query_result(env):
    _, broker, _ = env
    with broker.execute_query_iter(DRUID_JSON["TPCH Q1"], chunk_bytes=256) as it:
        rows = list(it)
    assert rows == broker.execute_query(DRUID_JSON["TPCH Q1"])


def test_servers_info(env):
    _, _, coord = env
    assert coord.servers_info()[0]["type"] == "historical"


def test_datasource_info(env):
    _, broker, coord = env
    assert "tpch" in broker.datasources()
    assert coord.datasource_info("tpch") and coord.segments("tpch", full=False)


@pytest.mark.parametrize("sql", [
    "select l_returnflag, l_linestatus, count(*), sum(l_extendedprice) as s from orderLineItemPartSupplier "
    "group by l_returnflag, l_linestatus",                                                           # basicAgg
    "select o_orderkey, sum(l_extendedprice) as price, o_orderdate, o_shippriority from orderLineItemPartSupplier "
    "where c_mktsegment = 'BUILDING' group by o_orderkey, o_orderdate, o_shippriority",             # tpchQ3
])
def test_sql_through_planner(env, sql):
    s, _, _ = env
    d = s.sql(sql)
    assert len(d.druid_queries()) == 1
    got = sorted(d.collect())
    exp = sorted(s.sql(sql.replace("orderLineItemPartSupplier", "orderLineItemPartSupplierBase")).collect())
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        assert all((abs(x - y) <= 1e-6 * max(1.0, abs(y))) if isinstance(x, float) else x == y for x, y in zip(a, b))
