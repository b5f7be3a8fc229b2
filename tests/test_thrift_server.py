"""HiveServer2 Thrift endpoint: SASL-PLAIN and noSasl clients, metadata calls, errors, concurrency
(the reference's HiveThriftServer2 entry point + JDBC clients)."""
import threading

import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.server.hive_client import HiveError, connect
from spark_druid_olap_amd.server.hive_server import HiveThriftServer
from spark_druid_olap_amd.session import Session


@pytest.fixture(scope="module")
def server(ds_small, df_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    srv = HiveThriftServer(s, port=0).start()
    yield srv
    srv.stop()


@pytest.mark.parametrize("sasl", [True, False])
def test_query_roundtrip(server, sasl, df_small):
    with connect(port=server.port, sasl=sasl) as c:
        cur = c.cursor().execute("select l_returnflag, count(*) c, sum(l_extendedprice) s "
                                 "from orderLineItemPartSupplier group by l_returnflag order by l_returnflag")
        assert cur.description == [("l_returnflag", "string"), ("c", "bigint"), ("s", "double")]
        rows = cur.fetchall()
        exp = df_small.groupby("l_returnflag").agg(c=("l_extendedprice", "size"), s=("l_extendedprice", "sum"))
        assert [r[0] for r in rows] == list(exp.index)
        assert [r[1] for r in rows] == list(exp.c)
        for r, s in zip(rows, exp.s):
            assert r[2] == pytest.approx(s)
        cur.close()


def test_paging_nulls_and_errors(server):
    with connect(port=server.port) as c:
        cur = c.cursor()
        cur.arraysize = 7
        cur.execute("select o_orderkey, cast(null as string) n from orderLineItemPartSupplierBase limit 20")
        rows = cur.fetchall()
        assert len(rows) == 20 and all(r[1] is None for r in rows)
        with pytest.raises(HiveError):
            c.cursor().execute("select nosuchcol from orderLineItemPartSupplier")
        rows = c.cursor().execute("explain druid rewrite select count(*) from orderLineItemPartSupplier").fetchall()
        assert any("TimeSeriesQuerySpec" in r[0] for r in rows)


def test_metadata_calls(server):
    with connect(port=server.port) as c:
        r = c.call("GetTables", {"sessionHandle": c.session, "schemaName": "default", "tableName": "%"})
        cur = c.cursor()
        cur.op = r["operationHandle"]
        tabs = {row[2].lower() for row in cur.fetchall()}
        assert "orderlineitempartsupplier" in tabs
        r = c.call("GetColumns", {"sessionHandle": c.session, "tableName": "orderLineItemPartSupplier"})
        cur.op = r["operationHandle"]
        assert len(cur.fetchall()) == len(tpch.FLAT_SCHEMA)


def test_concurrent_clients(server):
    errs = []

    def client(i):
        try:
            with connect(port=server.port, sasl=bool(i % 2)) as c:
                for _ in range(3):
                    rows = c.cursor().execute("select s_region, count(*) from orderLineItemPartSupplier "
                                              "group by s_region").fetchall()
                    assert len(rows) == 5
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=client, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
