"""Druid-compatible HTTP API over the engine + the Druid clients (DruidClient,
broker/coordinator/overlord clients, retry utils)."""
import json
import os

import pytest

from spark_druid_olap_amd.client.druid_client import (DruidCoordinatorClient, DruidOverlordClient,
                                                      DruidQueryServerClient)
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
from spark_druid_olap_amd.server.druid_http import DruidHTTPServer
from spark_druid_olap_amd.session import Session
from spark_druid_olap_amd.utils.errors import DruidDataSourceException


@pytest.fixture(scope="module")
def srv(ds_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    h = DruidHTTPServer(s, port=0).start()
    yield h
    h.stop()


def test_native_queries_roundtrip(srv, ds_small):
    c = DruidQueryServerClient("127.0.0.1", srv.port)
    for name, q in DRUID_JSON.items():
        r = c.execute_query(q)
        assert isinstance(r, list) and r, name
        if q["queryType"] == "groupBy":
            assert {"version", "timestamp", "event"} <= set(r[0])
    q1 = c.execute_query(DRUID_JSON["TPCH Q1"])
    assert sum(e["event"]["alias-1"] for e in q1) == ds_small.num_rows
    ts = c.execute_query({"queryType": "timeseries", "dataSource": "tpch", "granularity": "all",
                          "intervals": ["1992-01-01/1999-01-01"],
                          "aggregations": [{"type": "count", "name": "c"}]})
    assert ts[0]["result"]["c"] == ds_small.num_rows
    tb = c.time_boundary("tpch")
    assert tb["minTime"].startswith("1992")
    md = c.metadata("tpch")
    assert md["columns"]["l_returnflag"]["cardinality"] == 3
    assert "tpch" in c.datasources()


def test_coordinator_and_errors(srv):
    co = DruidCoordinatorClient("127.0.0.1", srv.port)
    assert co.segments("tpch", full=False)
    assert co.servers_info()[0]["type"] == "historical"
    with pytest.raises(DruidDataSourceException):
        DruidQueryServerClient("127.0.0.1", srv.port).execute_query({"queryType": "groupBy", "dataSource": "nope",
                                                                     "dimensions": [], "intervals": []})


@pytest.mark.skipif(not os.path.exists("/root/reference/src/test/resources/zip_code.json.template"),
                    reason="reference checkout not mounted")
def test_overlord_index_task(srv):
    ref = "/root/reference/src/test/resources"
    text = open(f"{ref}/zip_code.json.template").read().replace(":DATA_DIR:", f"{ref}/zipCodes/sample")
    ov = DruidOverlordClient("127.0.0.1", srv.port)
    tid = ov.submit_task(json.loads(text))
    st = ov.wait_until_task_completes(tid, timeout_s=30, poll_s=0.05)
    assert st["status"] == "SUCCESS"
    r = DruidQueryServerClient("127.0.0.1", srv.port).execute_query(
        {"queryType": "timeseries", "dataSource": "zipCodes", "granularity": "all",
         "intervals": ["2015-01-01/2017-01-01"], "aggregations": [{"type": "count", "name": "c"}]})
    assert r[0]["result"]["c"] >= 1


def test_query_history_page(ds_small):
    import requests

    s = Session(engine=Engine(use_native=False), conf={"spark.sparklinedata.enable.druid.query.history": "true"})
    s.register_datasource(ds_small)
    h = DruidHTTPServer(s, port=0).start()
    try:
        DruidQueryServerClient("127.0.0.1", h.port).execute_query(DRUID_JSON["TPCH Q1"])
        r = requests.get(f"http://127.0.0.1:{h.port}/sparklinedata/druid/queries", timeout=10)
        assert r.status_code == 200 and r.headers["Content-Type"].startswith("text/html")
        assert "Druid Query Details" in r.text and "GroupByQuerySpec" in r.text or "groupBy" in r.text
        js = requests.get(f"http://127.0.0.1:{h.port}/sparklinedata/druid/queries.json", timeout=10).json()
        assert len(js) == 1 and js[0]["numRows"] == 4
    finally:
        h.stop()


def test_delete_cancels_a_running_query(srv, monkeypatch):
    """DELETE /druid/v2/{queryId} aborts a query that is already executing: the engine stops at
    its next stage boundary (here: between the segment batches of a historical-style query)."""
    import threading
    import time as _t
    import urllib.request

    from spark_druid_olap_amd.engine import executor as X

    started = threading.Event()
    real = X.PreparedQuery._scan

    def slow_scan(self, prog, prep):
        started.set()
        _t.sleep(0.3)
        return real(self, prog, prep)
    monkeypatch.setattr(X.PreparedQuery, "_scan", slow_scan)
    # many segment batches -> many scans with a checkpoint before each
    monkeypatch.setattr(srv.session.engine, "execute",
                        lambda spec, ds, nseg=None, _e=srv.session.engine: _e.prepare(spec, ds, 1).run())
    q = {"queryType": "timeseries", "dataSource": "tpch", "granularity": "all",
         "intervals": ["1992-01-01/1999-01-01"], "aggregations": [{"type": "count", "name": "c"}],
         "context": {"queryId": "cancel-me"}}
    out = {}

    def run():
        c = DruidQueryServerClient("127.0.0.1", srv.port)
        t0 = _t.time()
        try:
            out["r"] = c.execute_query(q)
        except DruidDataSourceException as e:
            out["err"] = str(e)
        out["s"] = _t.time() - t0
    th = threading.Thread(target=run)
    th.start()
    assert started.wait(30)
    req = urllib.request.Request(f"http://127.0.0.1:{srv.port}/druid/v2/cancel-me", method="DELETE")
    urllib.request.urlopen(req).read()
    th.join(60)
    assert "err" in out and "cancel" in out["err"].lower(), out
    assert out["s"] < 10  # far less than scanning every monthly segment batch at 0.3 s each


def test_streamed_results_iterator(srv, ds_small):
    """A large groupBy (every order) is sent chunked and parsed row by row by the client's
    ResultIterator -- the same rows as the buffered call; closing early drops the connection."""
    c = DruidQueryServerClient("127.0.0.1", srv.port)
    q = {"queryType": "groupBy", "dataSource": "tpch", "granularity": "all", "intervals": ["1992-01-01/1999-01-01"],
         "dimensions": ["o_orderkey"], "aggregations": [{"type": "longSum", "name": "q", "fieldName": "l_quantity"}]}
    full = c.execute_query(q)
    assert len(full) > 4096  # above the server's streaming threshold
    with c.execute_query_iter(q, chunk_bytes=4096) as it:
        rows = list(it)
    assert rows == full and it.rows == len(full)
    it2 = c.execute_query_iter(q, chunk_bytes=1024)
    first = [next(it2) for _ in range(10)]
    it2.close()
    assert first == full[:10]
    # the cancel hook reaches the server (DELETE /druid/v2/{queryId})
    it3 = c.execute_query_iter({**q, "context": {"queryId": "stream-cancel-1"}})
    next(it3)
    it3.cancel()
    assert it3.query_id == "stream-cancel-1"
