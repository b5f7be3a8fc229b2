"""Serving metrics: latency percentiles, QPS and errors per endpoint, recorded by the
HiveServer2 servers and the Druid HTTP API, served as JSON and Prometheus text."""
import json
import urllib.request

import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.server.hive_client import HiveError, connect
from spark_druid_olap_amd.session import Session
from spark_druid_olap_amd.utils.metrics import ServerMetrics


def test_percentiles_and_window():
    m = ServerMetrics(window=100)
    for i in range(1, 201):
        m.record("x", float(i), ok=i % 50 != 0)
    s = m.snapshot()["x"]
    assert s["count"] == 200 and s["errors"] == 4
    # the window holds the last 100 latencies: 101..200
    assert s["p50_ms"] == pytest.approx(150.5) and s["max_ms"] == 200.0
    assert s["qps_1m"] > 0
    txt = m.prometheus()
    assert 'sdo_latency_ms{endpoint="x",quantile="0.99"}' in txt and 'sdo_requests_total{endpoint="x"} 200' in txt


@pytest.mark.parametrize("native", [False, True])
def test_servers_record_and_expose(ds_small, df_small, native):
    from spark_druid_olap_amd.server.druid_http import DruidHTTPServer
    from spark_druid_olap_amd.server.gateway import make_server

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    srv = make_server(s, port=0, native=native).start()
    http = DruidHTTPServer(s, "127.0.0.1", 0).start()
    try:
        with connect(port=srv.port) as c:
            for _ in range(5):
                c.cursor().execute("select l_returnflag, count(*) from orderLineItemPartSupplier group by l_returnflag")
            with pytest.raises(HiveError):
                c.cursor().execute("select nosuch from orderLineItemPartSupplier")
        body = json.dumps({"queryType": "timeseries", "dataSource": "tpch", "granularity": "all",
                           "intervals": ["1992-01-01/1999-01-01"],
                           "aggregations": [{"type": "count", "name": "n"}]}).encode()
        req = urllib.request.Request(f"http://127.0.0.1:{http.port}/druid/v2/", data=body,
                                     headers={"Content-Type": "application/json"})
        urllib.request.urlopen(req).read()
        snap = json.loads(urllib.request.urlopen(f"http://127.0.0.1:{http.port}/sparklinedata/metrics").read())
        ep = "gateway" if native else "thrift"
        assert snap[ep]["count"] >= 6 and snap[ep]["errors"] >= 1 and snap[ep]["p99_ms"] >= snap[ep]["p50_ms"] > 0
        assert snap["druid_http"]["count"] == 1
        prom = urllib.request.urlopen(f"http://127.0.0.1:{http.port}/metrics").read().decode()
        assert f'sdo_requests_total{{endpoint="{ep}"}}' in prom
    finally:
        http.stop()
        srv.stop()
