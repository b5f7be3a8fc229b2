"""Service discovery + membership watches (the reference's ZooKeeper/Curator layer,
sd/client/CuratorConnection.scala:41-235; tc/CuratorConnectionTest.scala:26-61)."""
import json
import subprocess
import sys
import time

from spark_druid_olap_amd.client.discovery import (CHILD_ADDED, CHILD_REMOVED, Discovery, FileRegistry,
                                                   MemoryRegistry)
from spark_druid_olap_amd.client.druid_client import discover_clients
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
from spark_druid_olap_amd.server.druid_http import DruidHTTPServer
from spark_druid_olap_amd.session import Session


def test_service_discovery_and_watches():
    d = Discovery(MemoryRegistry(), "/druid", qualify_names=True)
    seen = []
    d.watch_membership(lambda ev, p: seen.append((ev, p)))
    assert d.get_broker() is None
    d.announce_service("broker", "10.0.0.1", 8082)
    assert d.get_broker() == ("10.0.0.1", 8082)
    assert d.reg.children("/druid/discovery/druid:broker")  # zkQualifyDiscoveryNames
    d.announce_server("gpu:3", {"type": "historical"})
    d.reg.poll()
    d.announce_segment("gpu:3", "tpch_1993-01-01_1993-02-01_v1_0")
    d.reg.poll()
    assert d.segments("gpu:3") == ["tpch_1993-01-01_1993-02-01_v1_0"]
    d.unannounce("/druid/segments/gpu:3/tpch_1993-01-01_1993-02-01_v1_0")
    d.reg.poll()
    evs = [e for e, _ in seen]
    assert evs == [CHILD_ADDED, CHILD_ADDED, CHILD_REMOVED]


def test_session_clients_found_through_discovery(ds_small):
    s = Session(engine=Engine(use_native=False))
    s.attach_discovery("mem://test-discovery")
    s.register_datasource(ds_small)
    h = DruidHTTPServer(s, port=0).start()
    try:
        broker, coord, ov = discover_clients("mem://test-discovery")
        r = broker.execute_query(DRUID_JSON["TPCH Q1"])
        assert sum(e["event"]["alias-1"] for e in r) == ds_small.num_rows
        assert coord.servers_info()
        # the historical (this rank) announced every segment of the datasource
        assert len(s.discovery.segments("gpu:0")) == len(ds_small.segments)
    finally:
        h.stop()
    assert s.discovery.get_broker() is None


def test_membership_change_clears_metadata_cache(ds_small):
    s = Session(engine=Engine(use_native=False))
    s.attach_discovery("mem://test-cache-clear")
    s.register_datasource(ds_small)
    s.discovery.reg.poll()
    g0 = s.catalog.cluster.meta_generation
    p0 = s.catalog.cluster.generation
    s.discovery.announce_server("gpu:7", {"type": "historical"})
    s.discovery.reg.poll()
    assert s.catalog.cluster.meta_generation > g0
    # the plan-cache key (registry generation) does not move on an asynchronous discovery event:
    # ranks observe those at different moments, and their plans must stay in lock-step
    assert s.catalog.cluster.generation == p0


CHILD = """
import sys, time
sys.path.insert(0, {root!r})
from spark_druid_olap_amd.client.discovery import Discovery, FileRegistry
d = Discovery(FileRegistry({path!r}))
d.announce_service("broker", "127.0.0.1", 18082)
print("ready", flush=True)
time.sleep(60)
"""


def test_file_registry_across_processes(tmp_path):
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, "-c", CHILD.format(root=root, path=str(tmp_path))],
                         stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "ready"
        d = Discovery(FileRegistry(str(tmp_path)))
        seen = []
        d.reg.watch_children("/druid/discovery/broker", lambda ev, path: seen.append(ev))
        assert d.get_broker() == ("127.0.0.1", 18082)
    finally:
        p.kill()
        p.wait()
    # the owner is gone: its ephemeral node expires
    assert d.get_broker() is None
    d.reg.poll()
    assert seen == [CHILD_REMOVED]
