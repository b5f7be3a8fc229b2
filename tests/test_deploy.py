"""Deployment path (the reference's spin-up tool + start script, ``tools/spinup-tool/spinup.sh``,
``scripts/start-sparklinedatathriftserver.sh``): the server process ingests a Druid index task at
startup, persists its shard to the segment store, and a restarted server resumes from the store
with the same answers -- driven over the HiveServer2 wire protocol."""
import os
import subprocess
import sys
import time

import pytest

from spark_druid_olap_amd.server.hive_client import connect

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _start(args, tmp_path, tag):
    pf = tmp_path / f"port.{tag}"
    env = dict(os.environ, PYTHONPATH=ROOT, SDO_NATIVE_GATEWAY="0", CUDA_VISIBLE_DEVICES="")
    p = subprocess.Popen([sys.executable, "-m", "spark_druid_olap_amd.server.hive_server", "--port", "0",
                          "--ui-port", "-1", "--port-file", str(pf)] + args, cwd=ROOT, env=env,
                         stdout=subprocess.DEVNULL, stderr=open(tmp_path / f"log.{tag}", "w"))
    t0 = time.time()
    while not pf.exists():
        if p.poll() is not None or time.time() - t0 > 180:
            p.kill()
            raise AssertionError(open(tmp_path / f"log.{tag}").read()[-3000:])
        time.sleep(0.2)
    return p, int(pf.read_text())


def _ask(port):
    with connect(port=port) as c:
        return sorted(c.cursor().execute(
            "select platform, count(*), approx_count_distinct(user) from events group by platform").fetchall())


def test_server_ingests_persists_and_resumes(tmp_path):
    from tests.test_sketch_rollup import _spec, _write

    import json

    data = tmp_path / "data"
    data.mkdir()
    _write(str(data / "events.tsv"), n=3000)
    spec = tmp_path / "events.json"
    spec.write_text(json.dumps(_spec(str(data))))
    ddl = tmp_path / "ddl.sql"
    ddl.write_text("CREATE TABLE eventsBase(ts string, platform string, country string, user string, amount double) "
                   "USING csv OPTIONS (path 'x');"
                   "CREATE TABLE events USING org.sparklinedata.druid OPTIONS (sourceDataframe 'eventsBase', "
                   "timeDimensionColumn 'ts', druidDatasource 'events', "
                   "columnInfos '[{\"column\": \"user\", \"hllMetric\": \"uniq_users\"}]')")
    store = tmp_path / "store"
    p, port = _start(["--ingest", str(spec), "--segments", str(store), "--init-sql", str(ddl)], tmp_path, "a")
    try:
        first = _ask(port)
    finally:
        p.terminate()
        p.wait(30)
    assert (store / "events" / "rank0" / "manifest.json").exists()
    assert len(first) == 3 and sum(r[1] for r in first) == 3000
    p, port = _start(["--segments", str(store), "--init-sql", str(ddl)], tmp_path, "b")
    try:
        assert _ask(port) == first
    finally:
        p.terminate()
        p.wait(30)
