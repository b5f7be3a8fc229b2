"""RCCL actually executes the engine's collectives (verdict r5 #3a): a one-rank ``nccl`` process group
with the collectives forced on (tools/rccl_smoke.py) runs every primitive the multi-GPU path uses
and the headline + TPC-H queries through it, against the same queries without a process group."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_rccl_one_rank_smoke(tmp_path):
    from spark_druid_olap_amd.utils.launch import spawn_ranks

    out = tmp_path / "rccl.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("SDO_GLOO_GPU", None)
    rc = spawn_ranks(1, [sys.executable, os.path.join(ROOT, "tools", "rccl_smoke.py"), "--out", str(out),
                         "--sf", "1"], env=env)
    assert rc == 0
    r = json.loads(out.read_text())
    print(json.dumps(r)[:3000])
    assert r["backend"] == "nccl" and r["forced"], r
    assert all(r["primitives"].values()), r["primitives"]
    assert all(r["engine_equal"].values()), r["engine_equal"]
    assert r["engine_rows"]["TPCH Q3"] > 0 and r["engine_rows"]["TPCH Q1"] > 0
