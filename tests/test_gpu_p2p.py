"""Peer-to-peer one-shot merge (parallel/p2p.py, ops/csrc/p2p.hip; verdict r3 #3) on the leased GPU:
two rank processes share the card (gloo for the handle exchange and the reference merge, IPC
mappings of each other's mailbox), and the P2P kernel's merge must equal the all-gather merge --
synthetic states over several epochs, a failed rank's status word, and the headline SQL queries."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_p2p_merge_two_ranks_on_one_gpu(tmp_path):
    from spark_druid_olap_amd.utils.launch import spawn_ranks

    out = tmp_path / "p2p.json"
    env = dict(os.environ, SDO_GLOO_GPU="1", MASTER_ADDR="127.0.0.1", SDO_P2P_TIMEOUT_S="20")
    rc = spawn_ranks(2, [sys.executable, os.path.join(ROOT, "tools", "p2p_check.py"), "--out", str(out),
                         "--sf", "0.2"], env=env)
    assert rc == 0
    r = json.loads(out.read_text())
    print(json.dumps(r)[:3000])
    assert r["exchange"], "IPC mailboxes could not be mapped"
    assert r["synthetic_equal"] and r["failed_status_seen"]
    assert all(r["engine_equal"].values()), r["engine_equal"]
    assert r["engine_rows"]["TPCH Q1"] > 0 and r["engine_rows"]["TPCH Q5"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_p2p_selftest_failure_falls_back(tmp_path):
    """One rank's known-value self-test fails (test hook): no rank uses the exchange, and every
    headline statement completes over the collective path with the same answers."""
    from spark_druid_olap_amd.utils.launch import spawn_ranks

    out = tmp_path / "p2p_selftest.json"
    env = dict(os.environ, SDO_GLOO_GPU="1", MASTER_ADDR="127.0.0.1", SDO_P2P_SELFTEST_FAIL="1")
    rc = spawn_ranks(2, [sys.executable, os.path.join(ROOT, "tools", "p2p_check.py"), "--out", str(out),
                         "--sf", "0.05", "--scenario", "selftest_fail"], env=env)
    assert rc == 0
    r = json.loads(out.read_text())
    print(json.dumps(r)[:3000])
    assert r["p2p_stats"] == {"built": True, "enabled": False}, r["p2p_stats"]
    assert all(r["engine_equal"].values()), r["engine_equal"]
    assert r["engine_rows"]["TPCH Q1"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_p2p_soft_timeout_retries_over_collectives(tmp_path):
    """Rank 1 launches one merge 1.5 s late: rank 0's soft wait (0.5 s) expires, both ranks read
    the abandoned verdict, and the statement re-runs over the collective path -- one retry, the
    same answers, the exchange still enabled afterwards."""
    from spark_druid_olap_amd.utils.launch import spawn_ranks

    out = tmp_path / "p2p_delay.json"
    env = dict(os.environ, SDO_GLOO_GPU="1", MASTER_ADDR="127.0.0.1", SDO_P2P_DELAY="rank=1,s=1.5,times=1",
               SDO_P2P_TIMEOUT_S="0.5")
    rc = spawn_ranks(2, [sys.executable, os.path.join(ROOT, "tools", "p2p_check.py"), "--out", str(out),
                         "--sf", "0.05", "--scenario", "delay"], env=env)
    assert rc == 0
    r = json.loads(out.read_text())
    print(json.dumps(r)[:3000])
    st = r["p2p_stats"]
    assert st["enabled"] and st["total_retries"] == 1 and st["selftest"] is True, st
    assert st["retries"] == 0, st  # (consecutive count: reset by the completed epochs after it)
    assert sum(r["retried_statements"].values()) == 1, r["retried_statements"]
    assert all(r["engine_equal"].values()), r["engine_equal"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_p2p_late_peer_past_hard_deadline_times_out_everywhere(tmp_path):
    """Rank 1 (alive) launches its merge 3 s late with a 1 s hard deadline: rank 0 aborts the
    epoch; rank 1 must read that abort and ALSO report the timeout (not RETRY -- its re-run over
    collectives would pair with rank 0's next statement).  Both disable the exchange and the next
    run answers correctly over the collective path."""
    from spark_druid_olap_amd.utils.launch import spawn_ranks

    out = tmp_path / "p2p_late.json"
    env = dict(os.environ, SDO_GLOO_GPU="1", MASTER_ADDR="127.0.0.1", SDO_P2P_DELAY="rank=1,s=3,times=1",
               SDO_P2P_TIMEOUT_S="0.5", SDO_P2P_HARD_TIMEOUT_S="1")
    rc = spawn_ranks(2, [sys.executable, os.path.join(ROOT, "tools", "p2p_check.py"), "--out", str(out),
                         "--sf", "0.05", "--scenario", "late"], env=env)
    assert rc == 0
    r = json.loads(out.read_text())
    print(json.dumps(r)[:3000])
    assert r["late_outcomes"] == ["RankFailure", "RankFailure"], r["late_outcomes"]
    assert r["late_enabled_after"] == [False, False], r
    assert r["late_answer_equal"], r
