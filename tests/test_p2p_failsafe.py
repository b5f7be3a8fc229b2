"""Fail-safe plumbing of the peer-to-peer merge (parallel/p2p.py; verdict r4 "next" #1), on the CPU:
the status-word protocol's outcomes map to the right exceptions, an abandoned epoch re-runs the
statement with merges forced onto the collective path, P2P state that is compacted is checked
first (advisor r4: nested / grouping-sets consumers dropped it), and the exchange is never offered
to an SPMD execution slot's own process group."""
import pytest
import torch

from spark_druid_olap_amd.engine.partials import Partials
from spark_druid_olap_amd.parallel import fault, p2p
from spark_druid_olap_amd.parallel.fault import P2PRetry, RankFailure


def test_status_words_map_to_exceptions():
    fault.raise_if_failed([0, 0], 0, None)
    with pytest.raises(P2PRetry):
        fault.raise_if_failed([fault.STATUS_P2P_RETRY] * 3, 1, None)
    with pytest.raises(RankFailure) as e:
        fault.raise_if_failed([0, fault.STATUS_P2P_TIMEOUT], 0, None)
    assert not isinstance(e.value, P2PRetry) and "timed out" in str(e.value)
    with pytest.raises(RankFailure) as e:
        fault.raise_if_failed([0, fault.STATUS_FAILED], 0, None)
    assert not isinstance(e.value, P2PRetry) and "local scan" in str(e.value)


def test_compact_checks_p2p_status_first():
    acc = torch.tensor([[1, 5], [0, 0], [2, 7]], dtype=torch.int64)
    part = Partials("dense", acc, None, [])
    part.status_dev = torch.tensor([0, fault.STATUS_P2P_RETRY], dtype=torch.int64)
    part.status_rank = 0
    with pytest.raises(P2PRetry):
        part.compact()
    ok = Partials("dense", acc, None, [])
    ok.status_dev = torch.tensor([0, 0], dtype=torch.int64)
    sp = ok.compact()
    assert sp.keys.tolist() == [0, 2] and ok.status_dev is None


def _session():
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.session import Session

    ds = tpch.to_datasource(tpch.generate_flat(0.002, "cpu"), profile="bench")
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    return s


def test_abandoned_epoch_reruns_statement_on_collective_path(monkeypatch):
    """finalize raising P2PRetry (what every rank does when the kernel's verdicts say 'abandoned')
    makes PreparedQuery.run re-run the statement once with the exchange suppressed."""
    from spark_druid_olap_amd.engine import executor

    s = _session()
    q = "select l_returnflag, count(*) c, sum(l_quantity) q from orderLineItemPartSupplier group by l_returnflag"
    want = sorted(s.sql(q).to_pandas().itertuples(index=False, name=None))
    real = executor.finalize
    seen = []

    def flaky(prog, part, out_types=None):
        seen.append(bool(getattr(p2p._TLS, "off", False)))
        if len(seen) == 1:
            raise P2PRetry("test: abandoned epoch")
        return real(prog, part, out_types)

    monkeypatch.setattr(executor, "finalize", flaky)
    df = s.sql(q)
    got = sorted(df.to_pandas().itertuples(index=False, name=None))
    assert got == want
    assert seen == [False, True]  # the retry ran with P2P suppressed
    assert not getattr(p2p._TLS, "off", False)  # and only for the retry


def test_exchange_never_offered_to_slot_groups(monkeypatch):
    from spark_druid_olap_amd.parallel.world import World, slot_group

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    w = World(rank=0, size=2, backend="nccl")
    built = []
    monkeypatch.setattr(p2p, "PeerExchange", lambda world, dev: built.append(dev))
    monkeypatch.setattr(World, "device", lambda self: torch.device("cuda", 0))
    with slot_group(object()):
        assert p2p.exchange_for(w) is None
    with p2p.suppressed():
        assert p2p.exchange_for(w) is None
    assert not built


def test_retries_disable_exchange_after_limit(monkeypatch):
    from spark_druid_olap_amd.parallel.world import World

    w = World(rank=0, size=2, backend="nccl")
    monkeypatch.setattr(World, "device", lambda self: torch.device("cuda", 0))

    class Ex:
        retries = 0
        total_retries = 0
        disabled = False
        rank = 0

    ex = Ex()
    monkeypatch.setitem(p2p._EXCHANGES, p2p._key(w), ex)
    for i in range(p2p.MAX_RETRIES - 1):
        p2p.note_retry(w)
        assert not ex.disabled
    # a completed epoch in between resets the CONSECUTIVE count (every rank sees the same verdicts)
    p2p.raise_status([0, 0], 0)
    assert ex.retries == 0 and ex.total_retries == p2p.MAX_RETRIES - 1
    for i in range(p2p.MAX_RETRIES - 1):
        p2p.note_retry(w)
        assert not ex.disabled
    p2p.note_retry(w)
    assert ex.disabled and ex.total_retries == 2 * p2p.MAX_RETRIES - 1
