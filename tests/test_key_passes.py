"""Key-range passes (planner/cost.py plan_key_passes, engine/executor.py KeyRangePasses): a huge
dense group table is computed as P cache-sized passes over disjoint key ranges; answers must equal
the single-pass plan, including HAVING and ORDER BY ... LIMIT over the union."""
import pytest

from spark_druid_olap_amd.engine.columns import materialize
from spark_druid_olap_amd.engine.executor import Engine, KeyRangePasses
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.planner import cost
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.session import Session

Q18 = ("select c_name, o_custkey, o_orderkey, o_orderdate, max(o_totalprice) as o_totalprice, "
       "sum(l_quantity) as total_qty from orderLineItemPartSupplier group by c_name, o_custkey, o_orderkey, "
       "o_orderdate having sum(l_quantity) > 180 order by o_totalprice desc, o_orderdate limit 25")
OTHERS = [
    "select o_orderkey, count(*), sum(l_extendedprice), min(l_discount) from orderLineItemPartSupplier "
    "where l_shipmode = 'AIR' group by o_orderkey",
    "select o_orderkey, l_returnflag, sum(l_quantity) q from orderLineItemPartSupplier group by o_orderkey, "
    "l_returnflag order by q desc, o_orderkey limit 17",
]


def _sess(ds, df):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", df, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    return s


def _norm(rows):
    return [tuple(round(x, 6) if isinstance(x, float) else x for x in r) for r in rows]


@pytest.mark.parametrize("q", [Q18] + OTHERS)
def test_passes_equal_single_scan(ds_small, df_small, q, monkeypatch):
    want = _sess(ds_small, df_small).sql(q).collect()
    monkeypatch.setattr(cost, "FORCE_KEY_PASSES", 5)
    s = _sess(ds_small, df_small)
    d = s.sql(q)
    got = d.collect()
    preps = [getattr(x, "_prepared", None) for x in d.druid_queries()]
    assert any(isinstance(p, KeyRangePasses) and len(p.subs) == 5 for p in preps)
    if "limit" in q:
        assert _norm(got) == _norm(want)
    else:
        assert sorted(_norm(got)) == sorted(_norm(want))


def test_pass_keys_use_a_base_not_a_remap(ds_small, monkeypatch):
    from spark_druid_olap_amd.ops import desc as D

    monkeypatch.setattr(cost, "FORCE_KEY_PASSES", 3)
    q = S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("o_orderkey")],
                           aggregations=[S.FunctionAggregationSpec("longSum", "q", "l_quantity")],
                           intervals=["1992-01-01/1999-01-01"])
    kp = Engine(use_native=False).prepare(q, ds_small)
    assert isinstance(kp, KeyRangePasses)
    for sub, (lo, hi) in zip(kp.subs, kp.ranges):
        kc = sub.scans[0][1].keys[0]
        assert kc.kind == D.K_ID and kc.base == lo and kc.card <= hi - lo and kc.remap is None
    r = kp.run()
    single = Engine(use_native=False).prepare(q, ds_small, key_passes=False).run()
    assert r.num_rows == single.num_rows and sorted(r.data["q"].tolist()) == sorted(single.data["q"].tolist())
    assert len(set(materialize(r.data["o_orderkey"]).tolist())) == r.num_rows


@pytest.mark.gpu
def test_gpu_passes_equal_single_scan(monkeypatch):
    flat = tpch.generate_flat(0.05, "cuda")
    ds = tpch.to_datasource(flat, profile="bench")
    df = tpch.to_pandas(flat)

    def sess():
        s = Session(engine=Engine(use_native=True))
        s.register_datasource(ds)
        s.register_table("orderLineItemPartSupplierBase", df, schema=tpch.FLAT_SCHEMA)
        s.sql(tpch.druid_ddl(with_column_mapping=False))
        return s

    want = {q: sess().sql(q).collect() for q in [Q18] + OTHERS}
    monkeypatch.setattr(cost, "FORCE_KEY_PASSES", 4)
    s = sess()
    for q in [Q18] + OTHERS:
        got = s.sql(q).collect()
        if "limit" in q:
            assert _norm(got) == _norm(want[q]), q
        else:
            assert sorted(_norm(got)) == sorted(_norm(want[q])), q
