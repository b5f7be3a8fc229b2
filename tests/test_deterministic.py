"""Deterministic-reduction mode: floating-point sums accumulate in exact 64.32 fixed
point (two integer slots), so the result is bitwise identical under any accumulation order --
HIP atomics, per-wave LDS folds, segment batches ("historical" execution) and cross-rank merges.

CPU tests check the value against an fp64 oracle and bitwise equality across different segment
batchings (different partial-combine orders); the GPU test runs the HIP kernel repeatedly."""
import numpy as np
import pytest
import torch

from spark_druid_olap_amd.engine.columns import materialize
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.engine.lower import FIX_ONE, fixed_value
from spark_druid_olap_amd.query import spec as S

JS = S.JavascriptAggregationSpec("ratio", ["l_extendedprice", "l_discount", "l_tax"],
                                 "function(current, a, b, c) { return current + (a * (1 - b)) / (1 + c) / 3; }",
                                 "function(a,b){return a+b;}", "function(){return 0;}")
NEG = S.JavascriptAggregationSpec("neg", ["l_extendedprice", "l_discount"],
                                  "function(current, a, b) { return current + (b - 0.05) * a / 7; }",
                                  "function(a,b){return a+b;}", "function(){return 0;}")


def _query(det, dims=("l_returnflag", "l_linestatus")):
    ctx = S.QuerySpecContext(deterministic=True) if det else None
    return S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec(d) for d in dims],
                              aggregations=[S.FunctionAggregationSpec("count", "c"), JS, NEG],
                              intervals=["1992-01-01/1999-01-01"], context=ctx)


def _oracle(df, dims):
    v = (df.l_extendedprice * (1 - df.l_discount)) / (1 + df.l_tax) / 3
    w = (df.l_discount - 0.05) * df.l_extendedprice / 7
    g = df.assign(_v=v, _w=w).groupby(list(dims))
    return g._v.sum(), g._w.sum()


def _by_key(res, dims):
    keys = list(zip(*[materialize(res.data[d]).tolist() for d in dims]))
    return {k: (res.data["ratio"][i], res.data["neg"][i]) for i, k in enumerate(keys)}


def test_fixed_value_roundtrip():
    vals = np.array([0.0, 1.5, -1.5, -1e-20, 123456.789, -987654.321], dtype=np.float64)
    fl = np.floor(vals)
    hi, lo = fl.astype(np.int64), np.rint((vals - fl) * FIX_ONE).astype(np.int64)
    np.testing.assert_allclose(fixed_value(hi, lo), vals, atol=2.0 ** -32)
    t = fixed_value(torch.from_numpy(hi), torch.from_numpy(lo)).numpy()
    assert np.array_equal(t, fixed_value(hi, lo))


def test_deterministic_lowering_uses_integer_slots(ds_small):
    from spark_druid_olap_amd.ops import desc as D

    eng = Engine(use_native=False)
    pq = eng.prepare(_query(True), ds_small)
    prog = pq.scans[0][1]
    assert all(op != D.S_SUM_F for op, _ in prog.slots)
    kinds = {a.name: a.kind for a in prog.aggs}
    assert kinds["ratio"] == "sum_fx" and kinds["neg"] == "sum_fx"
    # the default mode keeps the single f64 slot
    prog2 = eng.prepare(_query(False), ds_small).scans[0][1]
    assert any(op == D.S_SUM_F for op, _ in prog2.slots)


def test_deterministic_sum_matches_fp64_oracle(ds_small, df_small):
    dims = ("l_returnflag", "l_linestatus")
    res = Engine(use_native=False).execute(_query(True, dims), ds_small)
    ov, ow = _oracle(df_small, dims)
    got = _by_key(res, dims)
    assert len(got) == len(ov)
    for k, (v, w) in got.items():
        assert v == pytest.approx(ov[k], rel=1e-12, abs=1e-6)
        assert w == pytest.approx(ow[k], rel=1e-12, abs=1e-6)


@pytest.mark.parametrize("dims", [("l_returnflag", "l_linestatus"), ("s_nation",), ()])
def test_bitwise_equal_across_segment_batchings(ds_small, dims):
    """Broker (one fused scan) vs historical execution with 1, 2 and 5 segments per partial: the
    partials are combined in different orders, the deterministic sums must not change a bit."""
    eng = Engine(use_native=False)
    q = _query(True, dims) if dims else S.TimeSeriesQuerySpec(
        "tpch", ["1992-01-01/1999-01-01"], aggregations=[JS, NEG], context=S.QuerySpecContext(deterministic=True))
    base = eng.execute(q, ds_small)
    for spq in (1, 2, 5):
        r = eng.execute(q, ds_small, segments_per_query=spq)
        for c in ("ratio", "neg"):
            a = np.asarray(base.data[c], dtype=np.float64)
            b = np.asarray(r.data[c], dtype=np.float64)
            if dims:
                ka = np.lexsort([materialize(base.data[d]).astype(str) for d in dims])
                kb = np.lexsort([materialize(r.data[d]).astype(str) for d in dims])
                a, b = a[ka], b[kb]
            assert a.tobytes() == b.tobytes(), (c, spq)


def test_engine_flag_and_env(monkeypatch, ds_small):
    monkeypatch.setenv("SDO_DETERMINISTIC", "1")
    eng = Engine(use_native=False)
    assert eng.deterministic
    prog = eng.prepare(_query(False), ds_small).scans[0][1]
    assert {a.kind for a in prog.aggs if a.name in ("ratio", "neg")} == {"sum_fx"}


def test_nested_outer_sum_deterministic(ds_small):
    """Nested groupBy: the outer float sum of inner float sums goes through the fixed point too."""
    inner = _query(True, ("l_returnflag", "l_linestatus"))
    outer = S.GroupByQuerySpec(S.QueryDataSourceSpec(inner), [S.DefaultDimensionSpec("l_returnflag")],
                               aggregations=[S.FunctionAggregationSpec("doubleSum", "tot", "ratio")],
                               intervals=["1992-01-01/1999-01-01"], context=S.QuerySpecContext(deterministic=True))
    eng = Engine(use_native=False)
    a = eng.execute(outer, ds_small)
    b = eng.execute(outer, ds_small, segments_per_query=3)
    ia, ib = np.argsort(materialize(a.data["l_returnflag"]).astype(str)), np.argsort(materialize(b.data["l_returnflag"]).astype(str))
    assert np.asarray(a.data["tot"])[ia].tobytes() == np.asarray(b.data["tot"])[ib].tobytes()


@pytest.mark.gpu
def test_gpu_deterministic_runs_bitwise_equal():
    """HIP kernel, 5 runs: f64-atomic order changes run to run, the fixed-point sums must not."""
    from spark_druid_olap_amd.models import tpch

    ds = tpch.to_datasource(tpch.generate_flat(0.05, "cuda"), profile="bench")
    eng = Engine(use_native=True)
    for dims in (("l_returnflag", "l_linestatus"), ("s_nation", "p_brand")):
        pq = eng.prepare(_query(True, dims), ds)
        ref = None
        for _ in range(5):
            r = pq.run()
            keys = np.lexsort([materialize(r.data[d]).astype(str) for d in dims])
            cur = b"".join(np.asarray(r.data[c], dtype=np.float64)[keys].tobytes() for c in ("ratio", "neg"))
            ref = cur if ref is None else ref
            assert cur == ref, dims
        # and the value agrees with the torch fp64 reference executor on the same shard
        cpu = Engine(use_native=False).execute(_query(False, dims), ds)
        ga, gb = _by_key(r, dims), _by_key(cpu, dims)
        for k, (v, w) in ga.items():
            assert v == pytest.approx(gb[k][0], rel=1e-11, abs=1e-5)
            assert w == pytest.approx(gb[k][1], rel=1e-11, abs=1e-5)


def test_sql_conf_switches_plans(ds_small):
    """``SET spark.sparklinedata.druid.deterministic=true`` re-prepares cached plans with fixed-point
    sums; the answer matches the default f64 plan to rounding."""
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.session import Session

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    q = ("select l_returnflag, sum(l_extendedprice / (1 + l_tax) / 3) as r from orderLineItemPartSupplier "
         "group by l_returnflag order by l_returnflag")
    a = s.sql(q).collect()
    s.sql("set spark.sparklinedata.druid.deterministic=true")
    d = s.sql(q)
    b = d.collect()
    preps = [getattr(x, "_prepared", None) for x in d.druid_queries()]
    assert preps and all(p is not None and p.deterministic for p in preps)
    assert [r[0] for r in a] == [r[0] for r in b]
    for x, y in zip(a, b):
        assert y[1] == pytest.approx(x[1], rel=1e-12)
