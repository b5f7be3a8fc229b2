"""Serving-time background compiles (engine/device_exec.py async_compile): a first-seen kernel shape
runs on the interpreter kernel while its JIT source compiles on a background thread; the session
re-prepares the statement once the compile is done and the next execution runs the JIT kernel.
The interim (interpreter) and final (JIT) answers must agree exactly."""
import pytest

pytestmark = pytest.mark.gpu

Q = ("select l_returnflag, l_linestatus, sum(l_quantity) q, count(*) c from orderLineItemPartSupplier "
     "where l_shipdate <= date '1998-08-11' and l_discount > 0.03 group by l_returnflag, l_linestatus")


def test_interim_interpreter_then_jit(tmp_path, monkeypatch):
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.ops import jit
    from spark_druid_olap_amd.sql import plan as P
    from spark_druid_olap_amd.session import Session

    monkeypatch.setenv("SDO_JIT_CACHE", str(tmp_path / "jit"))  # every shape is first-seen here
    monkeypatch.setattr(jit, "_handles", {})
    monkeypatch.setattr(DE, "ASYNC_JIT", True)
    import threading

    gate = threading.Event()  # (holds the background compile until the interim answer is in)
    job = DE._async_job
    monkeypatch.setattr(DE, "_async_job", lambda *a: (gate.wait(120), job(*a))[1])
    flat = tpch.generate_flat(0.05, "cuda")
    ds = tpch.to_datasource(flat, profile="bench")
    s = Session(engine=Engine())
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))

    df = s.sql(Q)
    with DE.async_compile():
        df.prepare()
    dq = P.find_all_deep(df.plan, P.DruidQuery)[0]
    interim = dq._prepared
    assert interim.jit_pending, "the first-seen shape did not compile in the background"
    assert all(sc.jit is None for _, _, sc in interim.scans)
    a = df.to_pandas()
    assert dq._prepared is interim
    gate.set()
    for f in interim.jit_pending:
        f.result(timeout=300)
    df2 = s.sql(Q)
    df2.prepare()
    final = dq._prepared
    assert final is not interim and not getattr(final, "jit_pending", None)
    assert all(sc.jit is not None for _, _, sc in final.scans)
    b = df2.to_pandas()

    import pandas as pd

    key = lambda x: x.sort_values(["l_returnflag", "l_linestatus"]).reset_index(drop=True)  # noqa: E731
    assert len(a) >= 3 and list(a.columns) == ["l_returnflag", "l_linestatus", "q", "c"]
    # the interpreter kernel (interim) and the JIT kernel (final) agree exactly
    pd.testing.assert_frame_equal(key(a), key(b), check_dtype=False)
