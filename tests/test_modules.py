"""Module SPI and UDFs (SparklineDataModule / ModuleLoader parity)."""
import sys
import types

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.session import Session


def test_udf_pushed_over_dictionary(ds_small, df_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    s.register_udf("first_letter", lambda v: str(v)[:1], "string")
    d = s.sql("select first_letter(s_nation) f, count(*) from orderLineItemPartSupplier "
              "where first_letter(c_nation) = 'F' group by first_letter(s_nation)")
    [q] = d.druid_query_specs()
    assert isinstance(q.dimensions[0], S.ExtractionDimensionSpec)
    exp = df_small[df_small.c_nation.str[:1] == "F"].groupby(df_small.s_nation.str[:1]).size().to_dict()
    assert dict(d.collect()) == exp


def test_module_loading(ds_small):
    m = types.ModuleType("sdo_test_module")
    seen = []

    def register_functions(session):
        session.register_udf("plus_one", lambda v: v + 1, "bigint")

    def rule(plan, session):
        seen.append(type(plan).__name__)
        return None

    def parse(text, session):
        if text.strip().lower() == "ping":
            return session._rows_df([("pong", "string")], [("pong",)])
        return None
    m.register_functions, m.logical_rules, m.parse = register_functions, [rule], parse
    sys.modules["sdo_test_module"] = m
    s = Session(engine=Engine(use_native=False), conf={"spark.sparklinedata.modules": "sdo_test_module"})
    assert s.sql("ping").collect() == [("pong",)]
    assert s.sql("select plus_one(41)").collect() == [(42,)]
    assert seen


def test_cancel_and_timeout(ds_small):
    import pytest

    from spark_druid_olap_amd.utils.cancel import CancelToken
    from spark_druid_olap_amd.utils.errors import QueryCancelled, QueryTimeout

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    d = s.sql("select l_returnflag, count(*) from orderLineItemPartSupplier group by l_returnflag")
    t = CancelToken()
    t.cancel()
    with pytest.raises(QueryCancelled):
        d.collect(token=t)
    with pytest.raises(QueryTimeout):
        d.collect(token=CancelToken(timeout_ms=1e-6))
    assert len(d.collect()) == 3
