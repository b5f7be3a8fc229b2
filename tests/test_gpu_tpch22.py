"""TPC-H 22-query sweep through the HIP scan kernels vs the plain-PyTorch reference executor on
the same device-resident index (exact for sums and counts)."""
import math

import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch, tpch22
from spark_druid_olap_amd.session import Session

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sessions():
    ds = tpch.to_datasource(tpch.generate_flat(0.05, "cuda"), profile="bench")
    out = []
    for native in (True, False):
        s = Session(engine=Engine(use_native=native))
        s.register_datasource(ds)
        s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
        s.sql(tpch.druid_ddl(with_column_mapping=False))
        out.append(s)
    return out


def _rows(d):
    def n(v):
        return None if isinstance(v, float) and math.isnan(v) else (round(v, 2) if isinstance(v, float) else v)
    return sorted((tuple(n(v) for v in r) for r in d.collect()), key=lambda r: tuple((x is None, str(x)) for x in r))


@pytest.mark.parametrize("name", [n for n, _ in tpch22.QUERIES])
def test_tpch22_native_vs_reference(sessions, name):
    nat, ref = sessions
    q = dict(tpch22.QUERIES)[name]
    d = nat.sql(q)
    assert d.druid_queries()
    a, b = _rows(d), _rows(ref.sql(q))
    assert len(a) == len(b)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            if isinstance(u, float) or isinstance(v, float):
                assert u == pytest.approx(v, rel=1e-9, abs=0.011), (name, x, y)
            else:
                assert u == v, (name, x, y)
