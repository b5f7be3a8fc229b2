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


def test_presence_byte_table_matches_reference():
    """Existence-only dense HBM scan with a one-byte-per-group table (nested inner levels)."""
    import torch

    from spark_druid_olap_amd.engine.device_exec import PreparedScan
    from spark_druid_olap_amd.engine.lower import Lowerer
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.ops.reference import run_reference
    from spark_druid_olap_amd.query import spec as S

    ds = tpch.to_datasource(tpch.generate_flat(0.05, "cuda"), profile="bench")
    f = S.SelectorFilterSpec("l_shipmode", "MAIL")
    prog = Lowerer(ds).lower_aggregate(["1992-01-01/1999-01-01"], f, [S.DefaultDimensionSpec("o_orderkey")], None, [])
    prep = PreparedScan(prog, mode=D.M_DENSE_GLOBAL, dense_max=1 << 34)
    assert prep.pres_bytes and prep.acc.dtype == torch.uint8
    got = prep.run()
    ref = run_reference(prog)
    ref_keys = ref.compact().keys
    assert torch.equal(torch.sort(got.keys).values, torch.sort(ref_keys.to(got.keys.device)).values)
