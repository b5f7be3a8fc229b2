"""HLL code planes (segment/hllcode.py): the precomputed per-row (bucket, rho) of a dimension gives
bit-identical HLL registers to hashing each row's id (ops/reference.py:hll_update_values, the host
twin of the kernels' hll_bucket_rho), on the torch engine (CPU) and on the HIP JIT / interpreter
kernels (GPU)."""
import pytest
import torch

from spark_druid_olap_amd.ops import desc as D
from spark_druid_olap_amd.query import spec as S


def _lower(ds, codes: bool, dims=("l_returnflag", "l_linestatus"), col="o_orderkey", filt=None):
    from spark_druid_olap_amd.engine.lower import Lowerer
    from spark_druid_olap_amd.segment import hllcode

    old = hllcode.ENABLED
    hllcode.ENABLED = codes
    try:
        aggs = [S.FunctionAggregationSpec("count", "c"), S.CardinalityAggregationSpec("u", [col], True)]
        return Lowerer(ds).lower_aggregate(["1992-01-01/1999-01-01"], filt, [S.DefaultDimensionSpec(d) for d in dims],
                                           S.Granularity.parse("all"), aggs)
    finally:
        hllcode.ENABLED = old


@pytest.fixture(scope="module")
def cpu_ds():
    from spark_druid_olap_amd.models import tpch

    return tpch.to_datasource(tpch.generate_flat(0.02, "cpu"), profile="bench")


def test_codes_match_hash(cpu_ds):
    from spark_druid_olap_amd.ops.reference import hll_update_values
    from spark_druid_olap_amd.segment import hllcode

    v = torch.tensor([0, 1, 2, 12345, (1 << 31) - 1, (1 << 32) - 1], dtype=torch.int64)
    for p in (4, 11):
        c = hllcode.codes(v, 0x6ae165e4, p)
        b, r = hll_update_values(v, 0x6ae165e4, p)
        assert torch.equal(c >> 5, b) and torch.equal(c & 31, r)
        assert int(c.max()) < (1 << 16)


def test_code_plane_lowering_and_registers(cpu_ds):
    from spark_druid_olap_amd.ops.reference import run_reference

    a, b = _lower(cpu_ds, True), _lower(cpu_ds, False)
    kinds_a = [x["kind"] for x in a.aops]
    assert D.A_HLL_CODE in kinds_a and D.A_HLL not in kinds_a
    assert D.A_HLL in [x["kind"] for x in b.aops]
    assert any("#hll" in c for c in a.pcols)
    pa, pb = run_reference(a), run_reference(b)
    assert torch.equal(pa.hll[0], pb.hll[0]) and int(pa.hll[0].max()) > 0
    assert torch.equal(pa.acc, pb.acc)


def test_code_plane_not_for_byte_dims_or_large_p(cpu_ds, monkeypatch):
    from spark_druid_olap_amd.segment import hllcode

    assert hllcode.code_column(cpu_ds, "l_returnflag", 11, 1) is None  # u8 ids: no fewer bytes
    assert hllcode.code_column(cpu_ds, "o_orderkey", 12, 1) is None    # bucket + rho > 16 bits
    monkeypatch.setattr(hllcode, "MAX_BYTES", 0)
    assert hllcode.code_column(cpu_ds, "o_custkey", 11, 7) is None     # plane budget


@pytest.mark.gpu
def test_code_plane_kernels_match_hashed():
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.models import tpch

    ds = tpch.to_datasource(tpch.generate_flat(0.05, "cuda"), profile="bench")
    filt = S.BoundFilterSpec("o_orderdate", "1994-01-01", "1996-01-01", False, True)
    for dims, f in ((("l_returnflag", "l_linestatus"), None), (("s_nation",), filt), ((), None),
                    (("c_nation", "s_nation"), filt)):  # global (u32 scan-time) registers
        a, b = _lower(ds, True, dims, filt=f), _lower(ds, False, dims, filt=f)
        assert D.A_HLL_CODE in [x["kind"] for x in a.aops]
        for jit in (True, False):  # JIT kernel and the interpreter
            old = DE.USE_JIT
            DE.USE_JIT = jit
            try:
                ra, rb = DE.PreparedScan(a).run(), DE.PreparedScan(b).run()
                if jit:
                    assert DE.PreparedScan(a).jit is not None
            finally:
                DE.USE_JIT = old
            assert torch.equal(ra.hll[0].cpu(), rb.hll[0].cpu()), (dims, jit)
            assert torch.equal(ra.acc.cpu(), rb.acc.cpu())
            assert int(ra.hll[0].max()) > 0
