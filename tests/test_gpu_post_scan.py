"""Post-scan HIP kernels (ops/csrc/post_scan.hip) against plain PyTorch references, and concurrent
execution of one prepared query on several stream slots (engine/scheduler.py)."""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


def _native():
    from spark_druid_olap_amd.ops import native

    return native


@pytest.mark.parametrize("n,density", [(1, 1.0), (63, 0.5), (64 * 1024 + 5, 0.1), (3_000_001, 0.01),
                                       (5_000_000, 0.9), (200_000, 0.0)])
def test_compact_rows_matches_nonzero(n, density):
    g = torch.Generator(device="cuda").manual_seed(n)
    bits = torch.rand(n, generator=g, device="cuda") < density
    nw = (n + 63) // 64
    padded = torch.zeros(nw * 64, dtype=torch.bool, device="cuda")
    padded[:n] = bits
    w = (padded.view(nw, 64).to(torch.int64) << torch.arange(64, device="cuda")).sum(1)
    got = _native().compact_rows(w.contiguous())
    exp = torch.nonzero(bits).flatten()
    assert torch.equal(got, exp)


@pytest.mark.parametrize("dtype", [torch.int64, torch.uint8])
def test_nonzero_rows_strided(dtype):
    g = torch.Generator(device="cuda").manual_seed(5)
    if dtype == torch.int64:
        acc = torch.randint(0, 3, (777_777, 3), generator=g, device="cuda", dtype=torch.int64)
        col = acc[:, 0]
    else:
        col = torch.randint(0, 2, (1_234_567,), generator=g, device="cuda").to(torch.uint8)
    got = _native().nonzero_rows(col)
    assert torch.equal(got, torch.nonzero(col).flatten())


@pytest.mark.parametrize("n", [1, 15, 16, 1023, 1024, 1025, 150_001, 3_000_000])
def test_nonzero_rows_contiguous_bytes(n):
    """The 16-byte-load path for contiguous byte tables (and its ragged tail)."""
    g = torch.Generator(device="cuda").manual_seed(n)
    col = (torch.rand(n, generator=g, device="cuda") < 0.3).to(torch.uint8) * 7
    got = _native().nonzero_rows(col)
    assert torch.equal(got, torch.nonzero(col).flatten())
    b = torch.rand(n, generator=g, device="cuda") < 0.5
    assert torch.equal(_native().nonzero_rows(b.view(torch.uint8)), torch.nonzero(b).flatten())


@pytest.mark.parametrize("n,nbins", [(1, 1), (1000, 7), (3_000_017, 1_000_003), (10_000_000, 64), (5_000_000, 16384), (5_000_000, 16385)])
def test_histogram_matches_bincount(n, nbins):
    g = torch.Generator(device="cuda").manual_seed(n)
    keys = torch.randint(0, nbins, (n,), generator=g, device="cuda", dtype=torch.int64)
    keys[::97] = nbins + 5  # out-of-range ids are ignored
    got = _native().histogram(keys, nbins)
    exp = torch.bincount(keys[keys < nbins], minlength=nbins)
    assert torch.equal(got, exp)


@pytest.mark.parametrize("kind", ["f64", "i64"])
@pytest.mark.parametrize("desc", [True, False])
@pytest.mark.parametrize("R,k", [(100, 7), (1_000_003, 100), (2_000_000, 1)])
def test_topk_keep_is_exact_superset(kind, desc, R, k):
    g = torch.Generator(device="cuda").manual_seed(R + k)
    acc = torch.zeros((R, 3), dtype=torch.int64, device="cuda")
    if kind == "f64":
        v = (torch.randn(R, generator=g, device="cuda", dtype=torch.float64) * 1e6)
        v[::97] = v[5]  # ties
        acc[:, 1] = v.view(torch.int64)
        ref = v
    else:
        v = torch.randint(-10 ** 12, 10 ** 12, (R,), generator=g, device="cuda", dtype=torch.int64)
        v[::89] = v[3]
        acc[:, 1] = v
        ref = v.to(torch.float64)
    keep = _native().topk_keep(acc, 1, kind == "f64", desc, k)
    key = ref if desc else -ref
    kth = torch.topk(key, k).values.min()
    must = torch.nonzero(key >= kth).flatten()
    # every row that ties or beats the k-th best is kept, and keep is ascending and duplicate-free
    assert torch.isin(must, keep).all()
    assert bool((keep[1:] > keep[:-1]).all())
    # the superset stays small (one 36-bit bucket beyond the top k)
    assert keep.numel() <= max(4 * k + 64, must.numel() + 64)
    # exact after order + limit
    sel = key[keep]
    top = torch.sort(sel, descending=True).values[:k]
    assert torch.equal(top, torch.sort(key, descending=True).values[:k])


def test_concurrent_slots_match_serial():
    """Two threads run the same prepared GPU query on different stream slots at the same time:
    each slot has its own accumulators, so results equal a serial run."""
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.engine.scheduler import StreamScheduler
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.query import spec as S

    ds = tpch.to_datasource(tpch.generate_flat(0.2, "cuda"), profile="bench")
    eng = Engine(use_native=True)
    qs = [S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("l_returnflag"), S.DefaultDimensionSpec("s_nation")],
                             aggregations=[S.FunctionAggregationSpec("count", "c"),
                                           S.FunctionAggregationSpec("doubleSum", "s", "l_extendedprice")],
                             intervals=["1992-01-01/1999-01-01"]),
          S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("o_orderkey")],
                             aggregations=[S.FunctionAggregationSpec("doubleSum", "s", "l_extendedprice")],
                             intervals=["1992-01-01/1999-01-01"])]
    preps = [eng.prepare(q, ds) for q in qs]
    serial = [sorted(p.run().rows()) for p in preps]
    sched = StreamScheduler(slots=3, device=torch.device("cuda", 0))
    errs, outs = [], {}

    def work(tid):
        try:
            for it in range(6):
                with sched.lease():
                    p = preps[(tid + it) % 2]
                    outs[(tid, it)] = ((tid + it) % 2, sorted(p.run().rows()))
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    for qi, rows in outs.values():
        assert rows == serial[qi]
    assert len(preps[0].scans[0][2]._slots) >= 2  # several slots really ran
