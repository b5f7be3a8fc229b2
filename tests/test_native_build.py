"""Native extension: descriptor layout parity with the host mirror, and hipRTC compilation of the
per-query JIT kernels for gfx950 (hipRTC needs no GPU, so this runs on CPU CI)."""
import os

import pytest
import torch


def test_descriptor_layout_matches():
    from spark_druid_olap_amd.ops import desc, native

    m = native.load()
    L, P = m.layout(), desc.layout()
    assert L == {k: L[k] for k in P} and all(L[k] == P[k] for k in P)
    assert m.ARCH == "gfx950"


def test_jit_kernels_compile_for_bench_queries(ds_small, tmp_path, monkeypatch):
    from spark_druid_olap_amd.engine.lower import Lowerer
    from spark_druid_olap_amd.models.bench_queries import bench_specs
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.ops import jit

    monkeypatch.setenv("SDO_JIT_CACHE", str(tmp_path))
    low = Lowerer(ds_small)
    for name, q in bench_specs()[:4]:
        prog = low.lower_aggregate(q.intervals, q.filter, q.dimensions, q.granularity, q.aggregations)
        js = jit.JitScan(prog, D.M_DENSE_LDS if prog.G < 1000 else D.M_HASH, 4, bool(prog.nhll), 2048, True,
                         load=False)
        assert js.lay.total <= 160 * 1024
        assert "sdo_jit_" in js.src
    assert len(list(tmp_path.glob("*.co"))) >= 3
