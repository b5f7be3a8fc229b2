"""Small dense executions replayed as HIP graphs (engine/device_exec.py run_graph_small): same
answers as the direct launches, over repeated runs (the graph is captured once per slot and
re-captured when literal specialization swaps the kernel)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(res):
    from spark_druid_olap_amd.engine.columns import materialize

    cols = list(res.columns)
    data = [np.asarray(materialize(res.data[c])) for c in cols]
    return cols, data


def test_graph_replay_matches_direct_launches():
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import bench_specs

    ds = tpch.to_datasource(tpch.generate_flat(0.05, "cuda"), profile="bench")
    eng = Engine()
    old = DE.USE_GRAPHS, DE.SPECIALIZE, DE.SPECIALIZE_AFTER
    DE.SPECIALIZE, DE.SPECIALIZE_AFTER = "sync", 1  # (as bench.py: the final kernel from run 1)
    try:
        graphed = 0
        for name, q in bench_specs():
            DE.USE_GRAPHS = False
            ref = eng.prepare(q, ds).run()
            DE.USE_GRAPHS = True
            pq = eng.prepare(q, ds)
            outs = [pq.run() for _ in range(4)]  # run 1 specializes, later runs replay the graph
            torch.cuda.synchronize()
            prep = pq.scans[0][2]
            if prep is not None and getattr(prep._bufs(), "fetch", None) is not None:
                graphed += 1
            rc, rd = _rows(ref)
            for o in outs:
                oc, od = _rows(o)
                assert oc == rc, name
                for c, x, y in zip(rc, rd, od):
                    if x.dtype.kind in "fc":
                        assert np.allclose(x.astype(float), y.astype(float), rtol=1e-9, equal_nan=True), (name, c)
                    else:
                        assert (x == y).all(), (name, c)
        assert graphed >= 5  # the small dense headline queries take the graph path
    finally:
        DE.USE_GRAPHS, DE.SPECIALIZE, DE.SPECIALIZE_AFTER = old
