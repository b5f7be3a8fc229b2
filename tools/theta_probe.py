#!/usr/bin/env python3
"""thetaSketch group-by on the device (verdict r3 #6 evidence): TPC-H flattened index at --sf, a
per-shipmode theta sketch of o_orderkey (k = 4096) and of c_name (k = 16384), run --iters times
after a warmup; prints per-run latency.  Under ``rocprofv3 --kernel-trace --stats`` the kernel list
shows the KMV selection as sdo::theta_* kernels and no torch sort.

  python tools/theta_probe.py --sf 10 --iters 10
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.query import spec as S

    ds = tpch.to_datasource(tpch.generate_flat(a.sf, "cuda"), profile="bench")
    q = S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("l_shipmode")],
                           aggregations=[S.ThetaSketchAggregationSpec("orders", "o_orderkey", 4096),
                                         S.ThetaSketchAggregationSpec("customers", "c_name", 16384)],
                           intervals=["1992-01-01/1999-01-01"])
    pq = Engine(use_native=True).prepare(q, ds)
    r = pq.run()
    ts = []
    for _ in range(a.iters):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = pq.run()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"theta group-by SF{a.sf:g}: median {statistics.median(ts):.3f} ms  min {min(ts):.3f} ms  "
          f"groups {r.num_rows}", flush=True)
    th = getattr(pq, "_theta_prep", None)
    if th:
        print(f"   select passes per aggregator (last run): {th.attempts}  target multipliers: {th._mult}  "
              f"histogram bits: {th.bits}", flush=True)
    for i in range(r.num_rows):
        print("  ", r.data["l_shipmode"][i], round(float(r.data["orders"][i])), round(float(r.data["customers"][i])))


if __name__ == "__main__":
    main()
