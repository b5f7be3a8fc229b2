"""Larger-than-HBM path: a TPC-H shard held in pinned host memory and streamed through the GPU
(segment/streamed.py), vs the same shard resident in HBM.

``python tools/streamed_bench.py --sf 20 --window-rows 33554432``: prints, per benchmark query,
resident and streamed latency, the bytes copied host->device and the effective H2D rate, and
checks that both answers agree."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=20)
    ap.add_argument("--window-rows", type=int, default=1 << 25)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.columns import materialize
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import bench_specs
    from spark_druid_olap_amd.segment.streamed import HostShard, StreamedQuery

    dev = tpch.to_datasource(tpch.generate_flat(a.sf, "cuda"), profile="bench")
    t0 = time.perf_counter()
    host = dev.to("cpu")
    shard = HostShard(host, "cuda", window_rows=a.window_rows)
    print(f"[streamed] sf={a.sf} rows={dev.num_rows} windows={len(shard.windows)} "
          f"host copy+pin {time.perf_counter() - t0:.1f}s", flush=True)
    eng = Engine()
    out = {}
    for name, q in bench_specs():
        pq = eng.prepare(q, dev)
        sq = StreamedQuery(eng, q, shard)
        rt, st = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r1 = pq.run()
            torch.cuda.synchronize()
            rt.append((time.perf_counter() - t) * 1e3)
            b0 = shard.bytes_copied
            t = time.perf_counter()
            r2 = sq.run()
            torch.cuda.synchronize()
            st.append((time.perf_counter() - t) * 1e3)
            nbytes = shard.bytes_copied - b0
        same = sorted(map(repr, zip(*[materialize(r1.data[c]).tolist() for c in r1.columns]))) == \
            sorted(map(repr, zip(*[materialize(r2.data[c]).tolist() for c in r2.columns])))
        ms = statistics.median(st)
        out[name] = {"resident_ms": round(statistics.median(rt), 3), "streamed_ms": round(ms, 2),
                     "h2d_gb": round(nbytes / 1e9, 3), "h2d_gb_per_s": round(nbytes / 1e9 / (ms / 1e3), 1),
                     "same": same}
        print(f"[streamed] {name[:40]:40s} {json.dumps(out[name])}", flush=True)
    print(json.dumps({"metric": "streamed_vs_resident", "sf": a.sf, "window_rows": a.window_rows, "queries": out}))
    if not all(v["same"] for v in out.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
