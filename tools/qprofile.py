#!/usr/bin/env python3
"""Per-query phase timing on the GPU: reset / kernel / post (HIP events), plus effective
bandwidth of the scan kernel (bytes of referenced columns over scanned rows / kernel time)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--unroll", type=str, default="2")
    ap.add_argument("--both", action="store_true")
    args = ap.parse_args()
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.engine.lower import column_tensor
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import bench_specs
    from spark_druid_olap_amd.ops import native

    flat = tpch.generate_flat(args.sf, "cuda")
    ds = tpch.to_datasource(flat, profile="bench")
    del flat
    torch.cuda.synchronize()
    eng = Engine()
    for un in [int(x) for x in args.unroll.split(",")]:
        DE.UNROLL = un
        for use_jit in ([True, False] if args.both else [True]):
            DE.USE_JIT = use_jit
            print(f"rows={ds.num_rows} unroll={DE.UNROLL} jit={use_jit}")
            run_all(eng, ds, args)


def run_all(eng, ds, args):
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.lower import column_tensor
    from spark_druid_olap_amd.models.bench_queries import bench_specs
    from spark_druid_olap_amd.ops import native

    for name, q in bench_specs():
        pq = eng.prepare(q, ds)
        _, prog, prep = pq.scans[0]
        for _ in range(2):
            pq.run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tk, tr = [], []
        for _ in range(args.iters):
            ev[0].record()
            prep._reset()
            ev[1].record()
            prep._launch(prep._bufs())
            ev[2].record()
            torch.cuda.synchronize()
            tr.append(ev[0].elapsed_time(ev[1]))
            tk.append(ev[1].elapsed_time(ev[2]))
        t0 = time.perf_counter()
        for _ in range(args.iters):
            res = pq.run()
        torch.cuda.synchronize()
        tq = (time.perf_counter() - t0) * 1e3 / args.iters
        rows = prog.rows_in_ranges
        byts = sum(column_tensor(ds, c).element_size() for c in prog.cols) * rows
        bw = byts / (min(tk) * 1e-3) / 1e9
        ju = prep.jit.U if prep.jit else 0
        print(f"{name[:40]:40s} mode={prep.mode} G={prog.G:<8d} grid={prep.grid:<5d} jitU={ju} "
              f"reset={min(tr):7.3f}ms kernel={min(tk):7.3f}ms query={tq:7.3f}ms rows={rows/1e6:7.1f}M "
              f"cols={len(prog.cols)} zones={len(prog.zones)} bm={len(prog.bm_leaves)} fin={int(prog.final_pre)} "
              f"colGB/s={bw:7.0f} " + " ".join(f"{k}={v:.2f}" for k, v in res.stats.items() if k.endswith("_ms")))


if __name__ == "__main__":
    main()
