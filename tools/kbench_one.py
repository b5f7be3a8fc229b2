#!/usr/bin/env python3
"""Run one benchmark query's scan kernel N times (for rocprofv3 --pmc / kernel-trace focus)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--query", default="Ship Date Range")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import bench_specs
    from spark_druid_olap_amd.ops import native

    flat = tpch.generate_flat(args.sf, "cuda")
    ds = tpch.to_datasource(flat, profile="bench")
    del flat
    eng = Engine()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from query_probe import extra_specs

    specs = dict(bench_specs() + extra_specs())
    names = args.query.split(",") if args.query != "all" else [n for n, _ in bench_specs()]
    for name in names:
        q = specs[name]
        pq = eng.prepare(q, ds)
        _, prog, prep = pq.scans[0]
        pq.run()
        torch.cuda.synchronize()
        js = prep.jit
        if js is not None:  # which kernel shape runs (tag = mode, U, copies, staging, shared table)
            pk = {c: getattr(v, "width", None) for c, v in (getattr(prog, "packed", None) or {}).items()}
            print(f"{name}: {js.name} U={js.U} ncopy={js.lay.ncopy} regstage={js.lay.regstage} "
                  f"LDS={js.lay.total} spills={js.spills} packed={pk} "
                  f"meta={ {k: js.meta.get(k) for k in ('.vgpr_count', '.sgpr_count', '.sgpr_spill_count', '.vgpr_spill_count', '.private_segment_fixed_size', 'amdhsa.target')} }",
                  flush=True)
        for _ in range(args.iters):
            b = prep._bufs()
            prep._reset(b)
            prep._launch(b)  # the specialized (JIT) kernel when one was built, else the interpreter
        torch.cuda.synchronize()
        print("done", name, flush=True)


if __name__ == "__main__":
    main()
