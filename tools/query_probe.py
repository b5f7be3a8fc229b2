"""Prepare and run each benchmark QuerySpec, printing progress and per-variant kernel timings.

  python tools/query_probe.py SF [variant ...] [-- query names]

A variant is ``base[b<workgroups per CU>][c<accumulator copies per wave>][u<max words per step>][slds|sreg][creg0]
[dw<N>][plain]``: target workgroups per CU, accumulator copies, word unroll cap, forced LDS-DMA / VGPR staging,
count-only scans through LDS atomics instead of register counters, the packed-kernel dense-walk threshold, plain
byte-width columns (see ops/jit.py); results of every variant are checked against the first one.  Used to locate slow
or hung kernels and to A/B kernel-generation choices on the GPU box."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _same(a, b):
    import numpy as np

    from spark_druid_olap_amd.engine.columns import materialize

    if a.num_rows != b.num_rows or list(a.columns) != list(b.columns):
        return False
    for c in a.columns:
        x, y = materialize(a.data[c]), materialize(b.data[c])
        if x.dtype.kind in "fc" or y.dtype.kind in "fc":
            if not np.allclose(np.asarray(x, dtype=float), np.asarray(y, dtype=float), rtol=1e-9, equal_nan=True):
                return False
        elif not (np.asarray(x) == np.asarray(y)).all():
            return False
    return True


def extra_specs():
    """Q1-shaped variants that isolate one cost each (key decode, HLL, sums)."""
    from spark_druid_olap_amd.models import bench_queries as BQ
    from spark_druid_olap_amd.query import spec as S

    dims = BQ._dims("l_returnflag", "l_linestatus")
    aggs = BQ._q1_aggs()
    return [("x:count-only", S.GroupByQuerySpec("tpch", dims, aggregations=aggs[:1], intervals=BQ.ALL)),
            ("x:no-hll", S.GroupByQuerySpec("tpch", dims, aggregations=aggs[:5], intervals=BQ.ALL)),
            ("x:hll-only", S.GroupByQuerySpec("tpch", dims, aggregations=aggs[5:], intervals=BQ.ALL)),
            ("x:sum-ext", S.GroupByQuerySpec("tpch", dims, aggregations=aggs[1:2], intervals=BQ.ALL)),
            ("x:nodims-count", S.GroupByQuerySpec("tpch", [], aggregations=aggs[:1], intervals=BQ.ALL)),
            ("x:nodims-sum-ext", S.GroupByQuerySpec("tpch", [], aggregations=aggs[1:2], intervals=BQ.ALL)),
            ("x:nodims-no-hll", S.GroupByQuerySpec("tpch", [], aggregations=aggs[:5], intervals=BQ.ALL)),
            ("x:count-1key", S.GroupByQuerySpec("tpch", BQ._dims("l_linestatus"), aggregations=aggs[:1],
                                                intervals=BQ.ALL)),
            ("x:count-2key-1", S.GroupByQuerySpec("tpch", BQ._dims("l_returnflag"), aggregations=aggs[:1],
                                                  intervals=BQ.ALL))]


def main():
    import torch

    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import bench_specs
    from spark_druid_olap_amd.parallel.world import init_world

    args = sys.argv[1:]
    only = []
    if "--" in args:
        only = args[args.index("--") + 1:]
        args = args[:args.index("--")]
    sf = float(args[0]) if args else 100
    variants = args[1:] or ["base"]
    world = init_world()
    dev = world.device()
    torch.cuda.set_device(dev)
    flat = tpch.generate_flat(sf, dev)
    ds = tpch.to_datasource(flat, profile="bench")
    del flat
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    eng = Engine(world)
    print(f"data ready sf={sf} rows={ds.num_rows}", flush=True)
    specs = bench_specs() + extra_specs()
    base = {}
    import re

    from spark_druid_olap_amd.ops import jit as J

    for var in variants:
        mb = re.search(r"b(\d+)", var)
        DE.JIT_BLOCKS = int(mb.group(1)) if mb else 3
        mc = re.search(r"c(\d+)", var)
        J.MAX_NCOPY = int(mc.group(1)) if mc else 16
        DE.JIT_STAGE = "lds" if "slds" in var else ("reg" if "sreg" in var else "auto")
        DE.BLOCKS_PER_CU = max(3, DE.JIT_BLOCKS)
        J.COUNT_REGS = "creg0" not in var
        md = re.search(r"dw(\d+)", var)
        J.DENSE_WORDS_PACKED = int(md.group(1)) if md else 16
        from spark_druid_olap_amd.segment import packed as PK
        PK.ENABLED = "plain" not in var  # (byte-width columns instead of the packed copies)
        mu = re.search(r"u(\d+)", var)
        DE.FORCE_U = int(mu.group(1)) if mu else 0
        print(f"== {var}", flush=True)
        for name, qs in specs:
            if only and name not in only and name.replace(" ", "_") not in only:  # (TPCH_Q1 for "TPCH Q1")
                continue
            t = time.time()
            pq = eng.prepare(qs, ds)
            sc = pq.scans[0][2]
            ts = []
            r = None
            for i in range(6):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                r = pq.run()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t1) * 1e3)
            j = getattr(sc, "jit", None)
            info = (f"mode={sc.mode} U={getattr(j, 'U', None)} grid={getattr(sc, 'grid', None)} "
                    f"lds={j.lay.total if j else None}")
            ok = ""
            if name in base:
                ok = "same" if _same(base[name], r) else "DIFFERENT"
            else:
                base[name] = r
            print(f"  {name[:40]:40s} med {statistics.median(ts[1:]):7.3f} ms  first {ts[0]:7.2f}  {info} "
                  f"prep {time.time() - t - sum(ts) / 1e3:.2f}s rows={r.num_rows} {ok} "
                  + " ".join(f"{k}={v:.2f}" for k, v in r.stats.items() if k.endswith("_ms")), flush=True)


if __name__ == "__main__":
    main()
