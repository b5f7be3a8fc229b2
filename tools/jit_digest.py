#!/usr/bin/env python3
"""Digest of every JIT kernel source the engine would generate for the benchmark suites (CPU only,
nothing compiled): the shape-shared and literal-specialized scan of every pushed query of the
8-query headline suite, the TPC-H 22 sweep and SSB, through the same plan / layout / staging
choices as ``engine/device_exec.py _jit_build``.  Refactors of the generator that must not change
the default kernels compare the digests before and after:

  python tools/jit_digest.py > /tmp/before.txt   ...   python tools/jit_digest.py | diff /tmp/before.txt -

``--spills`` compiles every kernel (hipRTC, no GPU needed) and flags those that use scratch;
``--dump DIR`` writes the sources.
"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.engine.lower import column_tensor
    from spark_druid_olap_amd.models import ssb, tpch, tpch22
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.ops import jit
    from spark_druid_olap_amd.planner.cost import plan_groupby
    from spark_druid_olap_amd.segment import packed as PK
    from spark_druid_olap_amd.session import Session

    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    if dump:
        os.makedirs(dump, exist_ok=True)
    spills = "--spills" in sys.argv  # compile (hipRTC, no GPU) and report kernels that use scratch
    if not spills:
        jit.compile_code = lambda src, name: b""  # generate only
    jit.compile_source = lambda src, name: -1
    DE.native.narrow4 = lambda: 1

    def digest(label, sess, ds, queries):
        for name, q in queries:
            try:
                dqs = sess.sql(q).druid_queries()
            except Exception as e:  # noqa: BLE001
                print(f"{label}/{name}: plan error {type(e).__name__}")
                continue
            for i, dq in enumerate(dqs):
                try:
                    pq = sess.engine.prepare(dq.spec, ds)
                except Exception as e:  # noqa: BLE001
                    print(f"{label}/{name}#{i}: prepare error {type(e).__name__}")
                    continue
                pq = getattr(pq, "inner", pq)
                for j, (_, prog, _) in enumerate(getattr(pq, "scans", [])):
                    gp = plan_groupby(prog, True, True)
                    mode = {"dense-lds": D.M_DENSE_LDS, "dense-global": D.M_DENSE_GLOBAL, "hash": D.M_HASH,
                            "partitioned": D.M_PART}[gp.mode]
                    prog.packed = {}
                    for c in (list(prog.fcols) + list(prog.pcols)) if mode in (D.M_DENSE_LDS, D.M_DENSE_GLOBAL, D.M_HASH) else []:
                        t = column_tensor(ds, c)
                        if not t.is_floating_point():
                            tt = t[:ds.num_rows].to(torch.int64) if t.dtype == torch.uint16 else t[:ds.num_rows]
                            lo, hi = int(tt.min()), int(tt.max())
                            if PK.worth_packing(t, PK.width_for(lo, hi)):
                                prog.packed[c] = PK.pack(t, ds.num_rows, lo, hi)
                    js = DE._jit_build(prog, mode, bool(prog.nhll) and gp.hll_lds, 1 << prog.hll_p, gp.shared,
                                       load=False)
                    if js is None:
                        print(f"{label}/{name}#{i}.{j}: no jit")
                        continue
                    sp = js.specialized()
                    h1 = hashlib.sha1(js.src.encode()).hexdigest()[:12]
                    h2 = hashlib.sha1(sp.src.encode()).hexdigest()[:12]
                    print(f"{label}/{name}#{i}.{j}: {gp.mode} U={js.U} lds={js.lay.total} {h1} {h2}")
                    for k in (js, sp) if spills else ():
                        if k.spills:
                            print(f"   SPILLS ({'literal' if k is sp else 'shape'}): "
                                  + " ".join(f"{x}={k.meta.get(x)}" for x in (".vgpr_count", ".vgpr_spill_count",
                                                                             ".private_segment_fixed_size")))
                    if dump:
                        tag = f"{label}_{name}_{i}_{j}".replace(" ", "_").replace("/", "_").replace(",", "")
                        for suffix, src in (("shape", js.src), ("lit", sp.src)):
                            with open(os.path.join(dump, f"{tag}.{suffix}.hip"), "w") as f:
                                f.write(src)

    flat = tpch.generate_flat(0.05, "cpu")
    ds = tpch.to_datasource(flat, profile="bench")
    for label, qs, conf in (("tpch8", tpch.BENCH_QUERIES, {"spark.sparklinedata.druid.approxCountDistinct": "true"}),
                            ("tpch22", tpch22.QUERIES, {})):
        s = Session(engine=Engine(use_native=False), conf=conf)
        s.register_datasource(ds)
        s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
        s.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
        digest(label, s, ds, qs)
    sds = ssb.to_datasource(ssb.generate_flat(0.01, "cpu"))
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(sds)
    ssb.register(s)
    digest("ssb", s, sds, ssb.ALL_QUERIES)


if __name__ == "__main__":
    main()
