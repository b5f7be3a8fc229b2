"""Print the lowered program and the generated JIT kernel source of the headline queries (CPU
only: the SQL is planned over a small synthetic shard, lowered and emitted, not run).

  python tools/jit_source.py [query name substring ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.ops import jit
    from spark_druid_olap_amd.planner.cost import plan_groupby
    from spark_druid_olap_amd.session import Session
    from spark_druid_olap_amd.ops import desc as D

    want = [a for a in sys.argv[1:] if not a.startswith("--")]
    queries = tpch.BENCH_QUERIES
    if "--tpch22" in sys.argv:
        from spark_druid_olap_amd.models import tpch22

        queries = tpch22.QUERIES
    flat = tpch.generate_flat(0.05, "cpu")
    ds = tpch.to_datasource(flat, profile="bench")
    sess = Session(engine=Engine(use_native=False), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    sess.register_datasource(ds)
    sess.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    sess.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    for name, q in queries:
        if want and not any(w.lower() in name.lower() for w in want):
            continue
        df = sess.sql(q)
        for dq in df.druid_queries():
            pq = sess.engine.prepare(dq.spec, ds)
            for _, prog, _ in pq.scans:
                gp = plan_groupby(prog, True, True)
                if os.environ.get("SDO_FORCE_PART") and jit.part_eligible(prog) and prog.G > 4096:
                    gp.mode = "partitioned"
                mode = {"dense-lds": D.M_DENSE_LDS, "dense-global": D.M_DENSE_GLOBAL, "hash": D.M_HASH,
                        "partitioned": D.M_PART}[gp.mode]
                print(f"==== {name}: G={prog.G} keys={[(k.name, k.kind, k.card) for k in prog.keys]} "
                      f"slots={prog.slots} plan={gp.describe()}")
                from spark_druid_olap_amd.segment import packed as PK

                if PK.ENABLED:  # bit-packed columns (CPU copies here)
                    from spark_druid_olap_amd.engine.lower import column_tensor

                    prog.packed = {}
                    for c in (list(prog.fcols) + list(prog.pcols)) if mode in (D.M_DENSE_LDS, D.M_DENSE_GLOBAL, D.M_HASH) else []:
                        t = column_tensor(ds, c)
                        if not t.is_floating_point():
                            tt = t[:ds.num_rows].to(torch.int64) if t.dtype == torch.uint16 else t[:ds.num_rows]
                            lo, hi = int(tt.min()), int(tt.max())
                            if PK.worth_packing(t, PK.width_for(lo, hi)):
                                prog.packed[c] = PK.pack(t, ds.num_rows, lo, hi)
                regstage = jit.prefer_regstage(prog)
                lay = jit.layout(prog, mode, 4, bool(prog.nhll) and gp.hll_lds, 1 << prog.hll_p,
                                 (160 * 1024) // 3 - 512, regstage, gp.shared)
                g = jit._Gen(prog, mode, 4, bool(prog.nhll) and gp.hll_lds, True, lay, 1 << prog.hll_p)
                src = g.source("sdo_jit_probe")
                print(src)
                if os.environ.get("SDO_JIT_COMPILE"):  # hipRTC for gfx950 (no GPU needed)
                    code = jit.compile_code(src, "sdo_jit_probe")
                    print(f"// compiled: {len(code)} bytes of gfx950 code object")
                    if os.environ.get("SDO_JIT_REGS"):  # register budget of the kernel (code-object notes)
                        import re
                        import subprocess
                        import tempfile

                        with tempfile.NamedTemporaryFile(suffix=".co") as f:
                            f.write(code)
                            f.flush()
                            notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name],
                                                   capture_output=True, text=True).stdout
                        regs = {k: (re.findall(r"\." + k + r":\s+(\d+)", notes) or ["?"])[0]
                                for k in ("sgpr_count", "vgpr_count", "sgpr_spill_count", "vgpr_spill_count")}
                        print(f"@@ {name}: {regs}", file=sys.stderr)


if __name__ == "__main__":
    main()
