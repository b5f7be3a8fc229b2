#!/usr/bin/env python3
"""ISA of the JIT scan kernel a benchmark query runs (CPU only: hipRTC compiles for gfx950 without
a GPU).  The query is planned and lowered over a small synthetic shard exactly as the engine does
(same group-by plan, same staging / unroll / layout choice as ``engine/device_exec.py _jit_build``,
bit-packed column widths of the SF being modelled), then compiled -- shape-shared and
literal-specialized -- and disassembled with llvm-objdump.  Reports, per kernel:

* VGPR / SGPR / spill counts and LDS bytes (code-object notes) and the resulting waves per SIMD;
* the hottest loop (the largest backward branch) with its instruction mix: vector-memory loads,
  LDS ops, s_waitcnt sites, VALU / SALU, and loads per 64 rows;

  python tools/jit_isa.py "TPCH Q1" [--dump] [--shape]
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LLVM = "/opt/rocm/lib/llvm/bin"


def notes(code: bytes) -> dict:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code)
        f.flush()
        txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
    out = {}
    for k in ("sgpr_count", "vgpr_count", "agpr_count", "sgpr_spill_count", "vgpr_spill_count",
              "group_segment_fixed_size", "private_segment_fixed_size"):
        m = re.findall(r"\." + k + r":\s+(\d+)", txt)
        out[k] = int(m[0]) if m else None
    return out


def disasm(code: bytes) -> list:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code)
        f.flush()
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--no-show-raw-insn", f.name],
                             capture_output=True, text=True).stdout
    ins = []
    for line in txt.splitlines():
        m = re.match(r"\s+([a-z_0-9]+)(\s.*)?//\s*([0-9A-Fa-f]+):(.*)", line)
        if m:
            t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", m.group(4))
            ins.append((int(m.group(3), 16), m.group(1), (m.group(2) or "").strip(),
                        int(t.group(1), 16) if t else None))
    return ins


def classify(op: str) -> str:
    if op.startswith(("buffer_load", "global_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("buffer_store", "global_store", "flat_store", "global_atomic", "buffer_atomic")):
        return "vmem_store/atomic"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem_load"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def loops(ins: list) -> list:
    """Backward branches: (size in instructions, start addr, end addr)."""
    addr_idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    base = ins[0][0] if ins else 0
    out = []
    for i, (a, op, arg, off) in enumerate(ins):
        if op.startswith(("s_cbranch", "s_branch")) and off is not None:
            tgt = base + off
            if tgt <= a and tgt in addr_idx:
                out.append((i - addr_idx[tgt] + 1, addr_idx[tgt], i))
    return sorted(out, reverse=True)


def report(name: str, js, code: bytes, dump: bool) -> None:
    nt = notes(code)
    ins = disasm(code)
    v = nt.get("vgpr_count") or 0
    waves = min(8, 512 // max(8, (v + 7) // 8 * 8)) if v else None
    lds = js.lay.total
    print(f"== {name}  kernel {js.name}{' (literals)' if js.literals else ''}: U={js.U} mode-layout "
          f"total LDS {lds} B, {len(ins)} instructions")
    print(f"   regs: {nt}  -> waves/SIMD by VGPRs: {waves}; workgroups/CU by LDS: {(160 * 1024) // max(lds, 1)}")
    mix = Counter(classify(op) for _, op, _, _ in ins)
    print("   whole kernel mix: " + ", ".join(f"{k}={n}" for k, n in mix.most_common()))
    ls = loops(ins)
    for size, lo, hi in ls[:3]:
        body = ins[lo:hi + 1]
        m2 = Counter(classify(op) for _, op, _, _ in body)
        waits = [arg for _, op, arg, _ in body if op.startswith("s_waitcnt")]
        print(f"   loop [{lo}..{hi}] {size} instrs: " + ", ".join(f"{k}={n}" for k, n in m2.most_common()))
        print(f"      s_waitcnt sites: {len(waits)}: " + "; ".join(waits[:12]) + (" ..." if len(waits) > 12 else ""))
        vm = [op for _, op, _, _ in body if classify(op) == "vmem_load"]
        print(f"      vmem loads: {Counter(vm).most_common()}")
        if dump:
            for a, op, arg, _ in body:
                print(f"        {a:6x}: {op} {arg}")


def main():
    import torch

    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.engine.lower import column_tensor
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.ops import jit
    from spark_druid_olap_amd.planner.cost import plan_groupby
    from spark_druid_olap_amd.segment import packed as PK
    from spark_druid_olap_amd.session import Session

    want = [a for a in sys.argv[1:] if not a.startswith("--")]
    dump = "--dump" in sys.argv
    flat = tpch.generate_flat(0.05, "cpu")
    ds = tpch.to_datasource(flat, profile="bench")
    sess = Session(engine=Engine(use_native=False), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    sess.register_datasource(ds)
    sess.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    sess.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from query_probe import extra_specs

    todo = [(n, [dq.spec for dq in sess.sql(q).druid_queries()]) for n, q in tpch.BENCH_QUERIES
            if not want or any(w.lower() in n.lower() for w in want)]
    todo += [(n, [qs]) for n, qs in extra_specs() if n in want]  # (tools/query_probe.py x:* isolation specs)
    for name, qspecs in todo:
        for spec in qspecs:
            pq = sess.engine.prepare(spec, ds)
            for _, prog, _ in pq.scans:
                gp = plan_groupby(prog, True, True)
                mode = {"dense-lds": D.M_DENSE_LDS, "dense-global": D.M_DENSE_GLOBAL, "hash": D.M_HASH,
                        "partitioned": D.M_PART}[gp.mode]
                prog.packed = {}
                for c in (list(prog.fcols) + list(prog.pcols)) if mode in DE.PACKED_MODES and prog.est_rows >= DE.PACK_MIN_SELECTIVITY * ds.num_rows and not any(int(f[0]) == D.F_IN_SET for f in prog.fops) else []:
                    t = column_tensor(ds, c)
                    if not t.is_floating_point():
                        tt = t[:ds.num_rows].to(torch.int64) if t.dtype == torch.uint16 else t[:ds.num_rows]
                        lo, hi = int(tt.min()), int(tt.max())
                        if PK.worth_packing(t, PK.width_for(lo, hi)):
                            prog.packed[c] = PK.pack(t, ds.num_rows, lo, hi)
                hll_lds = bool(prog.nhll) and gp.hll_lds
                js = DE._jit_build(prog, mode, hll_lds, 1 << prog.hll_p, gp.shared, load=False)
                if js is None:
                    print(f"== {name}: interpreter kernel (no JIT)")
                    continue
                print(f"#### {name}: G={prog.G} plan={gp.describe()}")
                kernels = [js] if "--shape" in sys.argv else [js.specialized()]
                for k in kernels:
                    if "--src" in sys.argv:
                        print(k.src)
                    report(name, k, jit.compile_code(k.src, k.name), dump)


if __name__ == "__main__":
    main()
