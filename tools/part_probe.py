#!/usr/bin/env python3
"""Radix-partition pipeline probe (ops/csrc/partition.hip): synthetic records in the producer's
chunk-region layout, then the level-1 count / scatter, level-2 count / scatter and the LDS
aggregation, each timed with HIP events and priced in GB/s of records moved -- the pieces of
TPC-H Q18 / Q16 / the BI plan's large group-bys, measured without the scan in front of them.

  python tools/part_probe.py [--n 600e6] [--g 150e6] [--rw 2] [--table 32768] [--fill 1.0]
                             [--pu 0,4,8] [--iters 3]

Checks the aggregated table against torch (count and value sum per key) once per variant."""
import argparse
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=600e6, help="records (rows the producer emitted)")
    ap.add_argument("--g", type=float, default=150e6, help="key space")
    ap.add_argument("--rw", type=int, default=2, help="record words (key + values)")
    ap.add_argument("--table", type=int, default=32 << 10, help="LDS bytes per sub-bucket table")
    ap.add_argument("--fill", type=float, default=1.0, help="fraction of each 4096-record chunk region used")
    ap.add_argument("--pu", default="0", help="scatter-tile records per thread variants (0 = by width)")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--cluster", type=int, default=0,
                    help="0: uniform keys; C: each chunk's keys sorted within a random window of G/C keys "
                         "(the index's order: time, then key within a day)")
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--fast", type=int, default=1, help="1: the split kernels' same-bucket-wave path (clustered keys)")
    ap.add_argument("--lds-min", default="0", help="scatter LDS request floor variants in bytes (fewer blocks per CU)")
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.ops import native

    nat = native.load()
    dev = torch.device("cuda")
    st = native._stream(dev)
    n, G, RW = int(a.n), int(a.g), a.rw
    CH = D.CHUNK_ROWS
    per_chunk = max(1, int(CH * a.fill))
    nch = (n + per_chunk - 1) // per_chunk
    u32 = torch.int32
    # records: chunk c holds [c*CH, c*CH + per_chunk); key in word 0, value 1 in word 1 (others 0)
    recs = torch.zeros((nch * CH, RW), dtype=u32, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    view = recs.view(nch, CH, RW)[:, :per_chunk]
    if a.cluster:
        span = max(1, G // a.cluster)
        base = torch.randint(0, max(1, G - span), (nch, 1), generator=gen, device=dev, dtype=torch.int64)
        k = base + torch.randint(0, span, (nch, per_chunk), generator=gen, device=dev, dtype=torch.int64)
        view[..., 0] = torch.sort(k, dim=1).values.to(u32)
        del k, base
    else:
        view[..., 0] = torch.randint(0, G, (nch, per_chunk), generator=gen, device=dev, dtype=torch.int64).to(u32)
    if RW > 1:
        view[..., 1] = 1
    seg_lo = (torch.arange(nch, dtype=torch.int64, device=dev) * CH).to(u32)
    pend = seg_lo + per_chunk
    ns = 2 if RW <= 2 else 3  # (RW 4: an i32 and an i64 field, like TopNSuppliersGlobal's records)
    shift = max(0, int(math.floor(math.log2(max(8, a.table // (8 * ns))))))
    gbits = max(1, int(math.ceil(math.log2(max(2, G)))))
    rem = max(0, gbits - shift)
    if rem <= 10:
        levels, p1, p2, K = 1, 1 << rem, 1, 1
        shift1 = shift
    else:
        b1 = min(10, (rem + 1) // 2)
        b2 = rem - b1
        levels, p1, p2 = 2, 1 << b1, 1 << b2
        K = max(1, min(64, 4096 // p1))
        shift1 = shift + b2
    nsub = p1 * p2
    k1 = max(1, min(nch, 2048))
    words = nch * CH * RW
    out1 = torch.empty(words, dtype=u32, device=dev)
    out2 = torch.empty(words, dtype=u32, device=dev) if levels == 2 else None
    c1 = torch.empty(p1 * k1, dtype=u32, device=dev)
    t1 = torch.empty(p1, dtype=u32, device=dev)
    base1 = torch.empty(p1 + 1, dtype=u32, device=dev)
    if levels == 2:
        c2 = torch.empty(nsub * K, dtype=u32, device=dev)
        t2 = torch.empty(nsub, dtype=u32, device=dev)
        base2 = torch.empty(nsub + 1, dtype=u32, device=dev)
    acc = torch.empty((G, ns), dtype=torch.int64, device=dev)
    mb = n * RW * 4 / 1e6
    print(f"cluster={a.cluster} fast={a.fast} n={n} G={G} RW={RW} chunks={nch} fill={a.fill} shift={shift} levels={levels} P1={p1} P2={p2} K={K} "
          f"k1={k1} records={mb:.0f} MB", flush=True)

    def run(pu, lds_min=0):
        nat.part_tune(pu, lds_min)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
        names = []
        ev[0].record()
        a1 = (recs.data_ptr(), RW, seg_lo.data_ptr(), pend.data_ptr(), 1, nch, k1, shift1, p1, c1.data_ptr())
        cl = 2 if a.fast else 0
        nat.part_split(*a1, 0, 0, cl, st)
        ev[1].record()
        names.append(("count1", 1))
        nat.part_scan(c1.data_ptr(), p1, k1, t1.data_ptr(), base1.data_ptr(), st)
        ev[2].record()
        names.append(("scan1", 0))
        nat.part_split(*a1, base1.data_ptr(), out1.data_ptr(), 1 | cl, st)
        ev[3].record()
        names.append(("scatter1", 2))
        recs_f, base_f = out1, base1
        if levels == 2:
            b1p = base1.data_ptr()
            a2 = (out1.data_ptr(), RW, b1p, b1p + 4, p1, 1, K, shift, p2, c2.data_ptr())
            nat.part_split(*a2, 0, 0, cl, st)
            ev[4].record()
            names.append(("count2", 1))
            nat.part_scan(c2.data_ptr(), nsub, K, t2.data_ptr(), base2.data_ptr(), st)
            ev[5].record()
            names.append(("scan2", 0))
            nat.part_split(*a2, base2.data_ptr(), out2.data_ptr(), 1 | cl, st)
            ev[6].record()
            names.append(("scatter2", 2))
            recs_f, base_f = out2, base2
        else:
            ev[4].record()
            ev[5].record()
            ev[6].record()
            names += [("-", 0), ("-", 0), ("-", 0)]
        if RW <= 2:
            slots, widths = ([1], [1]) if RW == 2 else ([0], [0])
        elif RW == 3:
            slots, widths = [1, 2], [1, 1]  # (TopVolumeCustomers: two i32 sums)
        else:
            slots, widths = [1, 2], [1, 2]
        if 1 + sum(widths) == RW:
            nat.part_agg(recs_f.data_ptr(), RW, base_f.data_ptr(), nsub, G, shift, slots, widths,
                         [D.S_SUM_I] * ns, [0] * ns, acc.data_ptr(), [], 1, 0, 0, 0, st)
        ev[7].record()
        names.append(("agg", 1))
        torch.cuda.synchronize()
        out = {}
        for i, (nm, passes) in enumerate(names):
            if nm == "-":
                continue
            out[nm] = ev[i].elapsed_time(ev[i + 1])
        return out

    for v, lm in [(int(x), int(y)) for x in a.pu.split(",") for y in a.lds_min.split(",")]:
        ts = []
        for it in range(a.iters + 1):
            r = run(v, lm)
            if it:
                ts.append(r)
        med = {k: sorted(t[k] for t in ts)[len(ts) // 2] for k in ts[0]}
        tot = sum(med.values())
        gbs = {"count1": mb / 1e3, "scatter1": 2 * mb / 1e3, "count2": mb / 1e3, "scatter2": 2 * mb / 1e3,
               "agg": mb / 1e3}
        line = " ".join(f"{k}={ms:.3f}ms" + (f"({gbs[k] / ms:.2f}TB/s)" if k in gbs and ms > 0 else "")
                        for k, ms in med.items())
        print(f"pu={v} lds_min={lm}: total {tot:.3f} ms  {line}", flush=True)
        if a.check and RW == 2:
            keys = view[..., 0].reshape(-1).to(torch.int64)
            cnt = torch.bincount(keys, minlength=G)
            ok = torch.equal(acc[:, 1].cpu(), cnt.cpu()) if G <= (1 << 28) else bool((acc[:, 1] == cnt).all())
            print(f"  check: value sums per key == bincount: {ok}", flush=True)
            del keys, cnt
    nat.part_tune(0)


if __name__ == "__main__":
    main()
