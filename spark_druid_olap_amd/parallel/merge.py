"""Cross-GPU merge of partial aggregates (the reference's broker merge / Spark shuffle +
final aggregate, ``asd/PostAggregate.scala:39-103``, re-designed for RCCL over xGMI).

* Small dense states (the common OLAP case: Q1 is 6 groups) are latency-bound: ONE
  ``all_gather_into_tensor`` of the packed state (accumulators + HLL registers as int64 words)
  followed by a local per-slot reduction -- one collective instead of one per reduce-op.
* Large dense states use bandwidth-optimal ring ``all_reduce`` over at most three buckets (int
  sums + status word, float sums, max + bitwise-NOT(min)) with one host sync at the end; HLL
  registers reduce with MAX -- mergeable sketches, which the reference could not merge across
  historicals, ``asd/PostAggregate.scala:62-70``.
* Sparse (hash) states are compacted per GPU, gathered (variable length), and merged by key.
  When the datasource is partitioned on a grouping key the groups are disjoint across ranks and
  the merge degenerates to a concatenation.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from ..engine.partials import Partials, merge_sparse
from ..ops import desc as D
from .fault import STATUS_FAILED, STATUS_OK, raise_if_failed
from .world import World

ONE_SHOT_BYTES = 4 << 20


def _reduce_stacked(prog, acc_all: torch.Tensor) -> torch.Tensor:
    """acc_all [ranks, R, nslots] -> [R, nslots] with per-slot ops."""
    out = torch.empty(acc_all.shape[1:], dtype=torch.int64, device=acc_all.device)
    for s, (op, init) in enumerate(prog.slots):
        col = acc_all[:, :, s]
        if op == D.S_SUM_I:
            out[:, s] = col.sum(dim=0)
        elif op == D.S_SUM_F:
            out[:, s] = col.contiguous().view(torch.float64).sum(dim=0).view(torch.int64)
        elif op == D.S_MIN_I:
            out[:, s] = col.amin(dim=0)
        else:
            out[:, s] = col.amax(dim=0)
    return out


def _merge_dense_bucketed(world: World, prog, part: Partials, status: int,
                          local_error: Optional[BaseException]) -> Partials:
    """Large dense state: at most three ring all-reduces (each per-xGMI-link bandwidth bound) plus
    one per HLL register block, with ONE host synchronisation after all of them were enqueued.

    * int sums + the status word (sum of the ranks' statuses is non-zero iff one failed);
    * float64 sums;
    * int max slots and the bitwise NOT of int min slots (``min x == ~max ~x``, no overflow at
      INT64_MIN unlike negation), so min and max share one MAX collective.
    A failed rank contributes a layout-compatible placeholder, so every rank issues the same
    collectives in the same order and then raises together (parallel/fault.py)."""
    acc = part.acc.clone()
    R = acc.shape[0]
    by_op = {op: [s for s, (o, _) in enumerate(prog.slots) if o == op]
             for op in (D.S_SUM_I, D.S_SUM_F, D.S_MIN_I, D.S_MAX_I)}
    si, sf, mn, mx = by_op[D.S_SUM_I], by_op[D.S_SUM_F], by_op[D.S_MIN_I], by_op[D.S_MAX_I]
    st = torch.full((1,), status, dtype=torch.int64, device=acc.device)
    b_sum = torch.cat([acc[:, si].reshape(-1), st]) if si else st
    world.all_reduce(b_sum, "sum")
    if sf:
        b_f = acc[:, sf].contiguous().view(torch.float64)
        world.all_reduce(b_f, "sum")
        acc[:, sf] = b_f.view(torch.int64)
    if mn or mx:
        b_max = torch.cat([acc[:, mx].reshape(-1), torch.bitwise_not(acc[:, mn]).reshape(-1)])
        world.all_reduce(b_max, "max")
        if mx:
            acc[:, mx] = b_max[: R * len(mx)].reshape(R, len(mx))
        if mn:
            acc[:, mn] = torch.bitwise_not(b_max[R * len(mx):].reshape(R, len(mn)))
    hll = []
    for h in part.hll:
        hh = h.clone()
        world.all_reduce(hh, "max")
        hll.append(hh)
    failed = int(b_sum[-1].item())
    if local_error is not None or failed:
        raise_if_failed([failed], world.rank, local_error)
    if si:
        acc[:, si] = b_sum[:-1].reshape(R, len(si))
    return Partials("dense", acc, None, hll)


def merge_partials(world: World, prog, part: Partials, disjoint_keys: bool = False,
                   local_error: Optional[BaseException] = None) -> Partials:
    """Merge this rank's partials with every other rank's.  ``local_error`` set = this rank failed
    its scan and ``part`` is a layout-compatible placeholder: the status word travels in the
    merge's own collective and every rank raises (parallel/fault.py)."""
    if not world.distributed:
        if local_error is not None:
            raise local_error
        return part
    status = STATUS_FAILED if local_error is not None else STATUS_OK
    if part.kind == "dense" and part.acc.numel() * 8 * world.size <= ONE_SHOT_BYTES:
        R, ns = part.acc.shape
        st = torch.full((1,), status, dtype=torch.int64, device=part.acc.device)
        pieces = [part.acc.reshape(-1)] + [h.reshape(-1).to(torch.int64) for h in part.hll] + [st]
        buf = torch.cat(pieces)
        g = world.all_gather_tensor(buf)  # [ranks, L]
        sts = g[:, -1]
        if local_error is not None or bool((sts != 0).any()):
            raise_if_failed(sts.tolist(), world.rank, local_error)
        acc_all = g[:, : R * ns].reshape(world.size, R, ns)
        acc = _reduce_stacked(prog, acc_all)
        off = R * ns
        hll = []
        for h in part.hll:
            n = h.numel()
            hll.append(g[:, off: off + n].amax(dim=0).to(torch.int32).reshape(h.shape))
            off += n
        return Partials("dense", acc, None, hll)
    if part.kind == "dense":
        return _merge_dense_bucketed(world, prog, part, status, local_error)
    # sparse
    sp = part.compact()
    # keys + accumulators travel as one [n, 1 + nslots] int64 block: one length exchange (which also
    # carries the status word) + one gather
    kv = torch.cat([sp.keys.reshape(-1, 1).to(torch.int64), sp.acc], dim=1)
    kvs, sts = world.all_gather_varlen(kv, status=status)
    if local_error is not None or any(sts):
        raise_if_failed(sts, world.rank, local_error)
    hlls = [world.all_gather_varlen(h) for h in sp.hll]
    parts = [Partials("sparse", kvs[i][:, 1:], kvs[i][:, 0], [h[i] for h in hlls]) for i in range(world.size)]
    if disjoint_keys:
        return Partials("sparse", torch.cat([p.acc for p in parts]), torch.cat([p.keys for p in parts]),
                        [torch.cat([p.hll[i] for p in parts]) for i in range(len(sp.hll))])
    return merge_sparse(parts, prog.slots)
