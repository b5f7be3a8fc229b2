"""Cross-GPU merge of partial aggregates (the reference's broker merge / Spark shuffle +
final aggregate, ``asd/PostAggregate.scala:39-103``, re-designed for RCCL over xGMI).

The path is the cost model's (``planner/cost.py plan_merge``), priced from the state's layout:

* Small dense states (the common OLAP case: Q1 is 6 groups) are latency-bound: ONE
  ``all_gather_into_tensor`` of the packed state (accumulators + HLL registers as int64 words)
  followed by a local per-slot reduction -- one collective instead of one per reduce-op.
* Large dense states use bandwidth-optimal ring ``all_reduce`` over at most three buckets (int
  sums + status word, float sums, max + bitwise-NOT(min)) with one host sync at the end; HLL
  registers reduce with MAX -- mergeable sketches, which the reference could not merge across
  historicals, ``asd/PostAggregate.scala:62-70``.
* Sparse (hash) states are compacted per GPU and shuffled by key hash with one
  ``all_to_all_single`` (the reference's hash-partitioned Exchange before Spark's final aggregate,
  ``asd/PostAggregate.scala:97-103``): each rank receives ~1/N of the partial rows, merges its key
  range locally, and only the merged (now disjoint) groups are gathered.  When the datasource is
  partitioned on a grouping key the groups are already disjoint across ranks and the merge
  degenerates to a concatenation (no shuffle).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from ..engine.partials import Partials, merge_sparse
from ..ops import desc as D
from .fault import STATUS_FAILED, STATUS_OK, raise_if_failed
from .world import World



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
    merged, sts = start_dense_merge(world, prog, part, status, "bucketed-allreduce").wait()
    if local_error is not None or any(sts):
        raise_if_failed(sts, world.rank, local_error)
    return merged


class DenseMerge:
    """An enqueued dense merge.  ``result()`` -> (merged partials, per-rank status words as a
    device tensor) without a host synchronisation (RCCL: the current stream waits for the
    collective); ``wait()`` -> (merged partials, status words as a list)."""

    def __init__(self, finish):
        self._finish = finish

    def result(self):
        return self._finish()

    def wait(self):
        part, sts = self._finish()
        return part, sts.tolist()


def start_dense_merge(world: World, prog, part: Partials, status: int, kind: Optional[str] = None) -> DenseMerge:
    """Enqueue the collectives of a dense merge (the cost model's one-shot gather or bucketed
    all-reduce) without waiting: segment-batched execution starts batch j's merge and scans batch
    j+1 while it runs (``PreparedQuery._run_pipelined``)."""
    kind = kind or merge_plan_for(world, part).kind
    if kind == "oneshot-allgather":
        R, ns = part.acc.shape
        st = torch.full((1,), status, dtype=torch.int64, device=part.acc.device)
        pieces = [part.acc.reshape(-1)] + [h.reshape(-1).to(torch.int64) for h in part.hll] + [st]
        pend = world.all_gather_tensor_async(torch.cat(pieces))  # [ranks, L]
        shapes = [h.shape for h in part.hll]

        def finish_gather():
            g = pend.wait()
            acc = _reduce_stacked(prog, g[:, : R * ns].reshape(world.size, R, ns))
            off = R * ns
            hll = []
            for shp in shapes:
                n = shp.numel()
                hll.append(g[:, off: off + n].amax(dim=0).to(torch.int32).reshape(shp))
                off += n
            return Partials("dense", acc, None, hll), g[:, -1]

        return DenseMerge(finish_gather)
    acc = part.acc.clone()
    R = acc.shape[0]
    by_op = {op: [s for s, (o, _) in enumerate(prog.slots) if o == op]
             for op in (D.S_SUM_I, D.S_SUM_F, D.S_MIN_I, D.S_MAX_I)}
    si, sf, mn, mx = by_op[D.S_SUM_I], by_op[D.S_SUM_F], by_op[D.S_MIN_I], by_op[D.S_MAX_I]
    st = torch.zeros((world.size,), dtype=torch.int64, device=acc.device)
    st[world.rank] = status
    b_sum = torch.cat([acc[:, si].reshape(-1), st]) if si else st
    p_sum = world.all_reduce_async(b_sum, "sum")
    p_f = p_max = None
    if sf:
        b_f = acc[:, sf].contiguous().view(torch.float64)
        p_f = world.all_reduce_async(b_f, "sum")
    if mn or mx:
        b_max = torch.cat([acc[:, mx].reshape(-1), torch.bitwise_not(acc[:, mn]).reshape(-1)])
        p_max = world.all_reduce_async(b_max, "max")
    p_hll = [world.all_reduce_async(h.clone(), "max") for h in part.hll]

    def finish_reduce():
        s = p_sum.wait()
        if p_f is not None:
            acc[:, sf] = p_f.wait().view(torch.int64)
        if p_max is not None:
            m = p_max.wait()
            if mx:
                acc[:, mx] = m[: R * len(mx)].reshape(R, len(mx))
            if mn:
                acc[:, mn] = torch.bitwise_not(m[R * len(mx):].reshape(R, len(mn)))
        hll = [p.wait() for p in p_hll]
        if si:
            acc[:, si] = s[:-world.size].reshape(R, len(si))
        return Partials("dense", acc, None, hll), s[-world.size:]  # one status word per rank

    return DenseMerge(finish_reduce)


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
    plan = merge_plan_for(world, part, disjoint_keys)
    if plan.kind == "oneshot-allgather":
        merged, sts = start_dense_merge(world, prog, part, status, plan.kind).wait()
        if local_error is not None or any(sts):
            raise_if_failed(sts, world.rank, local_error)
        return merged
    if plan.kind == "bucketed-allreduce":
        return _merge_dense_bucketed(world, prog, part, status, local_error)
    # sparse
    sp = part.compact()
    if disjoint_keys:
        return _gather_disjoint(world, sp, status, local_error)
    return _merge_sparse_shuffle(world, prog, sp, status, local_error)


def merge_plan_for(world: World, part: Partials, disjoint_keys: bool = False):
    """The cost model's merge choice (planner/cost.py plan_merge) for these partials: decided from
    the layout only, so every rank takes the same collective path."""
    from ..planner.cost import plan_merge

    return plan_merge(part.kind == "dense", dense_state_bytes(part) if part.kind == "dense" else 0, world.size,
                      disjoint_keys)


def dense_state_bytes(part: Partials) -> int:
    """Bytes one rank contributes to the one-shot gather: accumulators plus HLL registers (widened
    to int64 words in the gather buffer) -- the registers are usually the bulk (2048 per group per
    sketch at HLL_P=11)."""
    return (part.acc.numel() + sum(h.numel() for h in part.hll)) * 8


def _gather_disjoint(world: World, sp: Partials, status: int, local_error) -> Partials:
    """Groups are disjoint across ranks (grouped on the shard key): concatenate, no merge."""
    # keys + accumulators travel as one [n, 1 + nslots] int64 block: one length exchange (which also
    # carries the status word) + one gather
    kv = torch.cat([sp.keys.reshape(-1, 1).to(torch.int64), sp.acc], dim=1)
    kvs, sts = world.all_gather_varlen(kv, status=status)
    if local_error is not None or any(sts):
        raise_if_failed(sts, world.rank, local_error)
    hlls = [world.all_gather_varlen(h) for h in sp.hll]
    kv = torch.cat(kvs)
    return Partials("sparse", kv[:, 1:], kv[:, 0], [torch.cat(h) for h in hlls])


def shuffle_owner(keys: torch.Tensor, n: int) -> torch.Tensor:
    """Destination rank of each group key: a multiplicative hash, so the mixed-radix packed keys
    (whose low digits are the fastest key) spread evenly over the ranks."""
    h = (keys.to(torch.int64) * -7046029254386353131) >> 29  # 0x9E3779B97F4A7C15 as int64
    return torch.remainder(h, n)


def _merge_sparse_shuffle(world: World, prog, sp: Partials, status: int, local_error) -> Partials:
    """Hash-partitioned shuffle + local merge + gather of the merged groups."""
    n = world.size
    dest = shuffle_owner(sp.keys, n)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=n)
    kv = torch.cat([sp.keys.reshape(-1, 1).to(torch.int64), sp.acc], dim=1).index_select(0, order)
    recv, rc, sts = world.all_to_all_varlen(kv, counts, status=status)
    if local_error is not None or any(sts):
        raise_if_failed(sts, world.rank, local_error)
    hll = []
    for h in sp.hll:
        r, _ = world.all_to_all_varlen(h.index_select(0, order), counts)
        hll.append(r)
    mine = Partials("sparse", recv[:, 1:], recv[:, 0], hll)
    merged = merge_sparse([mine], prog.slots) if recv.shape[0] else mine
    # this rank owns a disjoint key range now: the final groups are a concatenation
    return _gather_disjoint(world, merged, STATUS_OK, None)
