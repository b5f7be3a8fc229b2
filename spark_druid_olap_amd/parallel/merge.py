"""Cross-GPU merge of partial aggregates (the reference's broker merge / Spark shuffle +
final aggregate, ``asd/PostAggregate.scala:39-103``, re-designed for RCCL over xGMI).

The path is the cost model's (``planner/cost.py plan_merge``), priced from the state's layout:

* Small dense states (the common OLAP case: Q1 is 6 groups) are latency-bound: ONE
  ``all_gather_into_tensor`` of the packed state (accumulators as 8-byte words, HLL registers as
  the bytes they are, the status word) followed by a local per-slot reduction -- one collective
  instead of one per reduce-op.
* Large dense states use bandwidth-optimal ring ``all_reduce`` over at most three buckets (int
  sums + status word, float sums, max + bitwise-NOT(min)) plus ONE u8 MAX all-reduce of every HLL
  register block, with one host sync at the end -- mergeable sketches, which the reference could
  not merge across historicals, ``asd/PostAggregate.scala:62-70``.
* Sparse (hash) states are compacted per GPU and shuffled by key hash with one
  ``all_to_all_single`` of packed rows (key, accumulators, register bytes; the reference's
  hash-partitioned Exchange before Spark's final aggregate, ``asd/PostAggregate.scala:97-103``):
  each rank receives ~1/N of the partial rows and merges its key range locally.  When the
  datasource is partitioned on a grouping key the groups are already disjoint and there is no
  shuffle.  Either way every rank then holds a DISJOINT slice of the final groups
  (``Partials.scattered``): HAVING and top-k pruning run there, distributed, and only the
  survivors travel -- to rank 0 alone when the caller only needs the result on the root
  (``gather_groups``), the reference's final aggregate collecting in one place
  (``asd/PostAggregate.scala:97-103``).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from ..engine.partials import Partials, merge_sparse
from ..ops import desc as D
from . import p2p
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


def _u8(h: torch.Tensor) -> torch.Tensor:
    """HLL registers as bytes (rho <= 65): placeholders and host-built blocks may be wider ints."""
    return h if h.dtype == torch.uint8 else h.clamp(0, 255).to(torch.uint8)


def _merge_dense_bucketed(world: World, prog, part: Partials, status: int,
                          local_error: Optional[BaseException]) -> Partials:
    """Large dense state: at most three ring all-reduces (each per-xGMI-link bandwidth bound) plus
    one for all HLL register blocks, with ONE host synchronisation after all of them were enqueued.

    * int sums + the status word (sum of the ranks' statuses is non-zero iff one failed);
    * float64 sums;
    * int max slots and the bitwise NOT of int min slots (``min x == ~max ~x``, no overflow at
      INT64_MIN unlike negation), so min and max share one MAX collective;
    * every HLL register block as one u8 MAX.
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
    hll = [_u8(h) for h in part.hll]
    dev = part.acc.device
    if kind == "oneshot-allgather":
        R, ns = part.acc.shape
        # one byte buffer per rank: accumulators (8-byte words), register bytes, status word
        st = torch.full((1,), status, dtype=torch.int64, device=dev)
        pieces = [part.acc.contiguous().view(torch.uint8).reshape(-1)] + [h.reshape(-1) for h in hll] + \
            [st.view(torch.uint8)]
        pend = world.all_gather_tensor_async(torch.cat(pieces))  # [ranks, L] uint8
        shapes = [h.shape for h in hll]

        def finish_gather():
            g = pend.wait()
            na = R * ns * 8
            acc = _reduce_stacked(prog, g[:, :na].contiguous().view(torch.int64).reshape(world.size, R, ns))
            off = na
            regs = []
            for shp in shapes:
                n = shp.numel()
                regs.append(g[:, off: off + n].amax(dim=0).reshape(shp))
                off += n
            return Partials("dense", acc, None, regs), g[:, off:].contiguous().view(torch.int64).reshape(-1)

        return DenseMerge(finish_gather)
    acc = part.acc.clone()
    R = acc.shape[0]
    by_op = {op: [s for s, (o, _) in enumerate(prog.slots) if o == op]
             for op in (D.S_SUM_I, D.S_SUM_F, D.S_MIN_I, D.S_MAX_I)}
    si, sf, mn, mx = by_op[D.S_SUM_I], by_op[D.S_SUM_F], by_op[D.S_MIN_I], by_op[D.S_MAX_I]
    st = torch.zeros((world.size,), dtype=torch.int64, device=dev)
    st[world.rank] = status
    b_sum = torch.cat([acc[:, si].reshape(-1), st]) if si else st
    p_sum = world.all_reduce_async(b_sum, "sum")
    p_f = p_max = p_hll = None
    if sf:
        b_f = acc[:, sf].contiguous().view(torch.float64)
        p_f = world.all_reduce_async(b_f, "sum")
    if mn or mx:
        b_max = torch.cat([acc[:, mx].reshape(-1), torch.bitwise_not(acc[:, mn]).reshape(-1)])
        p_max = world.all_reduce_async(b_max, "max")
    if hll:
        p_hll = world.all_reduce_async(torch.cat([h.reshape(-1) for h in hll]), "max")  # u8 registers
    shapes = [h.shape for h in hll]

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
        regs = []
        if p_hll is not None:
            flat, off = p_hll.wait(), 0
            for shp in shapes:
                regs.append(flat[off: off + shp.numel()].reshape(shp))
                off += shp.numel()
        if si:
            acc[:, si] = s[:-world.size].reshape(R, len(si))
        return Partials("dense", acc, None, regs), s[-world.size:]  # one status word per rank

    return DenseMerge(finish_reduce)


def merge_partials(world: World, prog, part: Partials, disjoint_keys: bool = False,
                   local_error: Optional[BaseException] = None, finish: str = "all",
                   defer_status: bool = False) -> Partials:
    """Merge this rank's partials with every other rank's.  ``local_error`` set = this rank failed
    its scan and ``part`` is a layout-compatible placeholder: the status word travels in the
    merge's own collective and every rank raises (parallel/fault.py).

    ``finish`` says where sparse results end up: ``"all"`` -- every rank gets every final group;
    ``"root"`` -- rank 0 gets them, the other ranks an empty slice; ``"local"`` -- every rank keeps
    its disjoint slice (``scattered``) for distributed HAVING / top-k before ``gather_groups``.
    Dense states are merged whole on every rank either way."""
    if not world.distributed:
        if local_error is not None:
            raise local_error
        return part
    status = STATUS_FAILED if local_error is not None else STATUS_OK
    plan = merge_plan_for(world, part, disjoint_keys)
    if plan.kind in ("oneshot-allgather", "bucketed-allreduce") and p2p.fits(prog, part):
        # small dense state: the peer-to-peer one-shot merge (one kernel per rank over IPC-mapped
        # mailboxes, parallel/p2p.py) -- chosen from the layout and the group's agreed exchange
        ex = p2p.exchange_for(world)
        if ex is not None:
            merged = ex.merge(prog, part, status)
            if local_error is not None:
                # (after publishing: the peers read this rank's failed status) -- unless every rank
                # abandoned the epoch, in which case this rank retries over RCCL with its peers
                sts = merged.status_dev.tolist()
                from .fault import STATUS_P2P_RETRY, P2PRetry

                if any(sts) and all(int(v) in (STATUS_OK, STATUS_P2P_RETRY) for v in sts) and \
                        STATUS_P2P_RETRY in [int(v) for v in sts]:
                    raise P2PRetry("peer-to-peer merge epoch abandoned by every rank: retrying over RCCL")
                raise local_error
            if not defer_status:
                p2p.check_status(merged)
            return merged
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
        if finish == "local":
            # no collective yet: the status word rides with the gather that follows (gather_groups)
            return Partials("sparse", sp.acc, sp.keys, sp.hll, scattered=True, status=status)
        return gather_groups(world, sp, finish == "root", status, local_error)
    return _merge_sparse_shuffle(world, prog, sp, status, local_error, finish)


def merge_plan_for(world: World, part: Partials, disjoint_keys: bool = False):
    """The cost model's merge choice (planner/cost.py plan_merge) for these partials: decided from
    the layout only, so every rank takes the same collective path."""
    from ..planner.cost import plan_merge

    # (a forced one-rank group -- the RCCL smoke -- takes the paths a pair of ranks would)
    n = world.size if world.size > 1 or not world.distributed else 2
    return plan_merge(part.kind == "dense", dense_state_bytes(part) if part.kind == "dense" else 0, n,
                      disjoint_keys)


def dense_state_bytes(part: Partials) -> int:
    """Bytes one rank contributes to the one-shot gather: 8-byte accumulator words plus the HLL
    register bytes (2048 per group per sketch at HLL_P=11 -- usually the bulk)."""
    return part.acc.numel() * 8 + sum(h.numel() for h in part.hll)


# ---------------------------------------------------------------------------------------------
# packed rows: one uint8 block [n, 8 * (1 + nslots) + nhll * m] per rank, so a shuffle or a gather
# is ONE collective whatever the number of sketches
def pack_rows(sp: Partials) -> torch.Tensor:
    n = int(sp.acc.shape[0])
    kv = torch.cat([sp.keys.reshape(-1, 1).to(torch.int64), sp.acc], dim=1).contiguous()
    parts = [kv.view(torch.uint8).reshape(n, 8 * kv.shape[1])] + [_u8(h).reshape(n, h.shape[1]) for h in sp.hll]
    return torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]


def unpack_rows(rows: torch.Tensor, nslots: int, hll_widths: List[int], scattered: bool = False) -> Partials:
    w = 8 * (1 + nslots)
    kv = rows[:, :w].contiguous().view(torch.int64).reshape(rows.shape[0], 1 + nslots)
    hll, off = [], w
    for m in hll_widths:
        hll.append(rows[:, off: off + m].contiguous())
        off += m
    # (contiguous: the native decode and top-k kernels take raw pointers -- a strided key column
    # read as contiguous mixed the count slot into the key ids, tools/rccl_smoke.py at SF1)
    return Partials("sparse", kv[:, 1:].contiguous(), kv[:, 0].contiguous(), hll, scattered=scattered)


def gather_groups(world: World, sp: Partials, root_only: bool, status: int = STATUS_OK,
                  local_error: Optional[BaseException] = None) -> Partials:
    """Concatenate every rank's disjoint groups: at rank 0 only (``root_only``: one all-to-all in
    which every rank sends its rows to the root and the others receive nothing -- the root takes in
    exactly the result, each peer over its own xGMI link), or on every rank (all-gather)."""
    ns = sp.acc.shape[1]
    widths = [int(h.shape[1]) for h in sp.hll]
    rows = pack_rows(sp)
    if root_only:
        got, sts = world.gather_varlen(rows, root=0, status=status)
    else:
        got, sts = world.all_gather_varlen(rows, status=status)
    if local_error is not None or any(sts):
        raise_if_failed(sts, world.rank, local_error)
    if not got:
        got = [rows[:0]]
    return unpack_rows(torch.cat(got) if len(got) > 1 else got[0], ns, widths)


def shuffle_owner(keys: torch.Tensor, n: int) -> torch.Tensor:
    """Destination rank of each group key: a multiplicative hash, so the mixed-radix packed keys
    (whose low digits are the fastest key) spread evenly over the ranks."""
    h = (keys.to(torch.int64) * -7046029254386353131) >> 29  # 0x9E3779B97F4A7C15 as int64
    return torch.remainder(h, n)


def _merge_sparse_shuffle(world: World, prog, sp: Partials, status: int, local_error,
                          finish: str = "all") -> Partials:
    """Hash-partitioned shuffle (one all-to-all of packed rows) + local merge; the result is this
    rank's disjoint key range (``finish="local"``) or gathered (``gather_groups``)."""
    n = world.size
    dest = shuffle_owner(sp.keys, n)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=n)
    rows = pack_rows(sp).index_select(0, order)
    recv, rc, sts = world.all_to_all_varlen(rows, counts, status=status)
    if local_error is not None or any(sts):
        raise_if_failed(sts, world.rank, local_error)
    mine = unpack_rows(recv, sp.acc.shape[1], [int(h.shape[1]) for h in sp.hll])
    merged = merge_sparse([mine], prog.slots) if recv.shape[0] else mine
    if finish == "local":
        return Partials("sparse", merged.acc, merged.keys, merged.hll, scattered=True)
    # this rank owns a disjoint key range now: the final groups are a concatenation
    return gather_groups(world, merged, finish == "root")
