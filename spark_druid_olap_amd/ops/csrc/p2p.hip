// Peer-to-peer one-shot merge of small dense partial aggregates over IPC-mapped device memory
// ("custom peer-to-peer one-shot reduce for sub-64 KB partials").
//
// The reference merges per-segment partials in one place -- the broker, or Spark's final aggregate
// after a shuffle (asd/PostAggregate.scala:97-103, sd/DruidRDD.scala:62-99).  Across GPUs the small
// dense states of typical OLAP queries (TPC-H Q1: 6 groups) are latency-bound: an RCCL all-gather, a
// torch reduction per slot and a host read of the status words cost several launches and a host
// round trip.  Here every rank owns a *mailbox* (uncached device memory, exported once with an IPC
// handle and opened by every peer), and ONE kernel per rank and merge:
//
//   1. waits until every peer is done with the epoch before (so the data slot it is about to
//      overwrite -- double-buffered by epoch parity -- is no longer read);
//   2. writes its packed partial -- accumulator words, HLL register bytes, its status word -- into
//      its own slot, then publishes the epoch in its header with a system-scope release;
//   3. waits (bounded by the SOFT timeout) for every peer's epoch and reduces the N mailboxes with
//      the per-slot operators (int sum, f64 sum, min, max; u8 max for HLL registers), reading peer
//      memory with system-scope loads (over xGMI across GPUs; through the same HBM when two ranks
//      share a card);
//   4. publishes its VERDICT for the epoch -- "I saw every peer's partial" or "I gave up" -- then
//      its done word, and waits (HARD timeout) for every peer's verdict;
//   5. publishes its FINAL word -- "aborted" when a hard wait expired -- and, if it did not abort,
//      waits (HARD timeout) for every peer's final word: an aborted epoch is a TIMEOUT everywhere.
//
// Every rank reads the same N verdict words, so every rank reaches the same outcome: all succeed,
// or -- when any rank's soft wait expired (a peer slow to arrive, or a coherence failure) -- all
// report P2P_STATUS_RETRY and the host re-runs the merge over RCCL (parallel/p2p.py).  Only a
// peer that never posts a verdict within the hard timeout (a dead process, or one later than the
// hard deadline -- every rank then sees the aborted final word) becomes a failed status word.
// No host synchronisation on the fast path: the caller's result copy carries the status words.  Every spin wait is bounded: no kernel that does not finish.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "p2p.h"

namespace sdo {

__device__ __forceinline__ uint64_t p2p_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t p2p_acquire(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void p2p_release(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// header words: [0] published epoch, [1] done epoch, [2 + (e & 1)] verdict of epoch e = (e << 1) | gave_up,
// [4 + (e & 1)] final word of epoch e = (e << 1) | aborted (posted after the hard wait for the done words)
__device__ __forceinline__ uint64_t* hdr(uint64_t base, int w) { return (uint64_t*)base + w; }

__device__ __forceinline__ uint64_t* slot_ptr(const P2PArgs& a, int r, uint64_t epoch) {
  return (uint64_t*)(a.mbox[r] + P2P_HEADER + (int64_t)(epoch & 1) * a.slot_bytes);
}

__device__ __forceinline__ unsigned all_mask(int n) { return n >= 32 ? 0xffffffffu : ((1u << n) - 1u); }

// Bounded wait until every peer's header word w reaches at least `want`; returns a bit mask of the
// ranks that did (all ranks' bits set = success).
__device__ unsigned wait_peers(const P2PArgs& a, int w, uint64_t want, int64_t ticks) {
  unsigned ok = 1u << a.rank;
  const uint64_t t0 = wall_clock64();
  const unsigned all = all_mask(a.nranks);
  while (ok != all) {
    for (int r = 0; r < a.nranks; ++r) {
      if (ok & (1u << r)) continue;
      if (p2p_acquire(hdr(a.mbox[r], w)) >= want) ok |= 1u << r;
    }
    if (ok == all) break;
    if ((int64_t)(wall_clock64() - t0) > ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  return ok;
}

// Bounded wait until every peer's final word of epoch e is posted (exactly epoch e: final words
// alternate by parity, and a word from epoch e - 2 must not count).
__device__ unsigned wait_fin(const P2PArgs& a, uint64_t e, int64_t ticks) {
  unsigned ok = 0;
  const uint64_t t0 = wall_clock64();
  const unsigned all = all_mask(a.nranks);
  while (ok != all) {
    for (int r = 0; r < a.nranks; ++r) {
      if (ok & (1u << r)) continue;
      if ((p2p_acquire(hdr(a.mbox[r], 4 + (int)(e & 1))) >> 1) == e) ok |= 1u << r;
    }
    if (ok == all) break;
    if ((int64_t)(wall_clock64() - t0) > ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  return ok;
}

// One workgroup of 1024 threads per merge (states are <= 64 KB: a few loads per thread).
__global__ void __launch_bounds__(1024) p2p_merge_kernel(P2PArgs a) {
  __shared__ unsigned s_prev, s_have, s_done, s_gaveup;
  const int tid = threadIdx.x;
  const uint64_t e = a.epoch;
  const unsigned all = all_mask(a.nranks);
  // 1. every peer finished epoch e - 1 (so nobody still reads the slot of parity e, last used in
  //    epoch e - 2, and every verdict word of parity e + 1 has been read)
  if (tid == 0) s_prev = e > 1 ? wait_peers(a, 1, e - 1, a.hard_ticks) : all;
  __syncthreads();
  // 2. publish this rank's partial (even after a failed wait: a late peer must still find data)
  uint64_t* mine = slot_ptr(a, a.rank, e);
  for (int64_t i = tid; i < a.nacc; i += blockDim.x) mine[i] = (uint64_t)a.acc_src[i];
  const uint64_t* hsrc = (const uint64_t*)a.hll_src;
  for (int64_t i = tid; i < a.nhll / 8; i += blockDim.x) mine[a.nacc + i] = hsrc[i];
  if (tid == 0) mine[a.nacc + a.nhll / 8] = (uint64_t)a.status;
  __threadfence_system();
  __syncthreads();
  if (tid == 0) p2p_release(hdr(a.mbox[a.rank], 0), e);
  // 3. every peer's partial of this epoch (soft bound)
  if (tid == 0) s_have = (s_prev == all) ? wait_peers(a, 0, e, a.soft_ticks) : (1u << a.rank);
  __syncthreads();
  const unsigned have = s_have;
  if (have == all) {
    // every rank folds the N partials in rank order 0..N-1 (its own in its place): f64 sums are
    // not associative, and ranks that summed in different orders could hold different bits for
    // one group -- and then take different HAVING / prune decisions on them
    for (int64_t i = tid; i < a.nacc; i += blockDim.x) {
      const int op = a.ops[i % a.nslots];
      int64_t v = 0;
      double f = 0.0;
      for (int r = 0; r < a.nranks; ++r) {
        const int64_t x = r == a.rank ? a.acc_src[i] : (int64_t)p2p_load(slot_ptr(a, r, e) + i);
        if (r == 0) {
          v = x;
          f = __longlong_as_double(x);
        } else if (op == 0) v += x;
        else if (op == 1) f += __longlong_as_double(x);
        else if (op == 2) v = x < v ? x : v;
        else v = x > v ? x : v;
      }
      a.acc_out[i] = op == 1 ? __double_as_longlong(f) : v;
    }
    uint64_t* hout = (uint64_t*)a.hll_out;
    for (int64_t i = tid; i < a.nhll / 8; i += blockDim.x) {
      uint64_t v = hsrc[i];
      for (int r = 0; r < a.nranks; ++r) {
        if (r == a.rank) continue;
        const uint64_t x = p2p_load(slot_ptr(a, r, e) + a.nacc + i);
        uint64_t m = 0;
#pragma unroll
        for (int b = 0; b < 64; b += 8) {
          const uint64_t p = (v >> b) & 0xff, q = (x >> b) & 0xff;
          m |= (p > q ? p : q) << b;
        }
        v = m;
      }
      hout[i] = v;
    }
  }
  // 4. verdict + done (after every read of the peers' slots), then every peer's verdict
  __threadfence_system();
  __syncthreads();
  if (tid == 0) {
    p2p_release(hdr(a.mbox[a.rank], 2 + (int)(e & 1)), (e << 1) | (have == all ? 0u : 1u));
    p2p_release(hdr(a.mbox[a.rank], 1), e);
    const unsigned done = wait_peers(a, 1, e, a.hard_ticks);
    unsigned gaveup = 0;
    for (int r = 0; r < a.nranks; ++r) {
      if (!(done & (1u << r))) continue;
      const uint64_t v = p2p_acquire(hdr(a.mbox[r], 2 + (int)(e & 1)));
      if ((v >> 1) != e || (v & 1)) gaveup |= 1u << r;
    }
    // 5. the final word: a rank whose hard wait expired (s_prev / done incomplete) ABORTS the
    //    epoch -- it reports TIMEOUT and disables its exchange.  A peer that arrives after that
    //    deadline (alive, only late: shard skew, a first-seen compile on one rank) would otherwise
    //    find the early rank's give-up verdict and done word and report RETRY, re-running over
    //    collectives that no longer pair up.  So every rank that completed its own waits also waits
    //    for every peer's final word, and an aborted (or missing) one is a TIMEOUT here too.
    const bool aborted = s_prev != all || done != all;
    p2p_release(hdr(a.mbox[a.rank], 4 + (int)(e & 1)), (e << 1) | (aborted ? 1u : 0u));
    unsigned fin_ok = all;
    if (!aborted) {
      const unsigned fin = wait_fin(a, e, a.hard_ticks);
      fin_ok = fin;
      for (int r = 0; r < a.nranks; ++r) {
        if (!(fin & (1u << r))) continue;
        if (p2p_acquire(hdr(a.mbox[r], 4 + (int)(e & 1))) & 1u) fin_ok &= ~(1u << r);
      }
    }
    s_done = done & fin_ok;
    s_gaveup = gaveup;
  }
  __syncthreads();
  if (tid < a.nranks) {
    const int r = tid;
    int64_t st;
    if (!(s_prev & (1u << r)) || !(s_done & (1u << r))) st = P2P_STATUS_TIMEOUT;
    else if (s_gaveup) st = P2P_STATUS_RETRY;  // every rank sees the same verdicts: all retry together
    else if (r == a.rank) st = a.status;
    else st = (int64_t)p2p_load(slot_ptr(a, r, e) + a.nacc + a.nhll / 8);
    a.status_out[r] = st;
  }
}

}  // namespace sdo
