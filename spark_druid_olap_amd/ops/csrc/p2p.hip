// Peer-to-peer one-shot merge of small dense partial aggregates over IPC-mapped device memory
// ("custom peer-to-peer one-shot reduce for sub-64 KB partials").
//
// The reference merges per-segment partials in one place -- the broker, or Spark's final aggregate
// after a shuffle (asd/PostAggregate.scala:97-103, sd/DruidRDD.scala:62-99).  Across GPUs the small
// dense states of typical OLAP queries (TPC-H Q1: 6 groups) are latency-bound: an RCCL all-gather, a
// torch reduction per slot and a host read of the status words cost several launches and a host
// round trip.  Here every rank owns a *mailbox* (one hipMalloc, exported once with hipIpcGetMemHandle
// and opened by every peer), and ONE kernel per rank and merge:
//
//   1. waits until every peer is done reading the mailbox slot it is about to overwrite
//      (double-buffered by epoch parity: slot e % 2 was last read in epoch e - 2);
//   2. writes its packed partial -- accumulator words, HLL register bytes, its status word -- into
//      its own slot, then publishes the epoch in its header with a system-scope release;
//   3. waits for every peer's epoch (system-scope acquire) and reduces the N mailboxes with the
//      per-slot operators (int sum, f64 sum, min, max; u8 max for HLL registers), reading peer
//      memory with system-scope loads (over xGMI across GPUs; through the shared memory side of
//      the same device when two ranks share a card);
//   4. writes every rank's status word next to the merged result and marks itself done.
//
// No host synchronisation: the caller's result copy carries the status words.  Every spin wait is
// bounded (wall clock, P2P_TIMEOUT_TICKS): a missing peer turns into a failed status word, never a
// kernel that does not finish.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdo {

constexpr int P2P_MAX_RANKS = 8;
constexpr int P2P_MAX_SLOTS = 64;
constexpr int64_t P2P_HEADER = 256;  // bytes: flag word, done word, error word, padding
constexpr int64_t P2P_STATUS_TIMEOUT = 3;  // status word of a rank that did not arrive in time

struct P2PArgs {
  uint64_t mbox[P2P_MAX_RANKS];  // every rank's mailbox base, as mapped in this process (own included)
  int nranks;
  int rank;
  uint64_t epoch;                // >= 1, strictly increasing per exchange
  int64_t slot_bytes;            // capacity of one data slot
  int64_t nacc;                  // accumulator words (rows x nslots)
  int64_t nhll;                  // HLL register bytes (multiple of 8)
  int nslots;
  int ops[P2P_MAX_SLOTS];        // SlotOp per slot
  const int64_t* acc_src;
  const uint8_t* hll_src;
  int64_t status;
  int64_t* acc_out;
  uint8_t* hll_out;
  int64_t* status_out;           // [nranks]
  int64_t timeout_ticks;         // wall_clock64 ticks (100 MHz)
};

__device__ __forceinline__ uint64_t p2p_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t p2p_acquire(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void p2p_release(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// header words: [0] published epoch, [1] done epoch
__device__ __forceinline__ uint64_t* hdr(uint64_t base, int w) { return (uint64_t*)base + w; }

__device__ __forceinline__ uint64_t* slot_ptr(const P2PArgs& a, int r, uint64_t epoch) {
  return (uint64_t*)(a.mbox[r] + P2P_HEADER + (int64_t)(epoch & 1) * a.slot_bytes);
}

// Bounded wait until every peer's header word w reaches at least `want`; returns a bit mask of the
// ranks that did (all ranks' bits set = success).
__device__ unsigned wait_peers(const P2PArgs& a, int w, uint64_t want) {
  unsigned ok = 1u << a.rank;
  const uint64_t t0 = wall_clock64();
  const unsigned all = (a.nranks >= 32) ? 0xffffffffu : ((1u << a.nranks) - 1u);
  while (ok != all) {
    for (int r = 0; r < a.nranks; ++r) {
      if (ok & (1u << r)) continue;
      if (p2p_acquire(hdr(a.mbox[r], w)) >= want) ok |= 1u << r;
    }
    if (ok == all) break;
    if ((int64_t)(wall_clock64() - t0) > a.timeout_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  return ok;
}

// One workgroup of 1024 threads per merge (states are <= 64 KB: a few loads per thread).
__global__ void __launch_bounds__(1024) p2p_merge_kernel(P2PArgs a) {
  __shared__ unsigned s_ok;
  const int tid = threadIdx.x;
  const uint64_t e = a.epoch;
  // 1. the slot of epoch e was last read in epoch e - 2: every peer must be done with it
  if (tid == 0) s_ok = e > 2 ? wait_peers(a, 1, e - 2) : ((1u << a.nranks) - 1u);
  __syncthreads();
  // 2. publish this rank's partial (even after a timeout: a late peer must still find data)
  uint64_t* mine = slot_ptr(a, a.rank, e);
  for (int64_t i = tid; i < a.nacc; i += blockDim.x) mine[i] = (uint64_t)a.acc_src[i];
  const uint64_t* hsrc = (const uint64_t*)a.hll_src;
  for (int64_t i = tid; i < a.nhll / 8; i += blockDim.x) mine[a.nacc + i] = hsrc[i];
  if (tid == 0) mine[a.nacc + a.nhll / 8] = (uint64_t)a.status;
  __threadfence_system();
  __syncthreads();
  if (tid == 0) p2p_release(hdr(a.mbox[a.rank], 0), e);
  // 3. every peer's partial of this epoch
  __shared__ unsigned s_have;
  if (tid == 0) s_have = wait_peers(a, 0, e);
  __syncthreads();
  const unsigned have = s_have;
  for (int64_t i = tid; i < a.nacc; i += blockDim.x) {
    const int op = a.ops[i % a.nslots];
    int64_t v = a.acc_src[i];
    double f = __longlong_as_double(v);
    for (int r = 0; r < a.nranks; ++r) {
      if (r == a.rank || !(have & (1u << r))) continue;
      const int64_t x = (int64_t)p2p_load(slot_ptr(a, r, e) + i);
      if (op == 0) v += x;
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
      if (r == a.rank || !(have & (1u << r))) continue;
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
  if (tid < a.nranks) {
    const int r = tid;
    int64_t st;
    if (r == a.rank) st = a.status;
    else if (!(have & (1u << r)) || !(s_ok & (1u << r))) st = P2P_STATUS_TIMEOUT;
    else st = (int64_t)p2p_load(slot_ptr(a, r, e) + a.nacc + a.nhll / 8);
    a.status_out[r] = st;
  }
  // 4. done reading every peer's slot of epoch e
  __threadfence_system();
  __syncthreads();
  if (tid == 0) p2p_release(hdr(a.mbox[a.rank], 1), e);
}

}  // namespace sdo
