// Radix-partitioned group-by for key spaces far beyond LDS (TPC-H Q18: 600M lines into
// 150M order groups, Q13: 149M orders into 15M customer counts).
//
// Random read-modify-write atomics on a table bigger than the L2 run at ~16-20 G updates/s on
// MI355X whether the table sits in HBM or in the 256 MB Infinity Cache (measured,
// planner/cost.py KEY_PASSES note): every update is its own cache-line transaction.  LDS atomics
// run two orders of magnitude faster, so the work is re-shaped until every group's updates meet in
// one workgroup's LDS:
//
//   producer  (the fused JIT scan, ops/jit.py M_PART, or part_keys_kernel over a key array)
//             count pass: per-block histogram of the top key bits (P1 buckets, LDS counters)
//             scatter pass: records (u32 key | value words) appended to the block's slice of each
//             bucket -- the block owns [base1[p] + inrow[p][b], ...), so one bucket's records from
//             one block land contiguously and every block keeps only P1 write fronts open (they
//             fit the XCD's L2, which merges the partial lines before they reach HBM)
//   split     (optional second level): K blocks per level-1 bucket re-partition it by the next
//             bits into P2 sub-buckets the same way (count, scan, scatter)
//   aggregate one workgroup per sub-bucket: a dense LDS table of the sub-bucket's 2^shift keys,
//             LDS atomics for every record, then ONE coalesced write of the table slice into the
//             group table -- every slot of the table is written, so no reset pass is needed
//
// Offsets are u32 (the host checks the record upper bound).  Counts of a [R][B] matrix are
// scanned per row (part_rowscan*) and the row totals once more (part_basescan), so a record's
// position is base[r] + inrow[r][b] + its LDS cursor.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "scan_desc.h"

namespace sdo {

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// exclusive block scan of one value per thread; NT threads (multiple of 64), lds >= NT/64 words
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t* lds, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan_u32(v);
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const uint32_t x = lds[i];
    pre += i < w ? x : 0u;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

// rows of <= 64 columns: one thread per row
__global__ void part_rowscan_small_kernel(uint32_t* __restrict__ c, int64_t R, int B, uint32_t* __restrict__ totals) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  uint32_t* row = c + r * B;
  uint32_t s = 0;
  for (int b = 0; b < B; ++b) {
    const uint32_t x = row[b];
    row[b] = s;
    s += x;
  }
  totals[r] = s;
}

// wider rows: one 256-thread block per row, each thread a contiguous run of the row
__global__ __launch_bounds__(256) void part_rowscan_kernel(uint32_t* __restrict__ c, int64_t R, int B,
                                                          uint32_t* __restrict__ totals) {
  __shared__ uint32_t lds[4];
  for (int64_t r = blockIdx.x; r < R; r += gridDim.x) {
    uint32_t* row = c + r * B;
    const int per = (B + 255) / 256;
    const int a = threadIdx.x * per, e = min(B, a + per);
    uint32_t s = 0;
    for (int b = a; b < e; ++b) s += row[b];
    uint32_t tot;
    uint32_t pre = block_excl_scan_u32<256>(s, lds, &tot);
    for (int b = a; b < e; ++b) {
      const uint32_t x = row[b];
      row[b] = pre;
      pre += x;
    }
    if (threadIdx.x == 0) totals[r] = tot;
  }
}

// base[0..R]: exclusive scan of the R row totals, base[R] = all records (one 1024-thread block)
__global__ __launch_bounds__(1024) void part_basescan_kernel(const uint32_t* __restrict__ totals, int64_t R,
                                                            uint32_t* __restrict__ base) {
  __shared__ uint32_t lds[16];
  const int64_t per = (R + 1023) / 1024;
  const int64_t a = threadIdx.x * per, e = a + per < R ? a + per : R;
  uint32_t s = 0;
  for (int64_t i = a; i < e; ++i) s += totals[i];
  uint32_t tot;
  uint32_t pre = block_excl_scan_u32<1024>(s, lds, &tot);
  for (int64_t i = a; i < e; ++i) {
    base[i] = pre;
    pre += totals[i];
  }
  if (threadIdx.x == 0) base[R] = tot;
}

// Level-1 producer over a plain key array (histograms: the Q13 customer counts): records are the
// u32 keys themselves (implicit count 1).  Same count / scatter protocol as the JIT scan producer.
__global__ __launch_bounds__(512) void part_keys_kernel(const int64_t* __restrict__ keys, int64_t n, int shift1,
                                                       int P1, uint32_t* __restrict__ counts1,
                                                       const uint32_t* __restrict__ base1, uint32_t* __restrict__ out,
                                                       int phase) {
  extern __shared__ uint32_t h[];
  const int B = gridDim.x;
  for (int q = threadIdx.x; q < P1; q += blockDim.x)
    h[q] = phase == 0 ? 0u : base1[q] + counts1[(int64_t)q * B + blockIdx.x];
  __syncthreads();
  const int64_t per = (n + B - 1) / B;
  const int64_t a = (int64_t)blockIdx.x * per, e = a + per < n ? a + per : n;
  for (int64_t i = a + threadIdx.x; i < e; i += blockDim.x) {
    const uint32_t k = (uint32_t)keys[i];
    const uint32_t p = k >> shift1;
    if (p >= (uint32_t)P1) continue;  // outside [0, P1 << shift1): never counted, never written
    if (phase == 0) {
      atomicAdd(&h[p], 1u);
    } else {
      const uint32_t pos = atomicAdd(&h[p], 1u);
      out[pos] = k;
    }
  }
  if (phase == 0) {
    __syncthreads();
    for (int q = threadIdx.x; q < P1; q += blockDim.x) counts1[(int64_t)q * B + blockIdx.x] = h[q];
  }
}

// Level 2: K blocks per level-1 bucket p split it into P2 sub-buckets by bits [shift2, shift2+log2 P2).
// counts2 is [P1 * P2][K] (row = p * P2 + q); phase 1 copies whole records (RW u32 words).
__global__ __launch_bounds__(512) void part_split_kernel(const uint32_t* __restrict__ in, int RW,
                                                        const uint32_t* __restrict__ base1, int K, int shift2, int P2,
                                                        uint32_t* __restrict__ counts2, const uint32_t* __restrict__ base2,
                                                        uint32_t* __restrict__ out, int phase) {
  extern __shared__ uint32_t h[];
  const int64_t p = blockIdx.x / K;
  const int k = blockIdx.x % K;
  const uint32_t lo = base1[p], hi = base1[p + 1];
  const uint64_t n = hi - lo;
  const uint32_t a = lo + (uint32_t)(n * k / K), e = lo + (uint32_t)(n * (k + 1) / K);
  const int64_t row0 = p * P2;
  for (int q = threadIdx.x; q < P2; q += blockDim.x)
    h[q] = phase == 0 ? 0u : base2[row0 + q] + counts2[(row0 + q) * K + k];
  __syncthreads();
  const uint32_t mask = (uint32_t)P2 - 1u;
  for (uint32_t i = a + threadIdx.x; i < e; i += blockDim.x) {
    const uint32_t* rec = in + (uint64_t)i * RW;
    const uint32_t key = rec[0];
    const uint32_t q = (key >> shift2) & mask;
    if (phase == 0) {
      atomicAdd(&h[q], 1u);
    } else {
      const uint32_t pos = atomicAdd(&h[q], 1u);
      uint32_t* o = out + (uint64_t)pos * RW;
      if (RW == 2) {
        *(uint2*)o = *(const uint2*)rec;
      } else {
        for (int w = 0; w < RW; ++w) o[w] = rec[w];
      }
    }
  }
  if (phase == 0) {
    __syncthreads();
    for (int q = threadIdx.x; q < P2; q += blockDim.x) counts2[(row0 + q) * K + k] = h[q];
  }
}

__device__ __forceinline__ void lds_fold(uint64_t* t, int op, int64_t v) {
  switch (op) {
    case S_SUM_I: atomicAdd((unsigned long long*)t, (unsigned long long)v); break;
    case S_SUM_F: unsafeAtomicAdd((double*)t, __longlong_as_double(v)); break;
    case S_MIN_I: atomicMin((long long*)t, (long long)v); break;
    default: atomicMax((long long*)t, (long long)v); break;
  }
}

// One workgroup per sub-bucket r: keys [r << shift, (r+1) << shift) of the dense group table.
// XCD-aware order: consecutive sub-buckets' tables are written by blocks on one XCD in turn (the
// hardware deals block ids round-robin over the 8 XCDs), which keeps each XCD's writes to
// neighbouring table lines.  The grid is a multiple of 8 blocks (>= nsub), so every r < nsub has
// exactly one block.
__global__ __launch_bounds__(512) void part_agg_kernel(const uint32_t* __restrict__ recs, int RW,
                                                      const uint32_t* __restrict__ base, int64_t nsub, int64_t G,
                                                      int shift, PartFields f, uint64_t* __restrict__ gacc) {
  extern __shared__ __attribute__((aligned(16))) uint64_t t[];
  const int64_t x = blockIdx.x;
  const int64_t per_xcd = gridDim.x / 8;
  const int64_t r = (x % 8) * per_xcd + x / 8;
  if (r >= nsub) return;
  const int64_t k0 = r << shift;
  if (k0 >= G) return;
  const int64_t nk = (G - k0) < ((int64_t)1 << shift) ? (G - k0) : ((int64_t)1 << shift);
  const int NS = f.nslots;
  for (int64_t i = threadIdx.x; i < nk * NS; i += blockDim.x) t[i] = (uint64_t)f.init[i % NS];
  __syncthreads();
  const uint32_t lo = base[r], hi = base[r + 1];
  for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t* rec = recs + (uint64_t)i * RW;
    const int64_t local = (int64_t)rec[0] - k0;
    if ((uint64_t)local >= (uint64_t)nk) continue;  // cannot happen for consistent buckets; never fault
    uint64_t* row = t + local * NS;
    int w = 1;
    for (int j = 0; j < f.nfields; ++j) {
      const int wd = f.width[j];
      int64_t v;
      if (wd == 0) v = 1;
      else if (wd == 1) v = (int64_t)(int32_t)rec[w];
      else v = (int64_t)((uint64_t)rec[w] | ((uint64_t)rec[w + 1] << 32));
      w += wd;
      const int s = f.slot[j];
      lds_fold(row + s, f.op[s], v);
    }
  }
  __syncthreads();
  uint64_t* g = gacc + k0 * NS;
  for (int64_t i = threadIdx.x; i < nk * NS; i += blockDim.x) g[i] = t[i];
}

}  // namespace sdo
