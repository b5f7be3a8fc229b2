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

// LDS bucket counters under clustered keys.  Producer chunk regions hold rows in time order and,
// within a day, in key order, so a wave's 64 consecutive records usually share ONE bucket: a plain
// per-lane atomic then serializes 64 ways on one LDS address (TPC-H Q18's level-1 count: 2.0 ms,
// against 0.84 ms on uniform keys, tools/part_probe.py).  When every active lane of the wave has
// the same bucket, one lane adds the lane count instead; otherwise each lane adds its own 1.  (The
// check is two ballots and a readlane: free next to the atomics it saves, ~nothing when keys are
// uniform.)
__device__ __forceinline__ void lds_count_add(uint32_t* h, uint32_t q, bool act, bool clustered) {
  if (!clustered) {  // (hashed keys: uniform buckets, the check would only cost)
    if (act) atomicAdd(&h[q], 1u);
    return;
  }
  const uint64_t am = __ballot(act);
  if (!am) return;
  const int leader = __builtin_ctzll(am);
  const uint32_t q0 = (uint32_t)__builtin_amdgcn_readlane((int)q, leader);
  if (__ballot(act && q == q0) == am) {
    if ((int)(threadIdx.x & 63) == leader) atomicAdd(&h[q0], (uint32_t)__popcll(am));
  } else if (act) {
    atomicAdd(&h[q], 1u);
  }
}

// Rank form, split in two so a tile's PU adds issue back to back and are waited for once: step 1
// issues the add (one lane for a uniform wave, else every active lane) and returns the uniform-wave
// mask (0: plain); step 2 turns the returned value into the lane's rank.
__device__ __forceinline__ uint64_t lds_rank_issue(uint32_t* h, uint32_t q, bool act, uint32_t& raw, bool clustered) {
  raw = 0u;
  if (!clustered) {
    if (act) raw = atomicAdd(&h[q], 1u);
    return 0ull;
  }
  const uint64_t am = __ballot(act);
  if (!am) return 0ull;
  const int leader = __builtin_ctzll(am);
  const uint32_t q0 = (uint32_t)__builtin_amdgcn_readlane((int)q, leader);
  const bool fast = __ballot(act && q == q0) == am;
  if (act && (!fast || (int)(threadIdx.x & 63) == leader)) raw = atomicAdd(&h[q], fast ? (uint32_t)__popcll(am) : 1u);
  return fast ? am : 0ull;
}

__device__ __forceinline__ uint32_t lds_rank_finish(uint64_t fm, uint32_t raw) {
  if (!fm) return raw;
  const int lane = threadIdx.x & 63;
  const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)raw, __builtin_ctzll(fm));
  return base + (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
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
  extern __shared__ __attribute__((aligned(16))) uint32_t h[];
  const int B = gridDim.x;
  for (int q = threadIdx.x; q < P1; q += blockDim.x)
    h[q] = phase == 0 ? 0u : base1[q] + counts1[(int64_t)q * B + blockIdx.x];
  __syncthreads();
  const int64_t per = (n + B - 1) / B;
  const int64_t a = (int64_t)blockIdx.x * per, e = a + per < n ? a + per : n;
  for (int64_t i0 = a; i0 < e; i0 += blockDim.x) {  // (block-uniform trip count: the bucket adds ballot)
    const int64_t i = i0 + threadIdx.x;
    const uint32_t k = i < e ? (uint32_t)keys[i] : 0u;
    const uint32_t p = k >> shift1;
    const bool act = i < e && p < (uint32_t)P1;  // outside [0, P1 << shift1): never counted, never written
    if (phase == 0) {
      lds_count_add(h, p, act, false);
    } else {
      uint32_t raw;
      const uint64_t fm = lds_rank_issue(h, p, act, raw, false);
      const uint32_t pos = lds_rank_finish(fm, raw);
      if (act) out[pos] = k;
    }
  }
  if (phase == 0) {
    __syncthreads();
    for (int q = threadIdx.x; q < P1; q += blockDim.x) counts1[(int64_t)q * B + blockIdx.x] = h[q];
  }
}

// Split: records of input segments are partitioned into P2 buckets by bits [shift2, shift2+log2 P2)
// of the key.  Input groups: group g owns segments [g*spg, (g+1)*spg), each [seg_lo[s], seg_hi[s]);
// its output buckets are rows g*P2 .. g*P2+P2-1 (counts2 is [groups * P2][K]).  K blocks per group:
// with one segment per group (a level-1 bucket) block k takes the k-th slice of its records, with
// many (the producer's chunk regions) the k-th slice of its segments.
//
// phase 0 counts (LDS histogram).  phase 1 scatters through an LDS tile sort: a tile of 512 x PU
// records is ranked per bucket (LDS atomics), reordered in LDS by bucket, and each thread then
// writes consecutive sorted records -- a bucket's run of the tile lands as one contiguous,
// coalesced store sequence instead of 64 scattered lines per wave instruction.  PU shrinks as
// records widen (the tile stays ~32 KB of LDS).

// Record addressing of a split pass: records [lo, lo + n) of one segment (Contig), or the
// concatenation of up to 512 small segments whose start offsets and exclusive length prefix sit in
// LDS (Packed: a selective producer leaves a few dozen records in each 4096-row chunk region, and a
// tile per region paid the tile's barriers for almost nothing -- TPC-H Q2's 8M-row inner level over
// 146K regions).  v -> record index.
// find / walk / at: a thread's records of one tile (v = t0 + tid + u * 512, increasing in u) look
// their region up once -- a binary search for the first, a short forward walk for the rest -- and
// keep the region index for the record copy, instead of a full search per record and use.
struct Contig {
  uint32_t lo;
  __device__ __forceinline__ uint64_t operator()(uint32_t v) const { return (uint64_t)lo + v; }
  __device__ __forceinline__ int find(uint32_t) const { return 0; }
  __device__ __forceinline__ int walk(uint32_t, int a) const { return a; }
  __device__ __forceinline__ uint64_t at(uint32_t v, int) const { return (uint64_t)lo + v; }
};
struct Packed {
  const uint32_t* slo;   // [ns] region starts (LDS)
  const uint32_t* spre;  // [ns + 1] exclusive prefix of the region lengths (LDS)
  int ns;
  __device__ __forceinline__ int find(uint32_t v) const {
    int a = 0, b = ns - 1;  // the last region whose prefix <= v
    while (a < b) {
      const int mid = (a + b + 1) >> 1;
      if (spre[mid] <= v) a = mid;
      else b = mid - 1;
    }
    return a;
  }
  __device__ __forceinline__ int walk(uint32_t v, int a) const {
    while (a + 1 < ns && spre[a + 1] <= v) ++a;  // (the same "last region whose prefix <= v")
    return a;
  }
  __device__ __forceinline__ uint64_t at(uint32_t v, int a) const { return (uint64_t)slo[a] + (v - spre[a]); }
  __device__ __forceinline__ uint64_t operator()(uint32_t v) const { return at(v, find(v)); }
};

template <bool CL>
__device__ __forceinline__ void split_range_count(const uint32_t* __restrict__ in, int RW, uint32_t lo, uint32_t hi,
                                                  int shift2, uint32_t mask, uint32_t* h) {
  if (RW == 2) {
    // two records per 16-byte load, 8 records per thread in flight
    uint32_t i = lo;
    if (i < hi && (i & 1u)) {  // align to a record pair
      if (threadIdx.x == 0) atomicAdd(&h[(in[(uint64_t)i * 2] >> shift2) & mask], 1u);
      ++i;
    }
    if (i >= hi) return;  // (empty, or the single odd record above)
    const uint32_t npair = (hi - i) / 2;
    const uint4* pr = (const uint4*)(in + (uint64_t)i * 2);
    for (uint32_t b0 = 0; b0 < npair; b0 += blockDim.x * 4) {  // (block-uniform trip count)
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t j = b0 + threadIdx.x + u * blockDim.x;
        if (j < npair) v[u] = pr[j];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool act = b0 + threadIdx.x + u * blockDim.x < npair;
        // (records 2j and 2j+1 of a lane are neighbours: each half combines across the wave)
        lds_count_add(h, act ? (v[u].x >> shift2) & mask : 0u, act, CL);
        lds_count_add(h, act ? (v[u].z >> shift2) & mask : 0u, act, CL);
      }
    }
    if (((hi - i) & 1u) && threadIdx.x == 0) atomicAdd(&h[(in[(uint64_t)(hi - 1) * 2] >> shift2) & mask], 1u);
    return;
  }
  for (uint32_t b0 = lo; b0 < hi; b0 += blockDim.x * 4) {  // (block-uniform trip count)
    uint32_t key[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t i = b0 + threadIdx.x + u * blockDim.x;
      key[u] = i < hi ? in[(uint64_t)i * RW] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool act = b0 + threadIdx.x + u * blockDim.x < hi;
      lds_count_add(h, (key[u] >> shift2) & mask, act, CL);
    }
  }
}

template <bool CL, class Map>
__device__ __forceinline__ void split_map_count(const uint32_t* __restrict__ in, int RW, Map map, uint32_t n, int shift2,
                                                uint32_t mask, uint32_t* h) {
  for (uint32_t b0 = 0; b0 < n; b0 += blockDim.x * 4) {  // (block-uniform trip count)
    uint32_t key[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t v = b0 + threadIdx.x + u * blockDim.x;
      key[u] = v < n ? in[map(v) * RW] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool act = b0 + threadIdx.x + u * blockDim.x < n;
      lds_count_add(h, (key[u] >> shift2) & mask, act, CL);
    }
  }
}

// pk_w (> 0, level 1 only): record word pk_w -- a small non-negative value -- leaves packed into the
// key word above bit shift2 (the key bits the bucket and sub-bucket imply), the other words after
// it: every later pass (level-2 split, aggregation) moves RW - 1 words per record.
template <int PU, bool CL, class Map>
__device__ __forceinline__ void split_range_scatter(const uint32_t* __restrict__ in, int RW, int RS, Map map, uint32_t n,
                                                    int shift2, uint32_t P2, uint32_t* cur, uint32_t* hist,
                                                    uint32_t* tstart, uint32_t* tile, uint32_t* scan_lds,
                                                    uint32_t* __restrict__ out, int pk_w = 0) {
  const uint32_t mask = P2 - 1u;
  constexpr uint32_t TILE = 512u * PU;
  for (uint32_t t0 = 0; t0 < n; t0 += TILE) {
    const uint32_t tn = n - t0 < TILE ? n - t0 : TILE;
    for (uint32_t q = threadIdx.x; q < P2; q += blockDim.x) hist[q] = 0u;
    __syncthreads();
    uint32_t q_[PU], r_[PU];
    int ra_[PU];
    uint2 v2[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const uint32_t j = threadIdx.x + u * blockDim.x;
      ra_[u] = 0;
      if (j < tn) {
        ra_[u] = u == 0 ? map.find(t0 + j) : map.walk(t0 + j, ra_[u - 1]);
        const uint64_t i = map.at(t0 + j, ra_[u]);
        if (RW == 2) {
          v2[u] = *(const uint2*)(in + i * 2);
        } else {
          v2[u].x = in[i * RW];
          v2[u].y = 0u;
        }
      }
    }
    uint64_t fm_[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const uint32_t j = threadIdx.x + u * blockDim.x;
      const bool act = j < tn;
      q_[u] = act ? (v2[u].x >> shift2) & mask : 0u;
      fm_[u] = lds_rank_issue(hist, q_[u], act, r_[u], CL);
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) r_[u] = lds_rank_finish(fm_[u], r_[u]);
    __syncthreads();
    // exclusive scan of the tile histogram -> bucket starts inside the tile; a thread's `per`
    // consecutive counters move as one 8- / 16-byte LDS access (consecutive lanes, consecutive
    // slots: no bank conflicts -- a scalar walk at stride `per` is a per-way conflict)
    const uint32_t per = (P2 + blockDim.x - 1) / blockDim.x;  // 1, 2, 4 or 8 (P2 a power of two)
    const uint32_t qa = threadIdx.x * per;
    uint32_t hv[8];
    if (qa < P2) {
      if (per == 8) {
        const uint4 a = ((const uint4*)hist)[2 * threadIdx.x], b = ((const uint4*)hist)[2 * threadIdx.x + 1];
        hv[0] = a.x; hv[1] = a.y; hv[2] = a.z; hv[3] = a.w; hv[4] = b.x; hv[5] = b.y; hv[6] = b.z; hv[7] = b.w;
      } else if (per == 4) {
        const uint4 a = ((const uint4*)hist)[threadIdx.x];
        hv[0] = a.x; hv[1] = a.y; hv[2] = a.z; hv[3] = a.w;
      } else if (per == 2) {
        const uint2 a = ((const uint2*)hist)[threadIdx.x];
        hv[0] = a.x; hv[1] = a.y;
      } else {
        hv[0] = hist[qa];
      }
    }
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if ((uint32_t)i < per && qa < P2) sum += hv[i];
    uint32_t tot;
    uint32_t pre = block_excl_scan_u32<512>(sum, scan_lds, &tot);
    if (qa < P2) {
      uint32_t ts[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ts[i] = pre;
        if ((uint32_t)i < per) pre += hv[i];
      }
      if (per == 8) {
        ((uint4*)tstart)[2 * threadIdx.x] = make_uint4(ts[0], ts[1], ts[2], ts[3]);
        ((uint4*)tstart)[2 * threadIdx.x + 1] = make_uint4(ts[4], ts[5], ts[6], ts[7]);
      } else if (per == 4) {
        ((uint4*)tstart)[threadIdx.x] = make_uint4(ts[0], ts[1], ts[2], ts[3]);
      } else if (per == 2) {
        ((uint2*)tstart)[threadIdx.x] = make_uint2(ts[0], ts[1]);
      } else {
        tstart[qa] = ts[0];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const uint32_t j = threadIdx.x + u * blockDim.x;
      if (j < tn) {
        const uint32_t d = tstart[q_[u]] + r_[u];
        if (RW == 2) {
          ((uint2*)tile)[d] = v2[u];
        } else if (RW == 1) {
          tile[d] = v2[u].x;  // (the key is the record)
        } else {
          const uint32_t* rec = in + map.at(t0 + j, ra_[u]) * RW;
          for (int w = 0; w < RW; ++w) tile[(uint64_t)d * RS + w] = rec[w];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const uint32_t j = threadIdx.x + u * blockDim.x;
      if (j < tn) {
        const uint32_t key = tile[(uint64_t)j * RS];
        const uint32_t q = (key >> shift2) & mask;
        const uint64_t pos = (uint64_t)cur[q] + (j - tstart[q]);
        if (pk_w > 0) {
          const uint32_t lo = key & ((1u << shift2) - 1u);
          const uint32_t w0 = lo | (tile[(uint64_t)j * RS + pk_w] << shift2);
          if (RW == 2) {
            out[pos] = w0;
          } else {
            const int RO = RW - 1;
            out[pos * RO] = w0;
            int o = 1;
            for (int w = 1; w < RW; ++w)
              if (w != pk_w) out[pos * RO + o++] = tile[(uint64_t)j * RS + w];
          }
        } else if (RW == 2) {
          *(uint2*)(out + pos * 2) = ((const uint2*)tile)[j];
        } else {
          for (int w = 0; w < RW; ++w) out[pos * RW + w] = tile[(uint64_t)j * RS + w];
        }
      }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < P2; q += blockDim.x) cur[q] += hist[q];
    __syncthreads();
  }
}

// dynamic LDS: phase 0: P2 words; phase 1: 3 * P2 + 512 * PU * RS words (RS: the tile's record
// stride -- RW, or RW + 1 for even widths >= 4 so a wave's consecutive records start on distinct banks)
// CL: the keys come in runs (dense keys of producer chunk regions and their level-1 buckets; not
// hashes): same-bucket waves add once (lds_count_add) -- a compile-time choice, so the hashed
// instantiation carries none of its code
template <int PU, bool CL>
__global__ __launch_bounds__(512) void part_split_kernel(const uint32_t* __restrict__ in, int RW, int RS,
                                                        const uint32_t* __restrict__ seg_lo,
                                                        const uint32_t* __restrict__ seg_hi, int spg, int K, int shift2,
                                                        int P2, uint32_t* __restrict__ counts2,
                                                        const uint32_t* __restrict__ base2, uint32_t* __restrict__ out,
                                                        int phase, int pk_w) {
  extern __shared__ __attribute__((aligned(16))) uint32_t h[];
  __shared__ uint32_t scan_lds[8];
  const int64_t g = blockIdx.x / K;
  const int k = blockIdx.x % K;
  const int64_t row0 = g * P2;
  for (int q = threadIdx.x; q < P2; q += blockDim.x)
    h[q] = phase == 0 ? 0u : base2[row0 + q] + counts2[(row0 + q) * K + k];
  __syncthreads();
  const uint32_t mask = (uint32_t)P2 - 1u;
  uint32_t* hist = h + P2;
  uint32_t* tstart = h + 2 * P2;
  uint32_t* tile = h + 3 * P2;
  if (spg == 1) {
    const uint32_t lo = seg_lo[g], hi = seg_hi[g];
    const uint64_t n = hi > lo ? hi - lo : 0;
    const uint32_t a = lo + (uint32_t)(n * k / K), e = lo + (uint32_t)(n * (k + 1) / K);
    if (phase == 0) split_range_count<CL>(in, RW, a, e, shift2, mask, h);
    else split_range_scatter<PU, CL>(in, RW, RS, Contig{a}, e - a, shift2, (uint32_t)P2, h, hist, tstart, tile, scan_lds,
                                     out, pk_w);
  } else {
    // the block's regions in groups of up to 512: lengths prefix-summed in LDS; groups of small
    // regions (< 1024 records on average) run as packed tiles, large ones region by region
    __shared__ uint32_t slo[512];
    __shared__ uint32_t spre[513];
    const int64_t s0 = g * spg + (int64_t)spg * k / K, s1 = g * spg + (int64_t)spg * (k + 1) / K;
    for (int64_t sb = s0; sb < s1; sb += 512) {
      const int ns = (int)(s1 - sb < 512 ? s1 - sb : 512);
      uint32_t len = 0, lo0 = 0;
      if ((int)threadIdx.x < ns) {
        lo0 = seg_lo[sb + threadIdx.x];
        const uint32_t hi0 = seg_hi[sb + threadIdx.x];
        len = hi0 > lo0 ? hi0 - lo0 : 0u;
      }
      uint32_t tot;
      const uint32_t pre = block_excl_scan_u32<512>(len, scan_lds, &tot);
      if ((int)threadIdx.x < ns) {
        slo[threadIdx.x] = lo0;
        spre[threadIdx.x] = pre;
      }
      if (threadIdx.x == 0) spre[ns] = tot;
      __syncthreads();
      // packed when the regions average under ~80% of a tile (a region-by-region pass runs one
      // part-empty tile per region: a date-filtered producer fills its 4096-row regions ~57%)
      // (the count pass keeps the round-5 rule: its per-record cost is the search itself)
      if (phase == 0 ? tot < 1024u * (uint32_t)ns : tot * 5u < 4u * 512u * (uint32_t)PU * (uint32_t)ns) {
        const Packed pm{slo, spre, ns};
        if (phase == 0) split_map_count<CL>(in, RW, pm, tot, shift2, mask, h);
        else split_range_scatter<PU, CL>(in, RW, RS, pm, tot, shift2, (uint32_t)P2, h, hist, tstart, tile, scan_lds, out,
                                         pk_w);
      } else {
        for (int si = 0; si < ns; ++si) {
          const uint32_t lo = slo[si], n = spre[si + 1] - spre[si];
          if (n == 0) continue;  // (uniform across the block: every thread reads the same LDS entry)
          if (phase == 0) split_range_count<CL>(in, RW, lo, lo + n, shift2, mask, h);
          else split_range_scatter<PU, CL>(in, RW, RS, Contig{lo}, n, shift2, (uint32_t)P2, h, hist, tstart, tile,
                                           scan_lds, out, pk_w);
        }
      }
      __syncthreads();  // (slo / spre are rewritten for the next group)
    }
  }
  if (phase == 0) {
    __syncthreads();
    for (int q = threadIdx.x; q < P2; q += blockDim.x) counts2[(row0 + q) * K + k] = h[q];
  }
}

template __global__ void part_split_kernel<32, false>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<32, true>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<16, false>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<16, true>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<8, false>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<8, true>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<4, false>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<4, true>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<2, false>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<2, true>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<1, false>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);
template __global__ void part_split_kernel<1, true>(const uint32_t*, int, int, const uint32_t*, const uint32_t*, int, int, int,
                                                       int, uint32_t*, const uint32_t*, uint32_t*, int, int);

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
__device__ __forceinline__ bool having_pass(const PartHaving& h, const uint64_t* row) {
  bool all = true, any = false;
  for (int j = 0; j < h.nterms; ++j) {
    const int64_t x = (int64_t)row[h.slot[j]];
    const double v = h.f64[j] ? __longlong_as_double(x) : (double)x / h.div[j];
    const bool t = h.op[j] == 0 ? v == h.c[j] : (h.op[j] == 1 ? v > h.c[j] : v < h.c[j]);
    all = all && t;
    any = any || t;
  }
  return h.conj ? all : any;
}

// HAVING mode: the groups of the sub-bucket that exist (presence count, slot 0, > 0) and pass the
// predicate are appended -- key + slots -- at a position reserved with one global atomic per block;
// writes past `cap` are dropped (the host sees out_count > cap and re-runs with room).
// Raise one LDS byte register to v (compare-and-swap on its dword; a relaxed read filters the
// updates that cannot raise it).
__device__ __forceinline__ void lds_max_u8(unsigned char* regs, int64_t idx, uint32_t v) {
  uint32_t* w = (uint32_t*)(regs + (idx & ~(int64_t)3));
  const uint32_t sh = (uint32_t)(idx & 3) * 8u;
  uint32_t old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (((old >> sh) & 0xffu) < v) {
    const uint32_t prev = atomicCAS(w, old, (old & ~(0xffu << sh)) | (v << sh));
    if (prev == old) break;
    old = prev;
  }
}

// Fused ORDER BY <slot> LIMIT k of the partitioned aggregation.  A group's sort value as an
// unsigned key, larger = better (doubles by their ordered bits, ascending orders inverted; NaN last
// either way, as 0 -- also the "no group" value).
__device__ __forceinline__ uint64_t topk_ord(uint64_t bits, int f64, int desc) {
  uint64_t u;
  if (f64) {
    const double d = __longlong_as_double((long long)bits);
    if (d != d) return 0ull;
    u = (bits >> 63) ? ~bits : (bits | 0x8000000000000000ull);
  } else {
    u = bits ^ 0x8000000000000000ull;
  }
  return desc ? u : ~u;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o), hi = __shfl_xor((uint32_t)(v >> 32), o);
    const uint64_t w = ((uint64_t)hi << 32) | lo;
    v = w > v ? w : v;
  }
  return v;
}

// The block's emission threshold for a fused top-k: max(its own k-th best sort value, the best
// k-th value an earlier block published in *gthr).  Any group below it has k better groups in one
// block, so it is not in the global top k (ties included: a group equal to the threshold is kept).
// A thread holds the sort values of its own table rows (at most PART_TOPK_RPT: tables of <= 4096
// keys); each wave extracts its k best by k rounds of a wave max (the lowest lane holding it pops
// that value), and wave 0 does the same over the 8 waves' lists.  The LDS table is read-only here.
constexpr int PART_TOPK_RPT = 8;

__device__ uint64_t part_topk_threshold(const uint64_t* t, int64_t nk, int NS, const PartHaving& hv,
                                        unsigned long long* gthr) {
  __shared__ uint64_t wtop[8 * PART_TOPK_MAX];
  __shared__ uint64_t blk_thr;
  const int k = hv.tk;
  uint64_t v[PART_TOPK_RPT];
#pragma unroll
  for (int j = 0; j < PART_TOPK_RPT; ++j) {
    const int64_t i = threadIdx.x + (int64_t)j * blockDim.x;
    v[j] = 0ull;
    if (i < nk) {
      const uint64_t* row = t + i * NS;
      if ((int64_t)row[0] > 0 && having_pass(hv, row)) v[j] = topk_ord(row[hv.tk_slot], hv.tk_f64, hv.tk_desc);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = 0; r < k; ++r) {
    uint64_t head = 0ull;
#pragma unroll
    for (int j = 0; j < PART_TOPK_RPT; ++j) head = v[j] > head ? v[j] : head;
    const uint64_t m = wave_max_u64(head);
    const unsigned long long b = __ballot(head == m);
    if (lane == __ffsll(b) - 1) {  // pop one copy of m
      bool done = false;
#pragma unroll
      for (int j = 0; j < PART_TOPK_RPT; ++j) {
        if (!done && v[j] == m) {
          v[j] = 0ull;
          done = true;
        }
      }
    }
    if (lane == 0) wtop[wave * PART_TOPK_MAX + r] = m;
  }
  __syncthreads();
  if (wave == 0) {
    const int nw = (int)(blockDim.x >> 6);
    const int nc = nw * k;  // candidates c = w * k + r, two per lane (k <= 16, 8 waves)
    uint64_t a0 = 0ull, a1 = 0ull;
    if (lane < nc) a0 = wtop[(lane / k) * PART_TOPK_MAX + lane % k];
    if (lane + 64 < nc) a1 = wtop[((lane + 64) / k) * PART_TOPK_MAX + (lane + 64) % k];
    if (a1 > a0) {
      const uint64_t x = a0;
      a0 = a1;
      a1 = x;
    }
    uint64_t m = 0ull;
    for (int r = 0; r < k; ++r) {
      m = wave_max_u64(a0);
      const unsigned long long b = __ballot(a0 == m);
      if (lane == __ffsll(b) - 1) {
        a0 = a1;
        a1 = 0ull;
      }
    }
    if (lane == 0) {
      // publish this block's k-th if it raises the global one (a relaxed read first: once the
      // threshold settles, most blocks issue no atomic)
      const uint64_t g = __hip_atomic_load(gthr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint64_t best = g > m ? g : m;
      if (m > g) {
        const uint64_t old = atomicMax(gthr, (unsigned long long)m);
        best = old > m ? old : m;
      }
      blk_thr = best;
    }
  }
  __syncthreads();
  return blk_thr;
}

__global__ __launch_bounds__(512) void part_agg_kernel(const uint32_t* __restrict__ recs, int RW,
                                                      const uint32_t* __restrict__ base, int64_t nsub, int64_t G,
                                                      int shift, PartFields f, PartHll hl, uint64_t* __restrict__ gacc,
                                                      PartHaving hv, int64_t* __restrict__ out_keys,
                                                      unsigned long long* __restrict__ out_count, int64_t cap) {
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
  // HLL byte registers after the slot table: [n][2^shift][2^p]
  const int64_t m = (int64_t)1 << hl.p;
  unsigned char* hr = (unsigned char*)(t + ((int64_t)1 << shift) * NS);
  for (int64_t i = threadIdx.x; i < (hl.n * (m << shift)) / 4; i += blockDim.x) ((uint32_t*)hr)[i] = 0u;
  __syncthreads();
  const uint32_t lo = base[r], hi = base[r + 1];
  constexpr int PU = 4;
  const uint32_t step = blockDim.x * PU;
  if (hl.n == 0 && RW == 2 && f.nfields == 1 && f.width[0] == 1) {
    // u32 key + one i32 value (TPC-H Q18: sum(l_quantity) per order): 8-byte record loads, PU in flight
    const int s0 = f.slot[0], op = f.op[s0];
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += step) {
      uint2 r2[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i < hi) r2[u] = *(const uint2*)(recs + (uint64_t)i * 2);
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        if (i0 + u * blockDim.x >= hi) break;
        const int64_t local = (int64_t)r2[u].x - k0;
        if ((uint64_t)local >= (uint64_t)nk) continue;
        lds_fold(t + local * NS + s0, op, (int64_t)(int32_t)r2[u].y);
      }
    }
  } else if (hl.n == 0 && RW == 1 && f.nfields == 1 && f.width[0] == PART_PACKED) {
    // one value packed into the key word by the level-1 split (TPC-H Q18: sum(l_quantity) per
    // order, 600M one-word records): the key's low bits locate the group, the high bits are the value
    const int s0 = f.slot[0], op = f.op[s0], ps = f.pk_shift;
    const uint32_t lmask = (1u << shift) - 1u;
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += step) {
      uint32_t kk[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i < hi) kk[u] = recs[i];
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        if (i0 + u * blockDim.x >= hi) break;
        const int64_t local = (int64_t)(kk[u] & lmask);
        if (local >= nk) continue;
        lds_fold(t + local * NS + s0, op, (int64_t)(kk[u] >> ps));
      }
    }
  } else if (hl.n == 0 && RW == 1 && f.nfields == 1 && f.width[0] == 0) {
    // key only (histograms, unfiltered counts)
    const int s0 = f.slot[0], op = f.op[s0];
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += step) {
      uint32_t kk[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i < hi) kk[u] = recs[i];
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        if (i0 + u * blockDim.x >= hi) break;
        const int64_t local = (int64_t)kk[u] - k0;
        if ((uint64_t)local >= (uint64_t)nk) continue;
        lds_fold(t + local * NS + s0, op, 1);
      }
    }
  } else if (RW <= 4 && hl.n == 0) {
    // narrow records without sketches (TopNSuppliersGlobal: key + f64 revenue + presence, 4 words):
    // PU records per thread loaded before any is folded, so PU loads are in flight, not one
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += step) {
      uint32_t r4[PU][4];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i < hi) {
          const uint32_t* rec = recs + (uint64_t)i * RW;
          if (RW == 4) {
            const uint4 q = *(const uint4*)rec;  // (16-byte records: 16-byte aligned)
            r4[u][0] = q.x; r4[u][1] = q.y; r4[u][2] = q.z; r4[u][3] = q.w;
          } else {
#pragma unroll
            for (int w = 0; w < 4; ++w) r4[u][w] = w < RW ? rec[w] : 0u;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        if (i0 + u * blockDim.x >= hi) break;
        // (a packed record's key word carries a value above pk_shift: the group is its low bits)
        const int64_t local = f.pk_shift ? (int64_t)(r4[u][0] & ((1u << shift) - 1u)) : (int64_t)r4[u][0] - k0;
        if ((uint64_t)local >= (uint64_t)nk) continue;  // cannot happen for consistent buckets; never fault
        uint64_t* row = t + local * NS;
        int w = 1;
        for (int j = 0; j < f.nfields; ++j) {
          const int wd = f.width[j];
          int64_t v;
          if (wd == PART_PACKED) {
            const int sl = f.slot[j];
            lds_fold(row + sl, f.op[sl], (int64_t)(r4[u][0] >> f.pk_shift));
            continue;
          }
          if (wd == 0) v = 1;
          else if (wd == 1) v = (int64_t)(int32_t)r4[u][w & 3];
          else v = (int64_t)((uint64_t)r4[u][w & 3] | ((uint64_t)r4[u][(w + 1) & 3] << 32));
          w += wd;
          const int sl = f.slot[j];
          lds_fold(row + sl, f.op[sl], v);
        }
      }
    }
  } else {
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      const uint32_t* rec = recs + (uint64_t)i * RW;
      const int64_t local = f.pk_shift ? (int64_t)(rec[0] & ((1u << shift) - 1u)) : (int64_t)rec[0] - k0;
      if ((uint64_t)local >= (uint64_t)nk) continue;  // cannot happen for consistent buckets; never fault
      uint64_t* row = t + local * NS;
      int w = 1;
      for (int j = 0; j < f.nfields; ++j) {
        const int wd = f.width[j];
        int64_t v;
        if (wd == PART_PACKED) {
          const int sl = f.slot[j];
          lds_fold(row + sl, f.op[sl], (int64_t)(rec[0] >> f.pk_shift));
          continue;
        }
        if (wd == 0) v = 1;
        else if (wd == 1) v = (int64_t)(int32_t)rec[w];
        else v = (int64_t)((uint64_t)rec[w] | ((uint64_t)rec[w + 1] << 32));
        w += wd;
        const int s = f.slot[j];
        lds_fold(row + s, f.op[s], v);
      }
      for (int h = 0; h < hl.n; ++h) {
        const uint32_t code = rec[w + h];
        unsigned char* gr = hr + (((int64_t)h << shift) + local) * m;
        if ((hl.stored >> h) & 1u) {
          // a stored sketch: union the row's sparse pairs (row id; all-ones = filtered out)
          if (code == 0xffffffffu) continue;
          const int64_t a = hl.sk_off[h][code], e = hl.sk_off[h][code + 1];
          for (int64_t j = a; j < e; ++j) {
            const uint32_t pk = (uint32_t)hl.sk_val[h][j];
            if (pk & 0xffu) lds_max_u8(gr, (int64_t)((pk >> 8) & (uint32_t)(m - 1)), pk & 0xffu);
          }
          continue;
        }
        if (code & 0xffu) lds_max_u8(gr, (int64_t)((code >> 8) & (uint32_t)(m - 1)), code & 0xffu);
      }
    }
  }
  __syncthreads();
  if (hv.nterms == 0 && hv.tk == 0) {
    uint64_t* g = gacc + k0 * NS;
    for (int64_t i = threadIdx.x; i < nk * NS; i += blockDim.x) g[i] = t[i];
    for (int h = 0; h < hl.n; ++h) {  // the sub-bucket's register rows, 16 bytes per thread step
      const uint4* src = (const uint4*)(hr + ((int64_t)h << shift) * m);
      uint4* dst = (uint4*)(hl.regs[h] + k0 * m);
      for (int64_t i = threadIdx.x; i < nk * m / 16; i += blockDim.x) dst[i] = src[i];
    }
    return;
  }
  __shared__ uint32_t scan_lds[8];
  __shared__ unsigned long long blk_base;
  // the emission threshold of a fused ORDER BY ... LIMIT tk (0: every surviving group)
  const uint64_t thr = hv.tk > 0 ? part_topk_threshold(t, nk, NS, hv, out_count + 1) : 0ull;
  uint32_t mine = 0;
  for (int64_t i = threadIdx.x; i < nk; i += blockDim.x) {
    const uint64_t* row = t + i * NS;
    mine += ((int64_t)row[0] > 0 && having_pass(hv, row) &&
             (thr == 0ull || topk_ord(row[hv.tk_slot], hv.tk_f64, hv.tk_desc) >= thr)) ? 1u : 0u;
  }
  uint32_t total;
  uint32_t pre = block_excl_scan_u32<512>(mine, scan_lds, &total);
  if (threadIdx.x == 0) blk_base = total ? atomicAdd(out_count, (unsigned long long)total) : 0ull;
  __syncthreads();
  if (total == 0) return;
  int64_t pos = (int64_t)blk_base + pre;
  for (int64_t i = threadIdx.x; i < nk; i += blockDim.x) {
    const uint64_t* row = t + i * NS;
    if (!((int64_t)row[0] > 0 && having_pass(hv, row) &&
          (thr == 0ull || topk_ord(row[hv.tk_slot], hv.tk_f64, hv.tk_desc) >= thr)))
      continue;
    if (pos < cap) {
      out_keys[pos] = k0 + i;
      for (int s = 0; s < NS; ++s) gacc[pos * NS + s] = row[s];
    }
    ++pos;
  }
}

}  // namespace sdo

namespace sdo {

// ---------------------------------------------------------------------------------------------
// Key spaces beyond 32 bits (TPC-H Q16's (brand, type, size, supplier) = 1.7e11 keys, ~12M present
// at SF100): records are bucketed by a 32-bit hash of the 64-bit key (record word 0; words 1-2 the
// key) through the same split kernels, and each sub-bucket -- ~HASH_SUB_KEYS distinct keys by the
// planner's estimate -- aggregates in an LDS open-addressing table (64-bit key compare-and-swap,
// then the slot operators), emitting its groups sparsely (key + slots) at a position reserved with
// one global atomic per workgroup.  A sub-bucket whose distinct keys overflow the table sets
// *overflow and drops them; the host re-partitions with more sub-buckets and runs again.
constexpr uint64_t HASH_EMPTY = ~0ull;

__device__ __forceinline__ uint32_t part_hash_probe(uint32_t h, int cap_log2) {
  // the partitioning consumed the hash's top bits; a multiplicative re-mix spreads the rest
  return (h * 0x9E3779B1u) >> (32 - cap_log2);
}

// HLL aggregators (hl.n > 0): each record ends with one (bucket << 8 | rho) word per HLL; every
// table slot keeps 2^p byte registers per HLL in LDS after the slot table, and a surviving group's
// registers are written to row `pos` of the [cap][2^p] output tables (hl.regs).
__global__ __launch_bounds__(512) void part_hash_agg_kernel(const uint32_t* __restrict__ recs, int RW,
                                                           const uint32_t* __restrict__ base, int64_t nsub,
                                                           int cap_log2, PartFields f, PartHll hl,
                                                           PartHaving hv, int64_t* __restrict__ out_keys,
                                                           uint64_t* __restrict__ out_acc,
                                                           unsigned long long* __restrict__ out_count, int64_t cap,
                                                           int* __restrict__ overflow) {
  extern __shared__ __attribute__((aligned(16))) uint64_t t[];
  const int64_t x = blockIdx.x;
  const int64_t per_xcd = gridDim.x / 8;
  const int64_t r = (x % 8) * per_xcd + x / 8;
  if (r >= nsub) return;
  const int C = 1 << cap_log2;
  const int NS = f.nslots;
  uint64_t* tk = t;           // [C] keys
  uint64_t* tv = t + C;       // [C][NS] slots
  const int64_t m = (int64_t)1 << hl.p;
  unsigned char* hr = (unsigned char*)(tv + (int64_t)C * NS);  // [n][C][2^p] byte registers
  for (int i = threadIdx.x; i < C; i += blockDim.x) tk[i] = HASH_EMPTY;
  for (int i = threadIdx.x; i < C * NS; i += blockDim.x) tv[i] = (uint64_t)f.init[i % NS];
  for (int64_t i = threadIdx.x; i < (hl.n * C * m) / 4; i += blockDim.x) ((uint32_t*)hr)[i] = 0u;
  __syncthreads();
  const uint32_t lo = base[r], hi = base[r + 1];
  bool full = false;
  for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t* rec = recs + (uint64_t)i * RW;
    const uint64_t key = (uint64_t)rec[1] | ((uint64_t)rec[2] << 32);
    uint32_t pos = part_hash_probe(rec[0], cap_log2);
    int slot = -1;
    for (int probe = 0; probe < C; ++probe) {
      const uint64_t prev = atomicCAS((unsigned long long*)&tk[pos], (unsigned long long)HASH_EMPTY,
                                      (unsigned long long)key);
      if (prev == HASH_EMPTY || prev == key) {
        slot = (int)pos;
        break;
      }
      pos = (pos + 1u) & (uint32_t)(C - 1);
    }
    if (slot < 0) {
      full = true;
      continue;
    }
    uint64_t* row = tv + (int64_t)slot * NS;
    int w = 3;
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
    for (int h = 0; h < hl.n; ++h) {
      const uint32_t code = rec[w + h];
      if (code & 0xffu) lds_max_u8(hr + ((int64_t)h * C + slot) * m, (int64_t)((code >> 8) & (uint32_t)(m - 1)),
                                   code & 0xffu);
    }
  }
  if (full) atomicOr(overflow, 1);
  __syncthreads();
  __shared__ uint32_t scan_lds[8];
  __shared__ unsigned long long blk_base;
  uint32_t mine = 0;
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    if (tk[i] == HASH_EMPTY) continue;
    mine += (hv.nterms == 0 || having_pass(hv, tv + (int64_t)i * NS)) ? 1u : 0u;
  }
  uint32_t total;
  uint32_t pre = block_excl_scan_u32<512>(mine, scan_lds, &total);
  if (threadIdx.x == 0) blk_base = total ? atomicAdd(out_count, (unsigned long long)total) : 0ull;
  __syncthreads();
  if (total == 0) return;
  int64_t pos = (int64_t)blk_base + pre;
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    if (tk[i] == HASH_EMPTY) continue;
    const uint64_t* row = tv + (int64_t)i * NS;
    if (hv.nterms && !having_pass(hv, row)) continue;
    if (pos < cap) {
      out_keys[pos] = (int64_t)tk[i];
      for (int s = 0; s < NS; ++s) out_acc[pos * NS + s] = row[s];
      for (int h = 0; h < hl.n; ++h) {  // (the group's registers: m / 16 16-byte copies)
        const uint4* src = (const uint4*)(hr + ((int64_t)h * C + i) * m);
        uint4* dst = (uint4*)(hl.regs[h] + pos * m);
        for (int64_t q = 0; q < m / 16; ++q) dst[q] = src[q];
      }
    }
    ++pos;
  }
}

}  // namespace sdo
