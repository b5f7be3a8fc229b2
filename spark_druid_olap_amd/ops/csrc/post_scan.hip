// Post-scan kernels for CDNA4 (gfx950): row compaction for Select/scan queries and threshold
// (top-k) selection over merged partial aggregates.
//
// Reference behaviour these implement:
//  * compact_rows -- the Select query's filtered-row cursor (SelectSpecWithIntervals + PagingSpec,
//    sd/DruidQuerySpec.scala:977-1070; paging loop asd/DruidSelectResultIterator.scala:116-137):
//    the scan kernel writes one 64-bit mask word per 64 rows; this turns the mask into sorted row ids
//    with one popcount pass, one workgroup-level scan of the per-block counts and one scatter pass.
//  * topk_* -- TopN / ORDER BY metric LIMIT k (TopNQuerySpec, sd/DruidQuerySpec.scala:767-822;
//    LimitSpec 437-456): a 4-level radix select (4 x 12 high bits of the order-preserving key) that
//    finds the 48-bit bucket of the k-th best value of a metric slot on the device without a host round
//    trip; every group whose key ties or beats that bucket is kept (a superset of the top k, exact
//    after the host's final order + limit).
//
// Wave64 everywhere: per-wave prefix sums use __shfl_up over 64 lanes, and block-level scans combine
// the (blockDim/64) wave totals through LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "post_scan.h"

namespace sdo {

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Exclusive scan of one int per thread across a block of up to 1024 threads.  Returns the
// thread's exclusive prefix; *total receives the block total.
__device__ __forceinline__ int block_excl_scan(int v, int* lds_waves, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  const int incl = wave_incl_scan(v);
  if (lane == 63) lds_waves[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    int w = lane < nw ? lds_waves[lane] : 0;
    const int wi = wave_incl_scan(w);
    if (lane < nw) lds_waves[lane] = wi - w;
    if (lane == nw - 1) lds_waves[32] = wi;
  }
  __syncthreads();
  const int out = lds_waves[wave] + incl - v;
  *total = lds_waves[32];
  __syncthreads();
  return out;
}

constexpr int CW_THREADS = 256;   // threads per compaction block
constexpr int CW_WORDS = 4;       // mask words per thread -> 1024 words (65536 rows) per block

// Pass 1: set rows per block.
__global__ void __launch_bounds__(CW_THREADS) compact_count_kernel(const uint64_t* __restrict__ mask, int64_t nwords,
                                                                  int* __restrict__ block_counts) {
  __shared__ int lds[40];
  const int64_t w0 = ((int64_t)blockIdx.x * CW_THREADS + threadIdx.x) * CW_WORDS;
  int c = 0;
#pragma unroll
  for (int i = 0; i < CW_WORDS; ++i)
    if (w0 + i < nwords) c += __popcll(mask[w0 + i]);
  int total;
  block_excl_scan(c, lds, &total);
  if (threadIdx.x == 0) block_counts[blockIdx.x] = total;
}

// Pass 2 (one workgroup): exclusive scan of the per-block counts -> int64 block offsets + total.
__global__ void __launch_bounds__(1024) compact_offsets_kernel(const int* __restrict__ block_counts, int64_t nblocks,
                                                              int64_t* __restrict__ offsets, int64_t* __restrict__ total) {
  __shared__ int lds[40];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nblocks; base += blockDim.x) {
    const int64_t i = base + threadIdx.x;
    const int v = i < nblocks ? block_counts[i] : 0;
    int tot;
    const int ex = block_excl_scan(v, lds, &tot);
    if (i < nblocks) offsets[i] = carry + ex;
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// Pass 3: every set bit writes its row id at (block offset + prefix within the block).
__global__ void __launch_bounds__(CW_THREADS) compact_write_kernel(const uint64_t* __restrict__ mask, int64_t nwords,
                                                                  const int64_t* __restrict__ offsets,
                                                                  int64_t* __restrict__ rows) {
  __shared__ int lds[40];
  const int64_t w0 = ((int64_t)blockIdx.x * CW_THREADS + threadIdx.x) * CW_WORDS;
  uint64_t w[CW_WORDS];
  int c = 0;
#pragma unroll
  for (int i = 0; i < CW_WORDS; ++i) {
    w[i] = (w0 + i < nwords) ? mask[w0 + i] : 0ull;
    c += __popcll(w[i]);
  }
  int total;
  int64_t pos = offsets[blockIdx.x] + block_excl_scan(c, lds, &total);
#pragma unroll
  for (int i = 0; i < CW_WORDS; ++i) {
    uint64_t m = w[i];
    const int64_t rbase = (w0 + i) << 6;
    while (m) {
      const int b = __ffsll((unsigned long long)m) - 1;
      rows[pos++] = rbase + b;
      m &= m - 1;
    }
  }
}

// Presence bitmask of a strided column (element i = base[i * stride] != 0; 1- or 8-byte elements):
// the "which groups exist" test of a dense accumulator table (slot 0 = row count) or of the
// one-byte existence table, as one ballot word per 64 groups for compact_rows.
__global__ void __launch_bounds__(256) nonzero_mask_kernel(const unsigned char* __restrict__ base, int esize,
                                                          int64_t n, int64_t stride, uint64_t* __restrict__ words) {
  const int lane = threadIdx.x & 63;
  const int64_t nwords = (n + 63) >> 6;
  const int64_t wstride = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = (((int64_t)blockIdx.x * blockDim.x) >> 6) + (threadIdx.x >> 6); w < nwords; w += wstride) {
    const int64_t i = (w << 6) + lane;
    bool nz = false;
    if (i < n) {
      nz = esize == 8 ? ((const int64_t*)base)[i * stride] != 0 : base[i * stride] != 0;
    }
    const uint64_t b = __ballot(nz);
    if (lane == 0) words[w] = b;
  }
}

// Per-bin counts of int64 group ids (nested count-only levels: TPC-H Q13's orders per customer):
// one no-return 32-bit device atomic per id, four ids in flight per thread, no min/max pre-pass
// (the bin count is known from the key radix).  Ids outside [0, nbins) are ignored.
__global__ void __launch_bounds__(256) histogram_kernel(const int64_t* __restrict__ keys, int64_t n, int64_t nbins,
                                                       unsigned int* __restrict__ counts) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    int64_t k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = keys[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((uint64_t)k[u] < (uint64_t)nbins) atomicAdd(counts + k[u], 1u);
  }
  for (; i < n; i += stride) {
    const int64_t k = keys[i];
    if ((uint64_t)k < (uint64_t)nbins) atomicAdd(counts + k, 1u);
  }
}

// Few bins (TPC-H Q13's outer level: 15M customers into ~30 order counts): every block counts
// into an LDS copy first and flushes it with one global atomic per non-empty bin -- global
// atomics on a handful of addresses would serialise.
__global__ void __launch_bounds__(256) histogram_lds_kernel(const int64_t* __restrict__ keys, int64_t n, int nbins,
                                                           unsigned int* __restrict__ counts) {
  extern __shared__ unsigned int h[];
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) h[b] = 0u;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = keys[i];
    if ((uint64_t)k < (uint64_t)nbins) atomicAdd(h + k, 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += blockDim.x)
    if (h[b]) atomicAdd(counts + b, h[b]);
}

// Contiguous one-byte tables (first-touch / existence bytes, bool masks): 16 bytes per lane per
// load, so a wave covers 1024 groups = 16 ballot words per iteration instead of one byte per lane
// (TPC-H Q3's 150 MB touch table: 183 us with byte loads).  Lane l holds a 16-bit mask of its
// bytes; word w of the chunk is lanes 4w..4w+3 packed, gathered with three lane shuffles.
__device__ __forceinline__ uint32_t nz4(uint32_t x) {
  return ((x & 0xFFu) != 0u) | (((x >> 8) & 0xFFu) != 0u) << 1 | (((x >> 16) & 0xFFu) != 0u) << 2 |
         ((x >> 24) != 0u) << 3;
}

__global__ void __launch_bounds__(256) nonzero_mask_u8_kernel(const unsigned char* __restrict__ base, int64_t n,
                                                             uint64_t* __restrict__ words) {
  const int lane = threadIdx.x & 63;
  const int64_t nwords = (n + 63) >> 6;
  const int64_t nchunks = (n + 1023) >> 10;
  const int64_t wstride = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t c = (((int64_t)blockIdx.x * blockDim.x) >> 6) + (threadIdx.x >> 6); c < nchunks; c += wstride) {
    const int64_t e0 = (c << 10) + (int64_t)lane * 16;
    uint32_t m = 0;
    if (e0 + 16 <= n) {
      const uint4 v = *(const uint4*)(base + e0);
      m = nz4(v.x) | nz4(v.y) << 4 | nz4(v.z) << 8 | nz4(v.w) << 12;
    } else {
      for (int j = 0; j < 16; ++j)
        if (e0 + j < n && base[e0 + j]) m |= 1u << j;
    }
    const uint64_t m1 = (uint64_t)(uint32_t)__shfl_down((int)m, 1);
    const uint64_t m2 = (uint64_t)(uint32_t)__shfl_down((int)m, 2);
    const uint64_t m3 = (uint64_t)(uint32_t)__shfl_down((int)m, 3);
    const int64_t w = (c << 4) + (lane >> 2);
    if ((lane & 3) == 0 && w < nwords) words[w] = (uint64_t)m | m1 << 16 | m2 << 32 | m3 << 48;
  }
}

// ---------------------------------------------------------------------------------------------
// top-k threshold over one accumulator slot of the merged partials ([rows, nslots] int64).
// The slot is mapped to an order-preserving unsigned key (larger = better) on the fly: f64 sums by
// their IEEE bits, integer slots by flipping the sign bit; ascending order inverts the key.
constexpr int TK_BITS = 12, TK_BINS = 1 << TK_BITS, TK_THREADS = 512, TK_LEVELS = 4;

__device__ __forceinline__ uint64_t ord_key(int64_t raw, int is_f64, int desc) {
  uint64_t u = (uint64_t)raw;
  if (is_f64) {
    u = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
  } else {
    u ^= 0x8000000000000000ull;
  }
  return desc ? u : ~u;
}

// Histogram of key bits [shift, shift+12) over the keys whose higher (12*level) bits equal the
// prefix chosen so far (state[0]).
__global__ void __launch_bounds__(TK_THREADS) topk_hist_kernel(const int64_t* __restrict__ acc, int64_t n, int nslots,
                                                              int slot, int is_f64, int desc,
                                                              const uint64_t* __restrict__ state, int level,
                                                              unsigned int* __restrict__ hist) {
  __shared__ unsigned int h[TK_BINS];
  for (int i = threadIdx.x; i < TK_BINS; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int shift = 64 - TK_BITS * (level + 1);
  const uint64_t prefix = level ? state[0] : 0ull;
  const int pshift = 64 - TK_BITS * level;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t k = ord_key(acc[i * nslots + slot], is_f64, desc);
    if (level == 0 || (k >> pshift) == prefix) atomicAdd(&h[(k >> shift) & (TK_BINS - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TK_BINS; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// One workgroup of TK_BINS/4 threads: walk the histogram from the top bin down until the k-th key
// is covered; extend the prefix with that bin and make k relative to it.  state = {prefix, k}.
__global__ void __launch_bounds__(TK_BINS / 4) topk_pick_kernel(unsigned int* __restrict__ hist,
                                                               uint64_t* __restrict__ state, int level) {
  __shared__ int lds[40];
  __shared__ int pick;
  __shared__ int64_t knew;
  const int t = threadIdx.x;
  const int owner = (TK_BINS / 4) - 1 - t;  // thread 0 owns the 4 highest bins
  unsigned int c[4];
  int s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = hist[owner * 4 + (3 - j)];
    s += (int)c[j];
  }
  int total;
  const int above = block_excl_scan(s, lds, &total);
  const int64_t k = (int64_t)state[1];
  if (t == 0) {
    pick = -1;
    knew = k;
  }
  __syncthreads();
  int64_t run = above;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (run < k && run + (int64_t)c[j] >= k) {
      pick = owner * 4 + (3 - j);
      knew = k - run;
    }
    run += (int64_t)c[j];
  }
  __syncthreads();
  if (t == 0) {
    const uint64_t b = pick < 0 ? 0ull : (uint64_t)pick;  // fewer than k keys: keep everything
    state[0] = (level == 0 ? 0ull : (state[0] << TK_BITS)) | b;
    state[1] = (uint64_t)knew;
    if (pick < 0) state[2] = 1;
  }
  for (int i = t; i < TK_BINS; i += blockDim.x) hist[i] = 0;
}

// keep bit per row: its key's top 12*TK_LEVELS bits >= the chosen prefix (every row that ties or
// beats the k-th best); one 64-bit word per 64 rows via a wave ballot, compacted by compact_rows.
__global__ void __launch_bounds__(256) topk_keep_kernel(const int64_t* __restrict__ acc, int64_t n, int nslots, int slot,
                                                       int is_f64, int desc, const uint64_t* __restrict__ state,
                                                       uint64_t* __restrict__ keep) {
  const int lane = threadIdx.x & 63;
  const int64_t nwords = (n + 63) >> 6;
  const int64_t wstride = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int shift = 64 - TK_BITS * TK_LEVELS;
  const uint64_t prefix = state[0];
  const bool all = state[2] != 0;
  for (int64_t w = (((int64_t)blockIdx.x * blockDim.x) >> 6) + (threadIdx.x >> 6); w < nwords; w += wstride) {
    const int64_t i = (w << 6) + lane;
    bool k = false;
    if (i < n) k = all || (ord_key(acc[i * nslots + slot], is_f64, desc) >> shift) >= prefix;
    const uint64_t b = __ballot(k);
    if (lane == 0) keep[w] = b;
  }
}

// Re-initialisation of a prepared scan's execution buffers in ONE launch (instead of one fill per
// buffer): the accumulator table gets its per-slot identity row (0 for sums/counts, +/-max for
// min/max), up to four HLL register arrays and the hash-overflow flag are zeroed.  Grid-stride,
// 64-bit vector stores.
struct ResetArgs {
  int64_t* acc;
  const int64_t* init;   // nslots identities
  int64_t rows;
  int nslots;
  int nz;                // zero regions in use
  uint64_t* z[4];        // zeroed regions (64-bit words)
  int64_t zn[4];         // their lengths in words
  int* overflow;
};

__global__ void __launch_bounds__(256) reset_bufs_kernel(ResetArgs a) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  const int64_t na = a.rows * a.nslots;
  for (int64_t i = tid; i < na; i += nth) a.acc[i] = a.init[i % a.nslots];
  for (int r = 0; r < a.nz; ++r) {
    uint64_t* z = a.z[r];
    for (int64_t i = tid; i < a.zn[r]; i += nth) z[i] = 0ull;
  }
  if (tid == 0 && a.overflow) *a.overflow = 0;
}

// ---- First-touch compaction of a dense HBM accumulator table (TPC-H Q3: 150M order groups, ~1M
// touched per run).  Pass 1 reads the byte table 16 bytes per lane (as nonzero_mask_u8_kernel),
// joins four lanes' 16-bit masks into the ballot word of 64 groups and counts per 65536-group block; compact_offsets_kernel scans the counts; pass 3
// writes each touched group's id and accumulator row, re-initialises the row and clears its byte --
// one launch instead of the mask / count / write / gather / index_copy / index_fill chain.
// The byte table is padded to a multiple of 64 groups (engine/device_exec.py _alloc).
__global__ void __launch_bounds__(CW_THREADS) touch_count_kernel(const uint4* __restrict__ touch, int64_t nwords,
                                                                uint64_t* __restrict__ words,
                                                                int* __restrict__ block_counts) {
  __shared__ int lds[40];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int c = 0;
  // a wave covers 16 words per step (64 lanes x 16 bytes); the block's 4 waves 64 words; 16 steps
  // cover the block's 1024 words
  for (int it = 0; it < CW_THREADS * CW_WORDS / 64; ++it) {
    const int64_t wb = (int64_t)blockIdx.x * CW_THREADS * CW_WORDS + it * 64 + wave * 16;
    const int64_t w = wb + (lane >> 2);
    uint32_t m = 0;
    if (w < nwords) {
      const uint4 v = touch[wb * 4 + lane];
      m = nz4(v.x) | (nz4(v.y) << 4) | (nz4(v.z) << 8) | (nz4(v.w) << 12);
    }
    const uint64_t m1 = (uint32_t)__shfl_down((int)m, 1, 64);
    const uint64_t m2 = (uint32_t)__shfl_down((int)m, 2, 64);
    const uint64_t m3 = (uint32_t)__shfl_down((int)m, 3, 64);
    if ((lane & 3) == 0 && w < nwords) {
      const uint64_t word = (uint64_t)m | (m1 << 16) | (m2 << 32) | (m3 << 48);
      words[w] = word;
      c += __popcll(word);
    }
  }
  int total;
  block_excl_scan(c, lds, &total);
  if (threadIdx.x == 0) block_counts[blockIdx.x] = total;
}

__global__ void __launch_bounds__(CW_THREADS) touch_gather_kernel(const uint64_t* __restrict__ words, int64_t nwords,
                                                                 const int64_t* __restrict__ offsets,
                                                                 int64_t* __restrict__ acc, int ns,
                                                                 const int64_t* __restrict__ init,
                                                                 unsigned char* __restrict__ touch,
                                                                 int64_t* __restrict__ out_idx,
                                                                 int64_t* __restrict__ out_acc) {
  __shared__ int lds[40];
  const int64_t w0 = ((int64_t)blockIdx.x * CW_THREADS + threadIdx.x) * CW_WORDS;
  uint64_t w[CW_WORDS];
  int c = 0;
#pragma unroll
  for (int i = 0; i < CW_WORDS; ++i) {
    w[i] = (w0 + i < nwords) ? words[w0 + i] : 0ull;
    c += __popcll(w[i]);
  }
  int total;
  int64_t pos = offsets[blockIdx.x] + block_excl_scan(c, lds, &total);
#pragma unroll
  for (int i = 0; i < CW_WORDS; ++i) {
    uint64_t m = w[i];
    const int64_t rbase = (w0 + i) << 6;
    while (m) {
      const int64_t r = rbase + (__ffsll((unsigned long long)m) - 1);
      m &= m - 1;
      out_idx[pos] = r;
      int64_t* a = acc + r * ns;
      int64_t* o = out_acc + pos * ns;
      for (int s = 0; s < ns; ++s) {
        o[s] = a[s];
        a[s] = init[s];
      }
      touch[r] = 0;
      ++pos;
    }
  }
}

// ---- Sparse result decode: the final host columns of a sparse group set (engine/partials.py
// finalize) in one pass -- key components ((id / stride) % card, through an FD map and a typed
// dictionary table, plus a range dictionary's start), aggregator slots (decimal scaling, ordered
// float decode) -- written at their SQL width into ONE buffer (column c at byte offset off[c]) for
// a single device-to-host copy, instead of a chain of torch element-wise / gather kernels and one
// copy per column.
__global__ void __launch_bounds__(256) sparse_decode_kernel(DecArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += stride) {
    const int64_t g = a.idx[r];
    for (int j = 0; j < a.ncols; ++j) {
      const DecCol& c = a.c[j];
      int64_t iv = 0;
      double dv = 0.0;
      bool is_d = false;
      if (c.kind == 0) {
        int64_t v = (g / c.stride) % c.card;
        if (c.orig) v = c.orig[v];
        if (c.lut_t == 1) iv = ((const int32_t*)c.lut)[v];
        else if (c.lut_t == 2) iv = ((const int64_t*)c.lut)[v];
        else if (c.lut_t == 3) { dv = ((const double*)c.lut)[v]; is_d = true; }
        else iv = v;
        iv += c.add;
      } else if (c.kind == 4) {
        iv = g;
      } else {
        const int64_t v = a.acc[r * a.ns + c.slot];
        if (c.kind == 1) {
          iv = v;
          if (c.div != 0.0) { dv = (double)v / c.div; is_d = true; }
        } else if (c.kind == 2) {
          iv = v >= 0 ? v : (v ^ 0x7FFFFFFFFFFFFFFFLL);
          dv = __longlong_as_double(iv);
          is_d = true;
        } else {
          iv = v;
        }
      }
      unsigned char* o = a.out + c.off;
      switch (c.out) {
        case 0: ((int16_t*)o)[r] = (int16_t)iv; break;
        case 1: ((int32_t*)o)[r] = (int32_t)iv; break;
        case 2: ((int64_t*)o)[r] = iv; break;
        case 3: ((double*)o)[r] = is_d ? dv : (double)iv; break;
        case 4: ((int64_t*)o)[r] = is_d ? __double_as_longlong(dv) : iv; break;
        default: ((int64_t*)o)[r] = (is_d ? (isfinite(dv) ? (int64_t)dv : 0) : iv); break;
      }
    }
  }
}

}  // namespace sdo
