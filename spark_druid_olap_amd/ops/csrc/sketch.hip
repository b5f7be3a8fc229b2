// Stored-sketch kernels for CDNA4 (gfx950): HyperUnique metrics that survive ingest-time rollup.
//
// Reference behaviour: a Druid index task stores a hyperUnique metric as an HLL sketch per rolled-up
// row (metricsSpec "hyperUnique", src/test/resources/zip_codeAll.json.template:49-52) and the
// HyperUniqueAggregationSpec (sd/DruidQuerySpec.scala:327-336) unions the sketches of the rows a
// query selects.  Here a rolled-up row keeps a SPARSE sketch: the distinct (bucket, max rho) pairs of
// the raw rows it absorbed, packed as (bucket << 8 | rho) int32 in a CSR layout (offsets per row).
//
//  * hll_pairs  -- ingest: the packed pair of every raw row's 64-bit value, bit-identical to the query
//    kernels' hll_bucket_rho (sdo_device.h), so a rolled-up index answers exactly like the raw one.
//  * hll_merge_stored -- query: union of the stored pairs of the selected rows into per-group
//    registers [G, 2^p] (the same byte register layout the scan kernel produces for query-time
//    cardinality, so cross-GPU merge, MFMA estimate and finalize are shared).  One wavefront per 64
//    selected rows, one lane per row walking its pairs: rows rarely hold more than a few pairs, and
//    registers saturate fast, so the plain read filters most atomics (as in hll_update8).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdo_device.h"

namespace sdo {

__global__ void __launch_bounds__(256) hll_pairs_kernel(const int64_t* __restrict__ vals, int64_t n, int p,
                                                       int64_t salt, int32_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t bucket, rho;
    dev::hll_bucket_rho(vals[i], salt, p, bucket, rho);
    out[i] = (int32_t)((bucket << 8) | rho);
  }
}

__global__ void __launch_bounds__(256) hll_merge_stored_kernel(const int64_t* __restrict__ rows,
                                                              const int64_t* __restrict__ gid, int64_t nsel,
                                                              const int64_t* __restrict__ offsets,
                                                              const int32_t* __restrict__ pairs, int p,
                                                              int64_t G, unsigned char* __restrict__ regs) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const uint32_t m = 1u << p;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsel; i += stride) {
    const int64_t r = rows[i];
    const int64_t g = gid[i];
    if (g < 0 || g >= G) continue;  // filtered-out row (host marks it -1)
    const int64_t e = offsets[r + 1];
    for (int64_t j = offsets[r]; j < e; ++j) {
      const uint32_t pk = (uint32_t)pairs[j];
      dev::hll_max8(regs, (uint64_t)g * m + ((pk >> 8) & (m - 1u)), pk & 0xffu);
    }
  }
}

}  // namespace sdo

namespace sdo {

// ---------------------------------------------------------------------------------------------
// Theta sketch (KMV) selection on the device: per group, the k smallest distinct 62-bit hashes of the
// selected rows (ThetaSketch metric, sd/metadata/DruidDataSource.scala:29,38; 16,384-entry sketches
// in src/test/resources/zip_codeAll.json.template:53-59).  Instead of sorting every (group, hash)
// pair, a radix select per group on the top THETA_BITS hash bits keeps only the candidates:
//
//  * theta_hist   -- histogram [G, 2^B] of the top B bits of every pair's hash (global atomics:
//    uniform hashes spread the updates; the group-major layout keeps one group's bins together);
//  * theta_thresh -- one workgroup per group scans its bins (block prefix sum) for the first bin at
//    which the running count reaches `target` (a margin over k: duplicates are counted), giving the
//    exclusive hash bound of the group's candidates, or "everything" when the group has fewer;
//  * theta_filter -- compacts the pairs below their group's bound (one atomic per wave for the
//    output cursor).
//
// The few candidates (~target per group) are then sorted, de-duplicated and cut to k (torch); a
// group whose candidates hold fewer than k distinct hashes although its bound excluded some pairs
// is re-selected with a larger target (engine/executor.py _theta_select).
__global__ void __launch_bounds__(256) theta_hist_kernel(const int64_t* __restrict__ g, const int64_t* __restrict__ h,
                                                        int64_t n, int bits, uint32_t* __restrict__ hist) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int shift = 62 - bits;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t b = ((uint64_t)h[i]) >> shift;
    atomicAdd(&hist[((uint64_t)g[i] << bits) + b], 1u);
  }
}

// one 1024-thread workgroup per group: bins are scanned in chunks of 1024 (a thread per bin)
__global__ void __launch_bounds__(1024) theta_thresh_kernel(const uint32_t* __restrict__ hist, int bits,
                                                            const int64_t* __restrict__ target,
                                                            int64_t* __restrict__ bound) {
  __shared__ uint32_t wsum[16];
  __shared__ int64_t s_found;
  __shared__ uint64_t s_base;
  const int64_t grp = blockIdx.x;
  const int nb = 1 << bits;
  const uint32_t* hg = hist + ((int64_t)grp << bits);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t want = (uint64_t)target[grp];
  if (tid == 0) {
    s_found = -1;
    s_base = 0;
  }
  __syncthreads();
  for (int c0 = 0; c0 < nb; c0 += 1024) {
    const uint32_t v = (c0 + tid < nb) ? hg[c0 + tid] : 0u;
    // inclusive prefix within the wave, then across the 16 waves
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(x, d, 64);
      if (lane >= d) x += t;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    const uint64_t incl = s_base + before + x;
    // the first bin whose running count reaches the target (bins are visited in order)
    const bool hit = incl >= want && incl - v < want && v > 0;
    if (hit) s_found = c0 + tid;
    __syncthreads();
    if (s_found >= 0) break;
    if (tid == 0) {
      uint32_t tot = 0;
      for (int w = 0; w < 16; ++w) tot += wsum[w];
      s_base += tot;
    }
    __syncthreads();
  }
  if (tid == 0) {
    // exclusive hash bound: every hash whose top bits are <= the found bin; "no bound" (2^62) when
    // the group never reached the target
    bound[grp] = s_found >= 0 ? (int64_t)((uint64_t)(s_found + 1) << (62 - bits)) : ((int64_t)1 << 62);
  }
}

__global__ void __launch_bounds__(256) theta_filter_kernel(const int64_t* __restrict__ g, const int64_t* __restrict__ h,
                                                          int64_t n, const int64_t* __restrict__ bound,
                                                          int64_t* __restrict__ out_g, int64_t* __restrict__ out_h,
                                                          unsigned long long* __restrict__ count, int64_t cap) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
    const int64_t i = i0 + threadIdx.x;
    bool keep = false;
    int64_t gi = 0, hi = 0;
    if (i < n) {
      gi = g[i];
      hi = h[i];
      keep = hi < bound[gi];
    }
    const uint64_t m = __ballot(keep);
    unsigned long long base = 0;
    if (lane == 0 && m) base = atomicAdd(count, (unsigned long long)__popcll(m));
    base = __shfl(base, 0, 64);
    if (keep) {
      const unsigned long long pos = base + __popcll(m & ((1ull << lane) - 1ull));
      if ((int64_t)pos < cap) {
        out_g[pos] = gi;
        out_h[pos] = hi;
      }
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Fused theta: the JIT producer (ops/jit.py A_THETA) writes (u32 group key, 62-bit KMV hash per
// theta aggregator) records straight into its chunk regions -- no row ids, no torch gather / hash
// of the selected rows, no compaction pass.  The radix select then reads the regions in place:
//
//  * theta_hist_regions -- per-workgroup LDS histograms [G, 2^B] (B sized by the host so they fit),
//    merged with one global add per non-empty bin -- the old global same-address atomics per pair
//    were a quarter of a 7-group theta query;
//  * theta_thresh       -- as above;
//  * theta_filter_regions -- the pairs below their group's bound, compacted with one atomic per wave.
__global__ void __launch_bounds__(256) theta_hist_regions_kernel(const uint32_t* __restrict__ recs, int rw, int hoff,
                                                                const uint32_t* __restrict__ seg_lo,
                                                                const uint32_t* __restrict__ seg_hi, int64_t nseg,
                                                                int G, int bits, uint32_t* __restrict__ hist,
                                                                int use_lds, int nt) {
  // nt sketches per record (hash t at words hoff + 2t): histogram rows t * G + g
  extern __shared__ uint32_t lh[];
  const int64_t nb = ((int64_t)G * nt) << bits;
  const int shift = 62 - bits;
  if (use_lds) {
    for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) lh[i] = 0u;
    __syncthreads();
  }
  constexpr int R = 4;  // records in flight per thread (loads issued before the atomics)
  for (int64_t sgi = blockIdx.x; sgi < nseg; sgi += gridDim.x) {
    const uint32_t lo = seg_lo[sgi], hi = seg_hi[sgi];
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += R * blockDim.x) {
      for (int t = 0; t < nt; ++t) {
        uint32_t g[R];
        uint64_t h[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const uint32_t i = i0 + u * blockDim.x;
          g[u] = 0xffffffffu;
          h[u] = 0;
          if (i < hi) {
            const uint32_t* r = recs + (uint64_t)i * rw;
            g[u] = r[0];
            h[u] = (uint64_t)r[hoff + 2 * t] | ((uint64_t)r[hoff + 2 * t + 1] << 32);
          }
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
          if (g[u] >= (uint32_t)G) continue;  // (past the region's end; never fault)
          const int64_t idx = (((int64_t)t * G + g[u]) << bits) + (int64_t)(h[u] >> shift);
          if (use_lds) atomicAdd(&lh[idx], 1u);
          else atomicAdd(&hist[idx], 1u);
        }
      }
    }
  }
  if (use_lds) {
    __syncthreads();
    for (int64_t i = threadIdx.x; i < nb; i += blockDim.x)
      if (lh[i]) atomicAdd(&hist[i], lh[i]);
  }
}

// One chunk region per block step: a count pass over the region's records (<= 4096: 16 per thread,
// kept as bits), a block scan, ONE global atomic for the region's output range, then a write pass
// (the records are re-read from L2).  A per-wave atomic on the single output cursor serialized
// ~1M atomics on one address at SF10 (10 of a 17 ms theta query).
__global__ void __launch_bounds__(256) theta_filter_regions_kernel(const uint32_t* __restrict__ recs, int rw, int hoff,
                                                                  const uint32_t* __restrict__ seg_lo,
                                                                  const uint32_t* __restrict__ seg_hi, int64_t nseg,
                                                                  int G, const int64_t* __restrict__ bound,
                                                                  int64_t* __restrict__ out_g, int64_t* __restrict__ out_h,
                                                                  unsigned long long* __restrict__ count, int64_t cap,
                                                                  int nt) {
  // nt <= 4 sketches per record: bit j * nt + t of `bits` = record j passes sketch t's bound
  // (bound[t * G + g]); its candidate is written as group t * G + g
  __shared__ uint32_t wsum[4];
  __shared__ unsigned long long s_base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t sgi = blockIdx.x; sgi < nseg; sgi += gridDim.x) {
    const uint32_t lo = seg_lo[sgi], hi = seg_hi[sgi];
    if (hi <= lo) continue;  // (uniform: every thread reads the same region bounds)
    uint64_t bits = 0;
    uint32_t mine = 0;
    const int per = 64 / nt;  // records per thread the bit set can hold (a region: <= 16)
    for (uint32_t j = 0, i = lo + threadIdx.x; i < hi && j < (uint32_t)per; ++j, i += blockDim.x) {
      const uint32_t* r = recs + (uint64_t)i * rw;
      const uint32_t g = r[0];
      if (g >= (uint32_t)G) continue;
      for (int t = 0; t < nt; ++t) {
        const uint64_t h = (uint64_t)r[hoff + 2 * t] | ((uint64_t)r[hoff + 2 * t + 1] << 32);
        if ((int64_t)h < bound[(int64_t)t * G + g]) {
          bits |= 1ull << (j * nt + t);
          ++mine;
        }
      }
    }
    // block exclusive scan of the per-thread counts
    uint32_t x = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(x, d, 64);
      if (lane >= d) x += t;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t pre = x - mine, tot = 0;
    for (int w = 0; w < 4; ++w) {
      tot += wsum[w];
      if (w < wave) pre += wsum[w];
    }
    if (threadIdx.x == 0) s_base = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
    __syncthreads();
    unsigned long long pos = s_base + pre;
    for (uint32_t j = 0, i = lo + threadIdx.x; j < (uint32_t)per && (bits >> (j * nt)); ++j, i += blockDim.x) {
      const uint32_t* r = recs + (uint64_t)i * rw;
      for (int t = 0; t < nt; ++t) {
        if (!((bits >> (j * nt + t)) & 1ull)) continue;
        if ((int64_t)pos < cap) {
          out_g[pos] = (int64_t)t * G + (int64_t)r[0];
          out_h[pos] = (int64_t)((uint64_t)r[hoff + 2 * t] | ((uint64_t)r[hoff + 2 * t + 1] << 32));
        }
        ++pos;
      }
    }
    __syncthreads();  // (wsum / s_base are rewritten for the next region)
  }
}

}  // namespace sdo
