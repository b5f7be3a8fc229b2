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
