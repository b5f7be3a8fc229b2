// Host-side launchers + pybind11 module for the CDNA4 OLAP kernels.  All device pointers cross
// the Python boundary as integers (torch.Tensor.data_ptr()) and streams as raw hipStream_t
// handles (torch.cuda.current_stream().cuda_stream), so this module needs no torch headers and
// builds in seconds with hipcc.  It must be imported after torch so that the HIP runtime torch
// loaded (same SONAME) is the one this module binds to.
#include <hip/hip_runtime.h>
#include <sys/prctl.h>
#include <hip/hiprtc.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <chrono>
#include <stdexcept>
#include <string>
#include <tuple>

#include "p2p.h"
#include <vector>
#include "scan_desc.h"
#include "post_scan.h"

namespace sdo {
template <int U>
__global__ void olap_scan_kernel(const ScanDesc* __restrict__ d);
__global__ void bitmap_build_kernel(const void* ids, int dtype, int64_t n, int64_t nwords, uint64_t* out,
                                    int64_t card);
__global__ void hll_estimate_kernel(const unsigned char* regs, int64_t G, int p, double* est);
__global__ void glds_probe_kernel(const unsigned char* src, uint32_t* out);
// post_scan.hip
__global__ void compact_count_kernel(const uint64_t* mask, int64_t nwords, int* block_counts);
__global__ void compact_offsets_kernel(const int* block_counts, int64_t nblocks, int64_t* offsets, int64_t* total);
__global__ void compact_write_kernel(const uint64_t* mask, int64_t nwords, const int64_t* offsets, int64_t* rows);
__global__ void topk_hist_kernel(const int64_t* acc, int64_t n, int nslots, int slot, int is_f64, int desc,
                                 const uint64_t* state, int level, unsigned int* hist);
__global__ void topk_pick_kernel(unsigned int* hist, uint64_t* state, int level);
__global__ void nonzero_mask_kernel(const unsigned char* base, int esize, int64_t n, int64_t stride, uint64_t* words);
__global__ void nonzero_mask_u8_kernel(const unsigned char* base, int64_t n, uint64_t* words);
__global__ void histogram_kernel(const int64_t* keys, int64_t n, int64_t nbins, unsigned int* counts);
__global__ void histogram_lds_kernel(const int64_t* keys, int64_t n, int nbins, unsigned int* counts);
__global__ void touch_count_kernel(const uint4* touch, int64_t nwords, uint64_t* words, int* block_counts);
__global__ void touch_gather_kernel(const uint64_t* words, int64_t nwords, const int64_t* offsets, int64_t* acc, int ns,
                                    const int64_t* init, unsigned char* touch, int64_t* out_idx, int64_t* out_acc);
__global__ void sparse_decode_kernel(DecArgs a);
struct ResetArgs {
  int64_t* acc;
  const int64_t* init;
  int64_t rows;
  int nslots;
  int nz;
  uint64_t* z[4];
  int64_t zn[4];
  int* overflow;
};
__global__ void reset_bufs_kernel(ResetArgs a);
__global__ void topk_keep_kernel(const int64_t* acc, int64_t n, int nslots, int slot, int is_f64, int desc,
                                 const uint64_t* state, uint64_t* keep);
// sketch.hip
__global__ void hll_pairs_kernel(const int64_t* vals, int64_t n, int p, int64_t salt, int32_t* out);
__global__ void hll_merge_stored_kernel(const int64_t* rows, const int64_t* gid, int64_t nsel, const int64_t* offsets,
                                        const int32_t* pairs, int p, int64_t G, unsigned char* regs);
// partition.hip
__global__ void part_rowscan_small_kernel(uint32_t* c, int64_t R, int B, uint32_t* totals);
__global__ void part_rowscan_kernel(uint32_t* c, int64_t R, int B, uint32_t* totals);
__global__ void part_basescan_kernel(const uint32_t* totals, int64_t R, uint32_t* base);
__global__ void part_keys_kernel(const int64_t* keys, int64_t n, int shift1, int P1, uint32_t* counts1,
                                 const uint32_t* base1, uint32_t* out, int phase);
template <int PU, bool CL>
__global__ void part_split_kernel(const uint32_t* in, int RW, int RS, const uint32_t* seg_lo, const uint32_t* seg_hi, int spg,
                                  int K, int shift2, int P2, uint32_t* counts2, const uint32_t* base2, uint32_t* out,
                                  int phase, int pk_w);
__global__ void part_hash_agg_kernel(const uint32_t* recs, int RW, const uint32_t* base, int64_t nsub, int cap_log2,
                                     PartFields f, PartHll hl, PartHaving hv, int64_t* out_keys, uint64_t* out_acc,
                                     unsigned long long* out_count, int64_t cap, int* overflow);
__global__ void part_agg_kernel(const uint32_t* recs, int RW, const uint32_t* base, int64_t nsub, int64_t G, int shift,
                                PartFields f, PartHll hl, uint64_t* gacc, PartHaving hv, int64_t* out_keys,
                                unsigned long long* out_count, int64_t cap);
__global__ void theta_hist_regions_kernel(const uint32_t* recs, int rw, int hoff, const uint32_t* seg_lo,
                                          const uint32_t* seg_hi, int64_t nseg, int G, int bits, uint32_t* hist,
                                          int use_lds, int nt);
__global__ void theta_filter_regions_kernel(const uint32_t* recs, int rw, int hoff, const uint32_t* seg_lo,
                                            const uint32_t* seg_hi, int64_t nseg, int G, const int64_t* bound,
                                            int64_t* out_g, int64_t* out_h, unsigned long long* count, int64_t cap,
                                            int nt);
__global__ void theta_hist_kernel(const int64_t* g, const int64_t* h, int64_t n, int bits, uint32_t* hist);
__global__ void theta_thresh_kernel(const uint32_t* hist, int bits, const int64_t* target, int64_t* bound);
__global__ void theta_filter_kernel(const int64_t* g, const int64_t* h, int64_t n, const int64_t* bound,
                                    int64_t* out_g, int64_t* out_h, unsigned long long* count, int64_t cap);
// p2p.hip (P2PArgs: p2p.h)
__global__ void p2p_merge_kernel(P2PArgs a);
}  // namespace sdo

namespace py = pybind11;

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Host waits for a stream (every native sync: fetch_small, sparse_decode, d2h, stream_sync).  HIP's
// own wait spins the thread's core for the whole wait (tools/sync_cpu_probe.py: CPU time == wall
// time), which is right for sub-millisecond scans and wasteful for a server's 10-50 ms partitioned
// group-bys, whose executor threads then burn the cores the clients and compile threads need
// (exec_thread_cpu_ms).  Hybrid: poll for g_wait_spin_us -- 2 ms, longer than every headline scan
// (TPC-H Q1 at SF100 waits ~1.05 ms), so their latency is unchanged -- then sleep between polls
// (20 us, then 40, then 50 us: a long wait ends at most ~50 us late, ~1 us of CPU per poll; naps
// capped at 200 us left a 0.25 ms gap after TopVolumeCustomers' aggregation,
// profiles/r6/rocprof_bi_topvolume_sf100_packed.txt).
static int64_t g_wait_spin_us = 2000;
static void set_wait_spin(int64_t us) {
  if (us < 0) throw std::invalid_argument("set_wait_spin: microseconds >= 0");
  g_wait_spin_us = us;
}
static void wait_stream(hipStream_t st, const char* what) {
  // (a thread's first sleeping wait drops its timer slack to 1 us: Linux otherwise rounds a 20 us
  // nap up by its default 50 us slack, and the statement's end is seen that much later)
  static thread_local bool slack_set = false;
  const auto t0 = std::chrono::steady_clock::now();
  int64_t nap = 20;
  while (true) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) check(e, what);
    const int64_t el =
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    if (el < g_wait_spin_us) continue;
    if (!slack_set) {
      prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
      slack_set = true;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(nap));
    nap = nap * 2 > 50 ? 50 : nap * 2;
  }
}

static void scan(uint64_t desc, int grid, int block, int lds, int unroll, uint64_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (block % 64 != 0 || block > 512 || block <= 0) throw std::invalid_argument("block must be a multiple of 64 <= 512");
  if (lds < 0 || lds > 160 * 1024) throw std::invalid_argument("lds bytes out of range");
  if (grid <= 0) return;
  const void* f;
  switch (unroll) {
    case 1: f = (const void*)sdo::olap_scan_kernel<1>; break;
    case 2: f = (const void*)sdo::olap_scan_kernel<2>; break;
    case 4: f = (const void*)sdo::olap_scan_kernel<4>; break;
    default: throw std::invalid_argument("unroll must be 1, 2 or 4");
  }
  if (lds > 65536) {
    check(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), "hipFuncSetAttribute");
  }
  void* args[] = {(void*)&desc};
  check(hipLaunchKernel(f, dim3(grid), dim3(block), args, (size_t)lds, s), "olap_scan_kernel launch");
}

static void bitmap_build(uint64_t ids, int dtype, int64_t n, int64_t nwords, uint64_t out, int64_t card,
                         uint64_t stream) {
  if (nwords <= 0) return;
  int64_t blocks = (nwords + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(sdo::bitmap_build_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const void*)ids, dtype, n, nwords, (uint64_t*)out, card);
  check(hipGetLastError(), "bitmap_build_kernel launch");
}

static void hll_estimate(uint64_t regs, int64_t G, int p, uint64_t est, uint64_t stream) {
  if (G <= 0) return;
  if (p < 4 || p > 18) throw std::invalid_argument("hll precision out of range");
  if (p < 7) throw std::invalid_argument("hll estimate needs >= 128 registers (128-register column chunks)");
  const unsigned blocks = (unsigned)((G + 31) / 32);
  hipLaunchKernelGGL(sdo::hll_estimate_kernel, dim3(blocks), dim3(8 * 64), 0, (hipStream_t)stream,
                     (const unsigned char*)regs, G, p, (double*)est);
  check(hipGetLastError(), "hll_estimate_kernel launch");
}

// ---------------------------------------------------------------------------------------------
// Stored HLL sketches (sketch.hip)
static unsigned grid_for(int64_t n, int64_t per_block, int64_t cap) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (unsigned)b;
}

static void hll_pairs(uint64_t vals, int64_t n, int p, int64_t salt, uint64_t out, uint64_t stream) {
  if (n <= 0) return;
  if (p < 4 || p > 18) throw std::invalid_argument("hll precision out of range");
  hipLaunchKernelGGL(sdo::hll_pairs_kernel, dim3(grid_for(n, 256, 65536)), dim3(256), 0, (hipStream_t)stream,
                     (const int64_t*)vals, n, p, salt, (int32_t*)out);
  check(hipGetLastError(), "hll_pairs_kernel launch");
}

static void hll_merge_stored(uint64_t rows, uint64_t gid, int64_t nsel, uint64_t offsets, uint64_t pairs, int p,
                             int64_t G, uint64_t regs, uint64_t stream) {
  if (nsel <= 0 || G <= 0) return;
  if (p < 4 || p > 18) throw std::invalid_argument("hll precision out of range");
  hipLaunchKernelGGL(sdo::hll_merge_stored_kernel, dim3(grid_for(nsel, 256, 65536)), dim3(256), 0,
                     (hipStream_t)stream, (const int64_t*)rows, (const int64_t*)gid, nsel, (const int64_t*)offsets,
                     (const int32_t*)pairs, p, G, (unsigned char*)regs);
  check(hipGetLastError(), "hll_merge_stored_kernel launch");
}

// ---------------------------------------------------------------------------------------------
// Row compaction (post_scan.hip): mask words -> sorted row ids.  65536 rows (1024 words) per block.
static int64_t compact_blocks(int64_t nwords) { return (nwords + 1023) / 1024; }

static void compact_count(uint64_t mask, int64_t nwords, uint64_t block_counts, uint64_t offsets, uint64_t total,
                          uint64_t stream) {
  const int64_t nb = compact_blocks(nwords);
  if (nb <= 0) return;
  if (nb > (int64_t)1 << 31) throw std::invalid_argument("mask too large");
  hipLaunchKernelGGL(sdo::compact_count_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream,
                     (const uint64_t*)mask, nwords, (int*)block_counts);
  check(hipGetLastError(), "compact_count_kernel launch");
  hipLaunchKernelGGL(sdo::compact_offsets_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                     (const int*)block_counts, nb, (int64_t*)offsets, (int64_t*)total);
  check(hipGetLastError(), "compact_offsets_kernel launch");
}

static void compact_write(uint64_t mask, int64_t nwords, uint64_t offsets, uint64_t rows, uint64_t stream) {
  const int64_t nb = compact_blocks(nwords);
  if (nb <= 0) return;
  hipLaunchKernelGGL(sdo::compact_write_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream,
                     (const uint64_t*)mask, nwords, (const int64_t*)offsets, (int64_t*)rows);
  check(hipGetLastError(), "compact_write_kernel launch");
}

// First-touch compaction (post_scan.hip touch_*): pass 1 + offsets; the caller reads the total,
// sizes the outputs and runs pass 3.  The byte table holds nwords * 64 bytes.
static void touch_count(uint64_t touch, int64_t nwords, uint64_t words, uint64_t block_counts, uint64_t offsets,
                        uint64_t total, uint64_t stream) {
  const int64_t nb = compact_blocks(nwords);
  if (nb <= 0) return;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sdo::touch_count_kernel, dim3((unsigned)nb), dim3(256), 0, s, (const uint4*)touch, nwords,
                     (uint64_t*)words, (int*)block_counts);
  check(hipGetLastError(), "touch_count_kernel launch");
  hipLaunchKernelGGL(sdo::compact_offsets_kernel, dim3(1), dim3(1024), 0, s, (const int*)block_counts, nb,
                     (int64_t*)offsets, (int64_t*)total);
  check(hipGetLastError(), "compact_offsets_kernel launch");
}

static void touch_gather(uint64_t words, int64_t nwords, uint64_t offsets, uint64_t acc, int ns, uint64_t init,
                         uint64_t touch, uint64_t out_idx, uint64_t out_acc, uint64_t stream) {
  const int64_t nb = compact_blocks(nwords);
  if (nb <= 0) return;
  if (ns < 1 || ns > sdo::MAX_SLOTS) throw std::invalid_argument("touch_gather: slot count");
  hipLaunchKernelGGL(sdo::touch_gather_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream,
                     (const uint64_t*)words, nwords, (const int64_t*)offsets, (int64_t*)acc, ns, (const int64_t*)init,
                     (unsigned char*)touch, (int64_t*)out_idx, (int64_t*)out_acc);
  check(hipGetLastError(), "touch_gather_kernel launch");
}

// Sparse result decode (post_scan.hip sparse_decode_kernel) into one device buffer, then one copy
// of ``nbytes`` into the pinned host buffer and one stream sync (GIL released while waiting).
// cols: (kind, out, lut_t, slot, stride, card, add, orig, lut, div, off)
using DecTuple = std::tuple<int, int, int, int, int64_t, int64_t, int64_t, uint64_t, uint64_t, double, int64_t>;
static void sparse_decode(uint64_t idx, uint64_t acc, int64_t n, int ns, std::vector<DecTuple> cols, uint64_t out,
                          int64_t nbytes, uint64_t host, uint64_t stream) {
  if ((int)cols.size() > sdo::DEC_MAX_COLS) throw std::invalid_argument("sparse_decode: too many columns");
  sdo::DecArgs a{};
  a.idx = (const int64_t*)idx;
  a.acc = (const int64_t*)acc;
  a.n = n;
  a.ns = ns;
  a.ncols = (int)cols.size();
  a.out = (unsigned char*)out;
  for (size_t j = 0; j < cols.size(); ++j) {
    auto& c = a.c[j];
    c.kind = std::get<0>(cols[j]);
    c.out = std::get<1>(cols[j]);
    c.lut_t = std::get<2>(cols[j]);
    c.slot = std::get<3>(cols[j]);
    c.stride = std::get<4>(cols[j]);
    c.card = std::get<5>(cols[j]);
    c.add = std::get<6>(cols[j]);
    c.orig = (const int64_t*)std::get<7>(cols[j]);
    c.lut = (const void*)std::get<8>(cols[j]);
    c.div = std::get<9>(cols[j]);
    c.off = std::get<10>(cols[j]);
    if (c.kind < 0 || c.kind > 4 || c.out < 0 || c.out > 5 || c.lut_t < 0 || c.lut_t > 3)
      throw std::invalid_argument("sparse_decode: column kind");
    if (c.kind == 0 && (c.stride <= 0 || c.card <= 0)) throw std::invalid_argument("sparse_decode: key stride/card");
    if ((c.kind == 1 || c.kind == 2 || c.kind == 3) && (c.slot < 0 || c.slot >= ns))
      throw std::invalid_argument("sparse_decode: slot");
    if (c.lut_t && !c.lut) throw std::invalid_argument("sparse_decode: table pointer");
    const int64_t width = c.out == 0 ? 2 : (c.out == 1 ? 4 : 8);
    if (c.off < 0 || c.off % width || c.off + n * width > nbytes) throw std::invalid_argument("sparse_decode: column offset");
  }
  hipStream_t st = (hipStream_t)stream;
  if (n > 0 && !cols.empty()) {
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(sdo::sparse_decode_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
    check(hipGetLastError(), "sparse_decode_kernel launch");
  }
  py::gil_scoped_release nogil;
  if (nbytes > 0) check(hipMemcpyAsync((void*)host, (const void*)out, nbytes, hipMemcpyDeviceToHost, st), "sparse_decode copy");
  wait_stream(st, "sparse_decode sync");
}

static void nonzero_mask(uint64_t base, int esize, int64_t n, int64_t stride, uint64_t words, uint64_t stream) {
  if (n <= 0) return;
  if (esize != 1 && esize != 8) throw std::invalid_argument("esize must be 1 or 8");
  int64_t nwords = (n + 63) / 64;
  if (esize == 1 && stride == 1 && (base & 15) == 0) {  // contiguous bytes: 16-byte loads
    int64_t nchunks = (n + 1023) / 1024;
    int64_t blocks = (nchunks + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(sdo::nonzero_mask_u8_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned char*)base, n, (uint64_t*)words);
    check(hipGetLastError(), "nonzero_mask_u8_kernel launch");
    return;
  }
  int64_t blocks = (nwords + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(sdo::nonzero_mask_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned char*)base, esize, n, stride, (uint64_t*)words);
  check(hipGetLastError(), "nonzero_mask_kernel launch");
}

static void histogram(uint64_t keys, int64_t n, int64_t nbins, uint64_t counts, uint64_t stream) {
  if (n <= 0 || nbins <= 0) return;
  if (nbins <= 16384) {  // LDS-privatised counts (64 KB at most)
    int64_t blocks = (n + 4095) / 4096;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(sdo::histogram_lds_kernel, dim3((unsigned)blocks), dim3(256), (unsigned)(nbins * 4),
                       (hipStream_t)stream, (const int64_t*)keys, n, (int)nbins, (unsigned int*)counts);
    check(hipGetLastError(), "histogram_lds_kernel launch");
    return;
  }
  int64_t blocks = (n + 1023) / 1024;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(sdo::histogram_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const int64_t*)keys, n, nbins, (unsigned int*)counts);
  check(hipGetLastError(), "histogram_kernel launch");
}

// One-launch re-initialisation of a prepared scan's buffers (post_scan.hip reset_bufs_kernel).
static void reset_bufs(uint64_t acc, uint64_t init, int64_t rows, int nslots, std::vector<uint64_t> zptr,
                       std::vector<int64_t> zwords, uint64_t overflow, uint64_t stream) {
  if (zptr.size() != zwords.size() || zptr.size() > 4) throw std::invalid_argument("at most 4 zero regions");
  sdo::ResetArgs a{};
  a.acc = (int64_t*)acc;
  a.init = (const int64_t*)init;
  a.rows = acc ? rows : 0;
  a.nslots = nslots;
  a.nz = (int)zptr.size();
  int64_t work = a.rows * nslots;
  for (size_t i = 0; i < zptr.size(); ++i) {
    a.z[i] = (uint64_t*)zptr[i];
    a.zn[i] = zwords[i];
    if (zwords[i] > work) work = zwords[i];
  }
  a.overflow = (int*)overflow;
  int64_t blocks = (work + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(sdo::reset_bufs_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  check(hipGetLastError(), "reset_bufs_kernel launch");
}

// Top-k threshold (post_scan.hip): 4 radix levels of histogram + pick, then the keep bitmask.
// state: 3 x uint64 {prefix, k, all} initialised to {0, k, 0}; hist: 4096 x uint32 zeroed.
static void topk_keep(uint64_t acc, int64_t n, int nslots, int slot, int is_f64, int desc, uint64_t state,
                      uint64_t hist, uint64_t keep, int grid, uint64_t stream) {
  if (n <= 0) return;
  if (slot < 0 || slot >= nslots) throw std::invalid_argument("bad slot");
  hipStream_t s = (hipStream_t)stream;
  for (int level = 0; level < 4; ++level) {  // TK_LEVELS
    hipLaunchKernelGGL(sdo::topk_hist_kernel, dim3(grid), dim3(512), 0, s, (const int64_t*)acc, n, nslots, slot, is_f64,
                       desc, (const uint64_t*)state, level, (unsigned int*)hist);
    check(hipGetLastError(), "topk_hist_kernel launch");
    hipLaunchKernelGGL(sdo::topk_pick_kernel, dim3(1), dim3(1024), 0, s, (unsigned int*)hist, (uint64_t*)state, level);
    check(hipGetLastError(), "topk_pick_kernel launch");
  }
  hipLaunchKernelGGL(sdo::topk_keep_kernel, dim3(grid), dim3(256), 0, s, (const int64_t*)acc, n, nslots, slot, is_f64,
                     desc, (const uint64_t*)state, (uint64_t*)keep);
  check(hipGetLastError(), "topk_keep_kernel launch");
}

// Returns 4 when 1/2-byte LDS-DMA elements land one dword per lane, 1 when packed (lane*size).
static int glds_probe() {
  unsigned char h_src[256];
  for (int i = 0; i < 256; ++i) h_src[i] = (unsigned char)(i + 1);
  unsigned char* d_src = nullptr;
  uint32_t* d_out = nullptr;
  check(hipMalloc(&d_src, 256), "hipMalloc");
  check(hipMalloc(&d_out, 128 * 4), "hipMalloc");
  check(hipMemcpy(d_src, h_src, 256, hipMemcpyHostToDevice), "hipMemcpy");
  hipLaunchKernelGGL(sdo::glds_probe_kernel, dim3(1), dim3(64), 0, 0, d_src, d_out);
  check(hipGetLastError(), "glds_probe launch");
  uint32_t h_out[128];
  check(hipMemcpy(h_out, d_out, sizeof(h_out), hipMemcpyDeviceToHost), "hipMemcpy");
  (void)hipFree(d_src);
  (void)hipFree(d_out);
  bool dword = true, packed = true;
  for (int l = 0; l < 64; ++l) {
    if ((h_out[l] & 0xff) != (uint32_t)((l + 1) & 0xff)) dword = false;
    if (((const unsigned char*)h_out)[l] != (unsigned char)(l + 1)) packed = false;
  }
  if (dword) return 4;
  if (packed) return 1;
  return -1;
}

// ---------------------------------------------------------------------------------------------
// Per-query JIT kernels (ops/jit.py): hipRTC compile -> code object bytes (cached on disk by the
// caller) -> hipModuleLoadData -> launch.  Compilation needs no GPU.
//
// A compile takes 0.3-2 s of host CPU: it runs with the GIL released, so serving threads (plan,
// launch, encode) keep running while a background literal specialization or a first-seen shape
// compiles (ops/jit.py compile_source runs different shapes' compiles in parallel).
static std::string rtc_compile_nogil(const std::string& src, const std::string& name,
                                     const std::vector<std::string>& opts) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), (name + ".hip").c_str(), 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    throw std::runtime_error("hiprtcCreateProgram failed");
  std::vector<const char*> o;
  for (auto& x : opts) o.push_back(x.c_str());
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)o.size(), o.data());
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  std::string log(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("hiprtc compile failed: " + log);
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::string code(cs, '\0');
  hiprtcGetCode(prog, &code[0]);
  hiprtcDestroyProgram(&prog);
  return code;
}

static py::bytes rtc_compile(const std::string& src, const std::string& name, const std::vector<std::string>& opts) {
  std::string code;
  {
    py::gil_scoped_release nogil;
    code = rtc_compile_nogil(src, name, opts);
  }
  return py::bytes(code);
}

struct JitKernel {
  hipModule_t mod;
  hipFunction_t fn;
};
static std::vector<JitKernel> g_jit;
static std::mutex g_jit_mu;

static int module_load(const std::string& code, const std::string& name) {
  JitKernel k;
  check(hipModuleLoadData(&k.mod, code.data()), "hipModuleLoadData");
  check(hipModuleGetFunction(&k.fn, k.mod, name.c_str()), "hipModuleGetFunction");
  std::lock_guard<std::mutex> g(g_jit_mu);
  g_jit.push_back(k);
  return (int)g_jit.size() - 1;
}

static void module_launch(int h, uint64_t desc, int grid, int block, int lds, uint64_t stream) {
  hipFunction_t fn;
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    if (h < 0 || h >= (int)g_jit.size()) throw std::invalid_argument("bad jit handle");
    fn = g_jit[h].fn;
  }
  if (block % 64 != 0 || block > 1024 || block <= 0) throw std::invalid_argument("bad block size");
  if (lds < 0 || lds > 160 * 1024) throw std::invalid_argument("lds bytes out of range");
  if (grid <= 0) return;
  void* args[] = {(void*)&desc};
  check(hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, (unsigned)lds, (hipStream_t)stream, args, nullptr),
        "jit kernel launch");
}

// Resident workgroups per CU of a JIT kernel at this block size and dynamic LDS (VGPR / SGPR / LDS
// limits of the compiled code): the persistent scan grid is sized to what is resident at once --
// a grid of 3 blocks per CU for a 117-VGPR kernel that fits 2 leaves a second, half-empty wave of
// workgroups (TPC-H Q1 at SF100: 1.56 -> 1.46 ms at 2 per CU).
static int module_occupancy(int h, int block, int lds) {
  hipFunction_t fn;
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    if (h < 0 || h >= (int)g_jit.size()) throw std::invalid_argument("bad jit handle");
    fn = g_jit[h].fn;
  }
  int n = 0;
  check(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, block, (size_t)lds), "occupancy");
  return n;
}

static py::dict module_attrs(int h) {
  hipFunction_t fn;
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    if (h < 0 || h >= (int)g_jit.size()) throw std::invalid_argument("bad jit handle");
    fn = g_jit[h].fn;
  }
  py::dict d;
  int v = 0;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_NUM_REGS, fn) == hipSuccess) d["num_regs"] = v;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, fn) == hipSuccess) d["local_bytes"] = v;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, fn) == hipSuccess) d["max_threads"] = v;
  return d;
}

// One host call per execution of a prepared scan: the fused reset of its slot buffers, then the
// specialized kernel (or the interpreter) -- the Python side caches every argument, so a small
// query's launch path is a single pybind call (the per-call Python work showed as ~25 us of a
// 0.2 ms query on the benchmark host).
static void run_scan(uint64_t acc, uint64_t init, int64_t rows, int nslots, std::vector<uint64_t> zptr,
                     std::vector<int64_t> zwords, uint64_t overflow, int jit, uint64_t desc, int grid, int block,
                     int lds, int unroll, uint64_t stream) {
  if (acc || !zptr.empty() || overflow) reset_bufs(acc, init, rows, nslots, zptr, zwords, overflow, stream);
  if (jit >= 0) module_launch(jit, desc, grid, block, lds, stream);
  else scan(desc, grid, block, lds, unroll, stream);
}

// Small dense result: HLL estimates of every register block (MFMA kernel) + the accumulator table
// and the estimates copied into one pinned host buffer + a stream synchronisation, in one call with
// the GIL released while the device works.
static void fetch_small(uint64_t acc, int64_t acc_bytes, std::vector<uint64_t> hll, int64_t G, int p,
                        uint64_t est_dev, uint64_t host, uint64_t stream) {
  hipStream_t st = (hipStream_t)stream;
  for (size_t i = 0; i < hll.size(); ++i) hll_estimate(hll[i], G, p, est_dev + i * (uint64_t)G * 8, stream);
  py::gil_scoped_release nogil;
  if (acc_bytes > 0)
    check(hipMemcpyAsync((void*)host, (const void*)acc, acc_bytes, hipMemcpyDeviceToHost, st), "fetch_small acc");
  if (!hll.empty())
    check(hipMemcpyAsync((void*)(host + acc_bytes), (const void*)est_dev, hll.size() * G * 8, hipMemcpyDeviceToHost, st),
          "fetch_small est");
  wait_stream(st, "fetch_small sync");
}

// fetch_small, then this scan's buffers reset for its next execution -- enqueued behind the copies
// while the scan still runs, so the reset leaves the next launch's critical path; the host waits
// for the copies only (an event recorded before the reset), not for the reset.
static void fetch_small_reset(uint64_t acc, int64_t acc_bytes, std::vector<uint64_t> hll, int64_t G, int p,
                              uint64_t est_dev, uint64_t host, uint64_t init, int64_t rows, int nslots,
                              std::vector<uint64_t> zptr, std::vector<int64_t> zwords, uint64_t overflow,
                              uint64_t stream) {
  hipStream_t st = (hipStream_t)stream;
  thread_local hipEvent_t ev = nullptr;
  if (!ev) check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "fetch_small_reset event");
  for (size_t i = 0; i < hll.size(); ++i) hll_estimate(hll[i], G, p, est_dev + i * (uint64_t)G * 8, stream);
  if (acc_bytes > 0)
    check(hipMemcpyAsync((void*)host, (const void*)acc, acc_bytes, hipMemcpyDeviceToHost, st), "fetch_small acc");
  if (!hll.empty())
    check(hipMemcpyAsync((void*)(host + acc_bytes), (const void*)est_dev, hll.size() * G * 8, hipMemcpyDeviceToHost, st),
          "fetch_small est");
  check(hipEventRecord(ev, st), "fetch_small_reset record");
  reset_bufs(acc, init, rows, nslots, zptr, zwords, overflow, stream);
  py::gil_scoped_release nogil;
  check(hipEventSynchronize(ev), "fetch_small_reset wait");
}

static void stream_sync(uint64_t stream) {
  py::gil_scoped_release nogil;
  wait_stream((hipStream_t)stream, "stream sync");
}

// Device int64 words -> host behind the stream's work, ONE wait (the partitioned aggregation's
// survivor count and overflow flag): a copy into this thread's pinned words, then the stream wait
// -- instead of a wait for the kernels and a second round trip for each .item().
static std::vector<int64_t> read_words(std::vector<uint64_t> ptrs, std::vector<int> bytes, uint64_t stream) {
  static thread_local int64_t* pin = nullptr;
  if (ptrs.size() > 16 || bytes.size() != ptrs.size()) throw std::invalid_argument("read_words: <= 16 (ptr, bytes)");
  for (int b : bytes)
    if (b != 4 && b != 8) throw std::invalid_argument("read_words: 4- or 8-byte words");
  std::vector<int64_t> out(ptrs.size());
  {
    py::gil_scoped_release nogil;
    if (!pin) check(hipHostMalloc((void**)&pin, 16 * sizeof(int64_t), hipHostMallocDefault), "read_words pin");
    for (size_t i = 0; i < ptrs.size(); ++i) {
      pin[i] = 0;
      check(hipMemcpyAsync(pin + i, (const void*)ptrs[i], (size_t)bytes[i], hipMemcpyDeviceToHost, (hipStream_t)stream),
            "read_words copy");
    }
    wait_stream((hipStream_t)stream, "read_words");
    for (size_t i = 0; i < ptrs.size(); ++i) out[i] = bytes[i] == 4 ? (int64_t)(int32_t)pin[i] : pin[i];
  }
  return out;
}

// ---------------------------------------------------------------------------------------------
// Radix-partitioned group-by (partition.hip).  Every launch below is sized from host-known layout
// numbers (buckets, blocks); record counts stay on the device (no synchronisation per run).
static void part_scan(uint64_t counts, int64_t R, int B, uint64_t totals, uint64_t base, uint64_t stream) {
  if (R <= 0 || B <= 0) return;
  hipStream_t s = (hipStream_t)stream;
  if (B <= 64) {
    hipLaunchKernelGGL(sdo::part_rowscan_small_kernel, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s,
                       (uint32_t*)counts, R, B, (uint32_t*)totals);
  } else {
    const int64_t g = R < 65536 ? R : 65536;
    hipLaunchKernelGGL(sdo::part_rowscan_kernel, dim3((unsigned)g), dim3(256), 0, s, (uint32_t*)counts, R, B,
                       (uint32_t*)totals);
  }
  check(hipGetLastError(), "part_rowscan launch");
  hipLaunchKernelGGL(sdo::part_basescan_kernel, dim3(1), dim3(1024), 0, s, (const uint32_t*)totals, R,
                     (uint32_t*)base);
  check(hipGetLastError(), "part_basescan launch");
}

static void part_keys(uint64_t keys, int64_t n, int shift1, int P1, uint64_t counts1, uint64_t base1, uint64_t out,
                      int phase, int grid, uint64_t stream) {
  if (n <= 0 || grid <= 0) return;
  if (P1 <= 0 || P1 > 16384) throw std::invalid_argument("part_keys: 1..16384 buckets");
  hipLaunchKernelGGL(sdo::part_keys_kernel, dim3(grid), dim3(512), (unsigned)(P1 * 4), (hipStream_t)stream,
                     (const int64_t*)keys, n, shift1, P1, (uint32_t*)counts1, (const uint32_t*)base1,
                     (uint32_t*)out, phase);
  check(hipGetLastError(), "part_keys_kernel launch");
}

// Probe knob (tools/part_probe.py A/B runs): records per thread of the scatter tile (0: by width).
static int g_part_pu = 0;
static int64_t g_part_lds_min = 0;  // (probe: pad the scatter's LDS request -> fewer blocks per CU)
static void part_tune(int pu, int64_t lds_min = 0) {
  if (pu != 0 && pu != 1 && pu != 2 && pu != 4 && pu != 8 && pu != 16 && pu != 32)
    throw std::invalid_argument("part_tune: pu in {0,1,2,4,8,16,32}");
  if (lds_min < 0 || lds_min > 160 * 1024 - 256) throw std::invalid_argument("part_tune: lds_min");
  g_part_pu = pu;
  g_part_lds_min = lds_min;
}

// groups x K blocks; group g's segments are [g*spg, (g+1)*spg) of seg_lo/seg_hi (a level-1 bucket
// table passes base1 and base1 + 1 with spg = 1).
static void part_split(uint64_t in, int RW, uint64_t seg_lo, uint64_t seg_hi, int64_t groups, int spg, int K,
                       int shift2, int P2, uint64_t counts2, uint64_t base2, uint64_t out, int phase, uint64_t stream) {
  if (groups <= 0 || K <= 0) return;
  if (P2 <= 0 || P2 > 4096 || (P2 & (P2 - 1))) throw std::invalid_argument("part_split: P2 a power of two <= 4096");
  if (RW < 1 || RW > 2 + 2 * sdo::MAX_SLOTS) throw std::invalid_argument("part_split: record width");
  if (spg < 1) throw std::invalid_argument("part_split: segments per group");
  // tile of 512 x PU records: longer same-bucket runs per tile store fuller lines, more LDS per
  // block costs residency.  3-word records (the BI plan's TopVolumeCustomers, 343M records over
  // 512 then 256 buckets at SF100): PU 4 / 8 / 16 scatter at 2.1 / 2.6-2.8 / 1.6-1.8 TB/s; 4-word
  // records 2.3-2.7 / 2.85 TB/s at PU 4 / 8 (tools/part_probe.py, profiles/r6/part_probe_*.txt)
  const int PU = g_part_pu ? g_part_pu : (RW <= 4 ? 8 : (RW <= 8 ? 2 : 1));
  // odd tile stride for even record widths >= 4 (conflict-free strided tile reads) when it fits
  int RS = RW;
  const int64_t lds_max = 160 * 1024 - 256;
  if (RW >= 4 && RW % 2 == 0 && ((int64_t)3 * P2 + (int64_t)512 * PU * (RW + 1)) * 4 <= lds_max) RS = RW + 1;
  // (phase bit 1: clustered keys, see partition.hip part_split_kernel; bits 8+: pk_w, the record
  // word a level-1 scatter packs into the key word above shift2 -- the output is RW - 1 words)
  int pk_w = (phase >> 8) & 0xff;
  phase &= 0xff;
  if ((phase & ~3) != 0) throw std::invalid_argument("part_split: phase");
  if (pk_w && (!(phase & 1) || pk_w >= RW || shift2 < 1 || shift2 > 31))
    throw std::invalid_argument("part_split: packed word");
  int64_t lds = (phase & 1) == 0 ? (int64_t)P2 * 4 : ((int64_t)3 * P2 + (int64_t)512 * PU * RS) * 4;
  if ((phase & 1) && lds < g_part_lds_min) lds = g_part_lds_min;
  if (lds > lds_max) throw std::invalid_argument("part_split: tile does not fit the LDS");
  const bool cl = (phase & 2) != 0;
  phase &= 1;
  const void* f = cl ? (PU == 32 ? (const void*)sdo::part_split_kernel<32, true>
                        : PU == 16 ? (const void*)sdo::part_split_kernel<16, true>
                        : PU == 8 ? (const void*)sdo::part_split_kernel<8, true>
                        : PU == 4 ? (const void*)sdo::part_split_kernel<4, true>
                        : PU == 2 ? (const void*)sdo::part_split_kernel<2, true> : (const void*)sdo::part_split_kernel<1, true>)
                     : (PU == 32 ? (const void*)sdo::part_split_kernel<32, false>
                        : PU == 16 ? (const void*)sdo::part_split_kernel<16, false>
                        : PU == 8 ? (const void*)sdo::part_split_kernel<8, false>
                        : PU == 4 ? (const void*)sdo::part_split_kernel<4, false>
                        : PU == 2 ? (const void*)sdo::part_split_kernel<2, false> : (const void*)sdo::part_split_kernel<1, false>);
  const uint32_t* in_ = (const uint32_t*)in;
  const uint32_t* lo_ = (const uint32_t*)seg_lo;
  const uint32_t* hi_ = (const uint32_t*)seg_hi;
  uint32_t* c2 = (uint32_t*)counts2;
  const uint32_t* b2 = (const uint32_t*)base2;
  uint32_t* o = (uint32_t*)out;
  void* args[] = {(void*)&in_, (void*)&RW, (void*)&RS, (void*)&lo_, (void*)&hi_, (void*)&spg, (void*)&K,
                  (void*)&shift2, (void*)&P2, (void*)&c2, (void*)&b2, (void*)&o, (void*)&phase, (void*)&pk_w};
  if (lds > 64 * 1024) check(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "part_split attr");
  check(hipLaunchKernel(f, dim3((unsigned)(groups * K)), dim3(512), args, (size_t)lds, (hipStream_t)stream),
        "part_split_kernel launch");
  check(hipGetLastError(), "part_split_kernel launch");
}

// having: [] for the dense table, else up to 4 (slot, is_f64, op, divisor, constant) terms; conj 1 = AND.
// With terms, gacc receives the surviving rows ([cap][nslots]), out_keys their keys, out_count
// (zeroed here) their number.
// hll: the [G][2^hll_p] byte register tables of the HLL aggregators the records carry (one word
// each after the value fields), empty for none.
static void part_agg_hll(uint64_t recs, int RW, uint64_t base, int64_t nsub, int64_t G, int shift, std::vector<int> slot,
                         std::vector<int> width, std::vector<int> ops, std::vector<int64_t> init, uint64_t gacc,
                         std::vector<std::tuple<int, int, int, double, double>> having, int conj, uint64_t out_keys,
                         uint64_t out_count, int64_t cap, std::vector<uint64_t> hll, int hll_p, uint64_t stream,
                         std::vector<std::tuple<uint64_t, uint64_t>> stored = {},
                         std::tuple<int, int, int, int> topk = {0, 0, 0, 1}) {
  if (nsub <= 0 || G <= 0) return;
  sdo::PartFields f{};
  if (slot.size() != width.size() || slot.size() > (size_t)sdo::MAX_SLOTS) throw std::invalid_argument("part_agg: fields");
  if (ops.size() != init.size() || ops.empty() || ops.size() > (size_t)sdo::MAX_SLOTS)
    throw std::invalid_argument("part_agg: slots");
  f.nfields = (int)slot.size();
  f.nslots = (int)ops.size();
  int words = 1;
  for (size_t j = 0; j < slot.size(); ++j) {
    // width PART_PACKED | shift << 8: a value the level-1 split packed into the key word above `shift`
    const int wd = width[j] & 0xff;
    if (wd == sdo::PART_PACKED) {
      const int ps = width[j] >> 8;
      if (f.pk_shift || ps < shift || ps > 31) throw std::invalid_argument("part_agg: packed field");
      f.pk_shift = ps;
    } else if (width[j] < 0 || width[j] > 2) {
      throw std::invalid_argument("part_agg: field");
    }
    if (slot[j] < 0 || slot[j] >= f.nslots) throw std::invalid_argument("part_agg: field");
    f.slot[j] = slot[j];
    f.width[j] = wd;
    words += wd == sdo::PART_PACKED ? 0 : wd;
  }
  sdo::PartHll hl{};
  if (hll.size() > (size_t)sdo::PART_MAX_HLL || (!hll.empty() && (hll_p < 4 || hll_p > 16)))
    throw std::invalid_argument("part_agg: HLL aggregators");
  hl.n = (int)hll.size();
  hl.p = hll.empty() ? 0 : hll_p;
  for (size_t h = 0; h < hll.size(); ++h) hl.regs[h] = (unsigned char*)hll[h];
  // stored sketches: the LAST stored.size() register tables, each with its (offsets, pairs) CSR
  if (stored.size() > hll.size()) throw std::invalid_argument("part_agg: stored sketches without register tables");
  for (size_t j = 0; j < stored.size(); ++j) {
    const size_t h = hll.size() - stored.size() + j;
    hl.stored |= 1u << h;
    hl.sk_off[h] = (const int64_t*)std::get<0>(stored[j]);
    hl.sk_val[h] = (const int32_t*)std::get<1>(stored[j]);
    if (!hl.sk_off[h] || !hl.sk_val[h]) throw std::invalid_argument("part_agg: null stored sketch");
  }
  words += hl.n;
  if (words != RW) throw std::invalid_argument("part_agg: record width does not match the fields");
  for (size_t s = 0; s < ops.size(); ++s) {
    f.op[s] = ops[s];
    f.init[s] = init[s];
  }
  const int64_t lds = ((int64_t)1 << shift) * (f.nslots * 8 + (int64_t)hl.n * ((int64_t)1 << hl.p));
  // (static LDS: the scan / base words and the fused top-k's per-wave lists, ~1.1 KiB)
  if (shift < 0 || lds > 160 * 1024 - 1536)
    throw std::invalid_argument("part_agg: sub-bucket table exceeds the LDS");
  if (lds > 64 * 1024)  // (the kernel's static LDS counts against the 160 KiB too: exactly the dynamic bytes)
    check(hipFuncSetAttribute((const void*)sdo::part_agg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
          "part_agg attr");
  const int64_t grid = (nsub + 7) / 8 * 8;
  if (grid > ((int64_t)1 << 31) - 8) throw std::invalid_argument("part_agg: too many sub-buckets");
  sdo::PartHaving hv{};
  if (having.size() > 4) throw std::invalid_argument("part_agg: at most 4 having terms");
  hv.nterms = (int)having.size();
  hv.conj = conj;
  for (size_t j = 0; j < having.size(); ++j) {
    hv.slot[j] = std::get<0>(having[j]);
    hv.f64[j] = std::get<1>(having[j]);
    hv.op[j] = std::get<2>(having[j]);
    hv.div[j] = std::get<3>(having[j]);
    hv.c[j] = std::get<4>(having[j]);
    if (hv.slot[j] < 0 || hv.slot[j] >= f.nslots || hv.op[j] < 0 || hv.op[j] > 2)
      throw std::invalid_argument("part_agg: having term");
  }
  // fused ORDER BY slot LIMIT k: out_count is then [count, threshold] (both reset here)
  hv.tk = std::get<0>(topk);
  hv.tk_slot = std::get<1>(topk);
  hv.tk_f64 = std::get<2>(topk) ? 1 : 0;
  hv.tk_desc = std::get<3>(topk) ? 1 : 0;
  if (hv.tk < 0 || hv.tk > sdo::PART_TOPK_MAX || hv.tk_slot < 0 || hv.tk_slot >= f.nslots)
    throw std::invalid_argument("part_agg: top-k");
  if (hv.tk && hl.n) throw std::invalid_argument("part_agg: top-k with HLL aggregators");
  if (hv.tk && ((int64_t)1 << shift) > 512 * 8) throw std::invalid_argument("part_agg: top-k over a table > 4096 keys");
  if (hv.nterms == 0 && hv.tk) hv.conj = 1;  // (no terms: every existing group passes)
  if ((hv.nterms || hv.tk) && (!out_keys || !out_count || cap < 0)) throw std::invalid_argument("part_agg: having output");
  if (hv.nterms || hv.tk)
    check(hipMemsetAsync((void*)out_count, 0, hv.tk ? 16 : 8, (hipStream_t)stream), "part_agg count reset");
  hipLaunchKernelGGL(sdo::part_agg_kernel, dim3((unsigned)grid), dim3(512), (unsigned)lds, (hipStream_t)stream,
                     (const uint32_t*)recs, RW, (const uint32_t*)base, nsub, G, shift, f, hl, (uint64_t*)gacc, hv,
                     (int64_t*)out_keys, (unsigned long long*)out_count, cap);
  check(hipGetLastError(), "part_agg_kernel launch");
}

// part_agg with a fused ORDER BY <tk_slot> LIMIT tk (partition.hip part_topk_threshold): out_count
// must hold two words
static void part_agg_topk(uint64_t recs, int RW, uint64_t base, int64_t nsub, int64_t G, int shift, std::vector<int> slot,
                          std::vector<int> width, std::vector<int> ops, std::vector<int64_t> init, uint64_t gacc,
                          std::vector<std::tuple<int, int, int, double, double>> having, int conj, uint64_t out_keys,
                          uint64_t out_count, int64_t cap, int tk, int tk_slot, int tk_f64, int tk_desc,
                          uint64_t stream) {
  if (tk < 1) throw std::invalid_argument("part_agg_topk: k >= 1");
  part_agg_hll(recs, RW, base, nsub, G, shift, slot, width, ops, init, gacc, having, conj, out_keys, out_count, cap, {},
               0, stream, {}, std::make_tuple(tk, tk_slot, tk_f64, tk_desc));
}

static void part_agg(uint64_t recs, int RW, uint64_t base, int64_t nsub, int64_t G, int shift, std::vector<int> slot,
                     std::vector<int> width, std::vector<int> ops, std::vector<int64_t> init, uint64_t gacc,
                     std::vector<std::tuple<int, int, int, double, double>> having, int conj, uint64_t out_keys,
                     uint64_t out_count, int64_t cap, uint64_t stream) {
  part_agg_hll(recs, RW, base, nsub, G, shift, slot, width, ops, init, gacc, having, conj, out_keys, out_count, cap, {},
               0, stream, {});
}

// ---------------------------------------------------------------------------------------------
// Theta (KMV) candidate selection (sketch.hip): histogram of the top `bits` hash bits per group,
// per-group bound for `target` candidates, compaction of the pairs below their bound.
static void theta_select(uint64_t g, uint64_t h, int64_t n, int64_t G, int bits, uint64_t hist, uint64_t target,
                         uint64_t bound, uint64_t out_g, uint64_t out_h, uint64_t count, int64_t cap,
                         uint64_t stream) {
  if (bits < 4 || bits > 16) throw std::invalid_argument("theta_select: 4..16 histogram bits");
  if (G <= 0 || G > (1 << 20)) throw std::invalid_argument("theta_select: 1..2^20 groups");
  hipStream_t s = (hipStream_t)stream;
  check(hipMemsetAsync((void*)hist, 0, (size_t)G << bits << 2, s), "theta hist clear");
  check(hipMemsetAsync((void*)count, 0, 8, s), "theta count clear");
  if (n > 0) {
    hipLaunchKernelGGL(sdo::theta_hist_kernel, dim3(grid_for(n, 256, 65536)), dim3(256), 0, s, (const int64_t*)g,
                       (const int64_t*)h, n, bits, (uint32_t*)hist);
    check(hipGetLastError(), "theta_hist_kernel launch");
  }
  hipLaunchKernelGGL(sdo::theta_thresh_kernel, dim3((unsigned)G), dim3(1024), 0, s, (const uint32_t*)hist, bits,
                     (const int64_t*)target, (int64_t*)bound);
  check(hipGetLastError(), "theta_thresh_kernel launch");
  if (n > 0) {
    hipLaunchKernelGGL(sdo::theta_filter_kernel, dim3(grid_for(n, 256, 65536)), dim3(256), 0, s, (const int64_t*)g,
                       (const int64_t*)h, n, (const int64_t*)bound, (int64_t*)out_g, (int64_t*)out_h,
                       (unsigned long long*)count, cap);
    check(hipGetLastError(), "theta_filter_kernel launch");
  }
}

// The same select over a theta producer's chunk-region records (sketch.hip theta_*_regions):
// record = u32 group key, then 2 words of 62-bit hash per theta from word `hoff`.  `nt` sketches
// (<= 4) are selected in ONE histogram and ONE filter pass over the records: rows t * G + g of the
// histogram / target / bound arrays, candidates written as group t * G + g.  The histogram is
// per-workgroup LDS when [nt G][2^bits] u32 fits 64 KiB (the host sizes bits for it), else global.
static void theta_select_regions(uint64_t recs, int rw, int hoff, uint64_t seg_lo, uint64_t seg_hi, int64_t nseg,
                                 int64_t G, int bits, uint64_t hist, uint64_t target, uint64_t bound, uint64_t out_g,
                                 uint64_t out_h, uint64_t count, int64_t cap, uint64_t stream, int nt,
                                 int reuse_bound) {
  // reuse_bound: `bound` already holds the rows' bounds (a repeated statement's last ones): filter only
  if (bits < 4 || bits > 16) throw std::invalid_argument("theta_select_regions: 4..16 histogram bits");
  if (G <= 0 || G > (1 << 20)) throw std::invalid_argument("theta_select_regions: 1..2^20 groups");
  if (nt < 1 || nt > 4) throw std::invalid_argument("theta_select_regions: 1..4 sketches per pass");
  if (rw < 3 || hoff < 1 || hoff + 2 * nt > rw) throw std::invalid_argument("theta_select_regions: record layout");
  hipStream_t s = (hipStream_t)stream;
  const int64_t GT = G * nt;
  if (!reuse_bound) check(hipMemsetAsync((void*)hist, 0, (size_t)GT << bits << 2, s), "theta hist clear");
  check(hipMemsetAsync((void*)count, 0, 8, s), "theta count clear");
  const int64_t lds = (int64_t)(GT << bits) * 4;
  const int use_lds = lds <= 64 * 1024 ? 1 : 0;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nseg, 4096));
  // (the histogram's workgroups each flush their LDS bins with global atomics onto the same
  // addresses: fewer, longer-running workgroups for it)
  const unsigned hgrid = use_lds ? (unsigned)std::max<int64_t>(1, std::min<int64_t>(nseg, 1024)) : grid;
  if (nseg > 0 && !reuse_bound) {
    hipLaunchKernelGGL(sdo::theta_hist_regions_kernel, dim3(hgrid), dim3(256), use_lds ? (size_t)lds : 0, s,
                       (const uint32_t*)recs, rw, hoff, (const uint32_t*)seg_lo, (const uint32_t*)seg_hi, nseg, (int)G,
                       bits, (uint32_t*)hist, use_lds, nt);
    check(hipGetLastError(), "theta_hist_regions_kernel launch");
  }
  if (!reuse_bound) {
    hipLaunchKernelGGL(sdo::theta_thresh_kernel, dim3((unsigned)GT), dim3(1024), 0, s, (const uint32_t*)hist, bits,
                       (const int64_t*)target, (int64_t*)bound);
    check(hipGetLastError(), "theta_thresh_kernel launch");
  }
  if (nseg > 0) {
    hipLaunchKernelGGL(sdo::theta_filter_regions_kernel, dim3(grid), dim3(256), 0, s, (const uint32_t*)recs, rw, hoff,
                       (const uint32_t*)seg_lo, (const uint32_t*)seg_hi, nseg, (int)G, (const int64_t*)bound,
                       (int64_t*)out_g, (int64_t*)out_h, (unsigned long long*)count, cap, nt);
    check(hipGetLastError(), "theta_filter_regions_kernel launch");
  }
}

// ---------------------------------------------------------------------------------------------
// Peer-to-peer mailboxes (p2p.hip): one allocation per (process group, rank), exported with an IPC
// handle and opened by every peer; the small dense merge is then one kernel per rank.
// The mailbox is UNCACHED device memory: the writer's stores and the peers' xGMI reads meet in
// HBM, with no L2 line of either GPU in between.  (A plain hipMalloc is the fallback when the
// uncached allocation cannot be exported; the kernel's system-scope fences / atomics cover it, and
// the exchange's known-value self-test decides whether the path is used at all, parallel/p2p.py.)
// Returns (pointer, IPC handle, "uncached" | "coarse").
static py::tuple p2p_alloc(int64_t bytes) {
  void* p = nullptr;
  const char* kind = "uncached";
  hipIpcMemHandle_t h;
  bool ok = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) == hipSuccess;
  if (ok && hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipFree(p);
    p = nullptr;
    ok = false;
  }
  if (!ok) {
    (void)hipGetLastError();
    kind = "coarse";
    check(hipMalloc(&p, (size_t)bytes), "p2p mailbox hipMalloc");
    check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
  }
  check(hipMemset(p, 0, (size_t)bytes), "p2p mailbox clear");
  check(hipDeviceSynchronize(), "p2p mailbox clear sync");
  return py::make_tuple((uint64_t)p, py::bytes((const char*)&h, sizeof(h)), kind);
}

static uint64_t p2p_open(py::bytes handle) {
  std::string s(handle);
  if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("p2p_open: bad IPC handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, s.data(), sizeof(h));
  void* p = nullptr;
  check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return (uint64_t)p;
}

static void p2p_close(uint64_t p) { (void)hipIpcCloseMemHandle((void*)p); }
static void p2p_free(uint64_t p) { (void)hipFree((void*)p); }

static void p2p_merge(std::vector<uint64_t> mbox, int rank, uint64_t epoch, int64_t slot_bytes, uint64_t acc_src,
                      int64_t nacc, uint64_t hll_src, int64_t nhll, std::vector<int> ops, int64_t status,
                      uint64_t acc_out, uint64_t hll_out, uint64_t status_out, double soft_s, double hard_s,
                      uint64_t stream) {
  sdo::P2PArgs a{};
  const int n = (int)mbox.size();
  if (n < 1 || n > sdo::P2P_MAX_RANKS) throw std::invalid_argument("p2p_merge: 1..8 ranks");
  if (rank < 0 || rank >= n) throw std::invalid_argument("p2p_merge: rank");
  if (ops.empty() || ops.size() > (size_t)sdo::P2P_MAX_SLOTS) throw std::invalid_argument("p2p_merge: 1..64 slots");
  if (nacc < 0 || nacc % (int64_t)ops.size() != 0) throw std::invalid_argument("p2p_merge: accumulator words");
  if (nhll < 0 || nhll % 8 != 0) throw std::invalid_argument("p2p_merge: HLL bytes must be a multiple of 8");
  if ((nacc + nhll / 8 + 1) * 8 > slot_bytes) throw std::invalid_argument("p2p_merge: state exceeds the mailbox");
  if (epoch < 1) throw std::invalid_argument("p2p_merge: epoch >= 1");
  for (int i = 0; i < n; ++i) {
    if (!mbox[i]) throw std::invalid_argument("p2p_merge: unmapped mailbox");
    a.mbox[i] = mbox[i];
  }
  for (size_t j = 0; j < ops.size(); ++j) {
    if (ops[j] < 0 || ops[j] > 3) throw std::invalid_argument("p2p_merge: slot op");
    a.ops[j] = ops[j];
  }
  a.nranks = n;
  a.rank = rank;
  a.epoch = epoch;
  a.slot_bytes = slot_bytes;
  a.nacc = nacc;
  a.nhll = nhll;
  a.nslots = (int)ops.size();
  a.acc_src = (const int64_t*)acc_src;
  a.hll_src = (const uint8_t*)hll_src;
  a.status = status;
  a.acc_out = (int64_t*)acc_out;
  a.hll_out = (uint8_t*)hll_out;
  a.status_out = (int64_t*)status_out;
  a.soft_ticks = (int64_t)(soft_s * 1e8);  // wall clock: 100 MHz
  a.hard_ticks = (int64_t)(hard_s * 1e8);
  hipLaunchKernelGGL(sdo::p2p_merge_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
  check(hipGetLastError(), "p2p_merge_kernel launch");
}

// Sparse aggregation of hash-partitioned 64-bit-key records (partition.hip part_hash_agg_kernel):
// one workgroup per sub-bucket with an LDS table of 2^cap_log2 keys; survivors (every group, or
// those passing `having`) appended to out_keys / out_acc; *overflow set when a sub-bucket held more
// distinct keys than its table.
// hll: the [cap][2^hll_p] byte register output tables of the HLL aggregators the records carry (one
// word each after the value fields), empty for none.
static void part_hash_agg_hll(uint64_t recs, int RW, uint64_t base, int64_t nsub, int cap_log2, std::vector<int> slot,
                              std::vector<int> width, std::vector<int> ops, std::vector<int64_t> init,
                              std::vector<std::tuple<int, int, int, double, double>> having, int conj, uint64_t out_keys,
                              uint64_t out_acc, uint64_t out_count, int64_t cap, uint64_t overflow,
                              std::vector<uint64_t> hll, int hll_p, uint64_t stream) {
  if (nsub <= 0) return;
  sdo::PartFields f{};
  if (slot.size() != width.size() || slot.size() > (size_t)sdo::MAX_SLOTS) throw std::invalid_argument("part_hash_agg: fields");
  if (ops.size() != init.size() || ops.empty() || ops.size() > (size_t)sdo::MAX_SLOTS)
    throw std::invalid_argument("part_hash_agg: slots");
  f.nfields = (int)slot.size();
  f.nslots = (int)ops.size();
  int words = 3;
  for (size_t j = 0; j < slot.size(); ++j) {
    if (slot[j] < 0 || slot[j] >= f.nslots || width[j] < 0 || width[j] > 2)
      throw std::invalid_argument("part_hash_agg: field");
    f.slot[j] = slot[j];
    f.width[j] = width[j];
    words += width[j];
  }
  sdo::PartHll hl{};
  if (hll.size() > (size_t)sdo::PART_MAX_HLL || (!hll.empty() && (hll_p < 4 || hll_p > 16)))
    throw std::invalid_argument("part_hash_agg: HLL aggregators");
  hl.n = (int)hll.size();
  hl.p = hll.empty() ? 0 : hll_p;
  for (size_t h = 0; h < hll.size(); ++h) {
    if (!hll[h] || (hll[h] & 15)) throw std::invalid_argument("part_hash_agg: HLL output table");
    hl.regs[h] = (unsigned char*)hll[h];
  }
  words += hl.n;
  if (words != RW) throw std::invalid_argument("part_hash_agg: record width does not match the fields");
  for (size_t s = 0; s < ops.size(); ++s) {
    f.op[s] = ops[s];
    f.init[s] = init[s];
  }
  if (cap_log2 < 6 || cap_log2 > 14) throw std::invalid_argument("part_hash_agg: table of 2^6..2^14 keys");
  const int64_t lds = ((int64_t)1 << cap_log2) * ((1 + f.nslots) * 8 + (int64_t)hl.n * ((int64_t)1 << hl.p));
  if (lds > 160 * 1024 - 256) throw std::invalid_argument("part_hash_agg: table exceeds 160 KiB of LDS");
  sdo::PartHaving hv{};
  if (having.size() > 4) throw std::invalid_argument("part_hash_agg: at most 4 having terms");
  hv.nterms = (int)having.size();
  hv.conj = conj;
  for (size_t j = 0; j < having.size(); ++j) {
    hv.slot[j] = std::get<0>(having[j]);
    hv.f64[j] = std::get<1>(having[j]);
    hv.op[j] = std::get<2>(having[j]);
    hv.div[j] = std::get<3>(having[j]);
    hv.c[j] = std::get<4>(having[j]);
    if (hv.slot[j] < 0 || hv.slot[j] >= f.nslots || hv.op[j] < 0 || hv.op[j] > 2)
      throw std::invalid_argument("part_hash_agg: having term");
  }
  if (!out_keys || !out_acc || !out_count || !overflow || cap < 0) throw std::invalid_argument("part_hash_agg: outputs");
  hipStream_t s = (hipStream_t)stream;
  check(hipMemsetAsync((void*)out_count, 0, 8, s), "part_hash_agg count reset");
  check(hipMemsetAsync((void*)overflow, 0, 4, s), "part_hash_agg overflow reset");
  const int64_t grid = (nsub + 7) / 8 * 8;
  if (grid > ((int64_t)1 << 31) - 8) throw std::invalid_argument("part_hash_agg: too many sub-buckets");
  const void* fn = (const void*)sdo::part_hash_agg_kernel;
  // (the kernel's own static LDS counts against the 160 KiB: ask for exactly the dynamic bytes)
  if (lds > 65536) check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "part_hash_agg attr");
  const uint32_t* r_ = (const uint32_t*)recs;
  const uint32_t* b_ = (const uint32_t*)base;
  int64_t* ok_ = (int64_t*)out_keys;
  uint64_t* oa_ = (uint64_t*)out_acc;
  unsigned long long* oc_ = (unsigned long long*)out_count;
  int* of_ = (int*)overflow;
  void* args[] = {(void*)&r_, (void*)&RW, (void*)&b_, (void*)&nsub, (void*)&cap_log2, (void*)&f, (void*)&hl, (void*)&hv,
                  (void*)&ok_, (void*)&oa_, (void*)&oc_, (void*)&cap, (void*)&of_};
  check(hipLaunchKernel(fn, dim3((unsigned)grid), dim3(512), args, (size_t)lds, s), "part_hash_agg_kernel launch");
}

static void part_hash_agg(uint64_t recs, int RW, uint64_t base, int64_t nsub, int cap_log2, std::vector<int> slot,
                          std::vector<int> width, std::vector<int> ops, std::vector<int64_t> init,
                          std::vector<std::tuple<int, int, int, double, double>> having, int conj, uint64_t out_keys,
                          uint64_t out_acc, uint64_t out_count, int64_t cap, uint64_t overflow, uint64_t stream) {
  part_hash_agg_hll(recs, RW, base, nsub, cap_log2, slot, width, ops, init, having, conj, out_keys, out_acc, out_count,
                    cap, overflow, {}, 0, stream);
}

static int desc_size() { return (int)sizeof(sdo::ScanDesc); }

static py::dict layout() {
  py::dict d;
  d["ScanDesc"] = sizeof(sdo::ScanDesc);
  d["ColRef"] = sizeof(sdo::ColRef);
  d["FOp"] = sizeof(sdo::FOp);
  d["KOp"] = sizeof(sdo::KOp);
  d["AOp"] = sizeof(sdo::AOp);
  d["EOp"] = sizeof(sdo::EOp);
  d["ZoneP"] = sizeof(sdo::ZoneP);
  d["Range"] = sizeof(sdo::Range);
  d["off_cols"] = offsetof(sdo::ScanDesc, cols);
  d["off_fops"] = offsetof(sdo::ScanDesc, fops);
  d["off_kops"] = offsetof(sdo::ScanDesc, kops);
  d["off_aops"] = offsetof(sdo::ScanDesc, aops);
  d["off_eops"] = offsetof(sdo::ScanDesc, eops);
  d["off_zones"] = offsetof(sdo::ScanDesc, zones);
  d["off_ranges"] = offsetof(sdo::ScanDesc, ranges);
  d["off_slot_init"] = offsetof(sdo::ScanDesc, slot_init);
  return d;
}

static py::dict device_info(int dev) {
  hipDeviceProp_t p;
  check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
  py::dict d;
  d["name"] = std::string(p.name);
  d["gcnArchName"] = std::string(p.gcnArchName);
  d["multiProcessorCount"] = p.multiProcessorCount;
  d["sharedMemPerBlock"] = (int64_t)p.sharedMemPerBlock;
  d["maxSharedMemoryPerMultiProcessor"] = (int64_t)p.maxSharedMemoryPerMultiProcessor;
  d["totalGlobalMem"] = (int64_t)p.totalGlobalMem;
  d["l2CacheSize"] = p.l2CacheSize;
  return d;
}

PYBIND11_MODULE(_sdo_native, m) {
  m.doc() = "MI355X (gfx950) OLAP scan kernels";
  m.def("scan", &scan, "launch the fused scan/filter/group-by kernel", py::arg("desc"), py::arg("grid"),
        py::arg("block"), py::arg("lds"), py::arg("unroll"), py::arg("stream"));
  m.def("bitmap_build", &bitmap_build);
  m.def("hll_estimate", &hll_estimate);
  m.def("compact_count", &compact_count);
  m.def("compact_write", &compact_write);
  m.def("topk_keep", &topk_keep);
  m.def("nonzero_mask", &nonzero_mask);
  m.def("touch_count", &touch_count);
  m.def("touch_gather", &touch_gather);
  m.def("sparse_decode", &sparse_decode);
  m.def("histogram", &histogram);
  m.def("reset_bufs", &reset_bufs);
  m.def("hll_pairs", &hll_pairs);
  m.def("hll_merge_stored", &hll_merge_stored);
  m.def("desc_size", &desc_size);
  m.def("rtc_compile", &rtc_compile);
  m.def("module_load", [](py::bytes code, const std::string& name) {
    std::string c(code);
    py::gil_scoped_release nogil;  // hipModuleLoadData: code-object load + relocation
    return module_load(c, name);
  });
  m.def("module_launch", &module_launch);
  m.def("module_occupancy", &module_occupancy);
  m.def("module_attrs", &module_attrs);
  m.def("theta_select", &theta_select);
  m.def("p2p_alloc", &p2p_alloc);
  m.def("p2p_open", &p2p_open);
  m.def("p2p_close", &p2p_close);
  m.def("p2p_free", &p2p_free);
  m.def("p2p_merge", &p2p_merge);
  m.def("run_scan", &run_scan);
  m.def("fetch_small", &fetch_small);
  m.def("fetch_small_reset", &fetch_small_reset);
  m.def("stream_sync", &stream_sync);
  m.def("read_words", &read_words);
  m.def("set_wait_spin", &set_wait_spin);
  m.def("glds_probe", &glds_probe);
  m.def("part_scan", &part_scan);
  m.def("part_keys", &part_keys);
  m.def("part_split", &part_split);
  m.def("part_tune", &part_tune, py::arg("pu"), py::arg("lds_min") = 0);
  m.def("part_hash_agg_hll", &part_hash_agg_hll);
  m.def("theta_select_regions", &theta_select_regions);
  m.def("part_agg", &part_agg);
  m.def("part_agg_topk", &part_agg_topk);
  m.def("part_agg_hll", [](uint64_t recs, int RW, uint64_t base, int64_t nsub, int64_t G, int shift, std::vector<int> slot,
                           std::vector<int> width, std::vector<int> ops, std::vector<int64_t> init, uint64_t gacc,
                           std::vector<std::tuple<int, int, int, double, double>> having, int conj, uint64_t out_keys,
                           uint64_t out_count, int64_t cap, std::vector<uint64_t> hll, int hll_p, uint64_t stream,
                           std::vector<std::tuple<uint64_t, uint64_t>> stored) {
    part_agg_hll(recs, RW, base, nsub, G, shift, slot, width, ops, init, gacc, having, conj, out_keys, out_count, cap,
                 hll, hll_p, stream, stored);
  });
  m.def("part_hash_agg", &part_hash_agg);
  m.def("layout", &layout);
  m.def("device_info", &device_info);
  m.attr("ARCH") = "gfx950";
}
