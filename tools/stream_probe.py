"""Streaming-read ceilings of one MI355X for the scan skeleton (ops/jit.py) -- what a kernel that
reads a bit-packed column can reach, by access pattern:

  x4          grid-stride uint4 loads (16 B / lane), sum of dwords          -- the plain ceiling
  x1          grid-stride dword loads (4 B / lane)
  pk24        the scan skeleton: 4096-row chunks dealt to waves, each lane's 24-bit field read as
              two dword loads at its bit offset (ld_pk), U words per step
  pk24_lds    the same chunks staged through LDS with uint4 loads, fields read from LDS
  torch       torch.sum of the same bytes as int32

  python tools/stream_probe.py [GB]

Prints GB/s per variant (median of 20 launches)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SRC = r'''
#include "sdo_device.h"
using namespace sdo;
using namespace sdo::dev;
struct P { const uint32_t* in; int64_t ndw; int64_t nchunks; unsigned long long* out; };

extern "C" __global__ __launch_bounds__(512) void sp_x4(const P* __restrict__ p) {
  const uint4* in = (const uint4*)p->in;
  const int64_t n4 = p->ndw / 4;
  uint64_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = in[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
  }
  for (; i < n4; i += stride) { const uint4 v = in[i]; acc += (uint64_t)v.x + v.y + v.z + v.w; }
  if (acc == 0x123456789abcdefull) p->out[0] = acc;  // (keeps the loads live, no same-address atomics)
}

extern "C" __global__ __launch_bounds__(512) void sp_x1(const P* __restrict__ p) {
  const uint32_t* in = p->in;
  const int64_t n = p->ndw;
  uint64_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 7 * stride < n; i += 8 * stride) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = in[i + u * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; i < n; i += stride) acc += in[i];
  if (acc == 0x123456789abcdefull) p->out[0] = acc;  // (keeps the loads live, no same-address atomics)
}

// 4096-row chunks of a 24-bit packed column: 64 words x 192 B = 12 KB per chunk
template <int U>
__device__ void pk24_body(const P* __restrict__ p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t pko = (((uint32_t)lane * 24u) >> 5) * 4u;
  const uint32_t psh = ((uint32_t)lane * 24u) & 31u;
  const int64_t total_waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  uint64_t acc = 0;
  for (int64_t c = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave; c < p->nchunks; c += total_waves) {
    const __amdgpu_buffer_rsrc_t rs = chunk_rsrc_pk((const unsigned char*)p->in, c, 24);
    for (int w0 = 0; w0 < 64; w0 += U) {
      uint64_t x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = ld_pk(rs, (uint32_t)(w0 + u) * 192u, pko);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += (uint64_t)pk_field<24>(x[u], psh);
    }
  }
  if (acc == 0x123456789abcdefull) p->out[0] = acc;  // (keeps the loads live, no same-address atomics)
}
extern "C" __global__ __launch_bounds__(512) void sp_pk24_u4(const P* __restrict__ p) { pk24_body<4>(p); }
extern "C" __global__ __launch_bounds__(512) void sp_pk24_u8(const P* __restrict__ p) { pk24_body<8>(p); }
extern "C" __global__ __launch_bounds__(512) void sp_pk24_u16(const P* __restrict__ p) { pk24_body<16>(p); }

// the same chunks staged into LDS (12 KB per wave, 256-thread blocks) with uint4 loads
extern "C" __global__ __launch_bounds__(256) void sp_pk24_lds(const P* __restrict__ p) {
  __shared__ __attribute__((aligned(16))) uint32_t st[4][3072 + 4];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t pko = ((uint32_t)lane * 24u) >> 5;
  const uint32_t psh = ((uint32_t)lane * 24u) & 31u;
  const int64_t total_waves = (int64_t)gridDim.x * 4;
  uint32_t* s = st[wave];
  uint64_t acc = 0;
  for (int64_t c = (int64_t)blockIdx.x * 4 + wave; c < p->nchunks; c += total_waves) {
    const uint4* src = (const uint4*)(p->in + c * 3072);
    uint4 v[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) v[k] = src[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 12; ++k) ((uint4*)s)[k * 64 + lane] = v[k];
    __builtin_amdgcn_wave_barrier();
#pragma unroll 8
    for (int w = 0; w < 64; ++w) {
      const uint64_t x = (uint64_t)s[w * 48 + pko] | ((uint64_t)s[w * 48 + pko + 1] << 32);
      acc += (uint64_t)pk_field<24>(x, psh);
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (acc == 0x123456789abcdefull) p->out[0] = acc;  // (keeps the loads live, no same-address atomics)
}
// ---- Q1-shaped: five bit-packed columns (24, 17, 14, 2, 1 bits) + one u16 column, 600M rows
struct Q { const uint32_t* col[6]; int64_t nchunks; unsigned long long* out; };

// current layout: word w of a chunk = 64 rows x W bits (2W dwords); lane l's field at bit l*W
template <int W>
__device__ __forceinline__ uint32_t cur_f(__amdgpu_buffer_rsrc_t r, int w, uint32_t pko, uint32_t psh) {
  return (uint32_t)pk_field<W>(ld_pk(r, (uint32_t)w * (8u * W), pko), psh);
}
extern "C" __global__ __launch_bounds__(512) void q1_cur(const Q* __restrict__ p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t pko24 = ((lane * 24u) >> 5) * 4u, psh24 = (lane * 24u) & 31u;
  const uint32_t pko17 = ((lane * 17u) >> 5) * 4u, psh17 = (lane * 17u) & 31u;
  const uint32_t pko14 = ((lane * 14u) >> 5) * 4u, psh14 = (lane * 14u) & 31u;
  const uint32_t pko2 = ((lane * 2u) >> 5) * 4u, psh2 = (lane * 2u) & 31u;
  const uint32_t pko1 = ((lane * 1u) >> 5) * 4u, psh1 = (lane * 1u) & 31u;
  const int64_t total_waves = (int64_t)gridDim.x * 8;
  uint64_t acc = 0;
  for (int64_t c = (int64_t)blockIdx.x * 8 + wave; c < p->nchunks; c += total_waves) {
    const auto r24 = chunk_rsrc_pk((const unsigned char*)p->col[0], c, 24);
    const auto r17 = chunk_rsrc_pk((const unsigned char*)p->col[1], c, 17);
    const auto r14 = chunk_rsrc_pk((const unsigned char*)p->col[2], c, 14);
    const auto r2 = chunk_rsrc_pk((const unsigned char*)p->col[3], c, 2);
    const auto r1 = chunk_rsrc_pk((const unsigned char*)p->col[4], c, 1);
    const auto r16 = chunk_rsrc((const unsigned char*)p->col[5], c * 4096, 4096, 1);
    for (int w0 = 0; w0 < 64; w0 += 8) {
      uint32_t a[8], b[8], e[8], f[8], g[8], h[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = cur_f<24>(r24, w0 + u, pko24, psh24);
        b[u] = cur_f<17>(r17, w0 + u, pko17, psh17);
        e[u] = cur_f<14>(r14, w0 + u, pko14, psh14);
        f[u] = cur_f<2>(r2, w0 + u, pko2, psh2);
        g[u] = cur_f<1>(r1, w0 + u, pko1, psh1);
        h[u] = ld_b<1>(r16, (uint32_t)(w0 + u) << 7, (uint32_t)lane << 1);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (uint64_t)a[u] + b[u] + e[u] + (f[u] << 3) + g[u] + h[u];
    }
  }
  if (acc == 0x123456789abcdefull) p->out[0] = acc;
}

// lane-interleaved layout: a chunk is 2 groups of 32 words; in group g lane l owns a W-dword
// stream holding its 32 rows' fields back to back; stream dword k sits at k*64 + l (one 256-byte
// coalesced dword load per k for the whole wave)
template <int W, int J0, int U>
struct IlB {
  static constexpr int K0 = (J0 * W) >> 5;
  static constexpr int K1 = ((J0 + U) * W - 1) >> 5;
  static constexpr int N = K1 - K0 + 1;
  uint32_t d[N + 1];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t gb, uint32_t lo4) {
#pragma unroll
    for (int k = 0; k < N; ++k) d[k] = __builtin_amdgcn_raw_buffer_load_b32(r, lo4, gb + (K0 + k) * 256u, 0);
    d[N] = 0u;
  }
  __device__ __forceinline__ uint32_t f(int u) const {
    const int bit = (J0 + u) * W - K0 * 32;
    const int k = bit >> 5, sh = bit & 31;
    const uint32_t x = sh + W <= 32 ? (d[k] >> sh) : __builtin_amdgcn_alignbit(d[k + 1], d[k], sh);
    return W == 32 ? x : (x & ((1u << W) - 1u));
  }
};
template <int J0>
__device__ __forceinline__ void q1_il_batch(const __amdgpu_buffer_rsrc_t* rs, const uint32_t* gb, uint32_t lo4,
                                            uint64_t& acc) {
  IlB<24, J0, 8> A; IlB<17, J0, 8> B; IlB<14, J0, 8> E; IlB<2, J0, 8> F; IlB<1, J0, 8> G; IlB<16, J0, 8> H;
  A.load(rs[0], gb[0], lo4); B.load(rs[1], gb[1], lo4); E.load(rs[2], gb[2], lo4);
  F.load(rs[3], gb[3], lo4); G.load(rs[4], gb[4], lo4); H.load(rs[5], gb[5], lo4);
#pragma unroll
  for (int u = 0; u < 8; ++u) acc += (uint64_t)A.f(u) + B.f(u) + E.f(u) + (F.f(u) << 3) + G.f(u) + H.f(u);
}
extern "C" __global__ __launch_bounds__(512) void q1_il(const Q* __restrict__ p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lo4 = (uint32_t)lane * 4u;
  constexpr int Ws[6] = {24, 17, 14, 2, 1, 16};
  const int64_t total_waves = (int64_t)gridDim.x * 8;
  uint64_t acc = 0;
  for (int64_t c = (int64_t)blockIdx.x * 8 + wave; c < p->nchunks; c += total_waves) {
    __amdgpu_buffer_rsrc_t rs[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) rs[i] = chunk_rsrc_pk((const unsigned char*)p->col[i], c, Ws[i]);
    for (int g = 0; g < 2; ++g) {
      uint32_t gb[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) gb[i] = (uint32_t)g * (256u * Ws[i]);
      q1_il_batch<0>(rs, gb, lo4, acc);
      q1_il_batch<8>(rs, gb, lo4, acc);
      q1_il_batch<16>(rs, gb, lo4, acc);
      q1_il_batch<24>(rs, gb, lo4, acc);
    }
  }
  if (acc == 0x123456789abcdefull) p->out[0] = acc;
}
'''


def main():
    import torch

    from spark_druid_olap_amd.ops import jit, native

    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 1.8
    nat = native.load()
    dev = torch.device("cuda", 0)
    nchunks = int(gb * 1e9) // (3072 * 4)
    ndw = nchunks * 3072
    buf = torch.randint(0, 1 << 30, (ndw + 64,), dtype=torch.int32, device=dev)
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    import numpy as np

    prm = np.zeros(4, dtype=np.int64)
    prm[:] = [buf.data_ptr(), ndw, nchunks, out.data_ptr()]
    pd = torch.from_numpy(prm).to(dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    code = jit.compile_code(SRC, "sp_x4")
    st = native._stream(dev)
    nbytes = ndw * 4
    print(f"{nbytes / 1e9:.2f} GB, {cus} CUs", flush=True)

    def run(name, grid, block, lds=0):
        h = nat.module_load(code, name)
        for _ in range(3):
            nat.module_launch(h, pd.data_ptr(), grid, block, lds, st)
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            nat.module_launch(h, pd.data_ptr(), grid, block, lds, st)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ms = statistics.median(ts)
        print(f"  {name:12s} grid {grid:6d} x {block:3d}  {ms:7.3f} ms  {nbytes / ms / 1e6:8.0f} GB/s", flush=True)

    for per_cu in (2, 4, 8):
        run("sp_x4", cus * per_cu, 512)
    for per_cu in (2, 4):
        run("sp_x1", cus * per_cu, 512)
    for u in (4, 8, 16):
        for per_cu in (2, 3, 4):
            run(f"sp_pk24_u{u}", cus * per_cu, 512)
    for per_cu in (2, 4, 6, 8):
        run("sp_pk24_lds", cus * per_cu, 256)
    # Q1-shaped: five packed columns + one u16 column over ROWS rows (same bytes in both layouts)
    rows = int(os.environ.get("Q1_ROWS", "600000000")) // 4096 * 4096
    del buf
    cols = [torch.randint(0, 1 << 30, (rows * w // 32 + 64,), dtype=torch.int32, device=dev) for w in (24, 17, 14, 2, 1, 16)]
    qp = np.zeros(8, dtype=np.int64)
    qp[:6] = [c.data_ptr() for c in cols]
    qp[6], qp[7] = rows // 4096, out.data_ptr()
    qd = torch.from_numpy(qp).to(dev)
    qbytes = sum(c.numel() * 4 for c in cols)
    print(f"Q1-shaped: {rows} rows, {qbytes / 1e9:.2f} GB", flush=True)
    pd_saved = pd

    def runq(name, grid):
        nonlocal pd
        pd = qd
        run(name, grid, 512)
        pd = pd_saved

    nbytes_saved = nbytes
    nbytes = qbytes
    for per_cu in (2, 3, 4):
        runq("q1_cur", cus * per_cu)
        runq("q1_il", cus * per_cu)
    nbytes = nbytes_saved
    return
    for _ in range(3):
        v.sum()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        v.sum()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = statistics.median(ts)
    print(f"  {'torch.sum':12s} {'':17s}  {ms:7.3f} ms  {nbytes / ms / 1e6:8.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
