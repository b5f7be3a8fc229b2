// CDNA4 (gfx950) fused segment-scan kernels: time-pruned row ranges -> zone-map chunk skipping ->
// filter (inverted bitmaps / dictionary-domain bitsets / ranges) -> group key -> aggregation
// (dense LDS accumulators with wave-level key de-duplication, dense global atomics, or a global
// open-addressing hash table) + HyperLogLog registers.  One launch replaces the per-segment
// cursor loop that Druid historicals run in Java for GroupBy / Timeseries / TopN / Search /
// Select queries (reference emits these specs at
// src/main/scala/org/sparklinedata/druid/DruidQuerySpec.scala:638-1070).
//
// Execution model (MI355X-first, not a translation of anything in the reference):
//   * a 64-bit bitmap word covers exactly the 64 rows one wavefront processes, so an inverted
//     bitmap leaf costs ONE scalar load per 64 rows and a whole wave skips empty words with a
//     uniform branch -- no per-row work at all for rows the filter rejects;
//   * column leaves load one value per lane and produce the same 64-bit mask via __ballot;
//   * U consecutive words are processed per step so every column read issues U independent
//     loads before the first wait (memory-level parallelism for HBM3E);
//   * inactive lanes load from the leader lane's address, so selective filters touch only the
//     cache lines of qualifying rows;
//   * dense group-by accumulators live in LDS (160 KiB per CU); per distinct key in a wave the
//     lanes are reduced with cross-lane shuffles and a single lane issues one LDS atomic;
//   * LDS partials are flushed to HBM once per workgroup with global atomics (persistent grid).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "scan_desc.h"

namespace sdo {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ int64_t f2ord(double f) {  // order-preserving double -> int64
  int64_t b = __double_as_longlong(f);
  return b >= 0 ? b : (b ^ 0x7fffffffffffffffLL);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t range_bits(int lo, int hi) {
  if (hi <= lo) return 0ull;
  uint64_t h = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  uint64_t l = lo <= 0 ? 0ull : ((1ull << lo) - 1ull);
  return h & ~l;
}

// ---------------------------------------------------------------------------------------------
// Batched column loads: U independent loads are issued inside one wave-uniform dtype branch so
// the compiler waits once per batch, not once per element.
template <int U>
__device__ __forceinline__ void load_int(const ColRef& c, const int64_t (&row)[U], int64_t (&v)[U]) {
  switch (c.dtype) {
    case DT_U8: {
      const uint8_t* p = (const uint8_t*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[row[u]];
    } break;
    case DT_I16: {
      const int16_t* p = (const int16_t*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[row[u]];
    } break;
    case DT_U16: {
      const uint16_t* p = (const uint16_t*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[row[u]];
    } break;
    case DT_I32: {
      const int32_t* p = (const int32_t*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[row[u]];
    } break;
    case DT_I64: {
      const int64_t* p = (const int64_t*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[row[u]];
    } break;
    case DT_F32: {
      const float* p = (const float*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = (int64_t)p[row[u]];
    } break;
    default: {
      const double* p = (const double*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = (int64_t)p[row[u]];
    } break;
  }
}

template <int U>
__device__ __forceinline__ void load_flt(const ColRef& c, const int64_t (&row)[U], double (&v)[U]) {
  switch (c.dtype) {
    case DT_F64: {
      const double* p = (const double*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[row[u]];
    } break;
    case DT_F32: {
      const float* p = (const float*)c.ptr;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = (double)p[row[u]];
    } break;
    default: {
      int64_t t[U];
      load_int<U>(c, row, t);
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = (double)t[u];
    } break;
  }
}

// ---------------------------------------------------------------------------------------------
// Filter program: postfix ops over a shifting register stack of wave masks (static indexing only:
// runtime-indexed register arrays would spill to scratch on CDNA).
template <int U>
struct MaskStack {
  uint64_t s[STACK_DEPTH][U];
  __device__ __forceinline__ void push(const uint64_t (&m)[U]) {
#pragma unroll
    for (int d = STACK_DEPTH - 1; d > 0; --d)
#pragma unroll
      for (int u = 0; u < U; ++u) s[d][u] = s[d - 1][u];
#pragma unroll
    for (int u = 0; u < U; ++u) s[0][u] = m[u];
  }
  template <int OP>
  __device__ __forceinline__ void binop() {
#pragma unroll
    for (int u = 0; u < U; ++u) s[0][u] = OP == 0 ? (s[1][u] & s[0][u]) : (s[1][u] | s[0][u]);
#pragma unroll
    for (int d = 1; d < STACK_DEPTH - 1; ++d)
#pragma unroll
      for (int u = 0; u < U; ++u) s[d][u] = s[d + 1][u];
  }
};

template <int U>
__device__ __forceinline__ void eval_filter(const ScanDesc* __restrict__ d, int off, int len,
                                            const int64_t (&word)[U], const int64_t (&row)[U],
                                            const uint64_t (&valid)[U], uint64_t (&out)[U]) {
  if (len == 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) out[u] = valid[u];
    return;
  }
  MaskStack<U> st;
  for (int i = off; i < off + len; ++i) {
    const FOp f = d->fops[i];
    uint64_t m[U];
    switch (f.op) {
      case F_TRUE:
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = ~0ull;
        st.push(m);
        break;
      case F_FALSE:
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = 0ull;
        st.push(m);
        break;
      case F_BITMAP: {
        const uint64_t* b = (const uint64_t*)f.bits;
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = valid[u] ? b[word[u]] : 0ull;
        st.push(m);
      } break;
      case F_BITMAP_OR: {
        const uint64_t* b = (const uint64_t*)f.bits;
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = 0ull;
        for (int64_t j = 0; j < f.hi; ++j) {
#pragma unroll
          for (int u = 0; u < U; ++u) m[u] |= valid[u] ? b[j * f.lo + word[u]] : 0ull;
        }
        st.push(m);
      } break;
      case F_ID_RANGE:
      case F_INT_RANGE: {
        int64_t v[U];
        load_int<U>(d->cols[f.col], row, v);
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = __ballot(v[u] >= f.lo && (f.op == F_ID_RANGE ? v[u] < f.hi : v[u] <= f.hi));
        st.push(m);
      } break;
      case F_IN_SET: {
        int64_t v[U];
        load_int<U>(d->cols[f.col], row, v);
        const uint64_t* b = (const uint64_t*)f.bits;
        uint64_t w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = b[((uint64_t)v[u]) >> 6];
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = __ballot((w[u] >> (v[u] & 63)) & 1ull);
        st.push(m);
      } break;
      case F_FLT_RANGE: {
        double v[U];
        load_flt<U>(d->cols[f.col], row, v);
        const bool los = f.flags & 1, his = f.flags & 2;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          bool a = los ? (v[u] > f.flo) : (v[u] >= f.flo);
          bool b = his ? (v[u] < f.fhi) : (v[u] <= f.fhi);
          m[u] = __ballot(a && b);
        }
        st.push(m);
      } break;
      case F_AND:
        st.template binop<0>();
        break;
      case F_OR:
        st.template binop<1>();
        break;
      case F_NOT:
#pragma unroll
        for (int u = 0; u < U; ++u) st.s[0][u] = ~st.s[0][u];
        break;
      default:
        break;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) out[u] = st.s[0][u] & valid[u];
}

// ---------------------------------------------------------------------------------------------
// Time bucketing: civil-from-days integer math, all in registers.
__device__ __forceinline__ void civil_from_days(int64_t z, int64_t& y, int64_t& m, int64_t& dd) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  y = yoe + era * 400;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  dd = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  y += (m <= 2);
}

__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

__device__ __forceinline__ int64_t time_field(int64_t ms, const KOp& k) {
  ms += k.tz_ms;
  switch (k.tfield) {
    case T_MS: return ms;
    case T_SECOND: return floordiv(ms, 1000);
    case T_MINUTE: return floordiv(ms, 60000);
    case T_HOUR: return floordiv(ms, 3600000);
    case T_DAY: return floordiv(ms, 86400000);
    case T_WEEK: return floordiv(floordiv(ms, 86400000) + 3, 7);
    case T_PERIOD: return floordiv(ms - k.origin_ms, k.period_ms);
    case T_HOD: return floordiv(ms, 3600000) - floordiv(ms, 86400000) * 24;
    case T_MOH: return floordiv(ms, 60000) - floordiv(ms, 3600000) * 60;
    case T_SOM: return floordiv(ms, 1000) - floordiv(ms, 60000) * 60;
    case T_DOW: {
      int64_t dy = floordiv(ms, 86400000);
      return floordiv(dy + 3, 7) * -7 + dy + 3 + 1;  // 1 = Monday .. 7 = Sunday
    }
    default: break;
  }
  const int64_t days = floordiv(ms, 86400000);
  int64_t y, m, dd;
  civil_from_days(days, y, m, dd);
  switch (k.tfield) {
    case T_MONTH: return y * 12 + (m - 1);
    case T_QUARTER: return y * 4 + (m - 1) / 3;
    case T_YEAR: return y;
    case T_MOY: return m;
    case T_DOM: return dd;
    case T_QOY: return (m - 1) / 3 + 1;
    case T_DOY: {
      // days since Jan 1 of y
      int64_t yy = y - 1;  // days_from_civil(y,1,1)
      const int64_t era = (yy >= 0 ? yy : yy - 399) / 400;
      const int64_t yoe = yy - era * 400;
      const int64_t doy = (153 * (1 + 9) + 2) / 5;  // March-based: Jan = month 10
      const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
      const int64_t jan1 = era * 146097 + doe - 719468;
      return days - jan1 + 1;
    }
    default: return days;
  }
}

// ---------------------------------------------------------------------------------------------
// Cross-lane reductions over a subset of lanes (others contribute the identity).
__device__ __forceinline__ int64_t wave_sum_i(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_sum_f(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int64_t wave_min_i(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int64_t t = __shfl_xor(v, o);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int64_t t = __shfl_xor(v, o);
    v = t > v ? t : v;
  }
  return v;
}

__device__ __forceinline__ void slot_atomic(uint64_t* p, int op, int64_t v) {
  switch (op) {
    case S_SUM_I: atomicAdd((unsigned long long*)p, (unsigned long long)v); break;
    case S_SUM_F: unsafeAtomicAdd((double*)p, __longlong_as_double(v)); break;
    case S_MIN_I: atomicMin((long long*)p, (long long)v); break;
    default: atomicMax((long long*)p, (long long)v); break;
  }
}

// open-addressing insert, returns slot or -1 on overflow
__device__ __forceinline__ int64_t hash_slot(uint64_t* keys, int64_t cap, uint64_t k, int* overflow) {
  const uint64_t EMPTY = ~0ull;
  uint64_t h = mix64(k) & (uint64_t)(cap - 1);
  for (int64_t probe = 0; probe < cap; ++probe) {
    uint64_t cur = __hip_atomic_load(keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == k) return (int64_t)h;
    if (cur == EMPTY) {
      unsigned long long prev = atomicCAS((unsigned long long*)(keys + h), EMPTY, k);
      if (prev == EMPTY || prev == k) return (int64_t)h;
    }
    h = (h + 1) & (uint64_t)(cap - 1);
  }
  atomicExch(overflow, 1);
  return -1;
}

// float expression VM (Druid javascript aggregators over several columns, reference
// src/main/scala/org/sparklinedata/druid/jscodegen/JSAggGenerator.scala:37-60)
template <int U>
__device__ __forceinline__ void eval_expr(const ScanDesc* __restrict__ d, int off, int len,
                                          const int64_t (&row)[U], double (&out)[U]) {
  double s0[U], s1[U], s2[U], s3[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { s0[u] = s1[u] = s2[u] = s3[u] = 0.0; }
  for (int i = off; i < off + len; ++i) {
    const EOp e = d->eops[i];
    if (e.op == E_COL || e.op == E_CONST) {
      double v[U];
      if (e.op == E_COL) {
        load_flt<U>(d->cols[e.col], row, v);
        if (e.c != 0.0) {
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] *= e.c;  // decimal scale
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = e.c;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) { s3[u] = s2[u]; s2[u] = s1[u]; s1[u] = s0[u]; s0[u] = v[u]; }
    } else if (e.op == E_NEG) {
#pragma unroll
      for (int u = 0; u < U; ++u) s0[u] = -s0[u];
    } else if (e.op == E_ABS) {
#pragma unroll
      for (int u = 0; u < U; ++u) s0[u] = fabs(s0[u]);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        double a = s1[u], b = s0[u], r;
        switch (e.op) {
          case E_ADD: r = a + b; break;
          case E_SUB: r = a - b; break;
          case E_MUL: r = a * b; break;
          case E_DIV: r = a / b; break;
          case E_MIN: r = fmin(a, b); break;
          default: r = fmax(a, b); break;
        }
        s0[u] = r; s1[u] = s2[u]; s2[u] = s3[u];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) out[u] = s0[u];
}

// ---------------------------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(512) void olap_scan_kernel(const ScanDesc* __restrict__ d) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const int mode = d->mode;
  const int nslots = d->nslots;
  const int64_t G = d->G;
  const int hll_p = d->hll_p;
  const int64_t hll_m = 1ll << hll_p;
  uint64_t* acc_lds = (uint64_t*)lds;

  if (mode == M_DENSE_LDS) {
    const int64_t n = G * nslots;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) acc_lds[i] = (uint64_t)d->slot_init[i % nslots];
    if (d->hll_lds) {
      uint32_t* r = (uint32_t*)(lds + n * 8);
      const int64_t nr = (int64_t)d->nhll * G * hll_m;
      for (int64_t i = threadIdx.x; i < nr; i += blockDim.x) r[i] = 0u;
    }
    __syncthreads();
  }
  uint64_t* gacc = (uint64_t*)d->out_acc;
  uint64_t* hkeys = (uint64_t*)d->out_keys;
  int* overflow = (int*)d->overflow;

  const int64_t total_waves = (int64_t)gridDim.x * wpb;
  const int64_t gw = (int64_t)blockIdx.x * wpb + wave;
  const int64_t num_rows = d->num_rows;

  for (int64_t c = gw; c < d->total_chunks; c += total_waves) {
    // linear chunk -> (range, absolute chunk)
    int r = 0;
    int64_t cc = c;
    while (r < d->nranges - 1 && cc >= d->ranges[r].nchunks) { cc -= d->ranges[r].nchunks; ++r; }
    const int64_t kchunk = d->ranges[r].chunk_begin + cc;
    int64_t clo = kchunk * CHUNK_ROWS, chi = clo + CHUNK_ROWS;
    if (clo < d->ranges[r].lo) clo = d->ranges[r].lo;
    if (chi > d->ranges[r].hi) chi = d->ranges[r].hi;
    if (chi > num_rows) chi = num_rows;
    if (chi <= clo) continue;
    // zone-map pruning (min/max of dictionary ids per 4096-row chunk)
    bool skip = false;
    for (int z = 0; z < d->nzones; ++z) {
      const ZoneP zp = d->zones[z];
      const int32_t zmin = ((const int32_t*)zp.zmin)[kchunk];
      const int32_t zmax = ((const int32_t*)zp.zmax)[kchunk];
      if ((int64_t)zmax < zp.lo || (int64_t)zmin >= zp.hi) { skip = true; break; }
    }
    if (skip) continue;

    const int64_t wbeg = clo >> 6, wend = (chi + 63) >> 6;
    for (int64_t w0 = wbeg; w0 < wend; w0 += U) {
      int64_t word[U], row[U];
      uint64_t valid[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        word[u] = w0 + u;
        const int64_t r0 = word[u] << 6;
        row[u] = r0 + lane;
        valid[u] = (word[u] < wend) ? range_bits((int)(clo > r0 ? clo - r0 : 0), (int)(chi - r0 > 64 ? 64 : chi - r0)) : 0ull;
      }
      uint64_t m[U];
      eval_filter<U>(d, 0, d->filter_len, word, row, valid, m);
      uint64_t any = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) any |= m[u];
      if (any == 0) continue;

      if (mode == M_MASK) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (valid[u] != 0 && lane == 0) ((uint64_t*)d->out_mask)[word[u]] = m[u];
        }
        if (lane == 0) {
          unsigned long long cnt = 0;
#pragma unroll
          for (int u = 0; u < U; ++u) cnt += __popcll(m[u]);
          atomicAdd((unsigned long long*)d->out_count, cnt);
        }
        continue;
      }

      // rows used for dependent loads: inactive lanes alias the first active lane's row
      int64_t lrow[U];
      bool act[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        act[u] = (m[u] >> lane) & 1ull;
        const int64_t lead = (word[u] << 6) + (m[u] ? __builtin_ctzll(m[u]) : 0);
        lrow[u] = act[u] ? row[u] : lead;
      }

      // ---- group key ----
      uint64_t key[U];
#pragma unroll
      for (int u = 0; u < U; ++u) key[u] = 0;
      for (int k = 0; k < d->nkops; ++k) {
        const KOp ko = d->kops[k];
        int64_t v[U];
        load_int<U>(d->cols[ko.col], lrow, v);
        if (ko.kind == K_REMAP) {
          const int32_t* rm = (const int32_t*)ko.remap;
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = rm[v[u]];
        } else if (ko.kind == K_TIME) {
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = time_field(v[u] * ko.unit_ms, ko) - ko.base;
        } else if (ko.kind == K_INT) {
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] -= ko.base;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          int64_t vv = v[u];
          if (ko.kind == K_TIME || ko.kind == K_INT) {  // clamp out-of-domain buckets (never hit for planned intervals)
            vv = vv < 0 ? 0 : (vv >= ko.card ? ko.card - 1 : vv);
          }
          key[u] += (uint64_t)vv * (uint64_t)ko.stride;
        }
      }
      // ---- slot resolution ----
      int64_t slot[U];
      if (mode == M_HASH) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          slot[u] = act[u] ? hash_slot(hkeys, d->hash_cap, key[u], overflow) : -1;
          if (slot[u] < 0) act[u] = false;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = __ballot(act[u]);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) slot[u] = (int64_t)key[u];
      }

      // ---- aggregators ----
      for (int a = 0; a < d->naggs; ++a) {
        const AOp ao = d->aops[a];
        uint64_t ma[U];
        if (ao.filt_len > 0) {
          eval_filter<U>(d, ao.filt_off, ao.filt_len, word, lrow, m, ma);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u) ma[u] = m[u];
        }
        if (ao.kind == A_HLL) {
          int64_t v[U];
          load_int<U>(d->cols[ao.col], lrow, v);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if ((ma[u] >> lane) & 1ull) {
              const uint64_t h = mix64((uint64_t)v[u] ^ (uint64_t)ao.salt);
              const uint32_t bucket = (uint32_t)(h >> (64 - hll_p));
              const uint64_t rest = (h << hll_p) | (1ull << (hll_p - 1));
              const uint32_t rho = (uint32_t)__builtin_clzll(rest) + 1u;
              const int64_t idx = slot[u] * hll_m + bucket;
              if (mode == M_DENSE_LDS && d->hll_lds) {
                atomicMax((uint32_t*)(lds + ao.hll_lds_off) + idx, rho);
              } else {
                atomicMax((uint32_t*)ao.hll_regs + idx, rho);
              }
            }
          }
          continue;
        }
        // value in int64 bits (float kinds: double bits, min/max: order-preserving int64)
        int64_t val[U];
        const int sop = d->slot_op[ao.slot];
        if (ao.kind == A_COUNT) {
#pragma unroll
          for (int u = 0; u < U; ++u) val[u] = 1;
        } else if (ao.kind == A_SUM_F || ao.kind == A_MIN_F || ao.kind == A_MAX_F) {
          double fv[U];
          if (ao.expr_len > 0) {
            eval_expr<U>(d, ao.expr_off, ao.expr_len, lrow, fv);
          } else {
            load_flt<U>(d->cols[ao.col], lrow, fv);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) val[u] = (ao.kind == A_SUM_F) ? __double_as_longlong(fv[u]) : f2ord(fv[u]);
        } else {
          load_int<U>(d->cols[ao.col], lrow, val);
        }
        uint64_t* accbase = (mode == M_DENSE_LDS) ? acc_lds : gacc;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          uint64_t pend = ma[u];
          if (!pend) continue;
          const bool mine = (pend >> lane) & 1ull;
          if (!d->dedup) {
            if (mine) slot_atomic(accbase + slot[u] * nslots + ao.slot, sop, val[u]);
            continue;
          }
          while (pend) {
            const int leader = __builtin_ctzll(pend);
            const uint64_t kk = readlane64((uint64_t)slot[u], leader);
            const uint64_t same = __ballot(mine && (uint64_t)slot[u] == kk) & pend;
            const bool in = (same >> lane) & 1ull;
            int64_t res;
            if (ao.kind == A_COUNT) {
              res = (int64_t)__popcll(same);
            } else if (sop == S_SUM_I) {
              res = wave_sum_i(in ? val[u] : 0);
            } else if (sop == S_SUM_F) {
              res = __double_as_longlong(wave_sum_f(in ? __longlong_as_double(val[u]) : 0.0));
            } else if (sop == S_MIN_I) {
              res = wave_min_i(in ? val[u] : INT64_MAX);
            } else {
              res = wave_max_i(in ? val[u] : INT64_MIN);
            }
            if (lane == leader) slot_atomic(accbase + kk * nslots + ao.slot, sop, res);
            pend &= ~same;
          }
        }
      }
    }
  }

  if (mode == M_DENSE_LDS) {
    __syncthreads();
    const int64_t n = G * nslots;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      const int s = (int)(i % nslots);
      const int64_t v = (int64_t)acc_lds[i];
      if (v != d->slot_init[s]) slot_atomic(gacc + i, d->slot_op[s], v);
    }
    if (d->hll_lds) {
      for (int a = 0; a < d->naggs; ++a) {
        const AOp ao = d->aops[a];
        if (ao.kind != A_HLL) continue;
        const uint32_t* r = (const uint32_t*)(lds + ao.hll_lds_off);
        uint32_t* g = (uint32_t*)ao.hll_regs;
        for (int64_t i = threadIdx.x; i < G * hll_m; i += blockDim.x) {
          const uint32_t v = r[i];
          if (v) atomicMax(g + i, v);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Inverted bitmap index build: one wave per 64-row word; per distinct id in the wave one lane
// writes the ballot word (no atomics: each (value, word) is written by exactly one wave).
__global__ __launch_bounds__(256) void bitmap_build_kernel(const void* ids, int dtype, int64_t n, int64_t nwords,
                                                           uint64_t* out, int64_t card) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t w = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); w < nwords; w += (int64_t)gridDim.x * wpb) {
    const int64_t r = (w << 6) + lane;
    int64_t id = -1;
    if (r < n) {
      switch (dtype) {
        case DT_U8: id = ((const uint8_t*)ids)[r]; break;
        case DT_I16: id = ((const int16_t*)ids)[r]; break;
        case DT_U16: id = ((const uint16_t*)ids)[r]; break;
        case DT_I32: id = ((const int32_t*)ids)[r]; break;
        default: id = ((const int64_t*)ids)[r]; break;
      }
    }
    uint64_t pend = __ballot(id >= 0 && id < card);
    while (pend) {
      const int leader = __builtin_ctzll(pend);
      const int64_t k = (int64_t)readlane64((uint64_t)id, leader);
      const uint64_t same = __ballot(id == k);
      if (lane == leader) out[k * nwords + w] = same;
      pend &= ~same;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// HyperLogLog finalize for G groups x m registers: sum(2^-M) and zero counts per group.
// The register matrix is multiplied by a ones vector on the matrix cores (MFMA 32x32x2 f32:
// A = 2^-M tile [32 groups x 2 regs], B = ones [2 x 32]), which is the batched sketch reduction
// the BASELINE north-star calls for; zero counting rides along as a second B column block.
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(64) void hll_estimate_kernel(const uint32_t* regs, int64_t G, int p,
                                                          double* est) {
  const int lane = threadIdx.x;
  const int64_t m = 1ll << p;
  const int64_t g0 = (int64_t)blockIdx.x * 32;
  // A operand: lane l holds A[i = l & 31][k = l >> 5] = 2^-M[g0+i][kbase + k]
  // B operand: lane l holds B[k = l >> 5][j = l & 31] = (j == 0) ? 1 : (j == 1 ? isZeroMarker : 0)
  f32x16 acc_sum = {0};
  f32x16 acc_zero = {0};
  const int i = lane & 31;
  const int kk = lane >> 5;
  const int64_t g = g0 + i;
  const float bsel = (i == 0) ? 1.0f : 0.0f;  // column 0 of B
  for (int64_t kb = 0; kb < m; kb += 2) {
    float a = 0.f, z = 0.f;
    if (g < G) {
      const uint32_t r = regs[g * m + kb + kk];
      a = __builtin_amdgcn_ldexpf(1.0f, -(int)r);
      z = r == 0 ? 1.f : 0.f;
    }
    acc_sum = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bsel, acc_sum, 0, 0, 0);
    acc_zero = __builtin_amdgcn_mfma_f32_32x32x2f32(z, bsel, acc_zero, 0, 0, 0);
  }
  // D[row][col]: col = lane & 31, row = (reg & 3) + 8*(reg >> 2) + 4*(lane >> 5). Column 0 holds sums.
  if ((lane & 31) == 0) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
      const int64_t gg = g0 + row;
      if (gg < G) {
        const double s = acc_sum[reg];
        const double zeros = acc_zero[reg];
        const double mm = (double)m;
        const double alpha = 0.7213 / (1.0 + 1.079 / mm);
        double e = alpha * mm * mm / s;
        if (e <= 2.5 * mm && zeros > 0) e = mm * log(mm / zeros);
        est[gg] = e;
      }
    }
  }
}

}  // namespace sdo

// explicit instantiations launched from bindings.cpp
template __global__ void sdo::olap_scan_kernel<1>(const sdo::ScanDesc* __restrict__);
template __global__ void sdo::olap_scan_kernel<2>(const sdo::ScanDesc* __restrict__);
template __global__ void sdo::olap_scan_kernel<4>(const sdo::ScanDesc* __restrict__);
