// Query-program descriptor shared by the host lowering (engine/lower.py builds the identical
// byte layout with numpy structured dtypes, see ops/desc.py) and the CDNA4 scan kernels.
//
// A Druid QuerySpec (reference: src/main/scala/org/sparklinedata/druid/DruidQuerySpec.scala:573-1127)
// is lowered into ONE of these per (query, GPU).  The kernel is an interpreter over the descriptor:
// every opcode is wave-uniform, so interpretation costs scalar branches only, and the
// per-row work is loads + a handful of VALU ops.  The layout is plain-old-data with explicit
// padding; never reorder fields without updating ops/desc.py (a unit test checks the sizes).
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#else
using __hip_internal::int8_t;
using __hip_internal::int16_t;
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint8_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#endif

namespace sdo {

constexpr int MAX_COLS = 24;      // cols[0..8): filter-phase columns, cols[8..24): payload columns
constexpr int PAYLOAD_BASE = 8;
constexpr int MAX_FOPS = 48;
constexpr int MAX_KOPS = 8;
constexpr int MAX_AOPS = 12;
constexpr int MAX_EOPS = 64;
constexpr int MAX_ZONES = 4;
constexpr int MAX_RANGES = 8;
constexpr int MAX_SLOTS = 16;
constexpr int MAX_BM = 8;           // inverted-bitmap leaves evaluated at chunk level
constexpr int STACK_DEPTH = 6;       // filter / expression register stack depth
constexpr int CHUNK_ROWS = 4096;     // zone-map granule == scheduling unit (64 words of 64 rows)
constexpr int CHUNK_WORDS = CHUNK_ROWS / 64;

enum DType : int32_t { DT_U8 = 0, DT_I16 = 1, DT_I32 = 2, DT_I64 = 3, DT_F32 = 4, DT_F64 = 5, DT_U16 = 6 };

// ---- filter opcodes (postfix program; evaluated on 64-bit wave masks, one bit per lane/row) ----
enum FOpCode : int32_t {
  F_TRUE = 0,
  F_BITMAP = 1,     // push bitmap leaf `lo` (chunk-level OR of bm_count rows of an inverted bitmap index)
  F_ID_RANGE = 2,   // push lo <= id < hi
  F_IN_SET = 3,     // push bitset[id]    (dictionary-domain predicate, evaluated once per dict entry)
  F_INT_RANGE = 4,  // push lo <= v <= hi   (integer / decimal-scaled metric or time)
  F_FLT_RANGE = 5,  // push flo <= v <= fhi (flags: bit0 lo-strict, bit1 hi-strict)
  F_AND = 6,
  F_OR = 7,
  F_NOT = 8,
  F_FALSE = 9,
  F_BITMAP_OR = 10,  // push OR of `hi` consecutive bitmap rows starting at bits (stride lo words)
  F_EXPR = 11        // push flo <= expr(eops[lo, lo+hi)) <= fhi (flags as F_FLT_RANGE; NaN fails)
};

struct ColRef {
  uint64_t ptr;
  int32_t dtype;
  int32_t meta;  // host-packed: lg | signed << 4 | float << 5 | LDS plane << 8
};

struct FOp {
  int32_t op;
  int32_t col;
  int32_t flags;
  int32_t pad;
  int64_t lo;
  int64_t hi;
  double flo;
  double fhi;
  uint64_t bits;
};

// ---- group-key components: key = sum(component * stride) ----
enum KKind : int32_t { K_ID = 0, K_REMAP = 1, K_TIME = 2, K_INT = 3 };
enum TField : int32_t {
  T_MS = 0, T_SECOND = 1, T_MINUTE = 2, T_HOUR = 3, T_DAY = 4, T_WEEK = 5, T_MONTH = 6,
  T_QUARTER = 7, T_YEAR = 8, T_MOY = 9, T_DOM = 10, T_DOW = 11, T_HOD = 12, T_MOH = 13,
  T_DOY = 14, T_SOM = 15, T_QOY = 16, T_PERIOD = 17
};

struct KOp {
  int32_t kind;
  int32_t col;
  int32_t tfield;
  int32_t pad;
  int64_t stride;
  int64_t base;
  int64_t card;
  int64_t unit_ms;    // time column storage unit
  int64_t tz_ms;      // fixed timezone offset applied before bucketing
  int64_t period_ms;  // T_PERIOD
  int64_t origin_ms;  // T_PERIOD
  uint64_t remap;     // int32 table for K_REMAP (dictionary-domain derived key)
};

// ---- aggregators ----
enum AKind : int32_t {
  A_COUNT = 0, A_SUM_I = 1, A_SUM_F = 2, A_MIN_I = 3, A_MAX_I = 4, A_MIN_F = 5, A_MAX_F = 6, A_HLL = 7,
  A_SUM_X = 8,  // exact decimal expression sum: llrint(expr) (expr pre-scaled by 10^scale) into S_SUM_I
  A_HLL_STORED = 9,  // union of the row's stored (rolled-up) HLL sketch into the group's registers (JIT only)
  A_ROWID = 10,      // emit producers: the row id as a record field (JIT only)
  A_HLL_CODE = 11    // HLL over a code column: u16 (bucket << 5 | rho) per row (segment/hllcode.py)
};
// accumulator slot update ops
enum SlotOp : int32_t { S_SUM_I = 0, S_SUM_F = 1, S_MIN_I = 2, S_MAX_I = 3 };

struct AOp {
  int32_t kind;
  int32_t col;        // input column (or -1 when expr_len > 0)
  int32_t expr_off;   // expression program (float VM) offset into eops
  int32_t expr_len;
  int32_t filt_off;   // per-aggregator filter program (Druid "filtered" aggregator)
  int32_t filt_len;
  int32_t slot;       // accumulator slot (non-HLL)
  int32_t hll_lds_off;// byte offset of this HLL's registers in LDS (when desc.hll_lds)
  uint64_t hll_regs;  // global byte registers [groups][1<<hll_p]
  int64_t salt;
  uint64_t sk_off;    // A_HLL_STORED: int64 [rows + 1] CSR offsets of the rows' stored sketches
  uint64_t sk_val;    //               int32 packed (bucket << 8 | rho) pairs
};

enum EOpCode : int32_t {
  E_COL = 0, E_CONST = 1, E_ADD = 2, E_SUB = 3, E_MUL = 4, E_DIV = 5, E_NEG = 6, E_ABS = 7,
  E_MIN = 8, E_MAX = 9,
  // unary math (floor ceil sqrt ln exp) and binary mod / pmod / pow
  E_FLOOR = 10, E_CEIL = 11, E_SQRT = 12, E_LOG = 13, E_EXP = 14, E_MOD = 15, E_PMOD = 16, E_POW = 17,
  E_LUT = 18  // push lut[id]: f64 dictionary-domain value of a dimension (pointer bits in c)
};
struct EOp {
  int32_t op;
  int32_t col;
  double c;
};

struct ZoneP {
  int32_t col;
  int32_t pad;
  int64_t lo;    // zone survives iff zmax >= lo && zmin < hi
  int64_t hi;
  uint64_t zmin; // int32 per chunk
  uint64_t zmax;
};

struct Range {
  int64_t lo;
  int64_t hi;
  int64_t chunk_begin;  // first absolute chunk index of this range
  int64_t nchunks;
};

enum Mode : int32_t { M_DENSE_LDS = 0, M_DENSE_GLOBAL = 1, M_HASH = 2, M_MASK = 3, M_PART = 4 };

struct ScanDesc {
  int32_t ncols, nfops, nkops, naggs;
  int32_t neops, nranges, nzones, nslots;
  int32_t mode;
  int32_t dedup;
  int32_t hll_lds;
  int32_t hll_p;
  int32_t nhll;
  int32_t lds_bytes;
  int32_t filter_len;   // main filter program = fops[0 .. filter_len)
  int32_t pad0;
  int64_t G;            // dense groups
  int64_t total_chunks;
  int64_t num_rows;
  uint64_t out_acc;     // u64 [G or cap][nslots]
  uint64_t out_keys;    // u64 [cap]   (hash mode)
  int64_t hash_cap;     // power of two
  uint64_t overflow;    // int32 flag (hash mode)
  uint64_t out_mask;    // u64 per 64-row word (mask mode)
  uint64_t out_count;   // u64 rows passing (mask mode)
  int64_t slot_init[MAX_SLOTS];
  int32_t slot_op[MAX_SLOTS];
  ColRef cols[MAX_COLS];
  FOp fops[MAX_FOPS];
  KOp kops[MAX_KOPS];
  AOp aops[MAX_AOPS];
  EOp eops[MAX_EOPS];
  ZoneP zones[MAX_ZONES];
  Range ranges[MAX_RANGES];
  // ---- v3: chunk-level bitmap pre-filter + per-wave LDS staging of column tiles (LDS-DMA) ----
  int32_t nfc;            // filter-phase columns: cols[0 .. nfc)
  int32_t npc;            // payload columns: cols[PAYLOAD_BASE .. PAYLOAD_BASE + npc)
  int32_t pre_off;        // bitmap-only conjuncts: fops[pre_off .. pre_off + pre_len), evaluated per chunk
  int32_t pre_len;
  int32_t final_pre;      // the pre-filter IS the whole filter (no per-row leaves)
  int32_t nbm;
  int32_t nplanes;        // 4-byte x 64-lane LDS planes per word (64-bit columns take two)
  int32_t lds_cache_off;  // byte offset of the per-wave staging regions in dynamic LDS
  int32_t lds_wave_bytes; // bytes per wave: nplanes * U * 256 + nbm * 512
  int32_t unroll;         // U (words per step) the host sized the regions for
  int32_t narrow4;        // LDS-DMA of 1/2-byte elements lands at lane*4 (probed at load time)
  int32_t pad2;
  uint64_t bm_bits[MAX_BM];
  int64_t bm_stride[MAX_BM];
  int64_t bm_count[MAX_BM];
  // radix-partitioned group-by (mode M_PART, partition.hip): the scan emits records instead of
  // updating a table.  part_recs: record storage (chunk c owns records [4096 c, 4096 c + 4096));
  // part_counts: each chunk's record end offset, stored at the chunk's position in workgroup order
  // (the chunks of producer block 0, then block 1, ...: ops/jit.py part_positions); part_base,
  // when set: the level-1 bucket histogram [part_n][gridDim.x] of the records each producer block
  // appended -- the split's count pass is then skipped.
  uint64_t part_recs;
  uint64_t part_counts;
  uint64_t part_base;
  int32_t part_shift;     // level-1 bucket = (record key >> part_shift) & (part_n - 1)
  int32_t part_n;         // level-1 buckets (a power of two <= PART_HIST_BUCKETS)
};

// Fields of a partition record (partition.hip part_agg_kernel): value j is width[j] u32 words
// (0 = implicit 1, 1 = i32, 2 = i64) folded into slot[j] with op[slot].
// width: u32 words of the field in the record (0: an implicit 1, 1: int32, 2: int64 / f64 bits) or
// PART_PACKED: a small non-negative value the level-1 split packed into the key word above bit
// pk_shift (the bits the sub-bucket already implies), so the record is one word narrower.
constexpr int32_t PART_PACKED = 3;
struct PartFields {
  int32_t nfields;
  int32_t nslots;
  int32_t slot[MAX_SLOTS];
  int32_t width[MAX_SLOTS];
  int32_t op[MAX_SLOTS];
  int64_t init[MAX_SLOTS];
  int32_t pk_shift;  // bit of the packed field in the key word (0: no packed field)
  int32_t pad_;
};

// HLL aggregators of the partitioned group-by (partition.hip part_agg_kernel): each record carries
// one (bucket << 8 | rho) word per HLL after its value fields; a sub-bucket's groups keep their
// byte registers in LDS and write them to their rows of the [G][2^p] register tables.  A stored
// (rolled-up hyperUnique) sketch -- bit h of `stored` -- carries the row id instead (0xffffffff: the
// aggregator's filter rejected the row), and the row's sparse (bucket << 8 | rho) pairs
// sk_val[sk_off[row] .. sk_off[row + 1]) are unioned into the group's registers.
constexpr int PART_MAX_HLL = 4;
struct PartHll {
  int32_t n;
  int32_t p;
  unsigned char* regs[PART_MAX_HLL];
  uint32_t stored;
  const int64_t* sk_off[PART_MAX_HLL];
  const int32_t* sk_val[PART_MAX_HLL];
};

// HAVING fused into the partitioned aggregation (partition.hip part_agg_kernel): up to 4
// comparisons of a slot value (int64 / scale divisor, or f64 bits) with a constant, AND-ed or
// OR-ed.  nterms == 0: write the dense table instead.
struct PartHaving {
  int32_t nterms;
  int32_t conj;           // 1: all terms, 0: any term
  int32_t slot[4];
  int32_t f64[4];         // slot holds double bits (else int64 divided by div)
  int32_t op[4];          // 0 equalTo, 1 greaterThan, 2 lessThan
  int32_t pad;
  double div[4];
  double c[4];
  // ORDER BY <slot> LIMIT tk fused as well (tk > 0, <= PART_TOPK_MAX; nterms may be 0): only groups
  // ranking at or above the block's tk-th best and the best tk-th any earlier block published
  // (out_count[1]) leave the kernel -- a superset of the global top tk with every tie, which the
  // host orders and limits exactly.  tk_f64: the slot holds double bits; tk_desc: larger first.
  int32_t tk;
  int32_t tk_slot;
  int32_t tk_f64;
  int32_t tk_desc;
};
constexpr int PART_TOPK_MAX = 16;

}  // namespace sdo
