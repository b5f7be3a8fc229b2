// Argument blocks shared by post_scan.hip and the host launchers (bindings.cpp).
#pragma once
#include <stdint.h>

namespace sdo {

constexpr int DEC_MAX_COLS = 16;
struct DecCol {
  int32_t kind;    // 0 key id, 1 integer slot, 2 ordered-float slot, 3 raw slot bits, 4 group id
  int32_t out;     // 0 int16, 1 int32, 2 int64, 3 f64 from the (integer) value, 4 raw 64-bit, 5 int64 from a double
  int32_t lut_t;   // 0 none, 1 int32 table, 2 int64 table, 3 f64 table
  int32_t slot;
  int64_t stride, card, add;
  const int64_t* orig;  // FD determinant's original ids (or null)
  const void* lut;
  double div;           // decimal scale divisor (0: none)
  int64_t off;          // byte offset of the column in the output buffer
};
struct DecArgs {
  const int64_t* idx;
  const int64_t* acc;
  int64_t n;
  int32_t ns, ncols;
  unsigned char* out;
  DecCol c[DEC_MAX_COLS];
};

}  // namespace sdo
