// Shared between p2p.hip (device) and bindings.cpp (host launch): the P2P merge kernel's arguments.
#pragma once
#include <stdint.h>

namespace sdo {

constexpr int P2P_MAX_RANKS = 8;
constexpr int P2P_MAX_SLOTS = 64;
constexpr int64_t P2P_HEADER = 256;        // bytes: publish, done, 2 verdict and 2 final words, padding
constexpr int64_t P2P_STATUS_TIMEOUT = 3;  // a peer never finished the epoch (hard wait expired)
constexpr int64_t P2P_STATUS_RETRY = 4;    // the epoch was abandoned by agreement: re-merge over RCCL

struct P2PArgs {
  uint64_t mbox[P2P_MAX_RANKS];  // every rank's mailbox base, as mapped in this process (own included)
  int nranks;
  int rank;
  uint64_t epoch;                // >= 1, strictly increasing per exchange
  int64_t slot_bytes;            // capacity of one data slot
  int64_t nacc;                  // accumulator words (rows x nslots)
  int64_t nhll;                  // HLL register bytes (multiple of 8)
  int nslots;
  int ops[P2P_MAX_SLOTS];        // SlotOp per slot
  const int64_t* acc_src;
  const uint8_t* hll_src;
  int64_t status;
  int64_t* acc_out;
  uint8_t* hll_out;
  int64_t* status_out;           // [nranks]
  int64_t soft_ticks;            // wall_clock64 ticks (100 MHz): wait for the peers' partials
  int64_t hard_ticks;            // wait for the peers' verdicts (they already arrived: only a dead peer)
};

}  // namespace sdo
