// ec_server.h -- shared layout of the stripe server (ec_server.hip) and its host side
// (ec_stripe_server.cpp, StripeServer).  Internal to liblstore_ec.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ec_kernels.h"

namespace lsec {

#ifndef LSEC_SRV_WG
#define LSEC_SRV_WG 32
#endif
constexpr int kSrvWG = LSEC_SRV_WG;  // server workgroups (one per CU they land on)
constexpr int kSrvSlotsPerWG = 31;  // post words 0-30 (two 64-byte lines); word 31 is the stop word
constexpr int kSrvSlots = kSrvWG * kSrvSlotsPerWG;
constexpr size_t kSrvSlotBytes = 96u << 10;  // chunk bytes of one slot (a part's inputs + outputs)
constexpr int kSrvMaxK = 32;        // inputs of one request the server takes
constexpr int kSrvMaxR = 8;         // outputs of one request the server takes
constexpr uint32_t kSrvBytewise = 1, kSrvBitsliced = 2;

// slot s of workgroup g's word i: consecutive slots belong to different workgroups, so the
// parts of one request (claimed as consecutive slots) are served in parallel
__host__ __device__ inline int srv_slot(int g, int i) { return i * kSrvWG + g; }
__host__ __device__ inline int srv_wg(int s) { return s % kSrvWG; }
__host__ __device__ inline int srv_word(int s) { return s / kSrvWG; }

// one request part: one column block of one stripe (size bytes of every shard)
struct SrvDesc {
  uint32_t kind, K, R, packet;
  uint64_t size;
  uint64_t cells;    // device address of row 0's cell 0; row r at cells + r * cstride cells
  uint32_t cstride, pad;
  uint64_t in[kSrvMaxK];   // device-visible addresses (page-locked host memory)
  uint64_t out[kSrvMaxR];
};

// page-locked coherent host memory shared by the host threads and the server
struct SrvShared {
  uint32_t post[kSrvWG][32];
  uint32_t done[kSrvSlots][16];  // done[s][0]; one 64-byte line per slot
  SrvDesc desc[kSrvSlots];
};

struct SrvArgs {
  SrvShared *shared;   // device address of the shared block
  int *votes;          // device memory: workgroups that voted to retire (zeroed before a launch)
  uint64_t idle_ticks; // 100 MHz wall clock ticks of idleness before a workgroup votes
  uint32_t hold;       // test hook: nonzero = poll but serve nothing (lsec_test_server_hold)
  uint32_t pad;
};

hipError_t launch_stripe_server(const SrvArgs &a, hipStream_t stream);

}  // namespace lsec
