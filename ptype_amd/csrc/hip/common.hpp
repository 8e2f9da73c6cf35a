// Common gfx950 helpers for the ptype device runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdexcept>
#include <string>

#include "records.hpp"
#include "tune.hpp"

#define PT_HIP_CHECK(expr)                                                                 \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " \
                               + __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")"); \
  } while (0)

namespace ptype {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// GPU registry table entry: 16 bytes so a lane probes with one dwordx4 load.
struct alignas(16) TableEntry {
  uint64_t key;   // 0 = empty, ~0 = tombstone
  uint32_t rank;  // owning GPU rank (one process per GPU)
  uint32_t mbox;  // local mailbox / actor-state index on that rank
};
static_assert(sizeof(TableEntry) == 16, "TableEntry must be 16 bytes");

constexpr uint64_t kKeyEmpty = 0ull;
constexpr uint64_t kKeyTomb = ~0ull;

// table stats words (uint64): live entries, tombstones, generation, max probe seen
enum TableStat { kStatLive = 0, kStatTomb = 1, kStatGen = 2, kStatMaxProbe = 3, kStatWords = 8 };

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  // splitmix64 finalizer: full-avalanche, cheap on the SALU/VALU
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// Probing starts at the 4-slot group (one 64-B line) the hash lands in, so a
// lookup issues the whole line as four independent dwordx4 loads and resolves
// almost every key with ONE memory latency (linear probing, load factor <= 0.5).
constexpr int kGroup = 4;
__host__ __device__ __forceinline__ uint64_t probe_start(uint64_t key, uint64_t mask) {
  return mix64(key) & mask & ~(uint64_t)(kGroup - 1);
}

// Actor ids used on the batch path map to table keys as id + 1 (0 is "empty").
__host__ __device__ __forceinline__ uint64_t actor_key(uint32_t actor) { return (uint64_t)actor + 1ull; }

// Route directory words (dense actor-id -> route word array, see K5b):
// 0xFFFFFFFF = not registered; kDirFallback = probe the hash table instead.
constexpr uint32_t kDirMissing = 0xffffffffu;
constexpr uint32_t kDirFallback = 0xfffffffeu;
// The directory's rank byte table (K5c, one byte per actor id, built with the
// directory): 0xFF = not registered; kRankFallback = probe the hash table.
constexpr uint8_t kRankMissing = 0xffu;
constexpr uint8_t kRankFallback = 0xfeu;

__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }

__device__ __forceinline__ unsigned mbcnt64(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Inclusive prefix sum across the 64 lanes of a wave with DPP row shifts (VALU,
// a few cycles each) instead of ds_bpermute shuffles (~100-cycle LDS-path round
// trips, six of them in a dependent chain): 4 row_shr steps scan each 16-lane
// row, then the three row totals are read as scalars and added to later rows.
__device__ __forceinline__ unsigned wave_incl_scan(unsigned v) {
  const unsigned lane = __lane_id();
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  const unsigned t0 = (unsigned)__builtin_amdgcn_readlane((int)v, 15);
  const unsigned t1 = (unsigned)__builtin_amdgcn_readlane((int)v, 31);
  const unsigned t2 = (unsigned)__builtin_amdgcn_readlane((int)v, 47);
  const unsigned row = lane >> 4;
  return v + (row > 0 ? t0 : 0u) + (row > 1 ? t1 : 0u) + (row > 2 ? t2 : 0u);
}

__device__ __forceinline__ uint64_t realtime_ticks() {  // 100 MHz constant clock
  return __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ void spin_ticks(uint64_t ticks) {
  if (!ticks) return;
  const uint64_t t0 = realtime_ticks();
  while (realtime_ticks() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// Two-level "last block out" ticket.  Same-address atomics serialise at the
// memory side (~8-10 ns each on MI355X: 8192 blocks taking one ticket word cost
// ~80 us, measured), so block b counts itself in group word b % kTicketGroups and
// the last block of each group counts the group in the top word: no word sees
// more than G / kTicketGroups + kTicketGroups atomics.  `words` holds
// kTicketWords u32, zero between launches (the winners reset them).  Call from
// ONE thread per block, after that block's own device-scope atomics have landed
// (their returned values consumed); returns true in exactly one block.
constexpr unsigned kTicketGroups = 64;
constexpr unsigned kTicketWords = kTicketGroups + 1;
__device__ __forceinline__ bool last_block_ticket(unsigned* words) {
  const unsigned G = gridDim.x, g = blockIdx.x % kTicketGroups;
  const unsigned in_group = (G - g + kTicketGroups - 1) / kTicketGroups;
  if (atomicAdd(&words[g], 1u) != in_group - 1) return false;
  atomicExch(&words[g], 0u);
  const unsigned groups = G < kTicketGroups ? G : kTicketGroups;
  if (atomicAdd(&words[kTicketGroups], 1u) != groups - 1) return false;
  atomicExch(&words[kTicketGroups], 0u);
  return true;
}

// A stream for PERSISTENT kernels (the dispatcher wave, the mailbox consumer).
// HIP maps ordinary streams round-robin onto a small pool of hardware queues per
// priority level (GPU_MAX_HW_QUEUES, 4 on the box), so a persistent kernel on a
// pooled stream sits in an in-order queue AHEAD of work that later streams put
// on the same queue -- including the very enqueue it waits for (a live mailbox
// session then stalls until the consumer's lifetime bound; a Send behind the
// dispatcher waits for its idle exit: measured 2975 ms, tools/pstream_probe.py).
// tune persistent_stream selects the placement (tune.hpp):
//   low    (default) a non-blocking stream at the lowest priority: its own queue
//          pool, which only persistent kernels use
//   cumask a CU-masked stream (a dedicated queue, never pooled) -- but HIP makes
//          it a BLOCKING stream, so legacy null-stream work waits for the
//          resident kernel (torch's default stream is the null stream)
//   pooled an ordinary non-blocking stream (the hazard above)
inline hipStream_t dedicated_stream(int device) {
  hipStream_t s = nullptr;
  const std::string mode = tune().persistent_stream;
  if (mode == "cumask") {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) {
      uint32_t mask[32];
      const uint32_t words = (uint32_t)((cus + 31) / 32) < 32u ? (uint32_t)((cus + 31) / 32) : 32u;
      for (uint32_t i = 0; i < words; ++i) mask[i] = 0xffffffffu;
      if (hipExtStreamCreateWithCUMask(&s, words, mask) == hipSuccess) return s;
    }
    (void)hipGetLastError();
  } else if (mode != "pooled") {
    // HIP reports the range [0 (normal), -1 (high)]; a value above 0 selects the
    // runtime's low-priority level, whose queue pool ordinary streams never use
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
        hipStreamCreateWithPriority(&s, hipStreamNonBlocking, mode == "high" ? greatest : least + 1) == hipSuccess)
      return s;
    (void)hipGetLastError();
  }
  PT_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return s;
}

}  // namespace ptype
