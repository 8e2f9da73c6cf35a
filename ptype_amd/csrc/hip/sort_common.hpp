// Counting-sort building blocks shared by the sorted epoch mailboxes
// (mailbox_sort.hip) and the sorted exchange (exchange_sorted.hip): a batch is
// cut into tiles of kSTile messages, each block owns a contiguous range of tiles
// (XCD-grouped, see virt_block), messages are resolved against the registry
// mirror, and a message's rank within its (tile, bucket) is computed in MESSAGE
// order by a wave match on the bucket bits plus per-wave counts -- a stable sort
// with no atomic per message.
#pragma once
#include "common.hpp"
#include "route_common.hpp"

namespace ptype {

// 512 threads (8 waves) per block, 4096-message tiles: with 256 shards a tile
// gives each shard a run of ~16 records (256 B, two whole lines) instead of ~8
// -- half-written lines evicted from L2 before their other half arrived made
// the 2048-message tiles write 1.9x the record bytes (PMC, r3).
constexpr int kST = 512;                 // count / scatter threads per block
constexpr int kSK = 8;                   // messages per thread per tile
constexpr int kSTile = kST * kSK;        // 4096 messages
constexpr int kSWave = kSK * kWave;  // a wave's contiguous run of a tile (512)



struct SortIn {  // by value
  const uint32_t* actor;
  const int64_t* a0;
  const int64_t* a1;
  const int64_t* a2;
  const uint16_t* mcol;
  uint32_t method_uniform;
  int64_t M;
  const TableEntry* table;
  uint64_t mask;
  const uint32_t* dir;
  const uint8_t* dirr;  // MODE 3: the directory's rank byte table (one byte per id: 4x fewer lines than dir)
  const uint32_t* pres;  // MODE 4: the directory's 2-bit presence map for rank_self (staged in LDS per block)
  uint32_t n_dir;
  uint32_t aw;
  int aw_shift;
  int rank_self;
  uint32_t origin_base;
  uint32_t G;      // blocks
  uint32_t tiles;  // ceil(M / kSTile)
  uint32_t tpb;    // tiles per block
  // 8-B ring records (stateless mailbox Sends, mailbox_sort.hip): nonzero = on; the field widths
  // (mailbox bits | a0 bits << 8 | a1 bits << 16, zigzag arguments) are the device word *r8w,
  // set by the previous Send's last block from its per-tile field maxima (r8max)
  uint32_t rec8;
  const uint32_t* r8w;
  uint32_t* r8max;
  // ordered 8-B records: a message whose fields do not fit keeps its ring slot as an
  // ESCAPE record (bit 63 set, place in the tile kept) and its {a0, mailbox} go here,
  // indexed by ring slot -- so the ring stays each actor's FIFO (no overflow, no hole)
  int64_t* r8esc;
  // wide pure records (a stateless batch of one pure method -- no state, no actor read --
  // whose arguments outgrew the 8-B fields): plane A holds {a0, a1} whole, and the
  // message's place in its tile is a u16 at the same slot of plane B's memory (18 B per
  // message instead of the 32-B long form).  The tile maxima are still kept (r8max), so
  // the next Send returns to 8-B records once its values fit again.
  uint32_t recw;
};

// Block b's range: XCD (b % 8) owns virtual blocks [x * G/8, (x+1) * G/8).
__device__ __forceinline__ uint32_t virt_block(uint32_t b, uint32_t G) {
  return (G >= 8 && (G & 7) == 0) ? (b & 7) * (G >> 3) + (b >> 3) : b;
}

// Route modes: 0 hash probe, 1 directory gather (rank, mailbox), 2 affine rule
// (computed), 3 rank byte gather -- stateless batches only: `mb` is then the
// actor id itself (the receiver's stateless handler needs no mailbox), except for
// ids the byte table sends to the hash table, which keep the probed mailbox.
template <int MODE, int SK = kSK>
__device__ __forceinline__ void resolve_k(const SortIn& in, const uint32_t (&a)[SK], int (&r)[SK],
                                          uint32_t (&mb)[SK]) {
  if constexpr (MODE == 3) {
    uint32_t w[SK];
#pragma unroll
    for (int k = 0; k < SK; ++k) w[k] = a[k] < in.n_dir ? (uint32_t)in.dirr[a[k]] : (uint32_t)kRankFallback;
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      r[k] = w[k] == kRankMissing ? -1 : (int)w[k];
      mb[k] = a[k];
      if (w[k] == kRankFallback) {
        if (a[k] != 0xffffffffu) lookup_entry(in.table, in.mask, actor_key(a[k]), r[k], mb[k]);
        else r[k] = -1;
      }
    }
  } else if constexpr (MODE == 1) {
    uint32_t w[SK];
#pragma unroll
    for (int k = 0; k < SK; ++k) w[k] = a[k] < in.n_dir ? in.dir[a[k]] : kDirFallback;
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      r[k] = w[k] == kDirMissing ? -1 : (int)(w[k] & 0xff);
      mb[k] = w[k] >> 8;
      if (w[k] == kDirFallback) {
        if (a[k] != 0xffffffffu) lookup_entry(in.table, in.mask, actor_key(a[k]), r[k], mb[k]);
        else r[k] = -1;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      if (MODE == 2 && a[k] < in.n_dir) {
        r[k] = in.aw_shift >= 0 ? (int)(a[k] & (in.aw - 1)) : (int)(a[k] % in.aw);
        mb[k] = in.aw_shift >= 0 ? a[k] >> in.aw_shift : a[k] / in.aw;
      } else if (a[k] == 0xffffffffu) {
        r[k] = -1;
        mb[k] = 0;
      } else {
        lookup_entry(in.table, in.mask, actor_key(a[k]), r[k], mb[k]);
      }
    }
  }
}

// Message i of tile t for (item k, lane) of wave w: a wave owns a contiguous run
// of the tile, so message order within a tile is (wave, item, lane).
// SK: messages per thread of the tile (kSK by default; the fused mailbox Send of a
// small batch takes smaller tiles, mailbox_sort.hip).
template <int SK = kSK>
__device__ __forceinline__ int64_t tile_index(uint32_t t, int k) {
  return (int64_t)t * (kST * SK) + (threadIdx.x / kWave) * (SK * kWave) + k * kWave + lane_id();
}

template <int SK = kSK>
__device__ __forceinline__ void load_actors(const SortIn& in, uint32_t t, uint32_t (&a)[SK]) {
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int64_t i = tile_index<SK>(t, k);
    a[k] = i < in.M ? __builtin_nontemporal_load(in.actor + i) : 0xffffffffu;
  }
}

// Lanes of this wave whose `key` (log_bits bits) equals this lane's, among `act`.
__device__ __forceinline__ uint64_t match_bits(uint32_t key, uint32_t log_bits, uint64_t act) {
  uint64_t m = act;
  for (uint32_t b = 0; b < log_bits; ++b) {
    const uint64_t bb = __ballot((key >> b) & 1u);
    m &= ((key >> b) & 1u) ? bb : ~bb;
  }
  return m;
}

// A tile's raw inputs, loaded one tile ahead of their use.
struct SortTileIn {
  uint32_t a[kSK];
  int64_t x0[kSK], x1[kSK], x2[kSK];
};

__device__ __forceinline__ void load_args(const SortIn& in, uint32_t t, SortTileIn& x) {
#pragma unroll
  for (int k = 0; k < kSK; ++k) {
    const int64_t i = tile_index(t, k);
    const bool ok = i < in.M;
    x.a[k] = ok ? __builtin_nontemporal_load(in.actor + i) : 0xffffffffu;
    x.x0[k] = ok ? __builtin_nontemporal_load(in.a0 + i) : 0;
    x.x1[k] = ok && in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
    x.x2[k] = ok && in.a2 ? __builtin_nontemporal_load(in.a2 + i) : 0;
  }
}

__device__ __forceinline__ bool fits_i32(int64_t v) { return v == (int64_t)(int32_t)v; }

// ---------------------------------------------------------------- one-pass sorts: decoupled look-back
// Per (tile, bucket) descriptors, u64 {epoch tag 24 | status 2 | value 38}, published
// with memory-side atomic exchanges and read with memory-side no-op atomics: the
// per-XCD L2s are not coherent within a kernel, so a plain or sc1 poll could keep
// reading a stale line (mailbox_dev.hpp ld_fresh).  The tag comes from a device
// word advanced once per Send, so earlier Sends' descriptors (and graph replays')
// read as unpublished without any clearing.  Users: mailbox_sort.hip
// mbx_onesweep_kernel, exchange_sorted.hip sx_onesweep_kernel.
constexpr uint64_t kDescA = 1ull << 38, kDescP = 2ull << 38, kDescVal = (1ull << 38) - 1;
__device__ __forceinline__ uint64_t desc_word(uint32_t tag, uint64_t status, uint64_t v) {
  return ((uint64_t)tag << 40) | status | v;
}
// A Send's descriptor tag from its device counter: 1..0xffffff for every counter
// value (2^24 - 1 distinct tags; a plain `(ctr & 0xffffff) + 1` reaches 0x1000000,
// whose shift out of the 24-bit field would publish tag 0 and stall every look-back).
__host__ __device__ __forceinline__ uint32_t epoch_tag(uint32_t ctr) { return ctr % 0xffffffu + 1u; }
constexpr uint32_t kLookbackSpins = 1u << 20;  // a bug guard (a lost descriptor must not hang the GPU)

// Sum of the descriptors of tiles q, q-1, ... (stride `stride` words apart, this
// column's) back to the first inclusive prefix: a window of kLbWin predecessors
// is read at once (memory-side atomics in flight together -- one round trip per
// window instead of one per tile); an unpublished entry is re-polled.
constexpr int kLbWin = 8;
__device__ __forceinline__ uint64_t lookback(unsigned long long* col, uint32_t stride, int64_t q, uint32_t tag,
                                             unsigned long long& timeouts) {
  uint64_t excl = 0;
  uint32_t spins = 0;
  while (q >= 0) {
    uint64_t x[kLbWin];
#pragma unroll
    for (int j = 0; j < kLbWin; ++j)
      x[j] = q - j >= 0 ? __hip_atomic_fetch_add(col + (size_t)(q - j) * stride, 0ull, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                        : desc_word(tag, kDescP, 0);  // before tile 0: 0
    int j = 0;  // entries consumed (unrolled with flags: a register array indexed at run time spills to scratch)
    bool done = false, stall = false;
#pragma unroll
    for (int k = 0; k < kLbWin; ++k) {
      if (done || stall) continue;
      if ((uint32_t)(x[k] >> 40) != tag) {  // not published yet: poll it again
        stall = true;
        continue;
      }
      excl += x[k] & kDescVal;
      ++j;
      if (x[k] & kDescP) done = true;
    }
    if (done) break;
    q -= j;
    if (stall) {
      if (++spins > kLookbackSpins) {
        ++timeouts;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return excl;
}

}  // namespace ptype
