// GPU-resident registry mirror (SURVEY C9 / kernels K5, K6, K7).
//
// The authoritative registry lives in the Raft-replicated MVCC store (host);
// this open-addressing hash table in HBM mirrors it for device-side routing so
// the batch path never leaves the GPU to resolve a destination.  Reference
// behaviour it mirrors: Register/Services/nodes (cluster/registry.go:51-166) and
// lease expiry (cluster/registry.go:59, 2 s TTL).
//
// Layout: 16-byte entries {u64 key, u32 rank, u32 mbox}; a side array of u64
// expiry deadlines (host monotonic ms, 0 = never); capacity is a power of two
// sized 2x the live count (1M actors -> 2M slots -> 32 MB + 16 MB, trivially
// resident in 288 GB HBM and mostly in the 256 MB Infinity Cache).
// Probing is linear; deletes leave tombstones that lookups skip and upserts do
// not reuse, the host rebuilds (pack -> clear -> upsert) when they pile up.
#include "common.hpp"

namespace ptype {

// Block-reduce two counters (sum, max) and publish them with ONE atomic each per
// block; the generation is bumped once per launch (block 0).  Per-wave atomics
// on the same words from ~16K waves serialize across the 8 XCDs.
__device__ __forceinline__ void publish_block_stats(unsigned long long sum, unsigned long long mx,
                                                    unsigned long long* __restrict__ sum_word,
                                                    unsigned long long* __restrict__ max_word,
                                                    unsigned long long* __restrict__ gen_word, bool negate_sum) {
  __shared__ unsigned long long s_sum[4], s_max[4];
  for (int off = 32; off > 0; off >>= 1) {
    sum += __shfl_xor(sum, off);
    const unsigned long long o = __shfl_xor(mx, off);
    mx = o > mx ? o : mx;
  }
  const unsigned w = threadIdx.x / kWave;
  if (lane_id() == 0) {
    s_sum[w] = sum;
    s_max[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, m = 0;
    for (unsigned k = 0; k < blockDim.x / kWave; ++k) {
      a += s_sum[k];
      m = s_max[k] > m ? s_max[k] : m;
    }
    if (a && sum_word) atomicAdd(sum_word, negate_sum ? (unsigned long long)(-(long long)a) : a);
    if (m && max_word) atomicMax(max_word, m);
    if (blockIdx.x == 0 && gen_word) atomicAdd(gen_word, 1ull);
  }
  __syncthreads();  // the shared slots may be reused by a following call
}

__device__ __forceinline__ uint64_t ld_key(const TableEntry* e) {
  return __hip_atomic_load(&e->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Upsert input: either SoA columns (keys / ranks / mboxes) or packed TableEntry
// records as K7 writes them (`packed`, a restore: no host-side column split).
struct UpsertIn {
  const uint64_t* keys = nullptr;
  const uint32_t* ranks = nullptr;
  const uint32_t* mboxes = nullptr;
  const TableEntry* packed = nullptr;
  __device__ __forceinline__ void get(int64_t i, uint64_t& key, uint64_t& val) const {
    if (packed) {
      const uint4 v = *reinterpret_cast<const uint4*>(&packed[i]);
      key = ((uint64_t)v.y << 32) | v.x;
      val = ((uint64_t)v.w << 32) | v.z;
    } else {
      key = keys[i];
      val = ((uint64_t)mboxes[i] << 32) | ranks[i];
    }
  }
};

__global__ __launch_bounds__(256) void table_upsert_kernel(TableEntry* __restrict__ t, uint64_t mask, UpsertIn in,
                                                           const uint64_t* __restrict__ exp_in,
                                                           uint64_t* __restrict__ exp_tbl, int64_t n,
                                                           unsigned long long* __restrict__ stats) {
  unsigned long long added = 0, maxp = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t key, v;
    in.get(i, key, v);
    if (key == kKeyEmpty || key == kKeyTomb) continue;
    uint64_t h = probe_start(key, mask);
    uint64_t probe = 0;
    bool ok = false;
    for (; probe <= mask; ++probe, h = (h + 1) & mask) {
      uint64_t cur = ld_key(&t[h]);
      if (cur == key) { ok = true; break; }
      if (cur == kKeyEmpty) {
        uint64_t expected = kKeyEmpty;
        if (__hip_atomic_compare_exchange_strong(&t[h].key, &expected, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          ++added;
          ok = true;
          break;
        }
        if (expected == key) { ok = true; break; }
      }
    }
    if (!ok) continue;  // table full: host sizes capacity >= 2x live, never hit in practice
    *reinterpret_cast<uint64_t*>(&t[h].rank) = v;
    if (exp_tbl) exp_tbl[h] = exp_in ? exp_in[i] : 0ull;
    if (probe > maxp) maxp = probe;
  }
  publish_block_stats(added, maxp, &stats[kStatLive], &stats[kStatMaxProbe], &stats[kStatGen], false);
}

__global__ __launch_bounds__(256) void table_delete_kernel(TableEntry* __restrict__ t, uint64_t mask,
                                                           const uint64_t* __restrict__ keys, int64_t n,
                                                           unsigned long long* __restrict__ stats,
                                                           uint8_t* __restrict__ found_out) {
  unsigned long long removed = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    bool hit = false;
    if (key != kKeyEmpty && key != kKeyTomb) {
      uint64_t h = probe_start(key, mask);
      for (uint64_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
        uint64_t cur = ld_key(&t[h]);
        if (cur == kKeyEmpty) break;
        if (cur == key) {
          uint64_t expected = key;
          if (__hip_atomic_compare_exchange_strong(&t[h].key, &expected, kKeyTomb, __ATOMIC_RELAXED,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            ++removed;
            hit = true;
          }
          break;
        }
      }
    }
    if (found_out) found_out[i] = hit ? 1 : 0;
  }
  publish_block_stats(removed, 0, &stats[kStatLive], nullptr, &stats[kStatGen], true);
  publish_block_stats(removed, 0, &stats[kStatTomb], nullptr, nullptr, false);
}

__global__ __launch_bounds__(256) void table_lookup_kernel(const TableEntry* __restrict__ t, uint64_t mask,
                                                           const uint64_t* __restrict__ keys, int64_t n,
                                                           int32_t* __restrict__ out_rank,
                                                           int32_t* __restrict__ out_mbox) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    int32_t rank = -1, mbox = -1;
    if (key != kKeyEmpty && key != kKeyTomb) {
      uint64_t h = probe_start(key, mask);
      for (uint64_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
        const uint4 e = *reinterpret_cast<const uint4*>(&t[h]);  // one dwordx4
        const uint64_t k = ((uint64_t)e.y << 32) | e.x;
        if (k == key) { rank = (int32_t)e.z; mbox = (int32_t)e.w; break; }
        if (k == kKeyEmpty) break;
      }
    }
    out_rank[i] = rank;
    if (out_mbox) out_mbox[i] = mbox;
  }
}

// K6: lease sweep -- tombstone every entry whose deadline passed.
__global__ __launch_bounds__(256) void table_sweep_kernel(TableEntry* __restrict__ t, uint64_t cap,
                                                          const uint64_t* __restrict__ exp_tbl, uint64_t now,
                                                          unsigned long long* __restrict__ stats) {
  unsigned long long removed = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = exp_tbl[i];
    if (e == 0 || e >= now) continue;
    uint64_t k = ld_key(&t[i]);
    if (k == kKeyEmpty || k == kKeyTomb) continue;
    if (__hip_atomic_compare_exchange_strong(&t[i].key, &k, kKeyTomb, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      ++removed;
  }
  publish_block_stats(removed, 0, &stats[kStatLive], nullptr, &stats[kStatGen], true);
  publish_block_stats(removed, 0, &stats[kStatTomb], nullptr, nullptr, false);
}

// K7: snapshot pack -- compact live entries (+ deadlines) into a dense buffer
// that the host copies to pinned DRAM with hipMemcpyAsync.  One wave ballot +
// one LDS scan per block + one global atomic per block for the output base.
// K tiles of 256 entries per block trip, item-major (coalesced reads): per-(tile,
// wave) counts in LDS, one block scan, ONE output reservation per trip.  One
// returning atomic per 256 entries (8 K per 2M-entry table, all on one word)
// serialised at L2: that was most of the pass.
template <int K>
__global__ __launch_bounds__(256) void table_pack_kernel(const TableEntry* __restrict__ t, uint64_t cap,
                                                         const uint64_t* __restrict__ exp_tbl,
                                                         TableEntry* __restrict__ out,
                                                         uint64_t* __restrict__ out_exp,
                                                         unsigned long long* __restrict__ out_count) {
  __shared__ unsigned wave_cnt[K][4];
  __shared__ unsigned long long block_base;
  const unsigned w = threadIdx.x / kWave;
  const uint64_t trip = (uint64_t)K * blockDim.x;
  for (uint64_t base = blockIdx.x * trip; base < cap; base += (uint64_t)gridDim.x * trip) {
    TableEntry e[K];
    bool live[K];
    unsigned pos[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t i = base + (uint64_t)k * blockDim.x + threadIdx.x;
      live[k] = false;
      if (i < cap) {
        const uint4 v = *reinterpret_cast<const uint4*>(&t[i]);
        e[k].key = ((uint64_t)v.y << 32) | v.x;
        e[k].rank = v.z;
        e[k].mbox = v.w;
        live[k] = e[k].key != kKeyEmpty && e[k].key != kKeyTomb;
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t m = __ballot(live[k]);
      pos[k] = mbcnt64(m);
      if (lane_id() == 0) wave_cnt[k][w] = __popcll(m);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan over (tile, wave), then the trip's reservation
      unsigned run = 0;
      for (int k = 0; k < K; ++k)
        for (unsigned q = 0; q < blockDim.x / kWave; ++q) {
          const unsigned c = wave_cnt[k][q];
          wave_cnt[k][q] = run;
          run += c;
        }
      block_base = run ? atomicAdd(out_count, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!live[k]) continue;
      const uint64_t i = base + (uint64_t)k * blockDim.x + threadIdx.x;
      const unsigned long long o = block_base + wave_cnt[k][w] + pos[k];
      out[o] = e[k];
      if (out_exp) out_exp[o] = exp_tbl ? exp_tbl[i] : 0ull;
    }
    __syncthreads();
  }
}

// K5b: route directory -- the registry flattened for the dense actor-id range
// [0, n_dir): dir[id] = rank | mbox << 8 (the route word), 0xFFFFFFFF for an id
// the registry does not hold, kDirFallback when the entry does not fit a route
// word (the data path then probes the hash table for that id).  The hash table
// stays the source of truth; this is its compiled form for the message hot path:
// a 4-B read per message from an L2-resident array instead of a 64-B probe line.
// `dir` must be pre-filled with 0xFF bytes.
//
// Affine check (affine_w > 0): count the ids of the range the table holds and
// the ones NOT placed by the strided rule (rank = id % W, mbox = id / W).  With
// every id present and no violation, the data path can compute route words
// arithmetically -- no directory gathers at all (`astats` = {present, violations}).
__global__ __launch_bounds__(256) void table_build_dir_kernel(const TableEntry* __restrict__ t, uint64_t cap,
                                                              uint32_t* __restrict__ dir, uint8_t* __restrict__ dirr,
                                                              uint64_t n_dir, uint32_t affine_w,
                                                              unsigned long long* __restrict__ astats) {
  unsigned long long present = 0, bad = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = *reinterpret_cast<const uint4*>(&t[i]);
    const uint64_t key = ((uint64_t)v.y << 32) | v.x;
    if (key == kKeyEmpty || key == kKeyTomb || key > n_dir) continue;  // actor_key(id) = id + 1
    dir[key - 1] = (v.z < 0xfeu && v.w < (1u << 24)) ? (v.z | (v.w << 8)) : kDirFallback;
    if (dirr) dirr[key - 1] = v.z < kRankFallback ? (uint8_t)v.z : kRankFallback;
    if (affine_w) {
      const uint64_t id = key - 1;
      ++present;
      bad += (v.z != id % affine_w || v.w != id / affine_w) ? 1 : 0;
    }
  }
  if (affine_w) {
    publish_block_stats(present, 0, &astats[0], nullptr, nullptr, false);
    publish_block_stats(bad, 0, &astats[1], nullptr, nullptr, false);
  }
}

// Blocks of the upsert / delete passes: each
// block publishes its counters with one same-address atomic, and those serialise
// at L2.  1M-actor inserts: 4096 blocks 5.7-5.9 G/s, 1024 7.5, 512 8.5, 256 7.9
// (profiles/r2_table_grid_sweep.txt).  (Skipping the max atomic behind an
// agent-scope read made it worse: 3.0 G/s at 4096.)
static unsigned table_blocks() {
  return 512u;
}

static inline unsigned grid_for(int64_t n, int per_block = 256, unsigned cap = 4096) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ---- host launchers (pointers are raw device addresses from torch tensors) ----
void launch_table_upsert(uintptr_t table, uint64_t cap, uintptr_t keys, uintptr_t ranks, uintptr_t mboxes,
                         uintptr_t exp_in, uintptr_t exp_tbl, int64_t n, uintptr_t stats, uintptr_t stream) {
  if (n <= 0) return;
  if (cap == 0 || (cap & (cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  UpsertIn in;
  in.keys = (const uint64_t*)keys;
  in.ranks = (const uint32_t*)ranks;
  in.mboxes = (const uint32_t*)mboxes;
  hipLaunchKernelGGL(table_upsert_kernel, dim3(grid_for(n, 256, table_blocks())), dim3(256), 0, as_stream(stream),
                     (TableEntry*)table, cap - 1, in, (const uint64_t*)exp_in, (uint64_t*)exp_tbl, n, (unsigned long long*)stats);
  PT_HIP_CHECK(hipGetLastError());
}

// Restore (K7 inverse): re-insert packed TableEntry records (+ their deadlines).
void launch_table_upsert_packed(uintptr_t table, uint64_t cap, uintptr_t entries, uintptr_t exp_in,
                                uintptr_t exp_tbl, int64_t n, uintptr_t stats, uintptr_t stream) {
  if (n <= 0) return;
  if (cap == 0 || (cap & (cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  UpsertIn in;
  in.packed = (const TableEntry*)entries;
  hipLaunchKernelGGL(table_upsert_kernel, dim3(grid_for(n, 256, table_blocks())), dim3(256), 0, as_stream(stream),
                     (TableEntry*)table, cap - 1, in, (const uint64_t*)exp_in, (uint64_t*)exp_tbl, n, (unsigned long long*)stats);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_table_delete(uintptr_t table, uint64_t cap, uintptr_t keys, int64_t n, uintptr_t stats,
                         uintptr_t found, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(table_delete_kernel, dim3(grid_for(n, 256, table_blocks())), dim3(256), 0, as_stream(stream),
                     (TableEntry*)table,
                     cap - 1, (const uint64_t*)keys, n, (unsigned long long*)stats, (uint8_t*)found);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_table_lookup(uintptr_t table, uint64_t cap, uintptr_t keys, int64_t n, uintptr_t out_rank,
                         uintptr_t out_mbox, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(table_lookup_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream),
                     (const TableEntry*)table, cap - 1, (const uint64_t*)keys, n, (int32_t*)out_rank,
                     (int32_t*)out_mbox);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_table_sweep(uintptr_t table, uint64_t cap, uintptr_t exp_tbl, uint64_t now, uintptr_t stats,
                        uintptr_t stream) {
  hipLaunchKernelGGL(table_sweep_kernel, dim3(grid_for((int64_t)cap)), dim3(256), 0, as_stream(stream),
                     (TableEntry*)table, cap, (const uint64_t*)exp_tbl, now, (unsigned long long*)stats);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_table_build_dir(uintptr_t table, uint64_t cap, uintptr_t dir, uint64_t n_dir, uint32_t affine_w,
                            uintptr_t astats, uintptr_t stream, uintptr_t dir_rank) {
  hipStream_t s = as_stream(stream);
  PT_HIP_CHECK(hipMemsetAsync((void*)dir, 0xff, n_dir * sizeof(uint32_t), s));
  if (dir_rank) PT_HIP_CHECK(hipMemsetAsync((void*)dir_rank, kRankMissing, n_dir, s));
  if (affine_w) PT_HIP_CHECK(hipMemsetAsync((void*)astats, 0, 2 * sizeof(unsigned long long), s));
  hipLaunchKernelGGL(table_build_dir_kernel, dim3(grid_for((int64_t)cap)), dim3(256), 0, s, (const TableEntry*)table,
                     cap, (uint32_t*)dir, (uint8_t*)dir_rank, n_dir, affine_w, (unsigned long long*)astats);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_table_pack(uintptr_t table, uint64_t cap, uintptr_t exp_tbl, uintptr_t out, uintptr_t out_exp,
                       uintptr_t out_count, uintptr_t stream) {
  constexpr int K = 8;  // 2048 entries per reservation
  hipLaunchKernelGGL(table_pack_kernel<K>, dim3(grid_for((int64_t)cap, 256 * K, 1024)), dim3(256), 0,
                     as_stream(stream),
                     (const TableEntry*)table, cap, (const uint64_t*)exp_tbl, (TableEntry*)out, (uint64_t*)out_exp,
                     (unsigned long long*)out_count);
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
