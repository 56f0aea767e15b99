// qb_route.hip — delivery of a record batch to the shards owning its groups
// (SURVEY.md §8e), gfx950: the device half of qb_dev_route_records.
//
// A node's inbound responses arrive at whichever rank's transport received
// them; each record must reach the rank whose shard holds its group (the
// contiguous ranges of qb_shard_range).  The leader step applies a group's
// records in batch order (raft.go:1099-1342 is a sequential fold), so the
// delivery is STABLE: a rank receives, from each source rank in rank order,
// that rank's records for it in their original order — the order
// etcd_amd/shard.py:route_records defines and the sharded tests check.
//
// Partition (this file): a stable counting partition of the batch by owner
// rank, with the group rebased to the owner's local index on the way:
//   R1 k_route_count    per tile of kTile records: per-owner counts
//   scan                owner-major [owner][tile] exclusive scan (qb_scan.h)
//   R2 k_route_scatter  per tile: each record's stable position =
//                       scan[owner][tile] + records of the same owner before
//                       it in the tile (wave ballots over peers, then waves
//                       and rounds in order), every column moved there
// The exchange (qb_comm.cpp) then sends owner p's contiguous run to rank p.
#include "qb_common.h"
#include "qb_scan.h"

namespace qb {
namespace route {

constexpr u32 kRounds = 4;
constexpr u32 kTile = kBlock * kRounds;  // records per workgroup, in round-major order
constexpr u32 kWaves = kBlock / 64;

struct Owner {
  u64 total, base, extra, big;  // big = extra * (base + 1): groups of the larger shards
  u32 world;
  // shard_range inverted: rank r < extra owns base + 1 groups, the rest base;
  // a group >= total goes to the last rank (its local index is then >= that
  // shard's size: the step counts it as a bad group, as the reference drops
  // a message for an unknown group).
  __device__ __forceinline__ u32 of(u64 g) const {
    if (g >= total) return world - 1;
    if (g < big) return u32(g / (base + 1));
    return u32(extra + (g - big) / base);
  }
  __device__ __forceinline__ u64 begin(u32 r) const {
    return u64(r) * base + (u64(r) < extra ? u64(r) : extra);
  }
};

inline Owner owner_of(u64 total, u32 world) {
  Owner o;
  o.total = total;
  o.world = world;
  o.base = total / world;
  o.extra = total % world;
  o.big = o.extra * (o.base + 1);
  return o;
}

__device__ __forceinline__ u64 lanes_below() {
  const u32 lane = threadIdx.x & 63u;
  return lane ? (~0ull >> (64u - lane)) : 0ull;
}

// The lanes of this wave whose owner equals this lane's (a loop over the
// distinct owners present in the wave: at most world iterations).
__device__ __forceinline__ u64 peers(u32 own, bool live) {
  u64 todo = __ballot(live), mine = 0;
  while (todo) {
    const u32 lead = u32(__builtin_ctzll(todo));
    const u32 o = u32(__shfl(int(own), int(lead), 64));
    const u64 m = __ballot(live && own == o);
    if (live && own == o) mine = m;
    todo &= ~m;
  }
  return mine;
}

__global__ __launch_bounds__(kBlock) void k_route_count(Owner ow, u64 M, const u32* __restrict__ rg,
                                                        u32* __restrict__ cnt, u32 ntiles) {
  __shared__ u32 c[QB_ROUTE_MAX_WORLD];
  for (u32 r = threadIdx.x; r < ow.world; r += kBlock) c[r] = 0;
  __syncthreads();
  const u64 t0 = u64(blockIdx.x) * kTile;
#pragma unroll
  for (u32 k = 0; k < kRounds; ++k) {
    const u64 j = t0 + u64(k) * kBlock + threadIdx.x;
    const bool live = j < M;
    const u32 own = live ? ow.of(rg[j]) : 0u;
    const u64 p = peers(own, live);
    // the lowest lane of each owner's peers counts them
    if (live && (p & lanes_below()) == 0) atomicAdd(&c[own], u32(__popcll(p)));
  }
  __syncthreads();
  for (u32 r = threadIdx.x; r < ow.world; r += kBlock) cnt[u64(r) * ntiles + blockIdx.x] = c[r];
}

struct Cols {
  const u32* group;
  const u8* flags;
  const u64 *index, *term, *hint, *log_term;
};
struct OutCols {
  u32* group;
  u8* flags;
  u64 *index, *term, *hint, *log_term;
};

__global__ __launch_bounds__(kBlock) void k_route_scatter(Owner ow, u64 M, Cols in,
                                                          const u32* __restrict__ pos,
                                                          u32 ntiles, OutCols out) {
  __shared__ u32 base[QB_ROUTE_MAX_WORLD];
  __shared__ u32 wc[kWaves][QB_ROUTE_MAX_WORLD];
  const u32 w = threadIdx.x >> 6;
  for (u32 r = threadIdx.x; r < ow.world; r += kBlock) base[r] = pos[u64(r) * ntiles + blockIdx.x];
  const u64 t0 = u64(blockIdx.x) * kTile;
  for (u32 k = 0; k < kRounds; ++k) {
    const u64 j = t0 + u64(k) * kBlock + threadIdx.x;
    const bool live = j < M;
    const u32 g = live ? in.group[j] : 0u;
    const u32 own = live ? ow.of(g) : 0u;
    for (u32 i = threadIdx.x; i < kWaves * QB_ROUTE_MAX_WORLD; i += kBlock) (&wc[0][0])[i] = 0;
    __syncthreads();  // base (first round / last round's update) and the cleared counts
    const u64 p = peers(own, live);
    const u32 rank_in_wave = u32(__popcll(p & lanes_below()));
    if (live && rank_in_wave == 0) wc[w][own] = u32(__popcll(p));
    __syncthreads();
    if (live) {
      u32 d = base[own] + rank_in_wave;
      for (u32 v = 0; v < w; ++v) d += wc[v][own];
      out.group[d] = u32(u64(g) - ow.begin(own));
      out.flags[d] = in.flags[j];
      out.index[d] = in.index[j];
      out.term[d] = in.term[j];
      if (in.hint) out.hint[d] = in.hint[j];
      if (in.log_term) out.log_term[d] = in.log_term[j];
    }
    __syncthreads();  // every lane has read base for this round
    for (u32 r = threadIdx.x; r < ow.world; r += kBlock) {
      u32 s = 0;
      for (u32 v = 0; v < kWaves; ++v) s += wc[v][r];
      base[r] += s;
    }
    __syncthreads();  // the update has read wc before the next round clears it
  }
}

}  // namespace route
}  // namespace qb

using namespace qb;

namespace {
size_t up256(size_t x) { return (x + 255) & ~size_t(255); }
u32 route_tiles(u64 M) { return u32((M + route::kTile - 1) / route::kTile); }
}  // namespace

// Workspace: the owner-major count matrix (+ its scan's block sums).
extern "C" size_t qb_route_partition_workspace_bytes(int world, uint64_t M) {
  if (world < 1 || world > QB_ROUTE_MAX_WORLD) return 0;
  const u64 n = u64(world) * route_tiles(M);
  return up256(sizeof(u32) * (n + 1)) + up256(sizeof(u32) * (scan::blocks(n) + 1));
}

extern "C" int qb_dev_route_partition(uint64_t total, int world, uint64_t M,
                                      const uint32_t* rec_group, const uint8_t* rec_flags,
                                      const uint64_t* rec_index, const uint64_t* rec_term,
                                      const uint64_t* rec_hint, const uint64_t* rec_log_term,
                                      uint32_t* send_group, uint8_t* send_flags,
                                      uint64_t* send_index, uint64_t* send_term,
                                      uint64_t* send_hint, uint64_t* send_log_term,
                                      uint32_t* send_off, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  QB_REQUIRE(world >= 1 && world <= QB_ROUTE_MAX_WORLD, "world must be 1..%d", QB_ROUTE_MAX_WORLD);
  QB_REQUIRE(M < (1ull << 32), "batch too large (M=%llu > 2^32-1)", (unsigned long long)M);
  QB_REQUIRE(send_off, "send_off is NULL");
  QB_REQUIRE(!rec_hint == !send_hint && !rec_log_term == !send_log_term,
             "hint / log_term: give both the input and the output column, or neither");
  hipStream_t st = as_stream(stream);
  if (M == 0) {
    const hipError_t e = hipMemsetAsync(send_off, 0, sizeof(u32) * (size_t(world) + 1), st);
    return e == hipSuccess ? QB_OK : hip_fail(e, "hipMemsetAsync(send_off)");
  }
  QB_REQUIRE(rec_group && rec_flags && rec_index && rec_term, "record column is NULL");
  QB_REQUIRE(send_group && send_flags && send_index && send_term, "send column is NULL");
  QB_REQUIRE(workspace && workspace_bytes >= qb_route_partition_workspace_bytes(world, M),
             "workspace too small (qb_route_partition_workspace_bytes)");
  const u32 nt = route_tiles(M);
  const u64 n = u64(world) * nt;
  char* ws = static_cast<char*>(workspace);
  u32* cnt = reinterpret_cast<u32*>(ws);
  u32* bsum = reinterpret_cast<u32*>(ws + up256(sizeof(u32) * (n + 1)));
  const route::Owner ow = route::owner_of(total, u32(world));
  hipLaunchKernelGGL(route::k_route_count, dim3(nt), dim3(kBlock), 0, st, ow, M, rec_group, cnt, nt);
  QB_CHECK_LAUNCH("k_route_count");
  scan::launch(cnt, n, bsum, st);
  QB_CHECK_LAUNCH("scan(route)");
  const route::Cols in{rec_group, rec_flags, reinterpret_cast<const u64*>(rec_index),
                       reinterpret_cast<const u64*>(rec_term), reinterpret_cast<const u64*>(rec_hint),
                       reinterpret_cast<const u64*>(rec_log_term)};
  const route::OutCols out{send_group, send_flags, reinterpret_cast<u64*>(send_index),
                           reinterpret_cast<u64*>(send_term), reinterpret_cast<u64*>(send_hint),
                           reinterpret_cast<u64*>(send_log_term)};
  hipLaunchKernelGGL(route::k_route_scatter, dim3(nt), dim3(kBlock), 0, st, ow, M, in, cnt, nt, out);
  QB_CHECK_LAUNCH("k_route_scatter");
  // send_off[r] = first record for rank r = cnt[r * nt] (the scan), send_off[world] = M
  const hipError_t e = hipMemcpy2DAsync(send_off, sizeof(u32), cnt, sizeof(u32) * nt, sizeof(u32),
                                        size_t(world), hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy2DAsync(send_off)");
  const hipError_t e2 = hipMemcpyAsync(send_off + world, cnt + n, sizeof(u32),
                                       hipMemcpyDeviceToDevice, st);
  return e2 == hipSuccess ? QB_OK : hip_fail(e2, "hipMemcpyAsync(send_off)");
}
