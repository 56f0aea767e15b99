// qb_delta.hip — the changed-commit delta of a shard (gfx950): the groups
// whose commit index moved this tick, compacted in group order as (global
// group, new commit) pairs, so the node-wide exchange (qb_comm.cpp:
// qb_dev_allgather_changed) moves 12 bytes per changed group instead of the
// whole commit vector (SURVEY.md §7 "gather only changed-commit deltas").
//
// Reference: a group surfaces a Ready when its HardState changed, the commit
// index being the part this tick moves (raft/node.go:573 newReady,
// raft/rawnode.go:157 HasReady); the tracker steps report exactly those
// groups in advanced_out (raft.go:585-588 maybeCommit returned true).
//
//   D1 k_delta_count  per tile of kTile groups: changed groups -> cnt[tile]
//   scan              exclusive scan of the tile counts (qb_scan.h)
//   D2 k_delta_write  per tile: each changed group's position = its tile's
//                     offset + changed groups before it in the tile (wave
//                     ballots, then waves in order); writes (g_base + g,
//                     commit[g]); the last tile also stores the total (u32 at
//                     cnt[ntiles], u64 at *count64)
#include "qb_common.h"
#include "qb_scan.h"

namespace qb {
namespace delta {

constexpr u32 kPer = 4;                  // groups per thread (one u32 of flags)
constexpr u32 kTile = kBlock * kPer;     // groups per workgroup
constexpr u32 kWaves = kBlock / 64;

__device__ __forceinline__ u32 load_flags(const u8* __restrict__ changed, u64 n, u64 g) {
  // four flag bytes as one word when whole and aligned, else byte by byte
  if (g + kPer <= n && (reinterpret_cast<uintptr_t>(changed + g) & 3u) == 0)
    return *reinterpret_cast<const u32*>(changed + g);
  u32 w = 0;
#pragma unroll
  for (u32 k = 0; k < kPer; ++k)
    if (g + k < n) w |= u32(changed[g + k]) << (8 * k);
  return w;
}

__device__ __forceinline__ u32 popc_flags(u32 w) {
  u32 c = 0;
#pragma unroll
  for (u32 k = 0; k < kPer; ++k) c += ((w >> (8 * k)) & 0xFFu) != 0;
  return c;
}

__global__ __launch_bounds__(kBlock) void k_delta_count(u64 n, const u8* __restrict__ changed,
                                                        u32* __restrict__ cnt) {
  __shared__ u32 ws[kWaves];
  const u64 g = u64(blockIdx.x) * kTile + u64(threadIdx.x) * kPer;
  u32 c = popc_flags(load_flags(changed, n, g));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += u32(__shfl_xor(int(c), o, 64));
  if ((threadIdx.x & 63u) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 t = 0;
#pragma unroll
    for (u32 w = 0; w < kWaves; ++w) t += ws[w];
    cnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kBlock) void k_delta_write(u64 n, const u8* __restrict__ changed,
                                                        const u64* __restrict__ commit, u64 g_base,
                                                        const u32* __restrict__ cnt, u32 ntiles,
                                                        u32* __restrict__ out_gid,
                                                        u64* __restrict__ out_commit,
                                                        u64* __restrict__ count64) {
  __shared__ u32 wsum[kWaves];
  const u64 g = u64(blockIdx.x) * kTile + u64(threadIdx.x) * kPer;
  const u32 w = load_flags(changed, n, g);
  const u32 mine = popc_flags(w);
  // exclusive prefix of the per-thread counts over the wave, then the waves
  u32 x = mine;
  const u32 lane = threadIdx.x & 63u;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = u32(__shfl_up(int(x), o, 64));
    if (lane >= u32(o)) x += y;
  }
  if (lane == 63u) wsum[threadIdx.x >> 6] = x;
  __syncthreads();
  u32 before = 0;
  for (u32 q = 0; q < (threadIdx.x >> 6); ++q) before += wsum[q];
  u32 pos = cnt[blockIdx.x] + before + x - mine;
#pragma unroll
  for (u32 k = 0; k < kPer; ++k) {
    if ((w >> (8 * k)) & 0xFFu) {
      out_gid[pos] = u32(g_base + g + k);
      out_commit[pos] = commit[g + k];
      ++pos;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *count64 = cnt[ntiles];
}

}  // namespace delta
}  // namespace qb

using namespace qb;

extern "C" size_t qb_compact_changed_workspace_bytes(uint64_t n) {
  const u64 nt = (n + delta::kTile - 1) / delta::kTile;
  return (sizeof(u32) * (nt + 1) + 255) / 256 * 256 +
         (sizeof(u32) * (scan::blocks(nt) + 1) + 255) / 256 * 256 + 256;
}

extern "C" int qb_dev_compact_changed(uint64_t n, const uint8_t* changed, const uint64_t* commit,
                                      uint64_t g_base, uint32_t* out_gid, uint64_t* out_commit,
                                      uint64_t* out_count, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  QB_REQUIRE(out_count, "out_count is NULL");
  QB_REQUIRE(n == 0 || (changed && commit && out_gid && out_commit), "NULL column");
  QB_REQUIRE(g_base + n <= 0xFFFFFFFFull, "global groups must fit uint32 (g_base + n = %llu)",
             (unsigned long long)(g_base + n));
  QB_REQUIRE(workspace && workspace_bytes >= qb_compact_changed_workspace_bytes(n),
             "workspace too small (qb_compact_changed_workspace_bytes)");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    const hipError_t e = hipMemsetAsync(out_count, 0, sizeof(u64), st);
    return e == hipSuccess ? QB_OK : hip_fail(e, "hipMemsetAsync(count)");
  }
  const u32 nt = u32((n + delta::kTile - 1) / delta::kTile);
  char* ws = static_cast<char*>(workspace);
  u32* cnt = reinterpret_cast<u32*>(ws);
  u32* bsum = reinterpret_cast<u32*>(ws + (sizeof(u32) * (u64(nt) + 1) + 255) / 256 * 256);
  hipLaunchKernelGGL(delta::k_delta_count, dim3(nt), dim3(kBlock), 0, st, n, changed, cnt);
  QB_CHECK_LAUNCH("k_delta_count");
  scan::launch(cnt, nt, bsum, st);
  hipLaunchKernelGGL(delta::k_delta_write, dim3(nt), dim3(kBlock), 0, st, n, changed,
                     reinterpret_cast<const u64*>(commit), g_base, cnt, nt, out_gid,
                     reinterpret_cast<u64*>(out_commit), reinterpret_cast<u64*>(out_count));
  QB_CHECK_LAUNCH("k_delta_write");
  return QB_OK;
}

// The receiving side: commit_all[gid[i]] = commit[i] for every gathered pair
// (padding entries carry gid = UINT32_MAX and are skipped).
namespace qb {
namespace delta {
__global__ __launch_bounds__(kBlock) void k_delta_scatter(u64 m, const u32* __restrict__ gid,
                                                          const u64* __restrict__ val, u64 total,
                                                          u64* __restrict__ commit_all) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= m) return;
  const u32 g = gid[i];
  if (g != 0xFFFFFFFFu && g < total) commit_all[g] = val[i];
}
}  // namespace delta
}  // namespace qb

extern "C" int qb_dev_scatter_changed(uint64_t m, const uint32_t* gid, const uint64_t* commit,
                                      uint64_t total, uint64_t* commit_all, void* stream) {
  if (m == 0) return QB_OK;
  QB_REQUIRE(gid && commit && commit_all, "NULL column");
  hipLaunchKernelGGL(delta::k_delta_scatter, dim3(unsigned((m + kBlock - 1) / kBlock)), dim3(kBlock),
                     0, as_stream(stream), m, gid, reinterpret_cast<const u64*>(commit), total,
                     reinterpret_cast<u64*>(commit_all));
  QB_CHECK_LAUNCH("k_delta_scatter");
  return QB_OK;
}
