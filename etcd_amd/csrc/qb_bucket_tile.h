// qb_bucket_tile.h — the LDS tile pieces of the level-1 bucketing (K3):
// the tracker steps' k_bk_scatter (qb_tracker_bucket.hip) and the composed
// wire -> tracker step's k_wire_scatter (qb_wire_tracker.hip).  DESIGN.md §3.3e.
#pragma once

#include "qb_bucket.h"

namespace qb {
namespace bk {

// ------------------------------------------------ LDS tile partition ----
// Counting sort of one tile (<= kTile records) by a small key, in LDS.  The
// caller provides each record's bin (or kNoBin); afterwards perm[e] is the
// tile index of the e-th record in bin order and start[b] the first e of
// bin b.  Payload columns are then moved with tile_move: coalesced global
// load into LDS, permuted LDS read, coalesced global store.
constexpr u16 kNoBin = 0xFFFF;
constexpr int kPartThreads = 1024;

struct alignas(16) TileLds {
  u16 bin[kTile];
  u16 rank[kTile];
  u16 perm[kTile];
  u64 stage[kTile];
  u8 cl[kTile];  // compact records: chunk-low, the next level's key
  u32 wsum[kPartThreads / 64];
};

// Exclusive scan of cnt[0..nb) in place (per-thread serial runs + wave
// shuffles + one LDS pass); returns the number of binned records.
__device__ __forceinline__ u32 tile_scan_bins(u32* cnt, u32 nb, u32* wsum) {
  const u32 T = blockDim.x;
  const u32 per = (nb + T - 1) / T;
  u32 run = 0;
  for (u32 j = 0; j < per; ++j) {
    const u32 b = threadIdx.x * per + j;
    if (b < nb) run += cnt[b];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = int(T >> 6);
  u32 x = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = u32(__shfl_up(int(x), o, 64));
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  u32 before = 0, total = 0;
  for (int q = 0; q < nw; ++q) {
    total += wsum[q];
    if (q < w) before += wsum[q];
  }
  u32 acc = before + x - run;
  for (u32 j = 0; j < per; ++j) {
    const u32 b = threadIdx.x * per + j;
    if (b < nb) {
      const u32 c = cnt[b];
      cnt[b] = acc;
      acc += c;
    }
  }
  __syncthreads();
  return total;
}

template <class Lds>
__device__ __forceinline__ void tile_perm(Lds& L, const u32* start, u32 nrec) {
  for (u32 k = threadIdx.x; k < nrec; k += blockDim.x) {
    const u16 b = L.bin[k];
    if (b != kNoBin) L.perm[start[b] + L.rank[k]] = u16(k);
  }
  __syncthreads();
}

// ---------------------------------------------------------------- K3 ----
// Level 1: one block per tile of the original records; bins = super-buckets.
// Every global load of the tile (group, flags and both payload columns) is
// issued before the first LDS step, so the loads overlap each other and the
// ranking.  Each super-bucket's run of the tile reserves its place in region
// b * 8 + x (x = the XCD slot, blockIdx % 8) with one returning atomic on the
// region's fill counter; what lies past the region's cap (a skewed batch)
// continues in the region's overflow pool parts (Pool, qb_bucket.h: at most
// two per run, drawn here).  Invalid records go to the stat shards.
constexpr int kPer = kTile / kPartThreads;  // records per thread
static_assert((kTile & (kTile - 1)) == 0, "pool offsets by shift and mask");
constexpr u32 kTileShift = 12;
static_assert((1u << kTileShift) == u32(kTile), "kTile = 2^kTileShift");
// Record index of region-relative position rel of super-bucket b's region x
// (the region grid, then the pool parts p0 / p1 drawn for the run that
// starts at gs), or ~0 when the run's pool part could not be drawn.
__device__ __forceinline__ u64 region_dst(const Geometry& geo, const Pool& pool, u32 b, u32 x,
                                          u32 rel, u32 gs, u32 p0, u32 p1) {
  if (rel < geo.cap) return u64(b * kRegionShards + x) * geo.cap + rel;
  const u32 q = rel - geo.cap, k = q >> kTileShift;
  const u32 k0 = ((gs > geo.cap ? gs : geo.cap) - geo.cap) >> kTileShift;
  const u32 pid = k == k0 ? p0 : p1;
  if (pid == kNoPart) return ~0ull;
  return pool.base + u64(pid) * kTile + (q & (u32(kTile) - 1u));
}
}  // namespace bk
}  // namespace qb
