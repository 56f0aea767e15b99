// qb_tracker_bucket.hip — one leader tick over G groups (FIXED layout):
// a batch of MsgAppResp records applied and the commit advanced, with the
// records bucketed by group so every update is an LDS atomic instead of a
// random-address HBM atomic.
//
// Reference semantics, identical to qb_tracker.hip (paths relative to raft/):
//   raft.Step term filter               raft.go:847-921
//   stepLeader MsgAppResp (quorum part) raft.go:1100-1109, 1237-1259
//   Progress.MaybeUpdate                tracker/progress.go:144-153
//   raft.maybeCommit / raftLog.maybeCommit  raft.go:585-588, log.go:328-334
//
// Pipeline (records are any-order; M ~ G at the BASELINE config 5):
//   memset           stat shards, flag words, region fills, chunk flags
//   K3 k_bk_scatter  per tile: counting sort by super-bucket in LDS; each
//                    super-bucket's run reserves its place in the region of
//                    this workgroup's XCD slot with one atomic and is written
//                    there contiguously; invalid records (group >= G, slot >=
//                    n) are counted and dropped (round 4: no histogram pass,
//                    no scan, no part table — DESIGN.md §3.3e)
//   K4 k_bk_split_*  per part of a region: the same LDS counting sort by
//                    chunk, written in place, plus the part's chunk run starts
//   K5 k_bk_apply<N> one workgroup per chunk of CH groups (its records are
//                    one short run per part of its super-bucket): classify (term
//                    filter, step-down ordering via an LDS atomic min of the
//                    batch index), MaybeUpdate as LDS atomic max, RecentActive
//                    as LDS atomic or, then maybeCommit for the chunk's groups
//                    and a coalesced write-back of match/next/active/committed.
#include "qb_bucket_tile.h"
#include "qb_tracker_slow.h"


namespace qb {
namespace bk {

// (two 1024-thread blocks per CU need <= 64 VGPRs and <= 80 SGPRs)
// COMPACT: the 8-byte records (the tracker steps) go from registers straight
// to their sorted LDS slot (round 3: K3 115 -> 112 us against the
// permutation walk); else the wide columns (the leader step) move through
// the permutation walk, one column at a time.
template <bool COMPACT>
__global__ __launch_bounds__(kPartThreads)
__attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8, 8))) void k_bk_scatter(
    Geometry geo, const u32* __restrict__ rg, const u8* __restrict__ rf,
    const u64* __restrict__ ri, const u64* __restrict__ rt, Cols out, u32* __restrict__ counts,
    u64* __restrict__ shards, u8* __restrict__ chunk_slow, Pool pool) {
  extern __shared__ __attribute__((aligned(16))) u32 dyn[];
  u32* start = dyn;               // NSB: count, then local exclusive start
  u32* gstart = dyn + geo.NSB;    // NSB: the run's offset in its region
  u32* pid0 = dyn + 2 * geo.NSB;  // NSB: pool parts of the run past the cap
  u32* pid1 = dyn + 3 * geo.NSB;
  __shared__ TileLds L;
  __shared__ u32 s_nesc;  // compact: this tile's escapes
  const u32 tile = geo.tile();
  if (tile >= geo.NT) return;
  if (threadIdx.x == 0) s_nesc = 0;  // (ordered before its use by the barriers below)
  const u64 t0 = u64(tile) * kTile;
  const u32 nrec = u32(geo.M - t0 < u64(kTile) ? geo.M - t0 : u64(kTile));
  u32 g[kPer], f[kPer];
  u64 vi[kPer], vt[kPer];
  // A full tile of aligned columns is read as 4 consecutive records per
  // lane (16-byte loads: 6 load instructions per thread instead of 16);
  // record k of thread j is then rk(j).  Runs within a bucket carry no
  // order (the LDS ranks are atomic), so the mapping is free.
  static_assert(kPer == 4, "vector loads assume 4 records per thread");
  const bool vec = nrec == u32(kTile) && (reinterpret_cast<uintptr_t>(rg) & 15u) == 0 &&
                   (reinterpret_cast<uintptr_t>(rf) & 3u) == 0 &&
                   (reinterpret_cast<uintptr_t>(ri) & 15u) == 0 &&
                   (reinterpret_cast<uintptr_t>(rt) & 15u) == 0;
  auto rk = [&](int j) -> u32 {
    return vec ? 4u * threadIdx.x + u32(j) : threadIdx.x + u32(j) * kPartThreads;
  };
  if (vec) {
    const u64 i = t0 + 4u * threadIdx.x;
    const uint4 gv = *reinterpret_cast<const uint4*>(rg + i);
    const u32 fv = *reinterpret_cast<const u32*>(rf + i);
    g[0] = gv.x;
    g[1] = gv.y;
    g[2] = gv.z;
    g[3] = gv.w;
#pragma unroll
    for (int j = 0; j < kPer; ++j) f[j] = (fv >> (8 * j)) & 0xFFu;
    // (ri is never null; the guard stays because without it the compiler's
    // allocation of the compact form spills 4 VGPRs instead of 1)
    if (ri) {
      const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(ri + i);
      const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(ri + i + 2);
      const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(rt + i);
      const ulonglong2 d = *reinterpret_cast<const ulonglong2*>(rt + i + 2);
      vi[0] = a.x;
      vi[1] = a.y;
      vi[2] = b.x;
      vi[3] = b.y;
      vt[0] = c.x;
      vt[1] = c.y;
      vt[2] = d.x;
      vt[3] = d.y;
    } else {
#pragma unroll
      for (int j = 0; j < kPer; ++j) vi[j] = vt[j] = 0ull;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const u32 k = rk(j);
      const bool in = k < nrec;
      g[j] = in ? rg[t0 + k] : 0xFFFFFFFFu;
      f[j] = in ? rf[t0 + k] : 0u;
      vi[j] = (in && ri) ? ri[t0 + k] : 0ull;
      vt[j] = (in && ri) ? rt[t0 + k] : 0ull;
    }
  }
  for (u32 b = threadIdx.x; b < geo.NSB; b += blockDim.x) start[b] = 0;
  __syncthreads();
  // bj: bin | chunk-low << 16 (kNoBin for an invalid record), rj: its rank;
  // compact: vj the encoded record (computed in the same pass, so the raw
  // columns die early: two 1024-thread blocks per CU hold <= 64 VGPRs)
  u32 bj[kPer], rj[kPer];
  u64 vj[kPer];
  u32 nbad = 0, nnon = 0;  // wave-uniform: invalid records
  u32 mside = 0;           // compact: side-form records
  u32 tj[kPer];            // compact: a side record's term (0 otherwise)
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const u32 k = rk(j);
    const bool ok = g[j] < geo.G && (f[j] & 0x0Fu) < geo.n;  // (k >= nrec has g = ~0)
    {
      const bool bad = k < nrec && g[j] >= geo.G;
      nbad += wave_popc(bad);
      nnon += wave_popc(k < nrec && !bad && !ok);
    }
    bj[j] = ok ? geo.sb_of(g[j]) : u32(kNoBin);
    rj[j] = ok ? atomicAdd(&start[bj[j]], 1u) : 0u;
    if constexpr (!COMPACT) {
      if (k < nrec) {
        L.bin[k] = u16(bj[j]);
        L.rank[k] = u16(rj[j]);
      }
    }
    bj[j] |= geo.cl_of_chunk(geo.chunk_of(g[j])) << 16;
    if constexpr (COMPACT) {
      vj[j] = geo.fmt.encode_side(g[j] & (geo.CH - 1u), f[j] & 0x0Fu, (f[j] & 0x80u) != 0, vi[j],
                                  vt[j], u32(t0 + k));
      const bool sr = ok && geo.fmt.term(vj[j]) == geo.fmt.tside();
      tj[j] = sr ? u32(vt[j]) : 0u;
      mside += sr ? 1u : 0u;
    }
  }
  if constexpr (COMPACT)
    if (mside) atomicAdd(&s_nesc, mside);
  __syncthreads();
  for (u32 b = threadIdx.x; b < geo.NSB; b += blockDim.x) {
    const u32 nbin = start[b];
    if (!nbin) continue;
    const u32 r = b * kRegionShards + blockIdx.x % kRegionShards;
    const u32 gs = atomicAdd(&counts[r], nbin);
    gstart[b] = gs;  // region-relative
    if (gs + nbin > geo.cap) {  // the run's tail continues in pool parts (<= 2)
      if constexpr (COMPACT)
        if (gs <= geo.cap) mark_heavy(pool, b);  // (the one run that crosses the cap)
      const u32 lo = gs > geo.cap ? gs : geo.cap;
      const u32 k0 = (lo - geo.cap) >> kTileShift, k1 = (gs + nbin - 1u - geo.cap) >> kTileShift;
      const u32 a = pool_acquire(pool, r, k0);
      pid0[b] = a;
      pid1[b] = k1 != k0 ? pool_acquire(pool, r, k1) : a;
    }
  }
  if ((threadIdx.x & 63) == 0 && (nbad | nnon)) {
    u64* sh = shards + u64(tile % kShards) * QB_STAT_COUNT;
    if (nbad) atomicAdd(sh + QB_STAT_BAD_GROUP, u64(nbad));
    if (nnon) atomicAdd(sh + QB_STAT_NON_MEMBER, u64(nnon));
  }
  const u32 nvalid = tile_scan_bins(start, geo.NSB, L.wsum);
  if constexpr (COMPACT) {
    // A tile where side records are not rare (more than 1/kSideDen of its
    // records: a stream of terms past the record's term field) keeps them —
    // the index in the record, the term in the side column at the record's
    // position — and writes the side column for every record of the tile, so
    // the column's lines are whole (the tile's runs); K4 carries it beside
    // the records and K5 reads it with them (round 5 gathered such records'
    // index and term from the batch: 1.43x the tick of small terms).  A tile
    // where they are rare turns them into escapes (no column writes: partial
    // lines cost more than a few records' gathers).
    const bool side = s_nesc * kSideDen > nvalid;  // (block-uniform)
    u32* t32 = reinterpret_cast<u32*>(L.rank);     // (rank + perm: unused by this form)
    // after the scan each record is stored at its sorted LDS slot with its
    // bin and chunk-low (and, side, its term), and the output pass reads the
    // slots in order
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const u32 b = bj[j] & 0xFFFFu;
      if (b == u32(kNoBin)) continue;
      const u32 e = start[b] + rj[j];
      u64 v = vj[j];
      if (!side && geo.fmt.term(v) == geo.fmt.tside()) v = geo.fmt.to_escape(v, u32(t0 + rk(j)));
      L.stage[e] = v;
      L.bin[e] = u16(b);
      L.cl[e] = u8(bj[j] >> 16);
      if (side) t32[e] = tj[j];
    }
    __syncthreads();
    if (side && threadIdx.x == 0) *out.sflag = 1u;
    const u32 x = blockIdx.x % kRegionShards;
    for (u32 e = threadIdx.x; e < nvalid; e += blockDim.x) {
      const u32 b = L.bin[e];
      const u32 gs = gstart[b];
      const u32 rel = gs + (e - start[b]);
      const u64 d = rel < geo.cap ? u64(b * kRegionShards + x) * geo.cap + rel
                                  : region_dst(geo, pool, b, x, rel, gs, pid0[b], pid1[b]);
      if (d != ~0ull) {
        out.mr[d] = L.stage[e];
        out.cl[d] = L.cl[e];
        if (side) out.side[d] = t32[e];
      } else {  // no pool part (never with the carve's sizing): the exact slow path
        chunk_slow[geo.chunk_of_sb_cl(b, L.cl[e])] = kChunkOverflow;
      }
    }
    return;
  } else {
    tile_perm(L, start, nrec);
    const u32 x = blockIdx.x % kRegionShards;
    // three columns, one at a time: index, term32, mr = meta | ridx << 32
    for (int col = 0; col < 3; ++col) {
      u64 v[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const u32 k = rk(j);
        if (col == 0) {
          v[j] = vi[j];
        } else if (col == 1) {
          v[j] = vt[j];
        } else {
          const u32 meta = (g[j] & (geo.CH - 1u)) | ((bj[j] >> 16) << 10) | ((f[j] & 0xFFu) << 17);
          v[j] = u64(meta) | (u64(u32(t0 + k)) << 32);
        }
      }
      if (vec) {  // two 16-byte LDS stores per lane (8-byte stores at a 32-byte stride conflict)
        *reinterpret_cast<ulonglong2*>(&L.stage[4u * threadIdx.x]) = ulonglong2{v[0], v[1]};
        *reinterpret_cast<ulonglong2*>(&L.stage[4u * threadIdx.x + 2]) = ulonglong2{v[2], v[3]};
      } else {
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (rk(j) < nrec) L.stage[rk(j)] = v[j];
      }
      __syncthreads();
      for (u32 e = threadIdx.x; e < nvalid; e += blockDim.x) {
        const u32 k = L.perm[e];
        const u32 b = L.bin[k];
        const u32 gs = gstart[b];
        const u32 rel = gs + (e - start[b]);
        const u64 val = L.stage[k];
        const u64 d = rel < geo.cap ? u64(b * kRegionShards + x) * geo.cap + rel
                                    : region_dst(geo, pool, b, x, rel, gs, pid0[b], pid1[b]);
        // (no part: impossible with geometry()'s pool sizing — every region
        // has kmax > its most parts, the pool >= M / kTile + the overflowing
        // regions — and the wide form has no slow path to send it to)
        if (d == ~0ull) continue;
        if (col == 0) out.index[d] = val;
        else if (col == 1) out.term32[d] = term_to32(val);
        else out.mr[d] = val;
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- K4 ----
// Level 2 over the region grid: part p = region r's j-th part (p = r * ppx
// + j; kTile records, the last one up to kTile + kWideSlack: region_parts;
// a part past its region's fill exits after one load); a counting sort of
// the part by chunk-low, written to the SAME range of buf2; cs[p][c] = first
// record of chunk-low c in part p (cs[p][128] = part end).  The wide columns
// (the leader step) move through the permutation walk.
constexpr u32 kWideTile = kTile + kWideSlack;
constexpr int kPerW = int(kWideTile / kPartThreads);  // records per thread
static_assert(kWideTile % kPartThreads == 0, "whole records per thread");
struct alignas(16) TileLdsW {
  u16 bin[kWideTile];
  u16 rank[kWideTile];
  u16 perm[kWideTile];
  u64 stage[kWideTile];
  u32 wsum[kPartThreads / 64];
};
// One part (nrec records at lo of `in`) sorted by chunk-low into the same
// range of `out`; cs row `row` gets the chunk starts.
__device__ __forceinline__ void split_wide_part(Cols in, Cols out, u32* __restrict__ cs, u32 lo,
                                                u32 nrec, u64 row) {
  __shared__ TileLdsW L;
  __shared__ u32 start[kChunksPerSb];
  // The payload columns are loaded now, with mr, and held in registers.
  u64 vi[kPerW], vt[kPerW], vm[kPerW];  // loaded together: one round trip
#pragma unroll
  for (int j = 0; j < kPerW; ++j) {
    const u32 k = threadIdx.x + j * kPartThreads;
    vi[j] = k < nrec ? in.index[lo + k] : 0ull;
    vt[j] = k < nrec ? u64(in.term32[lo + k]) : 0ull;
    vm[j] = k < nrec ? in.mr[lo + k] : 0ull;
  }
  if (threadIdx.x < kChunksPerSb) start[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPerW; ++j) {
    const u32 k = threadIdx.x + j * kPartThreads;
    if (k >= nrec) continue;
    const u16 b = u16((u32(vm[j]) >> 10) & 127u);
    L.bin[k] = b;
    L.rank[k] = u16(atomicAdd(&start[b], 1u));
    L.stage[k] = vm[j];
  }
  __syncthreads();
  tile_scan_bins(start, kChunksPerSb, L.wsum);
  if (threadIdx.x <= kChunksPerSb)
    cs[row * (kChunksPerSb + 1) + threadIdx.x] =
        lo + (threadIdx.x < kChunksPerSb ? start[threadIdx.x] : nrec);
  tile_perm(L, start, nrec);
  for (u32 e = threadIdx.x; e < nrec; e += blockDim.x) out.mr[lo + e] = L.stage[L.perm[e]];
  __syncthreads();
  for (int col = 0; col < 2; ++col) {
#pragma unroll
    for (int j = 0; j < kPerW; ++j) {
      const u32 k = threadIdx.x + j * kPartThreads;
      if (k < nrec) L.stage[k] = col == 0 ? vi[j] : vt[j];
    }
    __syncthreads();
    if (col == 1) {
      for (u32 e = threadIdx.x; e < nrec; e += blockDim.x)
        out.term32[lo + e] = u32(L.stage[L.perm[e]]);
    } else {
      for (u32 e = threadIdx.x; e < nrec; e += blockDim.x) out.index[lo + e] = L.stage[L.perm[e]];
    }
    __syncthreads();
  }
}

// Records of pool part pid: the rest of its region's fill past the part's
// start (a drawn part's positions below the fill are all written by K3).
__device__ __forceinline__ u32 pool_part_records(const Geometry& geo, const Pool& pool,
                                                 const u32* __restrict__ counts, u32 pid) {
  const u32 r = pool.owner_r[pid], k = pool.owner_k[pid];
  const u32 first = geo.cap + k * u32(kTile), fill = counts[r];
  const u32 n = fill > first ? fill - first : 0u;
  return n < u32(kTile) ? n : u32(kTile);
}

// K4's part for this workgroup: the region grid's part blockIdx.x, or —
// for the workgroups past `kparts`, one per part the pool can hold — the
// overflow pool's part blockIdx.x - kparts if it was drawn.  Returns false
// when there is none (a pool workgroup of a balanced batch returns after one
// load).  One call site of the part sort per kernel, and no loop: either a
// second call site or a loop over pool parts measured +21-27 VGPRs and +31
// SGPRs on the compact K4 (occupancy 8 -> 5).
template <bool WIDE>
__device__ __forceinline__ bool k4_item(const Geometry& geo, const Pool& pool,
                                        const u32* __restrict__ counts, u32 kparts, u32& lo,
                                        u32& nrec, u64& row, u32& sb) {
  if (blockIdx.x < kparts) {
    u32 r, j;
    if constexpr (WIDE) {
      // part-major order: workgroup b takes part j = b / R of region r = b % R
      // (R = NSB x 8), so the first parts of neighbouring regions go to
      // different XCDs whatever ppx is (region-major order put every first
      // part on the XCDs b % 8 = (r * ppx) % 8: two of eight for an even
      // ppx), and region (sb, x)'s first part runs on the XCD slot x that
      // wrote it in K3
      const u32 R = geo.NSB * kRegionShards;
      j = blockIdx.x / R;
      r = blockIdx.x - j * R;
    } else {
      // region-major order (the parts of a region on neighbouring
      // workgroups): with the tracker's ppx (5 at the bench) the first parts
      // still spread over the XCDs, and the part-major order measured +1 %
      // here (profiles/r04/leader/resv/)
      r = blockIdx.x / geo.ppx;
      j = blockIdx.x - r * geo.ppx;
    }
    u32 fill = counts[r];
    fill = fill < geo.cap ? fill : geo.cap;
    if constexpr (WIDE) {
      const u32 np = region_parts(fill, kWideSlack);
      if (j >= np) return false;  // no such part this call
      nrec = j + 1 == np ? fill - j * u32(kTile) : u32(kTile);
    } else {
      if (j * u32(kTile) >= fill) return false;  // no such part this tick
      nrec = fill - j * u32(kTile) < u32(kTile) ? fill - j * u32(kTile) : u32(kTile);
    }
    lo = r * geo.cap + j * u32(kTile);
    row = u64(r) * geo.ppx + j;
    sb = r / kRegionShards;
    return true;
  }
  const u32 drawn = *pool.ctr;
  const u32 np = drawn < pool.npool ? drawn : pool.npool;
  const u32 pid = blockIdx.x - kparts;
  if (pid >= np) return false;
  lo = u32(pool.base + u64(pid) * kTile);
  nrec = pool_part_records(geo, pool, counts, pid);
  row = geo.region_rows() + pid;
  sb = pool.owner_r[pid] / kRegionShards;
  return true;
}

__global__ __launch_bounds__(kPartThreads) void k_bk_split_wide(Geometry geo,
                                                                const u32* __restrict__ counts,
                                                                Cols in, Cols out,
                                                                u32* __restrict__ cs, Pool pool,
                                                                u32 kparts) {
  u32 lo, nrec, sb;
  u64 row;
  if (k4_item<true>(geo, pool, counts, kparts, lo, nrec, row, sb))
    split_wide_part(in, out, cs, lo, nrec, row);
}

// K4 for compact records (the tracker steps) in its own kernel: only the
// staged records and the chunk counters in LDS (33 KB instead of the shared
// tile's 61 KB) and 512 threads of 8 records, so four parts run per CU
// instead of two (round 3: fixed tick 583.5 -> 572.2 us).
constexpr int kSplitThreads = 512;
constexpr int kSplitPer = kTile / kSplitThreads;
// A part holding a chunk run of >= kHeavyRun records (a hot group): after
// the part is sorted by chunk-low into stage[] (its registers are dead by
// then, so this path costs the common one no VGPRs), each such run's records
// with equal lg | slot | reject | term are folded into one (qb_bucket.h,
// kDedupFlag) — the largest index and the count, in the side table at row *
// kDedupSlots + its LDS table slot — and the part is written out with the
// new run lengths.  Escapes, and records that find no table slot within 8
// probes, stay as they are.  start[] holds the exclusive bin starts (nrec
// records), and stays the old starts until the recount.
__device__ __forceinline__ u32 bin_of(const u32* start, u32 e) {
  u32 a = 0;  // start[a] <= e, 128 bins
#pragma unroll
  for (u32 st = 64; st >= 1; st >>= 1) a = start[a + st] <= e ? a + st : a;
  return a;
}
__device__ __forceinline__ void dedup_compact_part(const Geometry& geo, Cols out,
                                                   u32* __restrict__ cs, u32 lo, u32 nrec, u64 row,
                                                   u32 sb, Side side, const u64* stage, u32* start,
                                                   u32* wsum, bool sided) {
  const RecFmt fmt = geo.fmt;
  __shared__ u32 hkey[kDedupSlots];
  __shared__ u64 hmax[kDedupSlots];
  __shared__ u32 hcnt[kDedupSlots];
  __shared__ u32 cnt2[kChunksPerSb + 1];
  constexpr u32 kEmpty = 0xFFFFFFFFu;  // (a key's top bit is 0: chunk-low < 128)
  for (u32 i = threadIdx.x; i < kDedupSlots; i += kSplitThreads) {
    hkey[i] = kEmpty;
    hmax[i] = 0;
    hcnt[i] = 0;
  }
  if (threadIdx.x <= kChunksPerSb) cnt2[threadIdx.x] = 0;
  __syncthreads();
  const u32 hmask = (1u << kRecHdrBits) - 1u;
  const u32 ts = fmt.term_shift();
  u32 keep = 0;  // bit j: position threadIdx.x + j * kSplitThreads stays a record of its own
  u32 ksv[kSplitPer];  // the side word of each position (sided calls), moved with a kept record
  for (u32 j = 0; j < u32(kSplitPer); ++j) {
    const u32 e = threadIdx.x + j * kSplitThreads;
    ksv[j] = 0;
    if (e >= nrec) break;
    const u32 b = bin_of(start, e);
    const u32 nb = (b + 1 < kChunksPerSb ? start[b + 1] : nrec) - start[b];
    const u64 v = stage[e];
    // (the placement above wrote this workgroup's side words before its
    // barrier; no wave read these lines earlier in this launch)
    if (sided) ksv[j] = out.side[lo + e];
    bool merged = false;
    u32 hdr = u32(v) & hmask;
    bool foldable = nb >= kHeavyRun && fmt.term(v) != fmt.tesc();
    if (foldable && fmt.term(v) == fmt.tside()) {
      // a side record: folded under the term code kTermIsGroup when its term
      // is the group's, as a term-0 record (stale either way) when below it;
      // a higher one stays (its chunk goes to the slow path)
      const u64 g = u64(geo.chunk_of_sb_cl(sb, b)) * geo.CH + fmt.lg(v);
      const u64 gt = side.group_term[g];
      if (u64(ksv[j]) < gt) hdr &= (1u << ts) - 1u;
      else foldable = u64(ksv[j]) == gt;
    }
    if (foldable) {
      const u32 key = (b << kRecHdrBits) | hdr;
      const u32 h = (key * 2654435761u) >> 24;
      for (u32 q = 0; q < 8 && !merged; ++q) {
        const u32 sl = (h + q) & (kDedupSlots - 1u);
        const u32 old = atomicCAS(&hkey[sl], kEmpty, key);
        if (old == kEmpty || old == key) {
          atomicMax(&hmax[sl], v >> kRecHdrBits);
          atomicAdd(&hcnt[sl], 1u);
          merged = true;
        }
      }
    }
    if (!merged) {
      keep |= 1u << j;
      atomicAdd(&cnt2[b], 1u);
    }
  }
  __syncthreads();  // the table is complete
  const u32 hk = threadIdx.x < kDedupSlots ? hkey[threadIdx.x] : kEmpty;
  if (hk != kEmpty) atomicAdd(&cnt2[hk >> kRecHdrBits], 1u);
  __syncthreads();
  const u32 total = tile_scan_bins(cnt2, kChunksPerSb, wsum);  // cnt2 = the new bin starts
  if (threadIdx.x <= kChunksPerSb)
    cs[row * (kChunksPerSb + 1) + threadIdx.x] =
        lo + (threadIdx.x < kChunksPerSb ? cnt2[threadIdx.x] : total);
  __syncthreads();  // (cnt2 is a placement cursor from here on; every side word is read)
  for (u32 j = 0; j < u32(kSplitPer); ++j) {
    const u32 e = threadIdx.x + j * kSplitThreads;
    if (e >= nrec) break;
    if (!((keep >> j) & 1u)) continue;
    const u32 p = lo + atomicAdd(&cnt2[bin_of(start, e)], 1u);
    out.mr[p] = stage[e];
    if (sided) out.side[p] = ksv[j];
  }
  if (hk != kEmpty) {
    const u32 n = hcnt[threadIdx.x];
    const u64 mx = hmax[threadIdx.x], hdr = hk & hmask;
    const u32 t = fmt.term(hdr);
    const u32 c = geo.chunk_of_sb_cl(sb, hk >> kRecHdrBits);
    const u64 g = u64(c) * geo.CH + fmt.lg(hdr);
    const u64 gt = side.group_term[g];
    u64 rec = hdr | (mx << kRecHdrBits);  // a single record: itself (a side one: term gt)
    if (n > 1) {
      const u64 si = row * kDedupSlots + threadIdx.x;
      side.idx[si] = mx;
      side.tc[si] = (t == fmt.tside() ? kTermIsGroup : t) | (n << kDedupCountShift);
      const u64 tmask = u64(fmt.tesc()) << ts;
      rec = (hdr & ~tmask) | tmask | ((si | kDedupFlag) << kRecHdrBits);
      // the n - 1 records folded away, in the class K5 gives the record that
      // stands for them (a higher term sends the chunk to the slow path,
      // which counts every record itself: nothing to add)
      const u32 s = fmt.slot(hdr);
      u32 cls = 4;  // none
      if (side.off && s >= side.off[g + 1] - side.off[g]) {
        cls = 3;  // non-member (CSR: raft.go:1100-1104)
      } else {
        const u64 tt = t == fmt.tside() ? gt : u64(t);
        cls = tt < gt ? 0u : tt > gt ? 4u : fmt.rej(hdr) ? 2u : 1u;
      }
      if (cls < kExtClasses) atomicAdd(&side.ext[u64(c) * kExtClasses + cls], n - 1u);
    }
    const u32 p = lo + atomicAdd(&cnt2[hk >> kRecHdrBits], 1u);
    out.mr[p] = rec;
    if (sided) out.side[p] = u32(gt);  // (read only for a single side record: its term)
  }
}

__device__ __forceinline__ void split_compact_part(const Geometry& geo, Cols in, Cols out,
                                                   u32* __restrict__ cs, u32 lo, u32 nrec, u64 row,
                                                   u32 sb, Side side) {
  __shared__ u64 stage[kTile];
  __shared__ u32 start[kChunksPerSb];
  __shared__ u32 wsum[kSplitThreads / 64];
  // side records anywhere in this call (K3's flag word): the side column
  // moves with the records, every position of the part written (whole lines)
  const bool sided = *in.sflag != 0u;
  u64 vm[kSplitPer];  // loaded together: one round trip
  u32 vc[kSplitPer];
#pragma unroll
  for (int j = 0; j < kSplitPer; ++j) {
    const u32 k = threadIdx.x + j * kSplitThreads;
    vm[j] = k < nrec ? in.mr[lo + k] : 0ull;
    vc[j] = k < nrec ? u32(in.cl[lo + k]) : 0u;
  }
  if (threadIdx.x < kChunksPerSb) start[threadIdx.x] = 0;
  __syncthreads();
  // (each record's rank rides in its chunk-low word: vc = chunk-low | rank << 8,
  // so the side words cost no registers past the kernel's 64)
#pragma unroll
  for (int j = 0; j < kSplitPer; ++j) {
    const u32 k = threadIdx.x + j * kSplitThreads;
    vc[j] |= (k < nrec ? atomicAdd(&start[vc[j]], 1u) : 0u) << 8;
  }
  // a chunk with >= kHeavyRun records in this part (a hot group): the dedup
  // pass below (rare; block-uniform)
  // (needs the group terms to class what it folds: the step entry points
  // pass them, the bucket-only one does not)
  const bool heavy = __syncthreads_or(threadIdx.x < kChunksPerSb && side.group_term &&
                                      start[threadIdx.x] >= kHeavyRun);
  tile_scan_bins(start, kChunksPerSb, wsum);
  if (!heavy && threadIdx.x <= kChunksPerSb)
    cs[row * (kChunksPerSb + 1) + threadIdx.x] =
        lo + (threadIdx.x < kChunksPerSb ? start[threadIdx.x] : nrec);
#pragma unroll
  for (int j = 0; j < kSplitPer; ++j) {
    const u32 k = threadIdx.x + j * kSplitThreads;
    if (k < nrec) stage[start[vc[j] & 0xFFu] + (vc[j] >> 8)] = vm[j];
  }
  if (heavy) {  // (rare) the side words go to their sorted positions directly
    if (sided) {
#pragma unroll
      for (int j = 0; j < kSplitPer; ++j) {
        const u32 k = threadIdx.x + j * kSplitThreads;
        if (k < nrec) out.side[lo + start[vc[j] & 0xFFu] + (vc[j] >> 8)] = in.side[lo + k];
      }
    }
    __syncthreads();
    dedup_compact_part(geo, out, cs, lo, nrec, row, sb, side, stage, start, wsum, sided);
    return;
  }
  // the side words (block-uniform), loaded once the records' registers are
  // free; their latency runs under the record stores below
  u32 sv[kSplitPer];
  if (sided) {
#pragma unroll
    for (int j = 0; j < kSplitPer; ++j) {
      const u32 k = threadIdx.x + j * kSplitThreads;
      sv[j] = k < nrec ? in.side[lo + k] : 0u;
    }
  }
  __syncthreads();
  for (u32 e = threadIdx.x; e < nrec; e += kSplitThreads) out.mr[lo + e] = stage[e];
  if (sided) {
    // sorted through the records' LDS (now read): scattered LDS stores, then
    // coalesced global ones (scattered 4-byte global stores cost K4 ~2x)
    u32* s32 = reinterpret_cast<u32*>(stage);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSplitPer; ++j) {
      const u32 k = threadIdx.x + j * kSplitThreads;
      if (k < nrec) s32[start[vc[j] & 0xFFu] + (vc[j] >> 8)] = sv[j];
    }
    __syncthreads();
    for (u32 e = threadIdx.x; e < nrec; e += kSplitThreads) out.side[lo + e] = s32[e];
  }
}

// (the dedup path's registers would otherwise cost the common path its
// residency: 70 VGPRs / 102 SGPRs unbounded, 56 / 75 without the path)
__global__ __launch_bounds__(kSplitThreads)
__attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8, 8))) void k_bk_split_compact(
    Geometry geo, const u32* __restrict__ counts, Cols in, Cols out, u32* __restrict__ cs,
    Pool pool, u32 kparts, Side side) {
  // part p = region r's j-th kTile records (the region grid, qb_bucket.h),
  // then the overflow pool's parts
  u32 lo, nrec, sb;
  u64 row;
  if (k4_item<false>(geo, pool, counts, kparts, lo, nrec, row, sb))
    split_compact_part(geo, in, out, cs, lo, nrec, row, sb, side);
}

// ---------------------------------------------------------------- K5 ----
// Records arrive compact (one u64 each, RecFmt: lg, slot, reject, term,
// index; a side record's term is the u32 at its position in the side column,
// read with the record; an escape record carries its batch position and K5
// reads its exact index and term from the original batch).  A chunk none of whose records is
// above its group's term (the steady state) is applied here.  A chunk with a
// higher-term record (the sequential leader steps down there and ignores what
// follows, raft.go:875-879: batch order matters) is "slow": K5 leaves its
// state untouched, flags it, and k_bk_slow applies it from the original
// batch in batch order (the exact two-pass form of qb_tracker.hip).
// LDS: acc_match[n][CH] u64, acc_next[n][CH] u64 (if tracked), gterm[CH] u64,
// act[CH] u32.
// K5 threads per workgroup: 512, at most the chunk's group count (round 2:
// 512-thread workgroups, one group per thread, -12 us per tick).
__host__ __device__ constexpr u32 k5_block(int n) {
  return chunk_groups(u32(n)) < 512u ? chunk_groups(u32(n)) : 512u;
}

// SGPR cap: the hardware admits min(8, 800 / (ceil(sgpr / 16) * 16 + 16))
// waves per SIMD (MI355X_MICROARCH.md, residency), so the compiler's 92
// SGPRs held K5 at 3 workgroups per CU where its VGPRs and LDS allow 4;
// capped at 80 (a few SGPRs spill to VGPR lanes): -11 us per 16M-group tick.
template <int N, bool NEXT, bool MANY>
__device__ __forceinline__ void apply_chunk(
    const u32 c, const bool skip_heavy, const Geometry& geo, const Cols& recs,
    const u32* __restrict__ counts, const u32* __restrict__ cs, const EscArgs& esc,
    const u64* __restrict__ group_term, const u64* __restrict__ term_start,
    u64* __restrict__ match, u64* __restrict__ next, u16* __restrict__ active,
    u64* __restrict__ committed, u32* __restrict__ stepdown_at, u8* __restrict__ advanced,
    u8* __restrict__ chunk_slow, u32* __restrict__ any_slow, u64* __restrict__ shards,
    const u32* __restrict__ ptab, const HeavyArgs& hv) {
  constexpr u32 CH = chunk_groups(N);
  constexpr u32 B = k5_block(N);
  constexpr u32 GPT = CH / B;  // groups per thread in the commit phase
  __shared__ u32 tl[3];
  BlockTally<3> tally;
  __shared__ u64 acc_m[N * CH];
  __shared__ u64 acc_n[NEXT ? N * CH : 1];
  __shared__ u64 gterm[CH];
  __shared__ u32 act[CH];
  __shared__ u32 slow;
  const u64 g0 = u64(c) * CH;
  const u32 ng = u32(geo.G - g0 < CH ? geo.G - g0 : CH);
  // Load order: the group terms and this chunk's run table first, then the
  // commit phase's state (match rows, committed, term_start, RecentActive's
  // word), so the record pass waits for its own inputs only — vector loads
  // retire in order, and with the state issued first every wait of the
  // record chain (run table, then records) also waited for the state.  The
  // state's latency runs under the record pass.  Loads are branch-free
  // (clamped to the chunk's last group): exact wait counts need straight-line
  // code.
  const u32 sb = geo.sb_of_chunk(c), cl = geo.cl_of_chunk(c);
  // a record of this chunk that did not fit its reserved region (K3): the
  // whole chunk goes to the slow path
  const bool overflow = chunk_slow[c] == kChunkOverflow;
  // (the linear order's workgroup of a chunk the leading workgroups take:
  // its super-bucket is among the first hv.blocks / 128 heavy ones — read
  // with the run table's loads, tested once the table is built)
  const u32 hf = skip_heavy ? hv.sbflag[sb] : 0u;
  const bool heavy_sb = hf != 0u && hf - 1u < hv.blocks / kChunksPerSb;
  // side records in this call (K3's flag word): their side words are read
  // with the records
  const bool sided = *recs.sflag != 0u;
  // the records K4's dedup folded away (stale, applied, rejected)
  const u32 extv = esc.side.ext[u64(c) * kExtClasses + (threadIdx.x & 3u)];
  u64 gtr[GPT];
#pragma unroll
  for (u32 k = 0; k < GPT; ++k) {
    const u32 lg = threadIdx.x + k * B;
    gtr[k] = group_term[g0 + (lg < ng ? lg : ng - 1)];
  }
  __shared__ RunTableOf<MANY> rt;
  const RunTable::Regs rq = RunTable::issue_regions(cs, counts, sb, geo.ppx, geo.cap, cl);
  u64 v[GPT][N], cm[GPT], ts[GPT];
  u32 av[GPT];
#pragma unroll
  for (u32 k = 0; k < GPT; ++k) {
    const u32 lg = threadIdx.x + k * B;
    const u64 g = g0 + (lg < ng ? lg : ng - 1);
#pragma unroll
    for (int s = 0; s < N; ++s) v[k][s] = match[u64(s) * geo.G + g];
    cm[k] = committed[g];
    ts[k] = term_start[g];
    av[k] = active[g];
  }
  for (u32 k = threadIdx.x; k < N * CH; k += B) {
    acc_m[k] = 0;
    if constexpr (NEXT) acc_n[k] = 0;
  }
#pragma unroll
  for (u32 k = 0; k < GPT; ++k) {
    gterm[threadIdx.x + k * B] = gtr[k];
    act[threadIdx.x + k * B] = 0;
  }
  if (threadIdx.x == 0) slow = overflow ? 1u : 0u;
  if (threadIdx.x < 3) tl[threadIdx.x] = 0;
  // This chunk's records: one short run per part of its super-bucket,
  // flattened into one index space (RunTable) so every thread has a record
  // in flight at once; kRecPer records per thread, both columns of each
  // loaded before the first is classified.
  u32 total = rt.template finish<MANY>(rq, cs, counts, sb, geo.ppx, geo.cap, cl);
  __syncthreads();
  if (heavy_sb) return;  // block-uniform: the heavy workgroups apply this chunk
  constexpr int kRecPer = int(kK5Inflight / B);  // records in flight per workgroup
  const RecFmt fmt = geo.fmt;
  u64 rec[kRecPer];
  u32 srec[kRecPer];  // side words (a call with side records: K3's flag)
  // branch-free (clamped; an empty chunk reads record 0, which exists)
  auto fetch = [&](u32 f0, u32 tot) {
    u32 ix[kRecPer];
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) {
      const u32 f = f0 + u32(r) * B + threadIdx.x;
      ix[r] = tot ? rt.template locate_fixed<MANY>(f < tot ? f : tot - 1) : 0u;
    }
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) rec[r] = recs.mr[ix[r]];
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) srec[r] = sided ? recs.side[ix[r]] : 0u;
  };
  auto apply = [&](u32 f0, u32 tot) {
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) {
      const u32 f = f0 + u32(r) * B + threadIdx.x;
      bool stale = false, applied = false, rejected = false;
      if (f < tot) {
        const u64 x = rec[r];
        const u32 lg = fmt.lg(x), s = fmt.slot(x);
        u64 t = fmt.term(x), idx = fmt.payload(x);
        const u64 gt = gterm[lg];
        // a side record: its term from the side column; an escape: the exact
        // values from the batch, or a folded record's from the side table
        if (t == fmt.tside()) t = srec[r];
        else if (t == fmt.tesc()) unescape(esc, t, idx, gt);
        if (t > gt) {
          slow = 1;  // higher term: step-down order (raft.go:875-879)
        } else if (t < gt) {
          stale = true;                                   // raft.go:883-921
        } else {
          atomicOr(&act[lg], 1u << s);                    // raft.go:1107
          if (fmt.rej(x)) {
            rejected = true;                              // raft.go:1109: not MaybeUpdate
          } else {
            applied = true;
            atomicMax(&acc_m[s * CH + lg], idx);          // progress.go:146-150
            if constexpr (NEXT) atomicMax(&acc_n[s * CH + lg], idx + 1ull);  // :151
          }
        }
      }
      tally.add(0, stale);
      tally.add(1, applied);
      tally.add(2, rejected);
    }
  };
  // The first batch (at the bench's ~512 records per chunk, all of them) in
  // straight-line code: its wait is for its own loads and the state issued
  // before them, not a conservative drain at a loop head.
  fetch(0, total);
  // pinned: the records are loaded here, not sunk into apply's branches
#pragma unroll
  for (int r = 0; r < kRecPer; ++r) asm volatile("" : "+v"(rec[r]), "+v"(srec[r]));
  apply(0, total);
  // The rest of the region table, then the chunk's records in the overflow
  // pool (a skewed batch; none otherwise) in windows of 64 pool rows
  // through the same table — one loop, so the record pass is inlined twice
  // only (a loop per source cost 13 VGPRs).  Block-uniform control flow.
  {
    const u32 npool = rt.npool;
    u32 tot = total, w = 0;
    for (u32 f0 = B * kRecPer;;) {
      if (f0 >= tot) {
        if (w * 64u >= npool) break;
        __syncthreads();  // every reader of the previous table is done
        if (threadIdx.x < 64) rt.pool_window(w, cs, ptab, geo.kmax, geo.region_rows(), sb, cl);
        __syncthreads();
        ++w;
        tot = rt.pre[rt.nr];
        f0 = 0;
        continue;
      }
      fetch(f0, tot);
#pragma unroll
      for (int r = 0; r < kRecPer; ++r) asm volatile("" : "+v"(rec[r]), "+v"(srec[r]));
      apply(f0, tot);
      f0 += B * kRecPer;
    }
  }
  // the counts are final: staged before the barrier the block takes anyway,
  // published after it (a flush with barriers of its own at the end cost
  // 15 us per 16M-group tick)
  tally.stage(tl);
  if (threadIdx.x < 3 && extv) atomicAdd(&tl[threadIdx.x], extv);  // K4's folded records
  __syncthreads();
  if (slow) {  // block-uniform: state left for k_bk_slow, counts discarded
#pragma unroll
    for (u32 k = 0; k < GPT; ++k) {
      const u32 lg = threadIdx.x + k * B;
      if (lg < ng) stepdown_at[g0 + lg] = 0xFFFFFFFFu;
    }
    if (threadIdx.x == 0) {
      chunk_slow[c] = 1;
      atomicOr(any_slow, 1u);
    }
    return;
  }
  if (threadIdx.x == 0) chunk_slow[c] = 0;
  {
    const int slot[3] = {QB_STAT_STALE_TERM, QB_STAT_APPLIED, QB_STAT_REJECTED};
    BlockTally<3>::publish(tl, shard_of(shards), slot);
  }
  // maybeCommit for every group of the chunk + write-back (coalesced rows,
  // whole wave segments: segment_any, qb_bucket.h).
#pragma unroll
  for (u32 k = 0; k < GPT; ++k) {
    const u32 lg = threadIdx.x + k * B;
    const bool live = lg < ng;
    const u64 g = g0 + (live ? lg : 0u);
#pragma unroll
    for (int s = 0; s < N; ++s) {
      const u64 a = acc_m[s * CH + lg];
      const bool up = live && a > v[k][s];
      if (up) v[k][s] = a;
      if (segment_any(up) && live) match[u64(s) * geo.G + g] = v[k][s];
      if constexpr (NEXT) {
        if (live) {
          u64* q = next + u64(s) * geo.G + g;
          const u64 nn = acc_n[s * CH + lg];
          if (nn > *q) *q = nn;
        }
      }
    }
    const u64 ci = select_quorum<N>(v[k]);
    const bool adv = live && ci > cm[k] && ci >= ts[k];  // log.go:328-334
    const u32 na = live ? act[lg] : 0u;
    if (segment_any(adv) && live) committed[g] = adv ? ci : cm[k];
    if (advanced && live) advanced[g] = adv ? 1 : 0;
    if (segment_any(na != 0) && live) active[g] = u16(av[k] | na);
  }
}

template <int N, bool NEXT, bool MANY>
__global__ __launch_bounds__(k5_block(N)) __attribute__((amdgpu_num_sgpr(80))) void k_bk_apply(
    Geometry geo, Cols recs, const u32* __restrict__ counts, const u32* __restrict__ cs,
    EscArgs esc, const u64* __restrict__ group_term, const u64* __restrict__ term_start,
    u64* __restrict__ match, u64* __restrict__ next, u16* __restrict__ active,
    u64* __restrict__ committed, u32* __restrict__ stepdown_at, u8* __restrict__ advanced,
    u8* __restrict__ chunk_slow, u32* __restrict__ any_slow, u64* __restrict__ shards,
    const u32* __restrict__ ptab, HeavyArgs hv) {
  // One chunk per workgroup, one call site (a second call site or a loop
  // over chunks doubled the body's registers): the leading hv.blocks
  // workgroups take chunk i % 128 of the i / 128-th heavy super-bucket (the
  // first hv.blocks / 128 of them; later ones stay in the linear order), the
  // rest the chunks in reverse order — K4 wrote the last super-buckets last,
  // so their runs are the ones still in the 256 MB MALL when K5 starts.
  u32 c;
  const bool lead = blockIdx.x < hv.blocks;
  if (lead) {
    const u32 i = blockIdx.x;
    if (i >= *hv.nheavy * kChunksPerSb) return;  // (all of them in a balanced batch)
    c = geo.chunk_of_sb_cl(hv.heavy[i / kChunksPerSb], i % kChunksPerSb);
    if (c >= geo.NC) return;
  } else {
    c = geo.NC - 1u - (blockIdx.x - hv.blocks);
  }
  apply_chunk<N, NEXT, MANY>(c, !lead, geo, recs, counts, cs, esc, group_term, term_start, match,
                             next, active, committed, stepdown_at, advanced, chunk_slow, any_slow,
                             shards, ptab, hv);
}


template <int N, bool MANY>
void launch_apply_rows(const Geometry& geo, Cols recs, const u32* counts, const u32* cs,
                       const ApplyArgs& a, hipStream_t st) {
  const EscArgs esc{a.ri, a.rt, a.side};
  const dim3 grid(a.hv.blocks + geo.NC);
  if (a.next)
    hipLaunchKernelGGL((k_bk_apply<N, true, MANY>), grid, dim3(k5_block(N)), 0, st, geo, recs, counts,
                       cs, esc, a.gt, a.ts, a.match, a.next, a.active, a.committed, a.stepdown,
                       a.adv, a.chunk_slow, a.any_slow, a.stats, a.ptab, a.hv);
  else
    hipLaunchKernelGGL((k_bk_apply<N, false, MANY>), grid, dim3(k5_block(N)), 0, st, geo, recs, counts,
                       cs, esc, a.gt, a.ts, a.match, a.next, a.active, a.committed, a.stepdown,
                       a.adv, a.chunk_slow, a.any_slow, a.stats, a.ptab, a.hv);
}
template <int N>
void launch_apply(const Geometry& geo, Cols recs, const u32* counts, const u32* cs,
                  const ApplyArgs& a, hipStream_t st) {
  if (RunTable::many_rows(geo.ppx)) launch_apply_rows<N, true>(geo, recs, counts, cs, a, st);
  else launch_apply_rows<N, false>(geo, recs, counts, cs, a, st);
}

template <int N>
void launch_slow(const Geometry& geo, const ApplyArgs& a, const SlowArgs& s, u64* stats,
                 hipStream_t st) {
  hipLaunchKernelGGL((k_bk_slow<FixedLay<N>, ColSrc>), dim3(s.grid), dim3(kBlock), 0, st, geo,
                     FixedLay<N>{geo.G}, ColSrc{s.rg, s.rf, s.ri, s.rt}, a.gt, a.ts, a.chunk_slow, a.any_slow, s.bar, a.stepdown, a.match, a.next,
                     a.active, a.committed, a.adv, a.stats, stats);
}

template <int... Ns>
void dispatch_apply(std::integer_sequence<int, Ns...>, int n, const Geometry& geo, Cols recs,
                    const u32* counts, const u32* cs, const ApplyArgs& a, hipStream_t st) {
  ((n == Ns + 1 ? launch_apply<Ns + 1>(geo, recs, counts, cs, a, st) : void()), ...);
}

template <int... Ns>
void dispatch_slow(std::integer_sequence<int, Ns...>, int n, const Geometry& geo,
                   const ApplyArgs& a, const SlowArgs& s, u64* stats, hipStream_t st) {
  ((n == Ns + 1 ? launch_slow<Ns + 1>(geo, a, s, stats, st) : void()), ...);
}



}  // namespace bk
}  // namespace qb

using namespace qb;

namespace qb {
namespace bk {

// K4 of the compact form: each part of the region grid and of the pool
// sorted by chunk-low (bucket_records' second launch; the composed wire ->
// tracker step runs it after its own level 1, qb_wire_tracker.hip).
void launch_split_compact(const Geometry& geo, const Carve& cv, char* ws, const u64* group_term,
                          const u32* csr_off, hipStream_t st) {
  const unsigned kparts = geo.NSB * kRegionShards * geo.ppx;
  u32* sflag = side_flag_at(ws, cv);
  const Cols buf1 = compact_at(ws + cv.buf1, ws + cv.cl, ws + cv.side1, sflag),
             buf2 = compact_at(ws + cv.buf2, nullptr, ws + cv.side2, sflag);
  hipLaunchKernelGGL(k_bk_split_compact, dim3(kparts + geo.npool), dim3(kSplitThreads), 0, st, geo,
                     reinterpret_cast<u32*>(ws + cv.counts), buf1, buf2,
                     reinterpret_cast<u32*>(ws + cv.chunk_start), pool_at(ws, cv, geo), kparts,
                     side_at(ws, cv, group_term, csr_off));
}

ApplyArgs fixed_apply_args(const Geometry& geo, const Carve& cv, char* ws, const u64* ri,
                           const u64* rt, const u64* group_term, const u64* term_start, u64* match,
                           u64* next, u16* active, u64* committed, u32* stepdown_at, u8* advanced) {
  const Pool pool = pool_at(ws, cv, geo);
  return ApplyArgs{ri, rt, side_at(ws, cv), group_term, term_start, match, next, active, committed,
                   stepdown_at, advanced, reinterpret_cast<u8*>(ws + cv.chunk_flags),
                   reinterpret_cast<u32*>(ws + cv.flags), reinterpret_cast<u64*>(ws + cv.shards),
                   reinterpret_cast<const u32*>(ws + cv.ptab),
                   HeavyArgs{pool.sbflag, pool.heavy, pool.nheavy,
                             geo.NC < kHeavyBlocks ? geo.NC : kHeavyBlocks}};
}

// K5 of the FIXED step (k_bk_apply<n>) over buf2.
void launch_fixed_apply(u32 n, const Geometry& geo, const Carve& cv, char* ws, const ApplyArgs& a,
                        hipStream_t st) {
  const Cols recs = compact_at(ws + cv.buf2, nullptr, ws + cv.side2, side_flag_at(ws, cv));
  dispatch_apply(std::make_integer_sequence<int, QB_MAX_SLOTS>{}, int(n), geo, recs,
                 reinterpret_cast<const u32*>(ws + cv.counts),
                 reinterpret_cast<const u32*>(ws + cv.chunk_start), a, st);
}

int bucket_records(const Geometry& geo, const Carve& cv, char* ws, const u32* rec_group,
                   const u8* rec_flags, const u64* rec_index, const u64* rec_term, u64* shards,
                   hipStream_t st, bool compact, const u64* group_term, const u32* csr_off) {
  u32* cs = reinterpret_cast<u32*>(ws + cv.chunk_start);
  u32* counts = reinterpret_cast<u32*>(ws + cv.counts);
  u8* chunk_flags = reinterpret_cast<u8*>(ws + cv.chunk_flags);
  // Reserved regions (round 4): the stat shards, the flag words, the
  // regions' fill counters, the chunk flags (and the wide form's per-chunk
  // overflow counts) are adjacent in the carve — one memset — and K3 reserves
  // each tile's run of a super-bucket in its XCD slot's region with one
  // atomic per (tile, super-bucket): no histogram pass, no scan, no part
  // table (K1, K2 and the sums / parts kernel of round 3).  The chunk flags
  // must start at 0: K3 marks overflowing chunks and their readers test the
  // mark (a fresh workspace holds garbage; a stale mark would send a tracker
  // chunk to the slow path and reset its groups' stepdown_at).
  hipError_t e = hipMemsetAsync(ws + cv.shards, 0, cv.zero_end - cv.shards, st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(shards, counters)");
  if (geo.M == 0) return QB_OK;
  const unsigned kparts = geo.NSB * kRegionShards * geo.ppx;
  // K4's grid: the region grid's parts, then one workgroup per part the
  // overflow pool can hold (they return at once when none was drawn)
  const unsigned pblocks = geo.npool;
  const Pool pool = pool_at(ws, cv, geo);
  if (compact) {
    u32* sflag = side_flag_at(ws, cv);
    const Cols buf1 = compact_at(ws + cv.buf1, ws + cv.cl, ws + cv.side1, sflag);
    hipLaunchKernelGGL(k_bk_scatter<true>, dim3(geo.tile_grid()), dim3(kPartThreads),
                       4 * sizeof(u32) * geo.NSB, st, geo, rec_group, rec_flags, rec_index, rec_term,
                       buf1, counts, shards, chunk_flags, pool);
    QB_CHECK_LAUNCH("k_bk_scatter");
    launch_split_compact(geo, cv, ws, group_term, csr_off, st);
    QB_CHECK_LAUNCH("k_bk_split_compact");
    return QB_OK;
  }
  // wide: index, term32 (in a u64 column's space) and mr
  Cols buf1 = cols_at(ws + cv.buf1, cv.nrec_all, 3), buf2 = cols_at(ws + cv.buf2, cv.nrec_all, 3);
  buf1.term32 = reinterpret_cast<u32*>(buf1.term);
  buf2.term32 = reinterpret_cast<u32*>(buf2.term);
  hipLaunchKernelGGL(k_bk_scatter<false>, dim3(geo.tile_grid()), dim3(kPartThreads),
                     4 * sizeof(u32) * geo.NSB, st, geo, rec_group, rec_flags, rec_index, rec_term, buf1,
                     counts, shards, chunk_flags, pool);
  QB_CHECK_LAUNCH("k_bk_scatter");
  hipLaunchKernelGGL(k_bk_split_wide, dim3(kparts + pblocks), dim3(kPartThreads), 0, st, geo, counts,
                     buf1, buf2, cs, pool, kparts);
  QB_CHECK_LAUNCH("k_bk_split_wide");
  return QB_OK;
}

}  // namespace bk
}  // namespace qb

extern "C" size_t qb_fixed_tracker_workspace_bytes(uint32_t n, uint64_t G, uint64_t M) {
  if (n < 1 || n > QB_MAX_SLOTS) return 0;
  const bk::Carve cv = bk::carve(bk::geometry(n, G, M, 0, bk::kSbIl), 1);
  return cv.nrec_all <= 0xFFFFFFFFull ? cv.total : 0;  // 0: no workspace fits (u32 record index)
}

namespace {
// Shared checks of the tracker-step entry points; the geometry and carve of
// (n, G, M) are the same in all three, so a workspace bucketed by
// qb_dev_fixed_tracker_bucket is exactly what qb_dev_fixed_tracker_apply reads.
int fixed_tracker_check(uint32_t n, uint64_t G, uint64_t M, const void* workspace,
                        size_t workspace_bytes, bk::Geometry* geo, bk::Carve* cv) {
  QB_REQUIRE(n >= 1 && n <= QB_MAX_SLOTS, "n must be 1..%d", QB_MAX_SLOTS);
  QB_REQUIRE(M <= 0xFFFFFFFFull, "batch too large (M=%llu > 2^32-1)", (unsigned long long)M);
  QB_REQUIRE(G <= 0xFFFFFFFFull, "shard too large (G=%llu > 2^32-1)", (unsigned long long)G);
  *geo = bk::geometry(n, G, M, 0, bk::kSbIl);
  *cv = bk::carve(*geo, 1);
  // the reserved regions (NSB x 8 x cap records, about 2x M) are addressed
  // with u32 offsets by K3-K5
  QB_REQUIRE(cv->nrec_all <= 0xFFFFFFFFull,
             "batch too large for the bucket pass (M=%llu: %llu region records > 2^32-1)",
             (unsigned long long)M, (unsigned long long)cv->nrec_all);
  QB_REQUIRE(workspace && workspace_bytes >= cv->total,
             "workspace too small: need %zu bytes (qb_fixed_tracker_workspace_bytes)", cv->total);
  QB_REQUIRE(geo->NSB <= 4096, "shard too large for the bucket pass (G=%llu)",
             (unsigned long long)G);
  return QB_OK;
}
}  // namespace

namespace {
// The bucket half; group_term (nullable) lets K4 fold a hot group's records
// (the dedup needs the group terms to class what it folds away): the step
// passes it, the bucket-only entry point cannot.
int fixed_bucket(uint32_t n, uint64_t G, uint64_t M, const uint32_t* rec_group,
                 const uint8_t* rec_flags, const uint64_t* rec_index, const uint64_t* rec_term,
                 const uint64_t* group_term, void* workspace, size_t workspace_bytes,
                 void* stream) {
  if (G == 0) return QB_OK;
  QB_REQUIRE(M == 0 || (rec_group && rec_flags && rec_index && rec_term),
             "record pointer is NULL");
  bk::Geometry geo;
  bk::Carve cv;
  const int rc = fixed_tracker_check(n, G, M, workspace, workspace_bytes, &geo, &cv);
  if (rc != QB_OK) return rc;
  char* ws = static_cast<char*>(workspace);
  // (bucket_records zeroes the stat shards and the flag words itself)
  return bk::bucket_records(geo, cv, ws, rec_group, rec_flags, reinterpret_cast<const u64*>(rec_index),
                            reinterpret_cast<const u64*>(rec_term),
                            reinterpret_cast<u64*>(ws + cv.shards), as_stream(stream),
                            /*compact=*/true, reinterpret_cast<const u64*>(group_term));
}
}  // namespace

extern "C" int qb_dev_fixed_tracker_bucket(uint32_t n, uint64_t G, uint64_t M,
                                           const uint32_t* rec_group, const uint8_t* rec_flags,
                                           const uint64_t* rec_index, const uint64_t* rec_term,
                                           void* workspace, size_t workspace_bytes,
                                           void* stream) {
  return fixed_bucket(n, G, M, rec_group, rec_flags, rec_index, rec_term, nullptr, workspace,
                      workspace_bytes, stream);
}

extern "C" int qb_dev_fixed_tracker_apply(uint32_t n, uint64_t G, uint64_t M,
                                          const uint32_t* rec_group, const uint8_t* rec_flags,
                                          const uint64_t* rec_index, const uint64_t* rec_term,
                                          const uint64_t* group_term, const uint64_t* term_start,
                                          uint64_t* match, uint64_t* next, uint16_t* active,
                                          uint64_t* committed, uint32_t* stepdown_at,
                                          uint8_t* advanced_out, uint64_t* stats,
                                          void* workspace, size_t workspace_bytes, void* stream) {
  if (G == 0) return QB_OK;
  QB_REQUIRE(group_term && term_start && match && active && committed && stepdown_at && stats,
             "required state pointer is NULL");
  QB_REQUIRE(M == 0 || (rec_group && rec_flags && rec_index && rec_term),
             "record pointer is NULL");
  bk::Geometry geo;
  bk::Carve cv;
  const int rc = fixed_tracker_check(n, G, M, workspace, workspace_bytes, &geo, &cv);
  if (rc != QB_OK) return rc;
  hipStream_t st = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  u64* stt = reinterpret_cast<u64*>(stats);
  const auto* rg = reinterpret_cast<const u32*>(rec_group);
  const auto* ri = reinterpret_cast<const u64*>(rec_index);
  const auto* rtm = reinterpret_cast<const u64*>(rec_term);
  const bk::ApplyArgs a = bk::fixed_apply_args(
      geo, cv, ws, ri, rtm, reinterpret_cast<const u64*>(group_term),
      reinterpret_cast<const u64*>(term_start), reinterpret_cast<u64*>(match),
      reinterpret_cast<u64*>(next), active, reinterpret_cast<u64*>(committed), stepdown_at,
      advanced_out);
  bk::launch_fixed_apply(n, geo, cv, ws, a, st);
  QB_CHECK_LAUNCH("k_bk_apply");
  // chunks flagged slow by K5 (none in the steady state: the launch folds
  // the stat shards and returns) + the stat fold
  const bk::SlowArgs sa{rg, rec_flags, ri, rtm, reinterpret_cast<u32*>(ws + cv.flags) + 16,
                        bk::slow_blocks()};
  bk::dispatch_slow(std::make_integer_sequence<int, QB_MAX_SLOTS>{}, int(n), geo, a, sa, stt, st);
  QB_CHECK_LAUNCH("k_bk_slow");
  return QB_OK;
}

extern "C" int qb_dev_fixed_tracker_step(uint32_t n, uint64_t G, uint64_t M,
                                         const uint32_t* rec_group, const uint8_t* rec_flags,
                                         const uint64_t* rec_index, const uint64_t* rec_term,
                                         const uint64_t* group_term, const uint64_t* term_start,
                                         uint64_t* match, uint64_t* next, uint16_t* active,
                                         uint64_t* committed, uint32_t* stepdown_at,
                                         uint8_t* advanced_out, uint64_t* stats,
                                         void* workspace, size_t workspace_bytes, void* stream) {
  if (G == 0) return QB_OK;
  QB_REQUIRE(group_term && term_start && match && active && committed && stepdown_at && stats,
             "required state pointer is NULL");
  const int rc = fixed_bucket(n, G, M, rec_group, rec_flags, rec_index, rec_term, group_term,
                              workspace, workspace_bytes, stream);
  if (rc != QB_OK) return rc;
  return qb_dev_fixed_tracker_apply(n, G, M, rec_group, rec_flags, rec_index, rec_term, group_term,
                                    term_start, match, next, active, committed, stepdown_at,
                                    advanced_out, stats, workspace, workspace_bytes, stream);
}
