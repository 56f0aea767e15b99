// qb_bucket.h — device bucketing of record batches by group (shared by the
// bucketed tracker steps and the leader step): per-tile LDS counting sorts
// into reserved regions of super-buckets, then into chunks of CH groups
// (DESIGN.md §3.3, §3.3e).
#pragma once

#include "qb_common.h"
#include "qb_scan.h"

namespace qb {
namespace bk {

constexpr int kTile = 4096;          // records per scatter / split tile
constexpr int kChunksPerSb = 128;    // chunks per super-bucket (7 bits)
constexpr int kShards = 256;         // stat counter shards (one 64-byte line each)

// Bucketed record payload, structure of arrays, so every scatter store is
// one contiguous wave-wide write.  Two forms:
//
// Wide (the leader step): three columns — index (u64), term32 (u32, in a
//   u64 column's space) and mr = meta | ridx << 32 with
//   meta = lg (bits 0-9) | chunk-low (10-16) | record flags byte (17-24:
//          slot 17-20, kind 21-22, no-progress 23, reject 24),
//   ridx = batch index of the record (step-down ordering).
//   term32: the term as u32, or kTermEscape when it does not fit, in which
//   case the consumer reads the full term from the original batch by ridx.
//
// Compact (the tracker steps, Cols::compact): ONE u64 per record through
// both levels — what K5 needs and nothing else — plus a u8 chunk-low column
// between the levels (K4's sort key; K5 knows its chunk):
//   bits [0, lgb)            lg, the group within its chunk (lgb = log2 CH)
//   [lgb, lgb + slb)         slot (slb = 3 when the slot bound n <= 8, else 4)
//   bit lgb + slb            reject
//   [lgb + slb + 1, 24)      term (tb = 23 - lgb - slb bits: 10 or 11)
//   [24, 64)                 index (40 bits)
// The term field holds the term itself below tside() = 2^tb - 2 (1022 or
// 2046).  Round 6: a larger term below 2^32 - 1 with an
// index below 2^40 is a SIDE record — term field tside(), the index in the
// record, the term as a u32 in the side column at the record's position
// (Cols::side), carried through K4 beside the record — whenever its K3 tile
// has at least 1/8 of such records (kSideDen: a stream of realistic, long-
// lived terms); the side column then moves 4 bytes per record per level,
// in whole lines.  Anything else that does not fit (an index >= 2^40, a term
// >= 2^32 - 1, or a large term in a tile where they are rare) is an ESCAPE:
// term field tesc() = all ones, the index field the record's batch position,
// from which K5 reads the exact index and term in the original batch (two
// 8-byte gathers).  Raft indexes below 2^40 and terms below 1022 keep every
// record in 8 bytes; never a wrong answer.  (Round 5 wrote an escape-dense
// tile's exact (index, term) pairs to a 16-byte escape column at the buf1
// position, which K5 gathered across the region: a tick of terms >= 1023 cost
// 1.43x a small-term tick.  Round 2's packed form moved index + meta|term32,
// 16 bytes, four times per record: K3 write, K4 read + write, K5 read.)
struct Cols {
  u64* index;
  u64* term;
  u64* mr;
  u32* term32;
  u8* cl;        // compact: chunk-low of each record (K3 -> K4)
  u32 compact;
  u32* side;     // compact: the side column (a side record's u32 term at its position)
  u32* sflag;    // compact: the call's flag word, nonzero once a K3 tile wrote side records
};
constexpr u32 kTermEscape = 0xFFFFFFFFu;
// A K3 tile writes side records (and the side column for all its records)
// when more than 1/kSideDen of its records escape: then the escapes' gathers
// cost K5 more than the column costs K3-K5 (at 100 %: ~490 us vs ~50 us per
// 16M-record tick).
constexpr u32 kSideDen = 8;
// chunk_slow values: 1 = slow (k_bk_slow applies the chunk from the batch),
// 2 = deferred to the CSR step's second launch, 3 = a record of the chunk
// found no place (K3: the overflow pool was exhausted — never with the
// sizing below, kept as the exact fallback; K5 sends the chunk to the slow
// path).
constexpr u8 kChunkOverflow = 3;
__host__ __device__ __forceinline__ u32 term_to32(u64 t) {
  return t < u64(kTermEscape) ? u32(t) : kTermEscape;
}
constexpr u32 kIndexBits = 40;
constexpr u32 kRecHdrBits = 24;  // lg | slot | reject | term
// a side record's term and its index both fit the side form
__device__ __forceinline__ bool side_fits(u64 index, u64 term) {
  return (index >> kIndexBits) == 0 && term < u64(kTermEscape);
}
struct RecFmt {
  u32 lgb, slb, tb;
  __host__ __device__ u32 rej_shift() const { return lgb + slb; }
  __host__ __device__ u32 term_shift() const { return lgb + slb + 1; }
  __host__ __device__ u32 tesc() const { return (1u << tb) - 1u; }
  __host__ __device__ u32 tside() const { return (1u << tb) - 2u; }
  // (a large term is encoded as an escape here; K3 turns it into a side
  // record in a tile dense with them)
  __device__ __forceinline__ u64 encode(u32 lg, u32 slot, bool rej, u64 index, u64 term,
                                        u32 ridx) const {
    const bool esc = term >= u64(tside()) || (index >> kIndexBits) != 0;
    const u64 hdr = u64(lg) | (u64(slot) << lgb) | (u64(rej) << rej_shift()) |
                    (u64(esc ? tesc() : u32(term)) << term_shift());
    return hdr | ((esc ? u64(ridx) : index) << kRecHdrBits);
  }
  // K3 (round 6): a term past the field with an index and term that fit the
  // side form is encoded as a side record up front (term field tside(), the
  // index in the record); a tile that turns out not dense with them turns
  // them back into escapes (to_escape) — the raw columns die in the first pass
  __device__ __forceinline__ u64 encode_side(u32 lg, u32 slot, bool rej, u64 index, u64 term,
                                             u32 ridx) const {
    const bool iok = (index >> kIndexBits) == 0;
    const bool inl = iok && term < u64(tside());
    const bool sf = iok && !inl && term < u64(kTermEscape);
    const u32 tf = inl ? u32(term) : sf ? tside() : tesc();
    const u64 hdr = u64(lg) | (u64(slot) << lgb) | (u64(rej) << rej_shift()) | (u64(tf) << term_shift());
    return hdr | ((inl || sf ? index : u64(ridx)) << kRecHdrBits);
  }
  __device__ __forceinline__ u64 to_escape(u64 r, u32 ridx) const {
    return (r & ((1ull << term_shift()) - 1ull)) | (u64(tesc()) << term_shift()) |
           (u64(ridx) << kRecHdrBits);
  }
  __device__ __forceinline__ u32 lg(u64 r) const { return u32(r) & ((1u << lgb) - 1u); }
  __device__ __forceinline__ u32 slot(u64 r) const { return (u32(r) >> lgb) & ((1u << slb) - 1u); }
  __device__ __forceinline__ bool rej(u64 r) const { return (u32(r) >> rej_shift()) & 1u; }
  __device__ __forceinline__ u32 term(u64 r) const { return (u32(r) >> term_shift()) & tesc(); }
  __device__ __forceinline__ u64 payload(u64 r) const { return r >> kRecHdrBits; }
};

// Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8), each
// with its own L2.  xcd_major maps blockIdx to a logical tile so that tiles
// t, t+1, ... run on one XCD: the partial 128-byte lines that neighbouring
// tiles write into the same bucket (K3 runs, K1 histogram columns) meet in
// that XCD's L2 instead of reaching HBM as separate partial writes.  The grid
// must be a multiple of kXcds (Geometry::tile_grid); logical tiles >= the real count exit.
// Used only when a tile's mean run per super-bucket is shorter than two lines
// (kTile / NSB < 32 u64): config 5 (NSB = 256, 16-record runs) K3 241 -> 200
// us; the 4M-group leader step (NSB = 64, 64-record runs) measured its K3
// 41 -> 55 us with it, so it keeps the linear order.
constexpr u32 kXcds = 8;
// Overflow pool (round 5).  A region's records past its `cap` continue in
// kTile-record pool parts: part k of region r's overflow is pool part
// ptab[r * kmax + k] - 2 (0 = not drawn yet, 1 = being drawn), drawn from a
// pool counter by the first K3 workgroup that writes into it.  K4 sorts a
// pool part by chunk-low like a region part (its chunk-start row is
// region_rows() + the part's id), and the chunk's run table reads its pool
// rows after its region rows, in windows of 64 rows (RunTableT::pool_window).
// So a batch concentrated on a few super-buckets (10 % / 30 % of
// a 16M-record tick on one super-bucket took 2.6-2.9x a uniform tick through
// the slow path) is still sorted and applied through LDS; the round-4 slow
// path for capacity overflow and the leader's scanned overflow area (ADVICE
// r4: O(flagged chunks x overflow records)) are gone.
constexpr u32 kPartEmpty = 0, kPartBusy = 1, kPartBase = 2;
constexpr u32 kNoPart = 0xFFFFFFFFu;
struct Pool {
  u32* ptab;      // [NSB * 8 * kmax] (zeroed per call)
  u32* ctr;       // parts drawn (zeroed per call)
  u32* owner_r;   // [npool] region of each drawn part
  u32* owner_k;   // [npool] its index in the region's overflow
  u32 kmax, npool;
  u64 base;       // record index of pool part 0 (after the region grid)
  u32* sbflag;    // [NSB] 0, or 1 + the super-bucket's index in `heavy` (zeroed per call)
  u32* heavy;     // [NSB] super-buckets with a region past its cap, in K3's order
  u32* nheavy;    // their count (zeroed per call)
};
// K3: super-bucket sb's region just grew past its cap — list sb once as heavy
// (its chunks are applied first, by the heavy apply launch, which reads pool
// rows).
__device__ __forceinline__ void mark_heavy(const Pool& p, u32 sb) {
  if (atomicCAS(p.sbflag + sb, 0u, 0xFFFFFFFFu) == 0u) {
    const u32 i = atomicAdd(p.nheavy, 1u);
    p.heavy[i] = sb;
    __hip_atomic_store(p.sbflag + sb, i + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__host__ __device__ __forceinline__ u32 pool_parts_of(u32 fill, u32 cap) {
  return fill > cap ? (fill - cap + u32(kTile) - 1u) / u32(kTile) : 0u;
}
// Part k of region r's overflow (K3; every thread writing into it calls
// this): the part's id, or kNoPart when the pool or the region's table is
// exhausted (never with Geometry's sizing; the caller's records then take
// the exact slow path).  The first caller draws the id (CAS 0 -> 1, pool
// counter, publish id + 2); the others wait for the published id.  The
// wait always ends: the draw sits before the wait loop in straight-line
// code, so every wave publishes each part any of its lanes drew before any
// of its lanes starts waiting — a lane waits only on a part whose drawing
// lane has just its counter atomic and one store left, and is not itself
// waiting (two lanes of one wave never share a region: K3 gives each lane
// its own super-bucket).
__device__ __forceinline__ u32 pool_acquire(const Pool& p, u32 r, u32 k) {
  const bool in = k < p.kmax;
  u32* e = p.ptab + u64(r) * p.kmax + (in ? k : 0u);
  u32 v = in ? __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kNoPart;
  const bool won = v == kPartEmpty && atomicCAS(e, kPartEmpty, kPartBusy) == kPartEmpty;
  if (won) {
    const u32 id = atomicAdd(p.ctr, 1u);
    if (id < p.npool) {
      p.owner_r[id] = r;
      p.owner_k[id] = k;
    }
    v = id < p.npool ? id + kPartBase : kNoPart;
    __hip_atomic_store(e, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  while (v < kPartBase) {  // (a winner's v is already >= kPartBase)
    __builtin_amdgcn_s_sleep(2);
    v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return v == kNoPart ? kNoPart : v - kPartBase;
}

// Reserved regions per super-bucket (K3, both record forms): the workgroup
// on XCD x (blockIdx % 8) draws its runs from region x of each super-bucket,
// so a region is written by one XCD only and the partial lines at its runs'
// ends merge in that XCD's L2, and a fill counter takes 1/8 of the atomics.
// Measured (profiles/r04/tracker/ab_region_shards.log): 8 regions 534-548
// us per 16M-group tick, 4 / 2 / 1 regions (written by several XCDs)
// 569-606 us, round 3's scanned offsets 573-576 us.
constexpr u32 kRegionShards = kXcds;
// Rows of a chunk's run table (RunTable): kRegionShards regions x up to 32
// parts of kTile per super-bucket, so a region holds up to 131072 records
// (batches of up to ~8 records per group per call before the reserved
// regions overflow; round 4 started with 64 rows, i.e. ~2 per group).
constexpr u32 kMaxRows = 256;
// Parts of a region (K4): kTile records each, the last one up to kTile +
// slack so a region just past a multiple of kTile does not leave a part of a
// few records (each such part adds a run of ~1 record to every chunk's table:
// a line fetched per column for one record).  The wide form (the leader's
// K4, a 1024 x 5-record tile) takes kWideSlack; the compact form none.
constexpr u32 kWideSlack = 1024;
__host__ __device__ __forceinline__ u32 region_parts(u32 fill, u32 slack) {
  return fill <= u32(kTile) + slack ? (fill ? 1u : 0u) : (fill - slack + u32(kTile) - 1u) / u32(kTile);
}
// interleaved super-buckets (Geometry::il) for the tracker steps
constexpr bool kSbIl = true;
// K5 write-back (k_bk_apply, k_csr_apply): a wave whose 64-element segment
// of a slot row (or of committed / active) changed anywhere stores the whole
// segment, unchanged values rewritten, so every written line is whole —
// faster than storing only the changed lanes although more bytes are
// written (round 2: -20 us per 16M-group tick; round 3, CSR: -12 us).
// Narrower granules (32 / 64 bytes) measured +25 us (profiles/r03/k5_variants/).
__device__ __forceinline__ bool segment_any(bool p) { return __ballot(p) != 0; }
// Records a K5 workgroup has in flight per pass (both tracker steps);
// doubling it measured slower (profiles/r03/compact/).
constexpr u32 kK5Inflight = 1024;
__device__ __forceinline__ u32 xcd_major() {
  return (blockIdx.x % kXcds) * (gridDim.x / kXcds) + blockIdx.x / kXcds;
}

// Groups per K5 chunk (one workgroup; its LDS holds n accumulators per group).
__host__ __device__ constexpr u32 chunk_groups(u32 n) { return n <= 8 ? 512u : 256u; }
// CSR chunks: the LDS run buffer holds CH * WMAX slots.
__host__ __device__ constexpr u32 csr_chunk_groups(u32 /*wmax*/) { return 512u; }

struct Geometry {
  u64 G, M;
  u32 n, CH, NC, NSB, NT;
  u32 xcd;  // tiles of K1/K3 mapped XCD-major (see xcd_major)
  // CH and CH * kChunksPerSb are powers of two: group -> chunk / super-bucket
  // by shifts (a runtime u32 division is ~30 VALU instructions per record)
  u32 ch_shift, sb_shift;
  // il (interleaved super-buckets): super-bucket = the chunks of one XCD
  // within a window of 1024 consecutive chunks, i.e. chunk c is (c & 7) |
  // (c >> 10) << 3, chunk-low (c >> 3) & 127.  K5 dispatches chunk c as
  // workgroup c, round-robin over the XCDs, so a super-bucket's 128 chunks
  // run together on one XCD while K5 still walks the state in memory order.
  u32 il;
  RecFmt fmt;  // compact record layout (lg / slot / term bit widths)
  // Reserved regions: super-bucket sb's records from the tiles of shard x
  // (blockIdx % kRegionShards) go to region sb * kRegionShards + x of cap
  // records, cut into ppx parts of kTile.
  u32 cap, ppx;
  // Overflow pool: kmax parts per region at most (a region receives at most
  // its XCD slot's tiles' records), npool parts in all (enough for any
  // distribution of the batch: see geometry()).
  u32 kmax, npool;
  __host__ __device__ u64 region_rows() const { return u64(NSB) * kRegionShards * ppx; }
  __host__ __device__ u32 chunk_of(u32 g) const { return g >> ch_shift; }
  __host__ __device__ u32 sb_of_chunk(u32 c) const {
    return il ? (c & (kXcds - 1u)) | ((c >> 10) << 3) : c >> 7;
  }
  __host__ __device__ u32 cl_of_chunk(u32 c) const { return il ? (c >> 3) & 127u : c & 127u; }
  // the chunk of super-bucket sb with chunk-low cl (inverse of the two above)
  __host__ __device__ u32 chunk_of_sb_cl(u32 sb, u32 cl) const {
    return il ? (sb & (kXcds - 1u)) | (cl << 3) | ((sb >> 3) << 10) : sb * kChunksPerSb + cl;
  }
  __host__ __device__ u32 sb_of(u32 g) const { return il ? sb_of_chunk(g >> ch_shift) : g >> sb_shift; }
  __host__ __device__ u64 nbins() const { return u64(NSB) * NT; }
  u32 tile_grid() const { return xcd ? (NT + kXcds - 1) / kXcds * kXcds : NT; }
  __device__ __forceinline__ u32 tile() const { return xcd ? xcd_major() : blockIdx.x; }
};

inline Geometry geometry(u32 n, u64 G, u64 M, u32 ch = 0, bool il = false) {
  Geometry g{};
  g.il = il;
  g.G = G;
  g.M = M;
  g.n = n;
  g.CH = ch ? ch : chunk_groups(n);
  g.ch_shift = 0;
  while ((1u << g.ch_shift) < g.CH) ++g.ch_shift;
  g.sb_shift = g.ch_shift + 7;
  static_assert(kChunksPerSb == 128, "sb_shift = ch_shift + log2(kChunksPerSb)");
  g.NC = u32((G + g.CH - 1) / g.CH);
  g.NSB = il ? (g.NC + 1023u) / 1024u * kXcds : (g.NC + kChunksPerSb - 1) / kChunksPerSb;
  static_assert(kChunksPerSb * 8 == 1024, "il: 8 XCDs x 128 chunks per window");
  g.NT = u32((M + kTile - 1) / kTile);
  g.xcd = g.NSB > 0 && u32(kTile) / g.NSB < 32u;
  g.fmt.lgb = g.ch_shift;
  g.fmt.slb = n <= 8 ? 3u : 4u;
  g.fmt.tb = kRecHdrBits - 1u - g.fmt.lgb - g.fmt.slb;
  // reserved regions: twice a region's mean share plus 256 records, capped
  // by what the region's tiles can hold at most (a small batch never
  // overflows) and by the run table's kMaxRows rows per super-bucket
  const u64 S = kRegionShards;
  // a region's mean share for records spread evenly over the groups: the
  // fullest super-bucket holds mc of the NC chunks (interleaved: a window's
  // chunks of one XCD, up to 128), and the region gets the records of its
  // XCD slot's tiles, at most tps of the NT (tps = NT / S once NT >= S; a
  // batch of fewer tiles puts a whole tile's share in one region)
  const u64 mc = il ? (g.NC >= 1024 ? 128u : (g.NC + kXcds - 1) / kXcds)
                    : (g.NC < kChunksPerSb ? g.NC : kChunksPerSb);
  const u64 tps = (g.tile_grid() + S - 1) / S;
  const u64 den = u64(g.NC) * (g.NT ? g.NT : 1);
  const u64 m = g.NC ? (M * mc * tps + den - 1) / den : 0;
  // at most what the region's tiles can hold (and never more than the batch)
  u64 worst = tps * kTile;
  worst = worst < M ? worst : M;
  u64 cap = (2 * m + 256 + 255) / 256 * 256;  // (256-record granules)
  cap = cap < worst ? cap : (worst + 255) / 256 * 256;
  const u64 capmax = kMaxRows / S * kTile;  // the run table's rows per super-bucket
  cap = cap < 256 ? 256 : cap > capmax ? capmax : cap;
  g.cap = u32(cap);
  g.ppx = u32((cap + kTile - 1) / kTile);
  // pool: a region's overflow needs at most ceil((tps * kTile - cap) / kTile)
  // parts; all regions together at most sum(ceil(ovf_r / kTile)) <=
  // M / kTile + (overflowing regions), and a region overflows only past cap
  // records, so there are at most min(regions, M / cap) of them
  g.kmax = u32(tps + 1);
  const u64 regions = u64(g.NSB) * S;
  const u64 novf = (M + cap - 1) / cap;
  g.npool = M ? u32((M + kTile - 1) / kTile + (novf < regions ? novf : regions) + 1) : 0u;
  return g;
}

// Workspace carve (all offsets 256-byte aligned).  [shards, zero_end) is
// zeroed by one memset per call (bucket_records).
struct Carve {
  size_t shards, flags, counts, chunk_flags, ptab, sbflag, ext, user, zero_end, owner, heavy,
      side_idx, side_tc, chunk_start, buf1, buf2, cl, side1, side2, total;
  u64 nside;   // dedup side-table entries (compact form: kDedupSlots per chunk-start row)
  u64 nrec;    // records of the region grid (pool part 0 starts here)
  u64 nrec_all;  // records per column of buf1 / buf2: the region grid + the pool
};
inline size_t up256(size_t x) { return (x + 255) & ~size_t(255); }
// ncols = 3: the wide form (index, term32, mr; the leader step); ncols = 1:
// the compact form, whose u8 chunk-low column rides in the carve's cl area
// (the tracker steps).  user: bytes of the caller's own (at `user`) zeroed
// with the rest by bucket_records' memset.  Both forms' columns hold the
// region grid followed by the overflow pool (Pool).
constexpr u32 kFlagPoolCtr = 2;  // flag word: pool parts drawn
constexpr u32 kFlagHeavyCtr = 3;  // flag word: super-buckets whose regions overflowed
constexpr u32 kFlagSide = 4;      // flag word: a K3 tile wrote side records (Cols::sflag)
// K4 dedup (compact form, round 5): a chunk's run of at least kHeavyRun
// records in one part (a hot group: an even batch puts ~32 records of a chunk
// in a part; a batch capped at raft's 4 x 512 in-flight acks per group per
// tick stays below it — folding there cost K4 ~24 us for no K5 gain, so the
// threshold is 2048, not round 5's first 512) has its records with equal
// lg | slot | reject | term folded into
// one — the largest index and the count — through an LDS table of
// kDedupSlots entries.  A folded record is a compact escape whose payload
// holds kDedupFlag | its side-table entry (row * kDedupSlots + table slot):
// side_idx = the largest index, side_tc = term | count << kDedupCountShift.
// K5 applies it as `count` records of that class (MaybeUpdate is a max, the
// RecentActive bit an or; batch order only matters in a chunk with a
// higher-term record, which still goes to the slow path, which re-reads the
// original batch).  Escape payloads (batch positions) stay below 2^32.
// Side records fold too (round 6): K4 reads the side term and the group term
// and folds a side record equal to its group's term under term code
// kTermIsGroup (K5 reads the group term back for it), a stale one as term 0
// (stale against any group term it is below); a higher one is not folded.
constexpr u32 kHeavyRun = 2048;
constexpr u32 kDedupSlots = 256;
constexpr u64 kDedupFlag = 1ull << 39;
constexpr u32 kDedupCountShift = 12;
constexpr u32 kTermIsGroup = (1u << kDedupCountShift) - 1u;  // side_tc term code
constexpr u32 kExtClasses = 4;  // stale, applied, rejected, non-member
inline Carve carve(const Geometry& g, int ncols = 3, size_t user = 0) {
  Carve c{};
  size_t o = 0;
  c.shards = o;  o += up256(sizeof(u64) * QB_STAT_COUNT * kShards);
  c.flags = o;  o += 256;  // u32 words: any_slow (0), pool counter (2), slow-path barrier (16..)
  c.counts = o;  o += up256(sizeof(u32) * u64(g.NSB) * kRegionShards);  // region fills
  c.chunk_flags = o;  o += up256(u64(g.NC) + 1);  // u8 per chunk (chunk_slow)
  c.ptab = o;  o += up256(sizeof(u32) * u64(g.NSB) * kRegionShards * g.kmax);  // pool part table
  // per super-bucket: 0, or 1 + its index in the heavy list (a region of it
  // overflowed into the pool; K3)
  c.sbflag = o;  o += up256(sizeof(u32) * (u64(g.NSB) + 1));
  // per chunk: the records K4's dedup folded away, by class (stale, applied,
  // rejected, non-member) — added to the stats by K5 unless the chunk is slow
  c.ext = o;  o += ncols == 1 ? up256(sizeof(u32) * kExtClasses * (u64(g.NC) + 1)) : 0;
  c.user = o;  o += up256(user);
  c.zero_end = o;
  c.owner = o;  o += 2 * up256(sizeof(u32) * (u64(g.npool) + 1));
  c.heavy = o;  o += up256(sizeof(u32) * (u64(g.NSB) + 1));  // the heavy super-buckets (K3)
  // one row per part of the region grid (NSB x 8 x ppx), then one per pool part
  const u64 nrows = g.region_rows() + g.npool;
  c.nside = ncols == 1 ? nrows * kDedupSlots : 0;
  c.side_idx = o;  o += up256(sizeof(u64) * (c.nside ? c.nside : 1));
  c.side_tc = o;  o += up256(sizeof(u32) * (c.nside ? c.nside : 1));
  c.chunk_start = o;  o += up256(sizeof(u32) * nrows * (kChunksPerSb + 1));
  // (columns of at least one record: K5's branch-free loads read record 0 of
  // an empty chunk)
  c.nrec = u64(g.NSB) * kRegionShards * g.cap;
  c.nrec_all = c.nrec + u64(g.npool) * kTile;
  const u64 nrec = c.nrec_all ? c.nrec_all : 1;
  c.buf1 = o;  o += ncols * up256(sizeof(u64) * nrec);
  c.buf2 = o;  o += ncols * up256(sizeof(u64) * nrec);
  c.cl = o;  o += ncols == 1 ? up256(nrec) : 0;
  // compact form: the side columns beside buf1 (K3 -> K4) and buf2 (K4 -> K5)
  c.side1 = o;  o += ncols == 1 ? up256(sizeof(u32) * nrec) : 0;
  c.side2 = o;  o += ncols == 1 ? up256(sizeof(u32) * nrec) : 0;
  c.total = o;
  return c;
}
inline Pool pool_at(char* ws, const Carve& c, const Geometry& g) {
  Pool p{};
  p.ptab = reinterpret_cast<u32*>(ws + c.ptab);
  p.ctr = reinterpret_cast<u32*>(ws + c.flags) + kFlagPoolCtr;
  p.owner_r = reinterpret_cast<u32*>(ws + c.owner);
  p.owner_k = reinterpret_cast<u32*>(ws + c.owner + up256(sizeof(u32) * (u64(g.npool) + 1)));
  p.kmax = g.kmax;
  p.npool = g.npool;
  p.base = c.nrec;
  p.sbflag = reinterpret_cast<u32*>(ws + c.sbflag);
  p.heavy = reinterpret_cast<u32*>(ws + c.heavy);
  p.nheavy = reinterpret_cast<u32*>(ws + c.flags) + kFlagHeavyCtr;
  return p;
}
// The K4 dedup side table (compact form) and what K4 needs to class the
// records it folds away (the slow path, which re-reads the batch, ignores
// ext for its chunks).
struct Side {
  u64* idx;
  u32* tc;
  u32* ext;                // [NC][kExtClasses] (zeroed per call)
  const u64* group_term;   // the caller's, for the class of a folded record
  const u32* off;          // CSR: slot offsets (a slot past the group's count has
                           // no Progress); null for the FIXED layout
};
inline Side side_at(char* ws, const Carve& c, const u64* group_term = nullptr,
                    const u32* off = nullptr) {
  return Side{reinterpret_cast<u64*>(ws + c.side_idx), reinterpret_cast<u32*>(ws + c.side_tc),
              reinterpret_cast<u32*>(ws + c.ext), group_term, off};
}

inline Cols cols_at(char* base, u64 M, int ncols = 3) {
  const size_t col = up256(sizeof(u64) * (M ? M : 1));
  if (ncols == 1)
    return Cols{nullptr, nullptr, reinterpret_cast<u64*>(base), nullptr, nullptr, 0, nullptr, nullptr};
  return Cols{reinterpret_cast<u64*>(base), reinterpret_cast<u64*>(base + col),
              reinterpret_cast<u64*>(base + 2 * col), nullptr, nullptr, 0, nullptr, nullptr};
}
// The compact form's columns: the u64 records at `base`, the chunk-low bytes
// at `cl` (K3's output only), the side column at `side` and the flag word.
inline Cols compact_at(char* base, char* cl, char* side, u32* sflag) {
  return Cols{nullptr, nullptr, reinterpret_cast<u64*>(base), nullptr, reinterpret_cast<u8*>(cl),
              1, reinterpret_cast<u32*>(side), sflag};
}
inline u32* side_flag_at(char* ws, const Carve& c) {
  return reinterpret_cast<u32*>(ws + c.flags) + kFlagSide;
}


// Run table of one chunk: the chunk's run in each of up to kRuns parts of
// its super-bucket's regions, with an inclusive prefix of run lengths so
// flattened record f maps to a buffer index by binary search.
// Lane r's row of a run table (RunTableT::issue_regions).
struct RunRegs {
  u32 l, len, n, slack;
  u32 fill8;  // lanes 0..7: region x = lane's fill (the pool rows' count)
};
// R rows of LDS (kMaxRows for the MANY instantiations, 64 otherwise: the
// common kernels keep their LDS and so their occupancy).
template <u32 R>
struct RunTableT {
  static constexpr u32 kRuns = R;
  u32 lo[kRuns];
  u32 pre[kRuns + 1];
  u32 nr;
  u32 npool;     // the chunk's pool rows (finish); windows of 64 (pool_window)
  u32 ppre[kRegionShards + 1];  // pool rows of regions 0..x-1
  // issue_regions() loads lane r's run (every wave, branch-free: a row past
  // the table reads row 0 and counts nothing); finish() scans the lengths and
  // wave 0 publishes the table.  The caller synchronises before locate().
  // (Two halves, so a caller can keep the table's loads in flight ahead of
  // its own bulk loads: vector loads retire in order.)
  using Regs = RunRegs;
  // A chunk's runs: super-bucket sb's parts are rows sb * S * ppx + rr of the
  // region grid (S = kRegionShards), rr = x * ppx + j; part j of region x
  // exists iff j * kTile < its fill (counts, clamped to cap).
  __device__ __forceinline__ static void row_run(const u32* __restrict__ cs,
                                                 const u32* __restrict__ counts, u32 sb, u32 ppx,
                                                 u32 cap, u32 cl, u32 n, u32 rr_in, u32& l,
                                                 u32& len, u32 slack) {
    const bool in = rr_in < n;
    const u32 rr = in ? rr_in : 0u;
    const u32 x = rr / ppx, j = rr - x * ppx;
    const u64 row = (u64(sb) * n + rr) * (kChunksPerSb + 1);
    l = cs[row + cl];
    const u32 h = cs[row + cl + 1];
    u32 fill = counts[sb * kRegionShards + x];
    fill = fill < cap ? fill : cap;
    len = in && j < region_parts(fill, slack) ? h - l : 0u;
  }
  // Lane r loads row r and its region's count in one round trip (slack: the
  // form's last-part slack, region_parts).
  __device__ __forceinline__ static Regs issue_regions(const u32* __restrict__ cs,
                                                       const u32* __restrict__ counts, u32 sb,
                                                       u32 ppx, u32 cap, u32 cl, u32 slack = 0) {
    const u32 n = kRegionShards * ppx;
    Regs q;
    q.n = n;
    q.slack = slack;
    row_run(cs, counts, sb, ppx, cap, cl, n, threadIdx.x & 63u, q.l, q.len, slack);
    q.fill8 = counts[sb * kRegionShards + (threadIdx.x & (kRegionShards - 1u))];
    return q;
  }
  // Only the non-empty runs enter the table (a region's part past its fill
  // or without this chunk's records counts nothing), so the binary searches
  // of locate() go over fewer rows.  Returns the chunk's record count (every
  // lane).  MANY = false: up to 64 rows (8 parts per region), one pass from
  // the registers issue_regions() filled.  MANY = true (a batch of several
  // records per group: more than 8 parts per region, many_rows()): 64 rows
  // per pass, the rows past the first 64 loaded here.  The kernels are
  // instantiated for both, so the common one keeps its registers.
  __host__ __device__ static constexpr bool many_rows(u32 ppx) { return kRegionShards * ppx > 64; }
  template <bool MANY>
  __device__ __forceinline__ u32 finish(const Regs& q, const u32* __restrict__ cs,
                                        const u32* __restrict__ counts, u32 sb, u32 ppx, u32 cap,
                                        u32 cl) {
    const u32 r = threadIdx.x & 63u;
    u32 carry = 0, kb = 0;
    for (u32 p0 = 0; p0 < (MANY ? q.n : 1u); p0 += 64) {
      u32 l = q.l, len = q.len;
      if (MANY && p0) row_run(cs, counts, sb, ppx, cap, cl, q.n, p0 + r, l, len, q.slack);
      u32 x = len;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const u32 y = u32(__shfl_up(int(x), o, 64));
        if (r >= u32(o)) x += y;
      }
      const u64 ne = __ballot(len != 0);
      const u32 k = kb + u32(__popcll(ne & ((1ull << r) - 1ull)));
      if (threadIdx.x < 64 && ((ne >> r) & 1ull)) {
        lo[k] = l;
        pre[k + 1] = carry + x;
      }
      carry += u32(__shfl(int(x), 63, 64));
      kb += u32(__popcll(ne));
    }
    // the pool rows (round 5): region x's overflow parts, prefix over x
    {
      const u32 pp = r < kRegionShards ? pool_parts_of(q.fill8, cap) : 0u;
      u32 x = pp;
#pragma unroll
      for (int o = 1; o < int(kRegionShards); o <<= 1) {
        const u32 y = u32(__shfl_up(int(x), o, 64));
        if (r >= u32(o)) x += y;
      }
      if (threadIdx.x < kRegionShards) ppre[r + 1] = x;
      if (threadIdx.x == 0) ppre[0] = 0;
      const u32 tp = u32(__shfl(int(x), int(kRegionShards) - 1, 64));
      if (threadIdx.x == 0) npool = tp;
    }
    if (threadIdx.x == 0) {
      pre[0] = 0;
      nr = kb;
    }
    return carry;
  }
  // Window w of the chunk's pool rows (rows [64 w, 64 w + 64) of npool,
  // region-major): the table is rebuilt from them; returns their records
  // (wave 0's lanes; the others read pre[nr] after the caller's barrier).
  // Called by wave 0 after a barrier that published finish()'s npool /
  // ppre and retired every reader of the previous table.
  __device__ __forceinline__ u32 pool_window(u32 w, const u32* __restrict__ cs,
                                             const u32* __restrict__ ptab, u32 kmax,
                                             u64 region_rows, u32 sb, u32 cl) {
    const u32 r = threadIdx.x & 63u;
    const u32 rho = w * 64u + r;
    u32 l = 0, len = 0;
    if (rho < npool) {
      u32 x = 0;
#pragma unroll
      for (u32 i = 1; i < kRegionShards; ++i) x = ppre[i] <= rho ? i : x;
      const u32 e = ptab[u64(sb * kRegionShards + x) * kmax + (rho - ppre[x])];
      if (e != kNoPart && e >= kPartBase) {
        const u64 row = (region_rows + (e - kPartBase)) * (kChunksPerSb + 1) + cl;
        l = cs[row];
        len = cs[row + 1] - l;
      }
    }
    u32 x = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = u32(__shfl_up(int(x), o, 64));
      if (r >= u32(o)) x += y;
    }
    const u64 ne = __ballot(len != 0);
    const u32 k = u32(__popcll(ne & ((1ull << r) - 1ull)));
    if (threadIdx.x < 64 && ((ne >> r) & 1ull)) {
      lo[k] = l;
      pre[k + 1] = x;
    }
    if (threadIdx.x == 0) {
      pre[0] = 0;
      nr = u32(__popcll(ne));
    }
    return u32(__shfl(int(x), 63, 64));
  }
  __device__ __forceinline__ u32 locate(u32 f) const {
    u32 a = 0, b = nr;  // pre[a] <= f < pre[b]
    while (b - a > 1) {
      const u32 m = (a + b) >> 1;
      if (pre[m] <= f) a = m;
      else b = m;
    }
    return lo[a] + (f - pre[a]);
  }
  // locate() unrolled for a caller in straight-line code (no loop: exact
  // wait counts) for tables of at most 64 runs; MANY takes the loop.
  template <bool MANY>
  __device__ __forceinline__ u32 locate_fixed(u32 f) const {
    if constexpr (MANY) return locate(f);
    const u32 n = nr;
    u32 a = 0;
#pragma unroll
    for (u32 st = 32; st >= 1; st >>= 1) {
      const u32 m = a + st;
      const u32 pm = pre[m < n ? m : 0u];
      a = m < n && pm <= f ? m : a;
    }
    return lo[a] + (f - pre[a]);
  }
};
using RunTable = RunTableT<kMaxRows>;
template <bool MANY>
using RunTableOf = RunTableT<MANY ? kMaxRows : 64u>;

// K3-K4 of the bucketed pipeline: records (any order) -> buf2 holds each
// chunk's records as one run per part of its super-bucket's reserved regions;
// counts (region fills) and cs (chunk run starts per part) describe them
// (RunTable::issue_regions reads them).  One memset zeroes [cv.shards,
// cv.zero_end) first: stat shards, flag words, region fills, chunk flags and
// the pool part table.  Records with group >= G are dropped and counted into
// shards[QB_STAT_BAD_GROUP], and with n < 16 those with slot >= n into
// shards[QB_STAT_NON_MEMBER].  compact (carve with ncols = 1): the 8-byte
// compact record (RecFmt) through both levels, chunk-low in the carve's cl
// bytes between them.  Otherwise (carve with ncols = 3) the wide columns
// (index, term32, mr).  Records past a region's cap continue in its pool
// parts (Pool), sorted by K4 like region parts: cs row region_rows() + id.
int bucket_records(const Geometry& geo, const Carve& cv, char* ws, const u32* rec_group,
                   const u8* rec_flags, const u64* rec_index, const u64* rec_term, u64* shards,
                   hipStream_t st, bool compact, const u64* group_term = nullptr,
                   const u32* csr_off = nullptr);


}  // namespace bk
}  // namespace qb
