// qb_leader.hip — the leader inbox step over G raft groups (gfx950).
//
// A batch of responses (MsgAppResp, MsgHeartbeatResp, MsgSnapStatus,
// MsgUnreachable) is applied with the reference's sequential per-message
// semantics: every group's records in batch order, groups independent.
// Reference (paths relative to raft/):
//   raft.Step term filter                 raft.go:847-921
//   stepLeader                            raft.go:1099-1342
//   maybeSendAppend / bcastAppend         raft.go:423-492, 515-522
//   maybeCommit                           raft.go:585-588, log.go:328-334
//   raftLog.term / entries                log.go:268-299 (slice bounds 338-398)
//   findConflictByTerm                    log.go:150-171
//   Progress                              tracker/progress.go:85-212
//   Inflights                             tracker/inflights.go:55-132
//   readOnly.recvAck / advance            read_only.go:68-121
//   responseToReadIndexReq                raft.go:1737-1752
//
// Pipeline:
//   L1 bucket        bk::bucket_records (qb_bucket.h) sorts the records
//                    (wide columns) into chunks of 256 groups through LDS
//                    counting sorts into reserved regions (bad groups
//                    counted; a skewed batch's excess to the overflow area)
//   L2 k_ld_chunk_total  records per chunk, scanned within each block of
//                    256 chunks (+ the block's total); a chunk's base is that
//                    prefix plus the totals of the blocks before it (L3 adds
//                    them: no scan kernels)
//   L3 k_ld_chunk_runs  per chunk: LDS count per group, block scan (writes
//                    the per-group run starts), LDS-atomic scatter of the
//                    batch indexes into the groups' runs
//   (shards beyond the bucket geometry, > 134M groups, use per-record
//   global atomics instead: k_ld_count / scan / k_ld_scatter)
//   L4 k_ld_step     one thread per group: sort its run by batch index
//                    (records arrive in any order), then the sequential
//                    stepLeader over its Progress / log view / read queue;
//                    messages into an 8-slot per-group area of the workspace,
//                    spilling into 32-message chunks from a shared pool
//   L5 scan          exclusive scan of the message counts
//   L6 k_ld_emit     each group's messages copied to their final place
//                    (group order, emission order within a group)
// Only L4 is control-heavy; it touches a group's state only if the group has
// records.
#include <cstdlib>

#include "qb_bucket.h"
#include "qb_common.h"
#include "qb_scan.h"

namespace qb {
namespace ld {

constexpr u32 kFix = QB_LEADER_OUTBOX_SLOTS;    // messages per group kept in the fixed area
constexpr u32 kChunk = QB_LEADER_OUTBOX_CHUNK;  // messages per overflow chunk
constexpr u32 kEmitStage = 1024;  // messages per workgroup staged by k_ld_emit
constexpr u32 kNone = 0xFFFFFFFFu;
constexpr u8 kNoSlot = 0xFF;

struct Msg {
  u64 index, log_term, commit, aux;
  u32 group;
  u8 to, type;
  u16 reserved;
};
static_assert(sizeof(Msg) == sizeof(qb_msg_out), "qb_msg_out layout");
struct ReadSt {
  u64 index, ctx;
};
static_assert(sizeof(ReadSt) == sizeof(qb_read_state), "qb_read_state layout");

inline size_t up256(size_t x) { return (x + 255) & ~size_t(255); }

// The ABI's uint64_t is unsigned long; HIP atomics and qb helpers use u64.
__host__ __device__ __forceinline__ u64* U(uint64_t* p) { return reinterpret_cast<u64*>(p); }
__host__ __device__ __forceinline__ const u64* U(const uint64_t* p) {
  return reinterpret_cast<const u64*>(p);
}

constexpr u32 kCh = bk::chunk_groups(16);  // groups per bucket chunk (256)
static_assert(kCh == kBlock, "one thread per group of a chunk");

struct Carve {
  size_t cnt, bsum, cursor, perm, rflags, rterm, rindex, rhint, rlt, mcnt, mbs, mbsum, fix, chead,
      cnext, chunks, pool, shards;
  size_t bkt, ctot, cbsum, total;
  u64 nchunks;
  bool bucketed;
  bk::Geometry geo;
  bk::Carve bcv;
};
// outbox: the caller owns the message slots / chunks / counts
// (qb_dev_leader_step_outbox), so they are not carved.
inline Carve carve(u64 G, u64 M, bool outbox = false) {
  Carve c{};
  size_t o = 0;
  c.geo = bk::geometry(16, G, M);
  // the wide form's last part takes kWideSlack more records (bk::region_parts),
  // so a region has fewer parts: fewer run-table rows for every chunk
  const u32 wp = bk::region_parts(c.geo.cap, bk::kWideSlack);
  c.geo.ppx = wp ? wp : 1u;
  // the bucket pass addresses its region grid (NSB x 8 x cap records, about
  // 2x M) with u32 offsets: a geometry past that takes the atomic grouping
  c.bucketed = c.geo.NSB <= 4096 && bk::carve(c.geo, 3).nrec_all <= 0xFFFFFFFFull;
  const size_t pool_b = up256(sizeof(u32) * 2), shard_b = up256(sizeof(u64) * QB_LSTAT_COUNT * 64);
  if (c.bucketed) {
    // the message-chunk pool and the stat shards ride in the bucket carve's
    // user area: bucket_records' memset zeroes them (no memset of their own)
    c.bcv = bk::carve(c.geo, 3, pool_b + shard_b);
    c.bkt = o;   o += up256(c.bcv.total);
    c.pool = c.bkt + c.bcv.user;
    c.shards = c.pool + pool_b;
    c.ctot = o;  o += up256(sizeof(u32) * (u64(c.geo.NC) + 1));
    c.cbsum = o; o += up256(sizeof(u32) * ((u64(c.geo.NC) + kBlock - 1) / kBlock + 1));
  }
  c.cnt = o;    o += up256(sizeof(u32) * (G + 1));
  c.bsum = o;   o += up256(sizeof(u32) * (scan::blocks(G) + 1));
  c.cursor = o; o += up256(sizeof(u32) * (G + 1));
  c.perm = o;   o += up256(sizeof(u32) * (M + 1));
  c.rflags = o; o += up256(sizeof(u8) * (M + 1));
  c.rterm = o;  o += up256(sizeof(u64) * (M + 1));
  c.rindex = o; o += up256(sizeof(u64) * (M + 1));
  c.rhint = o;  o += up256(sizeof(u64) * (M + 1));
  c.rlt = o;    o += up256(sizeof(u64) * (M + 1));
  if (!outbox) {
    c.mcnt = o;   o += up256(sizeof(u32) * (G + 1));
    // per-workgroup message totals of k_ld_step (scanned), and their scan's
    // block sums
    c.mbs = o;    o += up256(sizeof(u32) * ((G + kBlock - 1) / kBlock + 1));
    c.mbsum = o;  o += up256(sizeof(u32) * (scan::blocks((G + kBlock - 1) / kBlock) + 1));
    c.fix = o;    o += up256(sizeof(Msg) * kFix * G);
    c.chead = o;  o += up256(sizeof(u32) * (G + 1));
    c.nchunks = M / 8 + 1024;  // 4 spilled messages per record on average
    c.cnext = o;  o += up256(sizeof(u32) * c.nchunks);
    c.chunks = o; o += up256(sizeof(Msg) * kChunk * c.nchunks);
  }
  if (!c.bucketed) {
    c.pool = o;   o += pool_b;
    c.shards = o; o += shard_b;
  }
  c.total = o;
  return c;
}

// The inbox's fields gathered into group order (position k of perm), so the
// step reads its records coalesced and one dependent hop earlier.
struct RecCols {
  u8* flags;
  u64* term;
  u64* index;
  u64* hint;      // reject records only
  u64* log_term;  // reject records only
};

struct Args {
  qb_leader_groups lg;
  qb_leader_inbox in;
  const u32* cnt;     // exclusive scan of per-group record counts, [G+1]
  u32* perm;          // batch indexes grouped by group (each run ascending)
  RecCols rec;        // the records in perm order
  u32* mcnt;          // messages per group (outbox); in-workgroup prefix (ordered)
  u32* mbs;           // ordered form: each workgroup's message total (else null)
  Msg* fix;           // [kFix][G]: message k of every group contiguous
  u32* chead;         // first overflow chunk per group
  u32* cnext;         // chunk links
  Msg* chunks;        // [nchunks * kChunk]
  u32* pool;          // [0] = next free chunk
  u64 nchunks;
  u64* shards;        // [64][QB_LSTAT_COUNT]
  u32* stepdown_at;
  u8* gflags;
  ReadSt* rs;         // outbox read_states: [readq_cap][G] (null: ReadStates are messages)
  u32* rcnt;          // ReadStates per group
};

// ------------------------------------------------------------ L1 / L3 ----
__global__ __launch_bounds__(kBlock) void k_ld_count(u64 G, u64 M, const u32* __restrict__ rg,
                                                     u32* __restrict__ cnt, u64* __restrict__ shards) {
  __shared__ u32 lds[1];
  BlockTally<1> tally;
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i];
    const bool bad = g >= G;
    if (!bad) atomicAdd(cnt + g, 1u);
    tally.add(0, bad);
  }
  const int slot[1] = {QB_LSTAT_BAD_GROUP};
  tally.flush(lds, shards + u64(blockIdx.x % 64) * QB_LSTAT_COUNT, slot);
}

__global__ __launch_bounds__(kBlock) void k_ld_scatter(u64 G, u64 M, const u32* __restrict__ rg,
                                                       u32* __restrict__ cursor,
                                                       u32* __restrict__ perm) {
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i];
    if (g < G) perm[atomicAdd(cursor + g, 1u)] = u32(i);
  }
}

// Sort a group's run of batch indexes ascending (runs are short: insertion
// sort; long runs: heapsort, both in place).
__device__ void sort_run(u32* a, u32 n) {
  if (n <= 32) {
    for (u32 i = 1; i < n; ++i) {
      const u32 v = a[i];
      u32 j = i;
      while (j > 0 && a[j - 1] > v) {
        a[j] = a[j - 1];
        --j;
      }
      a[j] = v;
    }
    return;
  }
  auto sift = [&](u32 root, u32 end) {
    for (;;) {
      u32 c = 2 * root + 1;
      if (c >= end) return;
      if (c + 1 < end && a[c + 1] > a[c]) ++c;
      if (a[root] >= a[c]) return;
      const u32 t = a[root];
      a[root] = a[c];
      a[c] = t;
      root = c;
    }
  };
  for (u32 i = n / 2; i-- > 0;) sift(i, n);
  for (u32 e = n - 1; e > 0; --e) {
    const u32 t = a[0];
    a[0] = a[e];
    a[e] = t;
    sift(0, e);
  }
}

// A group's run [r0, r0 + n) of perm: batch order, then its record fields
// gathered to the same positions.
__device__ void gather_run(const qb_leader_inbox& in, u32* perm, u32 r0, u32 n,
                           const RecCols& rc) {
  if (n > 1) sort_run(perm + r0, n);
  for (u32 k = r0; k < r0 + n; ++k) {
    const u32 i = perm[k];
    const u8 f = in.flags[i];
    rc.flags[k] = f;
    rc.term[k] = in.term[i];
    rc.index[k] = in.index[i];
    if (f & QB_REC_REJECT) {
      rc.hint[k] = in.hint ? in.hint[i] : 0ull;
      rc.log_term[k] = in.log_term ? in.log_term[i] : 0ull;
    }
  }
}

// A run whose fields are already gathered, in arbitrary order: insertion
// sort by batch index moving every field (runs are short); long runs are
// sorted by index alone and gathered again.
__device__ void order_run(const qb_leader_inbox& in, u32* perm, u32 r0, u32 n,
                          const RecCols& rc) {
  if (n > 32) {
    gather_run(in, perm, r0, n, rc);
    return;
  }
  for (u32 a = r0 + 1; a < r0 + n; ++a) {
    const u32 v = perm[a];
    const u8 f = rc.flags[a];
    const u64 t = rc.term[a], x = rc.index[a];
    const bool rej = (f & QB_REC_REJECT) != 0;
    const u64 h = rej ? rc.hint[a] : 0ull, lt = rej ? rc.log_term[a] : 0ull;
    u32 j = a;
    while (j > r0 && perm[j - 1] > v) {
      perm[j] = perm[j - 1];
      const u8 fj = rc.flags[j - 1];
      rc.flags[j] = fj;
      rc.term[j] = rc.term[j - 1];
      rc.index[j] = rc.index[j - 1];
      if (fj & QB_REC_REJECT) {
        rc.hint[j] = rc.hint[j - 1];
        rc.log_term[j] = rc.log_term[j - 1];
      }
      --j;
    }
    perm[j] = v;
    rc.flags[j] = f;
    rc.term[j] = t;
    rc.index[j] = x;
    if (rej) {
      rc.hint[j] = h;
      rc.log_term[j] = lt;
    }
  }
}

// Fallback path (no bucket geometry): one thread per group.
__global__ __launch_bounds__(kBlock) void k_ld_gather(u64 G, qb_leader_inbox in,
                                                      const u32* __restrict__ cnt,
                                                      u32* __restrict__ perm, RecCols rc) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  const u32 r0 = cnt[g], r1 = cnt[g + 1];
  if (r1 > r0) gather_run(in, perm, r0, r1 - r0, rc);
}

// --------------------------------------------------------- L2 / L3 (bk) ----
// Records of chunk c: the sum of its runs over the parts of its super-bucket's
// regions (bk::region_parts with the wide form's slack) and over their
// overflow pool parts (a skewed batch).
__global__ __launch_bounds__(kBlock) void k_ld_chunk_total(bk::Geometry geo,
                                                           const u32* __restrict__ counts,
                                                           const u32* __restrict__ cs,
                                                           const u32* __restrict__ ptab,
                                                           u32* __restrict__ cloc,
                                                           u32* __restrict__ bsum) {
  __shared__ u32 wsum[kBlock / 64];
  const u32 c = blockIdx.x * kBlock + threadIdx.x;
  u32 s = 0;
  if (c < geo.NC) {
    const u32 sb = geo.sb_of_chunk(c), cl = geo.cl_of_chunk(c);
    const u32 nrow = bk::kRegionShards * geo.ppx;
    for (u32 x = 0; x < bk::kRegionShards; ++x) {
      const u32 fill_all = counts[sb * bk::kRegionShards + x];
      const u32 fill = fill_all < geo.cap ? fill_all : geo.cap;
      const u32 np = bk::region_parts(fill, bk::kWideSlack);
      for (u32 j = 0; j < geo.ppx && j < np; ++j) {
        const u64 row = (u64(sb) * nrow + x * geo.ppx + j) * (bk::kChunksPerSb + 1) + cl;
        s += cs[row + 1] - cs[row];
      }
      const u32 npp = bk::pool_parts_of(fill_all, geo.cap);
      for (u32 k = 0; k < npp; ++k) {
        const u32 e = ptab[u64(sb * bk::kRegionShards + x) * geo.kmax + k];
        if (e == bk::kNoPart || e < bk::kPartBase) continue;
        const u64 row = (geo.region_rows() + (e - bk::kPartBase)) * (bk::kChunksPerSb + 1) + cl;
        s += cs[row + 1] - cs[row];
      }
    }
  }
  // exclusive prefix within the block, and the block's total
  const u32 lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  u32 inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = u32(__shfl_up(int(inc), o, 64));
    if (lane >= u32(o)) inc += y;
  }
  if (lane == 63u) wsum[w] = inc;
  __syncthreads();
  u32 before = 0, total = 0;
#pragma unroll
  for (u32 q = 0; q < kBlock / 64; ++q) {
    total += wsum[q];
    if (q < w) before += wsum[q];
  }
  if (c < geo.NC) cloc[c] = before + inc - s;
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

constexpr u32 kStageRecs = 1024;  // chunk records placed through LDS
constexpr u32 kLdsSortMax = 64;   // longer runs are ordered in HBM
struct ChunkStage {
  u64 mr[kStageRecs];
  u64 term[kStageRecs];
  u64 index[kStageRecs];
};
__device__ __forceinline__ ChunkStage& chunk_stage() {
  __shared__ ChunkStage s;
  return s;
}

// One workgroup per chunk of kCh groups (one thread per group): count the
// chunk's records per group in LDS, scan the counts (cnt[g] = the group's
// run start, cnt[G] = all valid records), then place every record's batch
// index in its group's run with an LDS cursor.  Order inside a run is
// arbitrary; the step sorts each run.  The chunk's records are its runs in
// the parts of its super-bucket's regions (one run table) and, after a
// skewed batch, in their overflow pool parts (windows of 64 pool rows
// through the same table: bk::RunTableT::pool_window).
template <bool MANY>
__global__ __launch_bounds__(kBlock) void k_ld_chunk_runs(bk::Geometry geo, bk::Cols recs,
                                                          const u32* __restrict__ counts,
                                                          const u32* __restrict__ cs,
                                                          const u32* __restrict__ ptab,
                                                          const u32* __restrict__ cloc,
                                                          const u32* __restrict__ bsum,
                                                          u32* __restrict__ cnt,
                                                          u32* __restrict__ perm,
                                                          qb_leader_inbox in, RecCols rc) {
  __shared__ bk::RunTableOf<MANY> rt;
  __shared__ u32 cur[kCh];
  __shared__ u32 wsum[kBlock / 64];
  const u32 c = blockIdx.x, t = threadIdx.x;
  const u32 sb = geo.sb_of_chunk(c), cl = geo.cl_of_chunk(c);
  const u32 clo = cloc[c];  // the chunk's prefix within its block of kBlock chunks
  __shared__ u32 s_bpre;
  cur[t] = 0;
  bk::RunRegs rq{};
  if (t < 64) {  // wave 0: the run table, and the totals of the blocks before this chunk's
    rq = bk::RunTable::issue_regions(cs, counts, sb, geo.ppx, geo.cap, cl, bk::kWideSlack);
    const u32 nb = c / kBlock;
    u32 bp = 0;
    for (u32 i = t; i < nb; i += 64) bp += bsum[i];
    rt.template finish<MANY>(rq, cs, counts, sb, geo.ppx, geo.cap, cl);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bp += u32(__shfl_xor(int(bp), o, 64));
    if (t == 0) s_bpre = bp;
  }
  __syncthreads();  // the run table is published
  const u32 total1 = rt.pre[rt.nr];  // the region records (workgroup-uniform)
  const u32 npool = rt.npool;        // the chunk's pool rows (workgroup-uniform)
  // Common case (round 3, one pass): no pool rows and at most kStageRecs
  // records — each record is loaded once, into registers (kRegRecs per
  // thread), counted from there and placed from there; otherwise the
  // records are read twice (count, then place) by the loops below.
  constexpr u32 kRegRecs = kStageRecs / kBlock;
  u64 rv[kRegRecs], ri[kRegRecs];
  u32 rt32[kRegRecs];
  const bool onepass = npool == 0 && total1 <= kStageRecs;  // block-uniform
  // the chunk's records one at a time (region runs, then the pool rows'
  // windows, after which the region table is rebuilt for the next pass);
  // every thread calls it (barriers inside when there are pool rows)
  auto each = [&](auto&& fn) {
    for (u32 f = t; f < total1; f += kBlock) {
      const u32 b = rt.locate(f);
      fn(recs.mr[b], recs.term32[b], recs.index[b]);
    }
    if (npool == 0) return;
    for (u32 w = 0; w * 64u < npool; ++w) {
      __syncthreads();
      if (t < 64) rt.pool_window(w, cs, ptab, geo.kmax, geo.region_rows(), sb, cl);
      __syncthreads();
      const u32 tot = rt.pre[rt.nr];
      for (u32 f = t; f < tot; f += kBlock) {
        const u32 b = rt.locate(f);
        fn(recs.mr[b], recs.term32[b], recs.index[b]);
      }
    }
    __syncthreads();
    if (t < 64) rt.template finish<MANY>(rq, cs, counts, sb, geo.ppx, geo.cap, cl);
    __syncthreads();
  };
  // the full term (a kTermEscape term32 is read from the batch by ridx)
  auto full_term = [&](u64 v, u32 t32) -> u64 {
    return t32 != bk::kTermEscape ? u64(t32) : in.term[u32(v >> 32)];
  };
  ChunkStage& cs_ = chunk_stage();
  // Two passes over the chunk's records — count per group, then place — with
  // ONE inlined walk (`each`): three walks (count, LDS placement, HBM
  // placement) with the pool windows held 90 VGPRs against 68 before them.
  // Common case: the records are placed in LDS, each group's run is put in
  // batch order there (runs of <= kLdsSortMax), and the chunk is written
  // out with coalesced stores; a chunk of more than kStageRecs records is
  // placed in HBM directly.
  u32 x = 0, start = 0, base = 0, ntot = 0;
  bool staged = true;
#pragma clang loop unroll(disable)
  for (u32 pass = 0; pass < 2u; ++pass) {
    if (pass == 1u) {  // the counts' scan: each group's run start
      __syncthreads();
      x = cur[t];
      u32 inc = x;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const u32 y = u32(__shfl_up(int(inc), o, 64));
        if ((t & 63u) >= u32(o)) inc += y;
      }
      if ((t & 63u) == 63u) wsum[t >> 6] = inc;
      __syncthreads();
      ntot = 0;  // the chunk's records: its region runs plus its pool runs (workgroup-uniform)
#pragma unroll
      for (u32 w = 0; w < kBlock / 64; ++w) {
        if (w < (t >> 6)) inc += wsum[w];
        ntot += wsum[w];
      }
      base = s_bpre + clo;
      start = inc - x;
      const u64 g = u64(c) * kCh + t;
      if (g < geo.G) cnt[g] = base + start;
      if (c + 1 == geo.NC && t == 0) cnt[geo.G] = base + ntot;
      cur[t] = start;
      staged = ntot <= kStageRecs;
      __syncthreads();  // every group's cur[] start is written
    }
    if (onepass) {
      if (pass == 0u) {
        u32 b[kRegRecs];
#pragma unroll
        for (u32 r = 0; r < kRegRecs; ++r) {
          const u32 f = t + r * kBlock;
          b[r] = f < total1 ? rt.locate(f) : 0u;
        }
#pragma unroll
        for (u32 r = 0; r < kRegRecs; ++r) {
          if (t + r * kBlock < total1) {
            rv[r] = recs.mr[b[r]];
            rt32[r] = recs.term32[b[r]];
            ri[r] = recs.index[b[r]];
          }
        }
#pragma unroll
        for (u32 r = 0; r < kRegRecs; ++r)
          if (t + r * kBlock < total1) atomicAdd(&cur[u32(rv[r]) & 1023u], 1u);
      } else {  // (staged: total1 <= kStageRecs)
#pragma unroll
        for (u32 r = 0; r < kRegRecs; ++r) {
          if (t + r * kBlock < total1) {
            const u64 v = rv[r];
            const u32 e = atomicAdd(&cur[u32(v) & 1023u], 1u);
            cs_.mr[e] = v;
            cs_.term[e] = full_term(v, rt32[r]);
            cs_.index[e] = ri[r];
          }
        }
      }
    } else {
      each([&](u64 v, u32 t32, u64 index) {
        const u32 e = atomicAdd(&cur[u32(v) & 1023u], 1u);
        if (pass == 0u) return;  // (count)
        if (staged) {
          cs_.mr[e] = v;
          cs_.term[e] = full_term(v, t32);
          cs_.index[e] = index;
          return;
        }
        const u32 k = base + e, i = u32(v >> 32);
        const u8 fl = u8(u32(v) >> 17);  // the record's flags byte (qb_bucket.h)
        perm[k] = i;
        rc.flags[k] = fl;
        rc.term[k] = full_term(v, t32);
        rc.index[k] = index;
        if (fl & QB_REC_REJECT) {
          rc.hint[k] = in.hint ? in.hint[i] : 0ull;
          rc.log_term[k] = in.log_term ? in.log_term[i] : 0ull;
        }
      });
    }
  }
  __syncthreads();
  if (staged) {
    if (x > 1 && x <= kLdsSortMax) {
      for (u32 a = start + 1; a < start + x; ++a) {
        const u64 v = cs_.mr[a], tv = cs_.term[a], iv = cs_.index[a];
        u32 j = a;
        while (j > start && (cs_.mr[j - 1] >> 32) > (v >> 32)) {
          cs_.mr[j] = cs_.mr[j - 1];
          cs_.term[j] = cs_.term[j - 1];
          cs_.index[j] = cs_.index[j - 1];
          --j;
        }
        cs_.mr[j] = v;
        cs_.term[j] = tv;
        cs_.index[j] = iv;
      }
    }
    __syncthreads();
    for (u32 e = t; e < ntot; e += kBlock) {
      const u64 v = cs_.mr[e];
      const u32 k = base + e, i = u32(v >> 32);
      const u8 fl = u8(u32(v) >> 17);  // the record's flags byte (qb_bucket.h)
      perm[k] = i;
      rc.flags[k] = fl;
      rc.term[k] = cs_.term[e];
      rc.index[k] = cs_.index[e];
      if (fl & QB_REC_REJECT) {
        rc.hint[k] = in.hint ? in.hint[i] : 0ull;
        rc.log_term[k] = in.log_term ? in.log_term[i] : 0ull;
      }
    }
    __syncthreads();  // perm complete (workgroup-visible) for the long runs
    if (x > kLdsSortMax) gather_run(in, perm, base + start, x, rc);
    return;
  }
  // A group with several records: its run (placed in arbitrary order) is
  // put in batch order and its fields gathered again in that order.
  if (x > 1) order_run(in, perm, base + start, x, rc);
}

// ------------------------------------------------------------------ L4 ----
// Per-group view of the leader (one thread).
struct Group {
  u64 g;
  u32 s0, ns;           // first slot, number of slots
  u32 j0;               // first slot in the staged span
  u32 mask_in, mask_out;
  u32 meta;
  u64 term, committed;
  u64 first, last;      // the log view's first / last index (requested with the group's fields)
  u32 nruns;
  u32 nmsg, stored;     // messages generated / stored (the pool can run out)
  u32 chunk;            // current overflow chunk
  u32 nrs;              // ReadStates stored (the outbox's read_states)
  bool dropped;
};

__device__ __forceinline__ u32 leader_slot(const Group& G_) { return G_.meta & 0xFFu; }
// Read-only log-view fields are re-read where used (L1 hits) instead of being
// held in registers for the whole step: this kernel is latency-bound and its
// occupancy is set by its VGPR count.  First / last index are the exception
// (round 5): requested with the group's fields, before the slot stage's
// barrier, so the commit check's log_term and the first MsgApp do not wait
// on a round trip of their own (118 VGPRs: still 4 waves per SIMD).
#define LG_FIRST(A, G_) ((G_).first)
#define LG_LAST(A, G_) ((G_).last)
#define LG_SNAP_I(A, G_) U((A).lg.snap_index)[(G_).g]
#define LG_SNAP_T(A, G_) U((A).lg.snap_term)[(G_).g]
#define LG_MAX_ENTS(A, G_) U((A).lg.max_ents)[(G_).g]
__device__ __forceinline__ u32 transferee(const Group& G_) { return (G_.meta >> 8) & 0xFFu; }

// raftLog.term (log.go:268-288, zeroTermOnErrCompacted): 0 outside
// [firstIndex-1, lastIndex]; otherwise the term of the run holding i.
__device__ u64 log_term(const Args& A, const Group& G_, u64 i) {
  const u64 dummy = LG_FIRST(A, G_) - 1;
  if (i < dummy || i > LG_LAST(A, G_)) return 0;
  u64 t = 0;
  const u64* rs = U(A.lg.run_start) + G_.g;  // run r at rs[r * G] (run-major)
  const u64* rt = U(A.lg.run_term) + G_.g;
  const u64 G = A.lg.G;
  for (u32 r = 0; r < G_.nruns; ++r)
    if (rs[r * G] <= i) t = rt[r * G];
  return t;
}

// log.go:150-171, one run at a time instead of one index at a time: inside a
// run every index has the run's term, so when that term is above `term` the
// whole run (down to the dummy entry) is skipped.
__device__ u64 find_conflict_by_term(const Args& A, const Group& G_, u64 index, u64 term) {
  if (index > LG_LAST(A, G_)) return index;
  const u64 dummy = LG_FIRST(A, G_) - 1;
  const u64* rs = U(A.lg.run_start) + G_.g;  // run r at rs[r * G] (run-major)
  const u64* rt = U(A.lg.run_term) + G_.g;
  const u64 G = A.lg.G;
  for (;;) {
    if (index < dummy || index > LG_LAST(A, G_)) return index;  // term 0 <= term
    u64 t = 0, start = 0;
    for (u32 r = 0; r < G_.nruns; ++r)
      if (rs[r * G] <= index) {
        t = rt[r * G];
        start = rs[r * G];
      }
    if (t <= term) return index;
    const u64 lo = start > dummy ? start : dummy;
    index = lo - 1;  // wraps at 0 exactly like the reference's index--
  }
}

__device__ void emit(const Args& A, Group& G_, u8 type, u32 to, u64 index, u64 log_term_,
                     u64 commit, u64 aux) {
  Msg m;
  m.index = index;
  m.log_term = log_term_;
  m.commit = commit;
  m.aux = aux;
  m.group = u32(G_.g);
  m.to = u8(to);
  m.type = type;
  m.reserved = 0;
  const u32 k = G_.nmsg++;
  if (G_.dropped) return;
  if (k < kFix) {
    A.fix[u64(k) * A.lg.G + G_.g] = m;
    G_.stored = k + 1;
    return;
  }
  const u32 kk = k - kFix;
  if (kk % kChunk == 0) {  // needs a new chunk
    const u32 c = atomicAdd(A.pool, 1u);
    if (c >= A.nchunks) {
      G_.dropped = true;
      return;
    }
    if (kk == 0) A.chead[G_.g] = c;
    else A.cnext[G_.chunk] = c;
    G_.chunk = c;
  }
  A.chunks[u64(G_.chunk) * kChunk + kk % kChunk] = m;
  G_.stored = k + 1;
}

// Progress accessors (slot j of the group).
// A slot's Progress: the kernel arguments (uniform, scalar registers) and the
// slot's index; addresses are formed at each use, so a live Pr costs a few
// vector registers instead of seven 64-bit pointers.  With S, match / next /
// inflight position / state byte live in the workgroup's LDS copy of its
// slot span (k_ld_step stages it with coalesced loads and writes it back);
// the inflight ring and pendingSnapshot stay in HBM.
constexpr u32 kSpanCap = 1536;  // staged slots per workgroup (6 per group)
struct SlotStage {
  u64 match[kSpanCap];
  u64 next[kSpanCap];
  u32 ipos[kSpanCap];
  u8 st[kSpanCap];
  u8 dirty[kSpanCap];  // fields of the slot whose value changed: written back
};
// dirty bits per staged field
constexpr u8 kDirtyMatch = 1, kDirtyNext = 2, kDirtyIpos = 4, kDirtySt = 8;

// A staged field: reads convert to the value; an assignment that changes it
// marks the field dirty, so the write-back stores only changed fields (a
// heartbeat response that leaves RecentActive set stores nothing; round 2
// wrote all four arrays of every slot the step touched).
template <class T, u8 BIT>
struct StagedRef {
  T& v;
  u8& d;
  __device__ __forceinline__ operator T() const { return v; }
  __device__ __forceinline__ const StagedRef& operator=(T x) const {
    if (x != v) {
      v = x;
      d |= BIT;
    }
    return *this;
  }
};
__device__ __forceinline__ SlotStage& slot_stage() {
  __shared__ SlotStage ss;
  return ss;
}

// The HBM form (span too wide to stage) tracks nothing: a per-thread byte.
__device__ __forceinline__ u8& dummy_dirty() {
  __shared__ u8 sink[kBlock];
  return sink[threadIdx.x];
}

template <bool S>
struct PrT {
  const Args* A;
  u64 p;  // slot index in the group arrays
  u32 j;  // slot index in the staged span (S)
  __device__ __forceinline__ auto match() const {
    if constexpr (S) return StagedRef<u64, kDirtyMatch>{slot_stage().match[j], slot_stage().dirty[j]};
    else return StagedRef<u64, 0>{U(A->lg.match)[p], dummy_dirty()};
  }
  __device__ __forceinline__ auto next() const {
    if constexpr (S) return StagedRef<u64, kDirtyNext>{slot_stage().next[j], slot_stage().dirty[j]};
    else return StagedRef<u64, 0>{U(A->lg.next)[p], dummy_dirty()};
  }
  __device__ __forceinline__ auto st() const {
    if constexpr (S) return StagedRef<u8, kDirtySt>{slot_stage().st[j], slot_stage().dirty[j]};
    else return StagedRef<u8, 0>{A->lg.pstate[p], dummy_dirty()};
  }
  __device__ __forceinline__ auto ipos() const {
    if constexpr (S) return StagedRef<u32, kDirtyIpos>{slot_stage().ipos[j], slot_stage().dirty[j]};
    else return StagedRef<u32, 0>{A->lg.infl_pos[p], dummy_dirty()};
  }
  __device__ __forceinline__ u64& psnap() const { return U(A->lg.pending_snapshot)[p]; }
  __device__ __forceinline__ u64* ibuf() const { return U(A->lg.infl_buf) + p * A->lg.inflight_cap; }
  __device__ __forceinline__ u32 K() const { return A->lg.inflight_cap; }
};
// Every Progress write goes through a PrT's StagedRef (maybe_commit only
// reads match), which marks the changed fields.
template <bool S>
__device__ __forceinline__ PrT<S> pr_of(const Args& A, const Group& G_, u32 j) {
  return PrT<S>{&A, u64(G_.s0) + j, G_.j0 + j};
}
__device__ __forceinline__ u32 st_state(u8 s) { return s & 3u; }

// inflights.go
template <class P>
__device__ __forceinline__ bool infl_full(const P& p) { return (p.ipos() >> 16) == p.K(); }
template <class P>
__device__ __forceinline__ void infl_reset(const P& p) { p.ipos() = 0; }
template <class P>
__device__ void infl_add(const P& p, u64 v) {
  const u32 pos = p.ipos();
  const u32 start = pos & 0xFFFFu, count = pos >> 16;
  u32 nxt = start + count;
  if (nxt >= p.K()) nxt -= p.K();
  p.ibuf()[nxt] = v;
  p.ipos() = start | ((count + 1) << 16);
}
template <class P>
__device__ void infl_free_le(const P& p, u64 to) {
  const u32 pos = p.ipos();
  const u32 start = pos & 0xFFFFu, count = pos >> 16;
  const u32 K = p.K();
  const u64* buf = p.ibuf();
  // i = the ring's prefix of entries <= to (inflights.go:95-122), read four
  // entries per round trip (clamped, branch-free) instead of one dependent
  // load per entry
  u32 i = 0;
  bool done = count == 0;
  while (!done && i < count) {
    u64 e[4];
#pragma unroll
    for (u32 q = 0; q < 4; ++q) {
      const u32 k = i + q < count ? i + q : count - 1;
      u32 idx = start + k;
      if (idx >= K) idx -= K;
      e[q] = buf[idx];
    }
#pragma unroll
    for (u32 q = 0; q < 4; ++q) {
      if (!done && i < count) {
        if (to < e[q]) done = true;
        else ++i;
      }
    }
  }
  if (i == 0) return;
  u32 idx = start + i;
  if (idx >= K) idx -= K;
  const u32 c2 = count - i;
  p.ipos() = c2 == 0 ? 0u : (idx | (c2 << 16));
}

// progress.go
template <class P>
__device__ __forceinline__ void reset_state(const P& p, u32 state) {
  p.st() = u8((p.st() & QB_PR_RECENT_ACTIVE) | state);  // ProbeSent = false
  p.psnap() = 0;
  infl_reset(p);
}
template <class P>
__device__ void become_probe(const P& p) {
  const u64 m1 = p.match() + 1;
  if (st_state(p.st()) == QB_PR_SNAPSHOT) {
    const u64 ps1 = p.psnap() + 1;
    reset_state(p, QB_PR_PROBE);
    p.next() = m1 > ps1 ? m1 : ps1;
  } else {
    reset_state(p, QB_PR_PROBE);
    p.next() = m1;
  }
}
template <class P>
__device__ __forceinline__ void become_replicate(const P& p) {
  reset_state(p, QB_PR_REPLICATE);
  p.next() = p.match() + 1;
}
template <class P>
__device__ __forceinline__ void become_snapshot(const P& p, u64 snapi) {
  reset_state(p, QB_PR_SNAPSHOT);
  p.psnap() = snapi;
}
template <class P>
__device__ __forceinline__ bool is_paused(const P& p) {
  const u8 s = p.st();
  switch (st_state(s)) {
    case QB_PR_PROBE: return (s & QB_PR_PROBE_SENT) != 0;
    case QB_PR_REPLICATE: return infl_full(p);
    default: return true;
  }
}
template <class P>
__device__ bool maybe_update(const P& p, u64 n) {
  bool updated = false;
  if (p.match() < n) {
    p.match() = n;
    updated = true;
    p.st() = u8(p.st() & ~QB_PR_PROBE_SENT);
  }
  const u64 n1 = n + 1;
  if (p.next() < n1) p.next() = n1;
  return updated;
}
template <class P>
__device__ bool maybe_decr_to(const P& p, u64 rejected, u64 hint) {
  if (st_state(p.st()) == QB_PR_REPLICATE) {
    if (rejected <= p.match()) return false;
    p.next() = p.match() + 1;
    return true;
  }
  if (p.next() - 1 != rejected) return false;
  const u64 h1 = hint + 1;
  const u64 mn = rejected < h1 ? rejected : h1;
  p.next() = mn > 1 ? mn : 1;
  p.st() = u8(p.st() & ~QB_PR_PROBE_SENT);
  return true;
}

// raft.go:432-492
template <bool S>
__device__ bool maybe_send_append(const Args& A, Group& G_, u32 to, bool send_if_empty) {
  const PrT<S> p = pr_of<S>(A, G_, to);
  if (is_paused(p)) return false;
  const u64 nx = p.next();
  const u64 term = log_term(A, G_, nx - 1);
  u64 n = 0;
  bool compacted = false;
  if (nx <= LG_LAST(A, G_)) {
    if (nx < LG_FIRST(A, G_)) compacted = true;
    else {
      const u64 avail = LG_LAST(A, G_) - nx + 1;
      n = avail < LG_MAX_ENTS(A, G_) ? avail : LG_MAX_ENTS(A, G_);
    }
  }
  if (n == 0 && !send_if_empty) return false;
  if (compacted) {
    if (!(p.st() & QB_PR_RECENT_ACTIVE)) return false;
    if (LG_SNAP_I(A, G_) == 0) return false;  // ErrSnapshotTemporarilyUnavailable
    emit(A, G_, QB_MSG_SNAP, to, LG_SNAP_I(A, G_), LG_SNAP_T(A, G_), 0, 0);
    become_snapshot(p, LG_SNAP_I(A, G_));
    return true;
  }
  emit(A, G_, QB_MSG_APP, to, nx - 1, term, G_.committed, n);
  if (n != 0) {
    const u32 s = st_state(p.st());
    if (s == QB_PR_REPLICATE) {
      const u64 last = nx + n - 1;
      p.next() = last + 1;
      infl_add(p, last);
    } else if (s == QB_PR_PROBE) {
      p.st() = u8(p.st() | QB_PR_PROBE_SENT);
    }
  }
  return true;
}

// tracker.go:177-179 -> joint.go:49-56 -> majority.go:126-172: the q-th
// largest match among a half's voters = the largest member value v with
// #{members >= v} >= q.  Runtime loops over the group's slots (its match
// values stay in L1 after the first touch): a register-resident 16-wide
// network cost ~60 VGPRs and halved the occupancy of this latency-bound
// kernel.
__device__ u64 half_ci(const u64* mp, u32 ns, u32 mask) {
  if (mask == 0) return kInf;
  const int q = __popc(mask) / 2 + 1;
  u64 best = 0;
  for (u32 i = 0; i < ns; ++i) {
    if (!((mask >> i) & 1u)) continue;
    const u64 vi = mp[i];
    if (vi <= best) continue;
    int c = 0;
    for (u32 j = 0; j < ns; ++j) c += ((mask >> j) & 1u) && mp[j] >= vi;
    if (c >= q) best = vi;
  }
  return best;
}

template <bool S>
__device__ bool maybe_commit(const Args& A, Group& G_) {
  const u64* mp = S ? slot_stage().match + G_.j0 : U(A.lg.match) + G_.s0;
  const u64 a = half_ci(mp, G_.ns, G_.mask_in), b = half_ci(mp, G_.ns, G_.mask_out);
  const u64 mci = a < b ? a : b;
  if (mci > G_.committed && log_term(A, G_, mci) == G_.term) {
    G_.committed = mci;
    return true;
  }
  return false;
}

template <bool S>
__device__ void bcast_append(const Args& A, Group& G_) {
  for (u32 s = 0; s < G_.ns; ++s)
    if (s != leader_slot(G_)) maybe_send_append<S>(A, G_, s, true);
}

// joint.go:61-75 over majority.go:178-210 with votes = acks (all true).
__device__ __forceinline__ u8 acks_vote(const Group& G_, u32 acks) {
  const u8 r1 = vote_from_counts(__popc(G_.mask_in), __popc(G_.mask_in & acks),
                                 __popc(G_.mask_in & acks));
  const u8 r2 = vote_from_counts(__popc(G_.mask_out), __popc(G_.mask_out & acks),
                                 __popc(G_.mask_out & acks));
  return joint_vote(r1, r2);
}

template <bool S>
__device__ void heartbeat_resp(const Args& A, Group& G_, u32 slot, const PrT<S>& p, u64 ctx) {
  p.st() = u8((p.st() | QB_PR_RECENT_ACTIVE) & ~QB_PR_PROBE_SENT);
  if (st_state(p.st()) == QB_PR_REPLICATE && infl_full(p)) {
    const u32 start = p.ipos() & 0xFFFFu;
    infl_free_le(p, p.ibuf()[start]);  // FreeFirstOne
  }
  if (p.match() < LG_LAST(A, G_)) maybe_send_append<S>(A, G_, slot, true);
  if (A.lg.read_only != QB_READ_ONLY_SAFE || ctx == 0) return;
  // read_only.go:68-79 recvAck
  const u32 cap = A.lg.readq_cap;
  // (a count past the queue's capacity is read as the capacity: no access
  // outside the caller's [readq_cap * G] arrays or the ReadState area)
  const u32 qlen = min((G_.meta >> 20) & 0x1Fu, cap);
  u64* qctx = U(A.lg.rq_ctx) + G_.g * cap;
  u64* qidx = U(A.lg.rq_index) + G_.g * cap;
  u32* qmeta = A.lg.rq_meta + G_.g * cap;
  // The queue's contexts four at a time (branch-free, clamped): one round
  // trip per four entries instead of one per entry of a dependent scan.
  u32 found = kNone;
  for (u32 k0 = 0; k0 < qlen && found == kNone; k0 += 4) {
    u64 c[4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i) c[i] = qctx[k0 + i < qlen ? k0 + i : qlen - 1];
#pragma unroll
    for (u32 i = 0; i < 4; ++i)
      if (found == kNone && k0 + i < qlen && c[i] == ctx) found = k0 + i;
  }
  u32 acks = 0;  // a nil map when the context is unknown
  if (found != kNone) {
    qmeta[found] |= 1u << slot;
    acks = qmeta[found] & 0xFFFFu;
  }
  if (acks_vote(G_, acks) != QB_VOTE_WON) return;
  if (found == kNone) return;  // advance finds nothing (read_only.go:113-121)
  // read_only.go:84-112 advance + raft.go:1304-1308 responses, oldest first.
  for (u32 k0 = 0; k0 <= found; k0 += 4) {  // loads of four entries issued together
    u32 mt[4];
    u64 ix[4], cx[4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
      const u32 k = k0 + i <= found ? k0 + i : found;
      mt[i] = qmeta[k];
      ix[i] = qidx[k];
      cx[i] = qctx[k];
    }
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
      if (k0 + i > found) break;
      const u32 from = mt[i] >> 16;
      if ((from == kNoSlot || from == leader_slot(G_)) && A.rs)  // r.readStates
        A.rs[u64(G_.nrs++) * A.lg.G + G_.g] = ReadSt{ix[i], cx[i]};
      else if (from == kNoSlot || from == leader_slot(G_))
        emit(A, G_, QB_READ_STATE, kNoSlot, ix[i], 0, 0, cx[i]);
      else
        emit(A, G_, QB_MSG_READ_INDEX_RESP, from, ix[i], 0, 0, cx[i]);
    }
  }
  const u32 rest = qlen - (found + 1);
  for (u32 k = 0; k < rest; ++k) {
    qctx[k] = qctx[k + found + 1];
    qidx[k] = qidx[k + found + 1];
    qmeta[k] = qmeta[k + found + 1];
  }
  G_.meta = (G_.meta & ~(0x1Fu << 20)) | (rest << 20);
}

template <bool S>
__device__ void app_resp(const Args& A, Group& G_, u32 slot, const PrT<S>& p, u64 index, bool reject,
                         u64 hint, u64 hint_term, u8& gfl) {
  p.st() = u8(p.st() | QB_PR_RECENT_ACTIVE);
  if (reject) {
    u64 next_probe = hint;
    if (hint_term > 0) next_probe = find_conflict_by_term(A, G_, hint, hint_term);
    if (maybe_decr_to(p, index, next_probe)) {
      if (st_state(p.st()) == QB_PR_REPLICATE) become_probe(p);
      maybe_send_append<S>(A, G_, slot, true);
    }
    return;
  }
  const bool old_paused = is_paused(p);
  if (!maybe_update(p, index)) return;
  const u32 s = st_state(p.st());
  if (s == QB_PR_PROBE) {
    become_replicate(p);
  } else if (s == QB_PR_SNAPSHOT && p.match() >= p.psnap()) {
    become_probe(p);
    become_replicate(p);
  } else if (s == QB_PR_REPLICATE) {
    infl_free_le(p, index);
  }
  if (maybe_commit<S>(A, G_)) {
    gfl |= QB_LFLAG_ADVANCED;
    if (G_.meta & QB_META_PENDING_READINDEX) {
      // releasePendingReadIndexMessages (raft.go:1813-1825) is the host's.
      G_.meta &= ~QB_META_PENDING_READINDEX;
      gfl |= QB_LFLAG_RELEASE_READS;
    }
    bcast_append<S>(A, G_);
  } else if (old_paused) {
    maybe_send_append<S>(A, G_, slot, true);
  }
  while (maybe_send_append<S>(A, G_, slot, false)) {
  }
  if (slot == transferee(G_) && p.match() == LG_LAST(A, G_))
    emit(A, G_, QB_MSG_TIMEOUT_NOW, slot, 0, 0, 0, 0);
}

template <class P>
__device__ void snap_status(const P& p, bool reject) {
  if (st_state(p.st()) != QB_PR_SNAPSHOT) return;
  if (reject) p.psnap() = 0;
  become_probe(p);
  p.st() = u8(p.st() | QB_PR_PROBE_SENT);
}

struct StepCounts {
  u32 applied = 0, stale = 0, higher = 0, non = 0, after = 0, msgs = 0, stored = 0, reads = 0;
};

// One group's records [r0, r1) of the gathered columns, in batch order (raft.go:847-921 term
// filter, then stepLeader per record).
// The group's fields and its first record, loaded by k_ld_step while the slot
// stage is in flight (QB_LD_PREFETCH): one HBM round trip fewer at the start
// of every workgroup.
struct Pre {
  u32 cfg, meta, f0;
  u64 term, committed, t0, i0;
  u64 first, last;  // the log view's first / last index (held by Group)
};
template <bool S>
__device__ __forceinline__ void step_group(const Args& A, u64 g, u32 r0, u32 r1, u32 s0, u32 s1, u32 sb,
                           const Pre& pre, u32& stepdown, u8& gfl, StepCounts& n) {
  Group G_;
  G_.g = g;
  G_.s0 = s0;
  G_.ns = s1 - s0;
  G_.j0 = s0 - sb;
  const u32 c = pre.cfg;
  G_.mask_in = c & 0xFFFFu;
  G_.mask_out = c >> 16;
  G_.meta = pre.meta;
  G_.term = pre.term;
  G_.committed = pre.committed;
  G_.first = pre.first;
  G_.last = pre.last;
  G_.nruns = min((G_.meta >> 16) & 0xFu, u32(QB_LEADER_MAX_RUNS));  // (the arrays' rows)
  G_.nmsg = 0;
  G_.stored = 0;
  G_.chunk = 0;
  G_.nrs = 0;
  G_.dropped = false;
  for (u32 k = r0; k < r1; ++k) {
    if (stepdown != kNone) {
      ++n.after;
      continue;
    }
    const u64 t = k == r0 ? pre.t0 : A.rec.term[k];
    const u32 f = k == r0 ? pre.f0 : u32(A.rec.flags[k]);
    if (t != 0 && t > G_.term) {  // raft.go:852-880: becomeFollower
      stepdown = A.perm[k];
      ++n.higher;
      continue;
    }
    if (t != 0 && t < G_.term) {  // raft.go:883-921: ignored
      ++n.stale;
      continue;
    }
    const u32 slot = f & 0x0Fu;
    if (slot >= G_.ns || (f & QB_REC_NO_PROGRESS)) {  // raft.go:1099-1104: no progress
      ++n.non;
      continue;
    }
    ++n.applied;
    const PrT<S> p = pr_of<S>(A, G_, slot);
    const u32 kind = (f >> 4) & 3u;
    const bool reject = (f & QB_REC_REJECT) != 0;
    if (kind == QB_IN_APP_RESP) {
      const u64 hint = reject ? A.rec.hint[k] : 0;
      const u64 ht = reject ? A.rec.log_term[k] : 0;
      app_resp<S>(A, G_, slot, p, k == r0 ? pre.i0 : A.rec.index[k], reject, hint, ht, gfl);
    } else if (kind == QB_IN_HEARTBEAT_RESP) {
      heartbeat_resp<S>(A, G_, slot, p, k == r0 ? pre.i0 : A.rec.index[k]);
    } else if (kind == QB_IN_SNAP_STATUS) {
      snap_status(p, reject);
    } else if (st_state(p.st()) == QB_PR_REPLICATE) {  // MsgUnreachable
      become_probe(p);
    }
  }
  if (stepdown != kNone) gfl |= QB_LFLAG_STEPPED_DOWN;
  A.lg.committed[g] = G_.committed;
  A.lg.meta[g] = G_.meta;
  n.msgs = G_.nmsg;
  n.stored = G_.stored;
  n.reads = G_.nrs;
}

// One thread per group.  The workgroup's groups own one contiguous slot span
// [off[g0], off[g0 + 256]); when it fits kSpanCap, its match / next /
// inflight positions / state bytes are staged in LDS with coalesced loads,
// stepped there, and written back coalesced (the step's Progress reads and
// read-modify-writes then cost LDS latency, not HBM round trips).  A larger
// span runs on the HBM arrays directly.
__global__ __launch_bounds__(kBlock) void k_ld_step(Args A) {
  __shared__ u32 lds[7];
  BlockTally<7> tally;
  const u64 G = A.lg.G;
  const u64 g0 = u64(blockIdx.x) * kBlock;
  const u64 g = g0 + threadIdx.x;
  const u64 gend = g0 + kBlock < G ? g0 + kBlock : G;
  const bool live = g < G;
  const u32 r0 = live ? A.cnt[g] : 0u, r1 = live ? A.cnt[g + 1] : 0u;
  const u32 s0 = live ? A.lg.off[g] : 0u, s1 = live ? A.lg.off[g + 1] : 0u;
  const u32 sb = A.lg.off[g0], span = A.lg.off[gend] - sb;
  const bool staged = span <= kSpanCap;  // workgroup-uniform
  if (threadIdx.x < 7) lds[threadIdx.x] = 0;  // the stat tally (staged below)
  const bool busy = __syncthreads_or(r1 > r0);
  if (!busy) {
    // No records for any group of the workgroup: only the outputs.
    if (live) {
      A.mcnt[g] = 0;
      if (A.rcnt) A.rcnt[g] = 0;
      if (A.stepdown_at) A.stepdown_at[g] = kNone;
      if (A.gflags) A.gflags[g] = 0;
    }
    if (A.mbs && threadIdx.x == 0) A.mbs[blockIdx.x] = 0;
    return;
  }
  // issued before the slot stage's loads so both round trips overlap
  Pre pre{};
  if (live && r1 > r0) {
    pre.cfg = A.lg.cfg[g];
    pre.meta = A.lg.meta[g];
    pre.term = A.lg.term[g];
    pre.committed = A.lg.committed[g];
    pre.t0 = A.rec.term[r0];
    pre.f0 = A.rec.flags[r0];
    pre.i0 = A.rec.index[r0];
    pre.first = U(A.lg.first_index)[g];
    pre.last = U(A.lg.last_index)[g];
  }
  SlotStage& ss = slot_stage();
  if (staged) {
    for (u32 j = threadIdx.x; j < span; j += kBlock) {
      ss.match[j] = U(A.lg.match)[sb + j];
      ss.next[j] = U(A.lg.next)[sb + j];
      ss.ipos[j] = A.lg.infl_pos[sb + j];
      ss.st[j] = A.lg.pstate[sb + j];
      ss.dirty[j] = 0;
    }
    __syncthreads();
  }
  StepCounts n;
  if (live) {
    u32 stepdown = kNone;
    u8 gfl = 0;
    if (r1 > r0) {
      if (staged) step_group<true>(A, g, r0, r1, s0, s1, sb, pre, stepdown, gfl, n);
      else step_group<false>(A, g, r0, r1, s0, s1, sb, pre, stepdown, gfl, n);
    }
    if (!A.mbs) A.mcnt[g] = n.stored;  // (ordered: the prefix below)
    if (A.rcnt) A.rcnt[g] = n.reads;
    if (A.stepdown_at) A.stepdown_at[g] = stepdown;
    if (A.gflags) A.gflags[g] = gfl;
  }
  // Per-wave sums of per-thread counts, staged into LDS before the barrier
  // the write-back needs anyway and published after it (a flush with two
  // barriers of its own at the end of the workgroup, as the tracker's K5 had)
  auto wsum = [](u32 v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
  tally.t[0] += wsum(n.applied);
  tally.t[1] += wsum(n.stale);
  tally.t[2] += wsum(n.higher);
  tally.t[3] += wsum(n.non);
  tally.t[4] += wsum(n.after);
  tally.t[5] += wsum(n.msgs);
  tally.t[6] += wsum(n.msgs - n.stored);
  // ordered form: the messages' place within the workgroup (a scan of the
  // stored counts over its 256 groups) and the workgroup's total, so no scan
  // kernel runs over the G counts (k_ld_emit adds the workgroups' prefix)
  __shared__ u32 mwave[kBlock / 64];
  u32 minc = n.stored;
  if (A.mbs) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = u32(__shfl_up(int(minc), o, 64));
      if ((threadIdx.x & 63u) >= u32(o)) minc += y;
    }
    if ((threadIdx.x & 63u) == 63u) mwave[threadIdx.x >> 6] = minc;
  }
  tally.stage(lds);
  __syncthreads();
  if (A.mbs) {
    u32 before = 0, total = 0;
#pragma unroll
    for (u32 q = 0; q < kBlock / 64; ++q) {
      total += mwave[q];
      if (q < (threadIdx.x >> 6)) before += mwave[q];
    }
    if (live) A.mcnt[g] = before + minc - n.stored;
    if (threadIdx.x == 0) A.mbs[blockIdx.x] = total;
  }
  {
    const int slot[7] = {QB_LSTAT_APPLIED, QB_LSTAT_STALE_TERM, QB_LSTAT_HIGHER_TERM,
                         QB_LSTAT_NON_MEMBER, QB_LSTAT_AFTER_STEPDOWN, QB_LSTAT_MSGS,
                         QB_LSTAT_MSGS_DROPPED};
    BlockTally<7>::publish(lds, A.shards + u64(blockIdx.x % 64) * QB_LSTAT_COUNT, slot);
  }
  if (staged) {
    for (u32 j = threadIdx.x; j < span; j += kBlock) {
      const u8 dm = ss.dirty[j];
      if (!dm) continue;
      if (dm & kDirtyMatch) U(A.lg.match)[sb + j] = ss.match[j];
      if (dm & kDirtyNext) U(A.lg.next)[sb + j] = ss.next[j];
      if (dm & kDirtyIpos) A.lg.infl_pos[sb + j] = ss.ipos[j];
      if (dm & kDirtySt) A.lg.pstate[sb + j] = ss.st[j];
    }
  }
}

// ------------------------------------------------------------------ L6 ----
// Each group's staged messages to their final place (msg_off = the scan of
// the counts), the workgroup's output range written with coalesced word
// stores.  Messages past msg_cap are counted as dropped.
__global__ __launch_bounds__(kBlock) void k_ld_emit(u64 G, const u32* __restrict__ moff,
                                                    const u32* __restrict__ mbs,
                                                    const u32* __restrict__ mbsum, u32 nblk,
                                                    const Msg* __restrict__ fix,
                                                    const u32* __restrict__ chead,
                                                    const u32* __restrict__ cnext,
                                                    const Msg* __restrict__ chunks,
                                                    Msg* __restrict__ out, u64 cap,
                                                    u32* __restrict__ msg_off,
                                                    u64* __restrict__ msg_total,
                                                    u64* __restrict__ shards) {
  __shared__ u32 lo[kBlock + 1];
  const u64 g0 = u64(blockIdx.x) * kBlock;
  const u32 ng = u32(G - g0 < kBlock ? G - g0 : kBlock);
  // group g's first message: its prefix within the step's workgroup (moff)
  // plus the workgroup's place (mbs scanned; two levels, off_at style)
  auto boff = [&](u32 i) -> u32 {
    return i < nblk ? mbs[i] + mbsum[i / scan::kScanPer] : mbs[nblk];
  };
  const u32 base = boff(blockIdx.x), next = boff(blockIdx.x + 1);
  for (u32 t = threadIdx.x; t <= ng; t += kBlock) lo[t] = t < ng ? moff[g0 + t] + base : next;
  __syncthreads();
  if (threadIdx.x < ng && msg_off) msg_off[g0 + threadIdx.x] = lo[threadIdx.x];
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    if (msg_off) msg_off[G] = lo[ng];
    *msg_total = lo[ng];
  }
  const u64 m0 = lo[0], m1 = lo[ng];
  const u64* fw = reinterpret_cast<const u64*>(fix);
  const u64* cw = reinterpret_cast<const u64*>(chunks);
  u64* ow = reinterpret_cast<u64*>(out);
  const u32 t = threadIdx.x;
  const u32 n = t < ng ? lo[t + 1] - lo[t] : 0u;
  const u64 w1 = (m1 < cap ? m1 : (m0 < cap ? cap : m0)) * 5;  // end of the words kept
  if (m1 - m0 <= kEmitStage && !__syncthreads_or(n > kFix)) {
    // The workgroup's messages (all in the fixed area) are gathered into LDS
    // row by row of the k-major area (coalesced reads), then stored as one
    // contiguous run of words (coalesced writes).
    __shared__ u64 words[kEmitStage * 5];
    const u32 mo = lo[t < ng ? t : 0] - u32(m0);
    for (u32 k = 0; k < kFix; ++k) {
      if (!__syncthreads_or(k < n)) break;
      if (k < n) {
        const u64* src = fw + (u64(k) * G + g0 + t) * 5;
#pragma unroll
        for (int w = 0; w < 5; ++w) words[(mo + k) * 5 + w] = src[w];
      }
    }
    __syncthreads();
    for (u64 w = m0 * 5 + t; w < w1; w += kBlock) ow[w] = words[w - m0 * 5];
  } else {
    // Word by word over the workgroup's output range (any message count).
    for (u64 w = m0 * 5 + t; w < w1; w += kBlock) {
      const u64 idx = w / 5;
      const u32 word = u32(w - idx * 5);
      // the group owning message idx: last a with lo[a] <= idx (binary search)
      u32 a = 0, b = ng;  // invariant lo[a] <= idx < lo[b]
      while (b - a > 1) {
        const u32 m = (a + b) >> 1;
        if (lo[m] <= idx) a = m;
        else b = m;
      }
      const u64 g = g0 + a;
      const u32 k = u32(idx - lo[a]);
      u64 v;
      if (k < kFix) {
        v = fw[(u64(k) * G + g) * 5 + word];
      } else {
        u32 c = chead[g];
        for (u32 hop = (k - kFix) / kChunk; hop; --hop) c = cnext[c];
        v = cw[(u64(c) * kChunk + (k - kFix) % kChunk) * 5 + word];
      }
      ow[w] = v;
    }
  }
  if (threadIdx.x == 0 && m1 > cap) {
    const u64 dropped = m1 - (m0 > cap ? m0 : cap);
    atomicAdd(shards + u64(blockIdx.x % 64) * QB_LSTAT_COUNT + QB_LSTAT_MSGS_DROPPED, dropped);
  }
}

// bshards: the bucket pass's shards (bad groups), or null.
// One wave per counter: lanes sum strided shards, then a shuffle reduction.
// chunks_used = the chunks actually drawn: the pool counter also counts
// failed draws (a group finding the pool exhausted), so it is clamped to
// nchunks.
__global__ void k_ld_fold(const u64* __restrict__ shards, const u64* __restrict__ bshards,
                          u64* __restrict__ stats, const u32* __restrict__ pool,
                          u32* __restrict__ chunks_used, u64 nchunks) {
  const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (chunks_used && threadIdx.x == 0) *chunks_used = u32(u64(*pool) < nchunks ? u64(*pool) : nchunks);
  if (k >= QB_LSTAT_COUNT) return;
  u64 s = shards[lane * QB_LSTAT_COUNT + k];
  if (bshards && k == QB_LSTAT_BAD_GROUP)
    for (int i = lane; i < bk::kShards; i += 64) s += bshards[i * QB_STAT_COUNT + QB_STAT_BAD_GROUP];
  for (int o = 32; o > 0; o >>= 1) {
    const u64 y = u64(__shfl_xor(static_cast<unsigned long long>(s), o, 64));
    s += y;
  }
  if (lane == 0) stats[k] += s;
}

}  // namespace ld
}  // namespace qb

using namespace qb;

extern "C" size_t qb_leader_workspace_bytes(uint64_t G, uint64_t M) {
  return ld::carve(G, M).total;
}

extern "C" size_t qb_leader_outbox_workspace_bytes(uint64_t G, uint64_t M) {
  return ld::carve(G, M, /*outbox=*/true).total;
}

namespace {

// Where the step leaves its messages: the workspace's k-major area + pool
// (qb_dev_leader_step, which then compacts them into group order), or the
// caller's outbox (qb_dev_leader_step_outbox).
struct MsgSink {
  ld::Msg* fix;
  u32* count;
  u32* chead;
  u32* cnext;
  ld::Msg* chunks;
  u64 nchunks;
  u32* chunks_used;  // outbox only
  ld::ReadSt* rs;    // outbox only, nullable
  u32* rcnt;
};

int leader_step_impl(const qb_leader_groups* lg, const qb_leader_inbox* in, const ld::Carve& c,
                     const MsgSink* sink, qb_msg_out* msgs, uint64_t msg_cap, uint64_t* msg_total,
                     uint32_t* msg_off, uint32_t* stepdown_at, uint8_t* gflags, uint64_t* stats,
                     char* ws, hipStream_t st) {
  const u64 G = lg->G, M = in->M;
  u32* cnt = reinterpret_cast<u32*>(ws + c.cnt);
  u32* bsum = reinterpret_cast<u32*>(ws + c.bsum);
  u32* perm = reinterpret_cast<u32*>(ws + c.perm);
  const ld::RecCols rcols{reinterpret_cast<u8*>(ws + c.rflags), reinterpret_cast<u64*>(ws + c.rterm),
                       reinterpret_cast<u64*>(ws + c.rindex), reinterpret_cast<u64*>(ws + c.rhint),
                       reinterpret_cast<u64*>(ws + c.rlt)};
  u32* pool = reinterpret_cast<u32*>(ws + c.pool);
  u64* shards = reinterpret_cast<u64*>(ws + c.shards);
  u64* bshards = nullptr;
  // QB_LEADER_OPT_ATOMIC_GROUPING selects the per-record-atomic grouping
  // even when the bucket geometry fits (both paths are tested).
  const bool force_atomic = (lg->options & QB_LEADER_OPT_ATOMIC_GROUPING) != 0;
  hipError_t e = hipSuccess;
  if (!c.bucketed || force_atomic) {  // (else bucket_records' memset zeroes them)
    // pool and stat shards are adjacent in the carve: one memset zeroes both
    e = hipMemsetAsync(pool, 0, c.shards - c.pool + sizeof(u64) * QB_LSTAT_COUNT * 64, st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(leader workspace)");
  }
  if (c.bucketed && !force_atomic) {
    char* bws = ws + c.bkt;
    bshards = reinterpret_cast<u64*>(bws + c.bcv.shards);
    u32* cloc = reinterpret_cast<u32*>(ws + c.ctot);
    u32* cbs = reinterpret_cast<u32*>(ws + c.cbsum);
    const u32* counts = reinterpret_cast<const u32*>(bws + c.bcv.counts);
    const u32* cs = reinterpret_cast<const u32*>(bws + c.bcv.chunk_start);
    const u32* ptab = reinterpret_cast<const u32*>(bws + c.bcv.ptab);
    // bucket_records zeroes bshards itself (before its first count)
    const int rc = bk::bucket_records(c.geo, c.bcv, bws, in->group, in->flags,
                                      ld::U(in->index), ld::U(in->term), bshards, st,
                                      /*compact=*/false);
    if (rc != QB_OK) return rc;
    hipLaunchKernelGGL(ld::k_ld_chunk_total, dim3((c.geo.NC + kBlock - 1) / kBlock),
                       dim3(kBlock), 0, st, c.geo, counts, cs, ptab, cloc, cbs);
    QB_CHECK_LAUNCH("k_ld_chunk_total");
    bk::Cols b2 = bk::cols_at(bws + c.bcv.buf2, c.bcv.nrec_all, 3);
    b2.term32 = reinterpret_cast<u32*>(b2.term);
    if (bk::RunTable::many_rows(c.geo.ppx))
      hipLaunchKernelGGL(ld::k_ld_chunk_runs<true>, dim3(c.geo.NC), dim3(kBlock), 0, st, c.geo, b2,
                         counts, cs, ptab, cloc, cbs, cnt, perm, *in, rcols);
    else
      hipLaunchKernelGGL(ld::k_ld_chunk_runs<false>, dim3(c.geo.NC), dim3(kBlock), 0, st, c.geo, b2,
                         counts, cs, ptab, cloc, cbs, cnt, perm, *in, rcols);
    QB_CHECK_LAUNCH("k_ld_chunk_runs");
  } else {
    u32* cursor = reinterpret_cast<u32*>(ws + c.cursor);
    e = hipMemsetAsync(cnt, 0, sizeof(u32) * (G + 1), st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(counts)");
    const unsigned rgrid = M ? (grid_for(M) < 2048 ? grid_for(M) : 2048) : 1;
    if (M) {
      hipLaunchKernelGGL(ld::k_ld_count, dim3(rgrid), dim3(kBlock), 0, st, G, M, in->group, cnt,
                         shards);
      QB_CHECK_LAUNCH("k_ld_count");
    }
    scan::launch(cnt, G, bsum, st);
    QB_CHECK_LAUNCH("scan(records)");
    if (M) {
      e = hipMemcpyAsync(cursor, cnt, sizeof(u32) * G, hipMemcpyDeviceToDevice, st);
      if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(cursor)");
      hipLaunchKernelGGL(ld::k_ld_scatter, dim3(rgrid), dim3(kBlock), 0, st, G, M, in->group,
                         cursor, perm);
      QB_CHECK_LAUNCH("k_ld_scatter");
      hipLaunchKernelGGL(ld::k_ld_gather, dim3(grid_for(G)), dim3(kBlock), 0, st, G, *in, cnt,
                         perm, rcols);
      QB_CHECK_LAUNCH("k_ld_gather");
    }
  }
  ld::Args A{};
  A.lg = *lg;
  A.in = *in;
  A.cnt = cnt;
  A.perm = perm;
  A.rec = rcols;
  A.mcnt = sink->count;
  A.mbs = msg_total ? reinterpret_cast<u32*>(ws + c.mbs) : nullptr;
  A.fix = sink->fix;
  A.chead = sink->chead;
  A.cnext = sink->cnext;
  A.chunks = sink->chunks;
  A.pool = pool;
  A.nchunks = sink->nchunks;
  A.shards = shards;
  A.stepdown_at = stepdown_at;
  A.gflags = gflags;
  A.rs = sink->rs;
  A.rcnt = sink->rcnt;
  hipLaunchKernelGGL(ld::k_ld_step, dim3(grid_for(G)), dim3(kBlock), 0, st, A);
  QB_CHECK_LAUNCH("k_ld_step");
  if (msg_total) {  // the group-ordered array: the workgroups' totals scanned, then the copy
    const u32 nblk = u32((G + kBlock - 1) / kBlock);
    u32* mbsum = reinterpret_cast<u32*>(ws + c.mbsum);
    // a local scan of the totals + the block sums' scan (the add-back is in
    // k_ld_emit); mbs[nblk] = all messages
    const u32 nsb = scan::blocks(nblk);
    hipLaunchKernelGGL(scan::k_scan_local, dim3(nsb), dim3(1024), 0, st, A.mbs, u64(nblk), mbsum);
    hipLaunchKernelGGL(scan::k_scan_sums, dim3(1), dim3(1024), 0, st, mbsum, nsb, A.mbs + nblk);
    QB_CHECK_LAUNCH("scan(message totals)");
    hipLaunchKernelGGL(ld::k_ld_emit, dim3(grid_for(G)), dim3(kBlock), 0, st, G, sink->count, A.mbs,
                       mbsum, nblk, A.fix, A.chead, A.cnext, A.chunks,
                       reinterpret_cast<ld::Msg*>(msgs), msg_cap, msg_off, ld::U(msg_total), shards);
    QB_CHECK_LAUNCH("k_ld_emit");
  }
  hipLaunchKernelGGL(ld::k_ld_fold, dim3(1), dim3(64 * QB_LSTAT_COUNT), 0, st, shards, bshards,
                     ld::U(stats), pool, sink->chunks_used, sink->nchunks);
  QB_CHECK_LAUNCH("k_ld_fold");
  return QB_OK;
}

int leader_check(const qb_leader_groups* lg, const qb_leader_inbox* in, uint64_t* stats) {
  QB_REQUIRE(lg && in, "qb_dev_leader_step: lg and in are required");
  const u64 G = lg->G, M = in->M;
  QB_REQUIRE(G < (1ull << 32) && M < (1ull << 32), "qb_dev_leader_step: G and M must be < 2^32");
  QB_REQUIRE(lg->inflight_cap >= 1 && lg->inflight_cap <= 4096,
             "qb_dev_leader_step: inflight_cap must be 1..4096");
  QB_REQUIRE(lg->readq_cap <= QB_LEADER_MAX_READQ, "qb_dev_leader_step: readq_cap must be 0..16");
  QB_REQUIRE(stats, "qb_dev_leader_step: stats is required");
  if (G == 0) return QB_OK;
  QB_REQUIRE(lg->off && lg->cfg && lg->meta && lg->term && lg->committed && lg->first_index &&
                 lg->last_index && lg->snap_index && lg->snap_term && lg->max_ents &&
                 lg->run_start && lg->run_term && lg->match && lg->next &&
                 lg->pending_snapshot && lg->pstate && lg->infl_pos && lg->infl_buf,
             "qb_dev_leader_step: a required group/progress array is NULL");
  QB_REQUIRE(lg->readq_cap == 0 || (lg->rq_ctx && lg->rq_index && lg->rq_meta),
             "qb_dev_leader_step: read queue arrays are required when readq_cap > 0");
  QB_REQUIRE(M == 0 || (in->group && in->flags && in->index && in->term),
             "qb_dev_leader_step: inbox group/flags/index/term are required");
  return QB_OK;
}

}  // namespace

extern "C" int qb_dev_leader_step(const qb_leader_groups* lg, const qb_leader_inbox* in,
                                  qb_msg_out* msgs, uint64_t msg_cap, uint64_t* msg_total,
                                  uint32_t* msg_off, uint32_t* stepdown_at, uint8_t* gflags,
                                  uint64_t* stats, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  QB_REQUIRE(msg_total, "qb_dev_leader_step: msg_total is required");
  const int rc = leader_check(lg, in, stats);
  if (rc != QB_OK || lg->G == 0) return rc;
  QB_REQUIRE(msg_cap == 0 || msgs, "qb_dev_leader_step: msgs is NULL");
  const ld::Carve c = ld::carve(lg->G, in->M);
  QB_REQUIRE(workspace && workspace_bytes >= c.total,
             "qb_dev_leader_step: workspace needs %zu bytes", c.total);
  char* ws = static_cast<char*>(workspace);
  const MsgSink sink{reinterpret_cast<ld::Msg*>(ws + c.fix), reinterpret_cast<u32*>(ws + c.mcnt),
                     reinterpret_cast<u32*>(ws + c.chead), reinterpret_cast<u32*>(ws + c.cnext),
                     reinterpret_cast<ld::Msg*>(ws + c.chunks), c.nchunks, nullptr, nullptr,
                     nullptr};
  return leader_step_impl(lg, in, c, &sink, msgs, msg_cap, msg_total, msg_off, stepdown_at, gflags,
                          stats, ws, as_stream(stream));
}

extern "C" int qb_dev_leader_step_outbox(const qb_leader_groups* lg, const qb_leader_inbox* in,
                                         const qb_leader_outbox* out, uint32_t* stepdown_at,
                                         uint8_t* gflags, uint64_t* stats, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  QB_REQUIRE(out, "qb_dev_leader_step_outbox: out is required");
  const int rc = leader_check(lg, in, stats);
  if (rc != QB_OK || lg->G == 0) return rc;
  QB_REQUIRE(out->slots && out->count && out->chunk_head && out->chunks_used,
             "qb_dev_leader_step_outbox: slots, count, chunk_head and chunks_used are required");
  QB_REQUIRE(out->nchunks == 0 || (out->chunks && out->chunk_next),
             "qb_dev_leader_step_outbox: chunks / chunk_next are required when nchunks > 0");
  QB_REQUIRE(out->nchunks < (1ull << 32), "qb_dev_leader_step_outbox: nchunks must be < 2^32");
  QB_REQUIRE(!out->read_states || out->read_count,
             "qb_dev_leader_step_outbox: read_count is required with read_states");
  const ld::Carve c = ld::carve(lg->G, in->M, /*outbox=*/true);
  QB_REQUIRE(workspace && workspace_bytes >= c.total,
             "qb_dev_leader_step_outbox: workspace needs %zu bytes", c.total);
  const MsgSink sink{reinterpret_cast<ld::Msg*>(out->slots), out->count, out->chunk_head,
                     out->chunk_next, reinterpret_cast<ld::Msg*>(out->chunks), out->nchunks,
                     out->chunks_used, reinterpret_cast<ld::ReadSt*>(out->read_states),
                     out->read_states ? out->read_count : nullptr};
  return leader_step_impl(lg, in, c, &sink, nullptr, 0, nullptr, nullptr, stepdown_at, gflags,
                          stats, static_cast<char*>(workspace), as_stream(stream));
}
