// qb_tracker_slow.h — pieces shared by the bucketed tracker steps (FIXED:
// qb_tracker_bucket.hip, CSR: qb_tracker_csr.hip): stat shards, the grid
// barrier, and the slow path that applies flagged chunks from the original
// batch in batch order.
//
//   raft.Step term filter / step-down   raft.go:847-921
//   stepLeader MsgAppResp (quorum part) raft.go:1100-1109, 1237-1259
//   Progress.MaybeUpdate                tracker/progress.go:144-153
//   raft.maybeCommit                    raft.go:585-588, log.go:328-334
#pragma once

#include "qb_bucket.h"
#include "qb_csr.h"

namespace qb {
namespace bk {

// The heavy super-buckets' chunks (a region of theirs overflowed into the
// pool: K3's list) are applied first, by the first kHeavyBlocks workgroups
// of the apply grid (one chunk each: the first 8 heavy super-buckets), so
// their long record passes overlap the other chunks instead of trailing them
// (the reverse chunk order put the chunks of super-bucket 0 last: a 30 %
// skew on it measured 838 us per tick with the pool alone); the workgroup
// that would have taken such a chunk in the linear order returns once it has
// read its super-bucket's flag.
constexpr u32 kHeavyBlocks = 1024;
struct HeavyArgs {
  const u32* sbflag;
  const u32* heavy;
  const u32* nheavy;
  u32 blocks;  // leading workgroups of the grid that take the heavy chunks
};
// K4's folded records (kDedupFlag) and the escapes: the exact index and term
// — the side table or the original batch.  (Side records carry their term
// in the side column, read with the record: RecFmt::tside.)
struct EscArgs {
  const u64 *ri, *rt;  // the original batch
  Side side;
};
// (A folded record counts once here; K4 added the records it folded away to
// the chunk's ext counters by class, which K5 adds unless the chunk is slow.)
// gt: the record's group term (a folded side record equal to it carries
// kTermIsGroup instead of the term).
__device__ __forceinline__ void unescape(const EscArgs& e, u64& t, u64& idx, u64 gt) {
  if (idx & kDedupFlag) {
    const u64 si = idx & (kDedupFlag - 1ull);
    idx = e.side.idx[si];
    t = e.side.tc[si] & kTermIsGroup;
    if (t == kTermIsGroup) t = gt;
  } else {
    const u32 ridx = u32(idx);
    idx = e.ri[ridx];
    t = e.rt[ridx];
  }
}

// Counters of block b go to shard b % kShards (QB_STAT_COUNT u64 each, one
// cache line), folded into the caller's stats by k_stats_fold.
__device__ __forceinline__ u64* shard_of(u64* shards) {
  return shards + u64(blockIdx.x % kShards) * QB_STAT_COUNT;
}

// One thread per shard (its 64-byte line in one go), wave sums by shuffles:
// a thread per counter walking the 256 shards serially took 7 us.  Run by
// one block of kShards threads (block 0 of k_bk_slow).
static_assert(kShards == kBlock, "the fold runs in one kBlock-thread block");
__device__ __forceinline__ void stats_fold_block(const u64* __restrict__ shards,
                                                 u64* __restrict__ stats) {
  __shared__ u64 part[kShards / 64][QB_STAT_COUNT];
  const int i = threadIdx.x, lane = i & 63, w = i >> 6;
  u64 x[QB_STAT_COUNT];
#pragma unroll
  for (int k = 0; k < QB_STAT_COUNT; ++k) x[k] = shards[i * QB_STAT_COUNT + k];
#pragma unroll
  for (int k = 0; k < QB_STAT_COUNT; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x[k] += __shfl_xor(x[k], o, 64);
    if (lane == 0) part[w][k] = x[k];
  }
  __syncthreads();
  if (i < QB_STAT_COUNT) {
    u64 s = 0;
#pragma unroll
    for (int q = 0; q < kShards / 64; ++q) s += part[q][i];
    stats[i] += s;
  }
}

// ------------------------------------------------------ slow chunks ----
// The flagged chunks' records, from the original batch in batch order,
// exactly as qb_tracker.hip's two passes (k_appresp_stepdown/apply) and
// k_commit_advance restricted to those chunks — in ONE launch: kSlowGrid
// blocks (at most a few per CU, all co-resident) run the three phases
// separated by grid barriers.  Without a flagged chunk (the steady state)
// block 0 folds the stat shards and every block returns after one scalar
// load: the former three launches (step-down, apply, finish) cost ~4.7 us
// each even as no-ops.
constexpr unsigned kSlowBlockMax = 256;

// Record sources of the slow path.  get(i, ...) is true when record i of the
// batch is a valid record (group < G, slot < n) of a flagged chunk, with its
// group, flags, index and term.  ColSrc: the batch's columns (the tracker
// steps); the composed wire -> tracker step decodes the message instead
// (qb_wire_tracker.hip).
struct ColSrc {
  const u32* rg;
  const u8* rf;
  const u64 *ri, *rt;
  __device__ __forceinline__ bool get(const Geometry& geo, const u8* __restrict__ chunk_slow,
                                      u64 i, u32& g, u32& f, u64& idx, u64& t) const {
    g = rg[i];
    f = rf[i];
    if (!(g < geo.G && (f & 0x0Fu) < geo.n && chunk_slow[geo.chunk_of(g)] == 1)) return false;
    t = rt[i];
    idx = ri[i];
    return true;
  }
};

// Tracker state layouts.  FIXED: n voters, slot-major rows of G (every slot
// below geo.n is a member).  CSR: group-major slots off[g] .. off[g+1]-1,
// cfg = mask_in | mask_out << 16 (learners in neither mask; slots past the
// group's count have no Progress, raft.go:1100-1104).
template <int N>
struct FixedLay {
  u64 G;
  __device__ __forceinline__ bool member(u32 g, u32 s) const { return true; }
  __device__ __forceinline__ u64 at(u32 g, u32 s) const { return u64(s) * G + g; }
  __device__ __forceinline__ u64 ci(const u64* __restrict__ match, u32 g) const {
    u64 v[N];
#pragma unroll
    for (int s = 0; s < N; ++s) v[s] = match[u64(s) * G + g];
    return select_quorum<N>(v);
  }
};

template <int WMAX>
struct CsrLay {
  const u32* off;
  const u32* cfg;
  __device__ __forceinline__ bool member(u32 g, u32 s) const { return s < off[g + 1] - off[g]; }
  __device__ __forceinline__ u64 at(u32 g, u32 s) const { return u64(off[g]) + s; }
  // every lane of the wave calls it (csr_ci's width is wave-uniform)
  __device__ __forceinline__ u64 ci(const u64* __restrict__ match, u32 g) const {
    const u32 a = off[g], s = off[g + 1] - a, c = cfg[g];
    return csr_ci<WMAX>(match + a, s > WMAX ? WMAX : s, c & 0xFFFFu, c >> 16);
  }
};

// Grid barrier over the co-resident blocks of k_bk_slow (MI355X_MICROARCH.md
// "barrier-counter": lane-0 release fence before the arrive, relaxed poll,
// acquire fence after).  ctr starts at 0 (zeroed with the stat shards by
// bucket_records' memset); barrier k waits for k * gridDim.x arrivals.
__device__ __forceinline__ void grid_barrier(u32* ctr, u32 target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
      __builtin_amdgcn_s_sleep(8);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <class Lay, class Src>
__global__ __launch_bounds__(kBlock) void k_bk_slow(
    Geometry geo, Lay lay, Src src, const u64* __restrict__ group_term,
    const u64* __restrict__ term_start, const u8* __restrict__ chunk_slow,
    const u32* __restrict__ any_slow, u32* __restrict__ bar, u32* __restrict__ stepdown_at,
    u64* __restrict__ match, u64* __restrict__ next, u16* __restrict__ active,
    u64* __restrict__ committed, u8* __restrict__ advanced, u64* __restrict__ shards,
    u64* __restrict__ stats) {
  if (*any_slow == 0) {
    if (blockIdx.x == 0) stats_fold_block(shards, stats);
    return;
  }
  __shared__ u32 tl[6];
  BlockTally<6> tally;  // higher, stale, applied, rejected, after, non-member
  const u64 stride = u64(gridDim.x) * kBlock;
  const u64 tid0 = u64(blockIdx.x) * kBlock + threadIdx.x;
  // Phase 1: the first higher-term record per group in batch order
  // (raft.go:875-879); K5 reset stepdown_at of every flagged chunk's groups.
  for (u64 i = tid0; i < geo.M; i += stride) {
    u32 g, f;
    u64 idx, t;
    bool higher = false;
    if (src.get(geo, chunk_slow, i, g, f, idx, t) && lay.member(g, f & 0x0Fu) &&
        t > group_term[g]) {
      atomicMin(stepdown_at + g, u32(i));
      higher = true;
    }
    tally.add(0, higher);
  }
  grid_barrier(bar, gridDim.x);
  // Phase 2: MaybeUpdate / RecentActive for records before the step-down.
  for (u64 i = tid0; i < geo.M; i += stride) {
    u32 g, f;
    u64 idx, t;
    bool stale = false, applied = false, rejected = false, after = false, non = false;
    const bool in = src.get(geo, chunk_slow, i, g, f, idx, t);
    if (in && !lay.member(g, f & 0x0Fu)) {
      non = true;  // raft.go:1100-1104 (slots >= geo.n were counted by K3)
    } else if (in) {
      const u64 gt = group_term[g];
      stale = t < gt;  // raft.go:883-921
      if (t == gt) {
        if (stepdown_at[g] < u32(i)) {
          after = true;  // the leader stepped down at an earlier record
        } else {
          const u32 s = f & 0x0Fu;
          // RecentActive (raft.go:1107) as an atomic or on the aligned word
          // holding active[g] (no 4-byte alignment asked of the caller)
          const uintptr_t a = reinterpret_cast<uintptr_t>(active + g);
          atomicOr(reinterpret_cast<u32*>(a & ~uintptr_t(3)), (1u << s) << ((a & 2u) * 8u));
          if (f & QB_REC_REJECT) {
            rejected = true;
          } else {
            applied = true;
            const u64 at = lay.at(g, s);
            atomicMax(match + at, idx);                  // progress.go:146-150
            if (next) atomicMax(next + at, idx + 1ull);  // progress.go:151
          }
        }
      }
    }
    tally.add(1, stale);
    tally.add(2, applied);
    tally.add(3, rejected);
    tally.add(4, after);
    tally.add(5, non);
  }
  const int slot[6] = {QB_STAT_HIGHER_TERM, QB_STAT_STALE_TERM, QB_STAT_APPLIED,
                       QB_STAT_REJECTED, QB_STAT_AFTER_STEPDOWN, QB_STAT_NON_MEMBER};
  tally.flush(tl, shard_of(shards), slot);
  grid_barrier(bar, 2 * gridDim.x);
  // Phase 3: maybeCommit for the flagged chunks' groups (log.go:328-334);
  // block 0 folds the (now complete) stat shards.
  if (blockIdx.x == 0) stats_fold_block(shards, stats);
  // whole waves iterate together (CsrLay::ci is wave-cooperative)
  for (u64 g0 = u64(blockIdx.x) * kBlock; g0 < geo.G; g0 += stride) {
    const u64 g = g0 + threadIdx.x;
    const bool mine = g < geo.G && chunk_slow[geo.chunk_of(u32(g))] == 1;
    if (__ballot(mine) == 0) continue;
    const u64 ci = lay.ci(match, mine ? u32(g) : u32(g0));
    if (!mine) continue;
    const u64 cm = committed[g];
    const bool adv = ci != kInf && ci > cm && ci >= term_start[g];  // log.go:328-334
    if (adv) committed[g] = ci;
    if (advanced) advanced[g] = adv ? 1 : 0;
  }
}

struct ApplyArgs {
  const u64 *ri, *rt;  // the original batch (escape records)
  Side side;           // K4's folded records
  const u64 *gt, *ts;
  u64 *match, *next;
  u16* active;
  u64* committed;
  u32* stepdown;
  u8* adv;
  u8* chunk_slow;
  u32* any_slow;
  u64* stats;
  const u32* ptab;  // the overflow pool's part table
  HeavyArgs hv;
};

// Host launchers of qb_tracker_bucket.hip shared with the composed wire ->
// tracker step (qb_wire_tracker.hip).
void launch_split_compact(const Geometry& geo, const Carve& cv, char* ws, const u64* group_term,
                          const u32* csr_off, hipStream_t st);
ApplyArgs fixed_apply_args(const Geometry& geo, const Carve& cv, char* ws, const u64* ri,
                           const u64* rt, const u64* group_term, const u64* term_start, u64* match,
                           u64* next, u16* active, u64* committed, u32* stepdown_at, u8* advanced);
void launch_fixed_apply(u32 n, const Geometry& geo, const Carve& cv, char* ws, const ApplyArgs& a,
                        hipStream_t st);

struct SlowArgs {
  const u32* rg;
  const u8* rf;
  const u64 *ri, *rt;
  u32* bar;
  unsigned grid;
};

// Blocks of k_bk_slow: at most 2 per CU (so all are resident at once for its
// grid barriers, whatever else is queued) and at most kSlowBlockMax.
inline unsigned slow_blocks() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 32;
  const unsigned b = 2u * unsigned(cus);
  return b < kSlowBlockMax ? b : kSlowBlockMax;
}

}  // namespace bk
}  // namespace qb
