// qb_tracker_csr.hip — one leader tick over G groups of the CSR layout
// (ragged voter counts, learners, joint configs): a batch of MsgAppResp
// records applied and the commit advanced, records bucketed by group on the
// device so every MaybeUpdate is an LDS atomic.
//
// Reference semantics (paths relative to the reference's raft/):
//   node.run / RawNode.Step: responses from a non-member are dropped first
//                                        node.go:356-360, rawnode.go:110-119
//   raft.Step term filter                raft.go:847-921
//   stepLeader MsgAppResp (quorum part)  raft.go:1100-1109, 1237-1259
//   Progress.MaybeUpdate                 tracker/progress.go:144-153
//   ProgressTracker.Committed            tracker/tracker.go:162-179 ->
//     JointConfig.CommittedIndex         quorum/joint.go:49-56 (learners have
//                                        a Progress and ack, but never count)
//   raft.maybeCommit (also on a joint transition, raft.go:1682)
//                                        raft.go:585-588, log.go:328-334
//
// Pipeline: K1-K4 are the FIXED step's bucketing (qb_bucket.h, records cut
// into chunks of CH consecutive groups, one run per part of the chunk's
// super-bucket).  K5 = k_csr_apply: one workgroup per chunk.  The chunk's
// groups own one contiguous slot run match[off[g0] .. off[g0 + CH]); an LDS
// accumulator per slot of the run takes the records' MaybeUpdate
// (ds_max_u64), the old run is streamed into registers meanwhile, then one
// coalesced pass writes the raised slots and leaves max(old, acc) in LDS, and
// each thread evaluates its group's JointConfig.CommittedIndex from LDS
// (compacted half sorts, qb_csr.h) and the maybeCommit gate.
//
// Two launches of K5: the first with an LDS run buffer of 8 slots per group
// (the workgroup's LDS sets the occupancy: 512 groups x 8 slots measured 847
// us per 16M-group step against 887 for 256 groups x 12), deferring a chunk
// whose run is longer; the second, with the table's max_slots per group,
// applies only the deferred chunks (a workgroup per chunk that returns at
// once otherwise, ~5 us).  Chunks with a higher-term record (batch order
// matters) go to the slow path (qb_tracker_slow.h) exactly as in the FIXED
// step.
#include "qb_tracker_slow.h"
#include "qb_wire_src.h"

namespace qb {
namespace bk {

// Threads per workgroup, and LDS slots per group of the first launch's run
// buffer (the measured choice: round 2, profiles/r02/ab_csr_*.log).
constexpr u32 kCsrBlock = 512;
constexpr int kCsrCapW = 8;
__host__ __device__ constexpr u32 csr_block() {
  return csr_chunk_groups(16) < kCsrBlock ? csr_chunk_groups(16) : kCsrBlock;
}
constexpr u8 kChunkDeferred = 2;  // chunk_slow value: run too long for the first launch

// CAPW: LDS slots per group; SECOND: the launch for the deferred chunks.
#define QB_CSR_APPLY_PARAMS                                                                      \
  Geometry geo, Cols recs, const u32 *__restrict__ counts, const u32 *__restrict__ cs,            \
      EscArgs esc,                                                                                 \
      const u32 *__restrict__ off, const u32 *__restrict__ cfg,                                   \
      const u64 *__restrict__ group_term, const u64 *__restrict__ term_start,                     \
      u64 *__restrict__ match, u64 *__restrict__ next, u16 *__restrict__ active,                  \
      u64 *__restrict__ committed, u32 *__restrict__ stepdown_at, u8 *__restrict__ advanced,      \
      u8 *__restrict__ chunk_slow, u32 *__restrict__ any_slow, u64 *__restrict__ shards,          \
      const u32 *__restrict__ ptab, HeavyArgs hv
#define QB_CSR_APPLY_ARGS                                                                      \
  geo, recs, counts, cs, esc, off, cfg, group_term, term_start, match, next, active, committed,  \
      stepdown_at, advanced, chunk_slow, any_slow, shards, ptab, hv

// One chunk c (the whole workgroup).
template <int WMAX, int CAPW, bool NEXT, bool SECOND, bool MANY>
__device__ __forceinline__ void csr_apply_chunk(const u32 c, const bool skip_heavy,
                                                QB_CSR_APPLY_PARAMS) {
  constexpr u32 CH = csr_chunk_groups(WMAX);
  constexpr u32 B = csr_block();
  constexpr u32 GPT = CH / B;          // groups per thread in the commit phase
  constexpr u32 CAP = CH * u32(CAPW);  // slot-run capacity
  constexpr u32 PER = (CAP + B - 1) / B;  // run slots per thread
  __shared__ u64 acc[CAP];
  __shared__ u64 accn[NEXT ? CAP : 1];
  __shared__ u32 offs[CH + 1];
  // group terms saturated to u32 (2 KB less LDS: four 512-thread workgroups
  // per CU fit in 40 KB); a term >= 2^32 - 1 is read again from group_term
  __shared__ u32 gterm[CH];
  __shared__ u32 act[CH];
  __shared__ u32 slow;
  __shared__ u32 tl[4];
  __shared__ RunTableOf<MANY> rtab;
  BlockTally<4> tally;  // stale, applied, rejected, non-member
  const u64 g0 = u64(c) * CH;
  const u32 ng = u32(geo.G - g0 < CH ? geo.G - g0 : CH);
  const u32 sb = geo.sb_of_chunk(c), cl = geo.cl_of_chunk(c);
  // a record of this chunk that did not fit its reserved region (K3): the
  // whole chunk goes to the slow path (checked before any deferral)
  const bool overflow = chunk_slow[c] == kChunkOverflow;
  // (the linear order's workgroup of a chunk the leading workgroups take:
  // see k_bk_apply; read with the first loads, tested once the table is built)
  const u32 hf = skip_heavy ? hv.sbflag[sb] : 0u;
  const bool heavy_sb = hf != 0u && hf - 1u < hv.blocks / kChunksPerSb;
  // side records in this call (K3's flag word): their side words are read
  // with the records
  const bool sided = *recs.sflag != 0u;
  // the records K4's dedup folded away (stale, applied, rejected, non-member)
  const u32 extv = esc.side.ext[u64(c) * kExtClasses + (threadIdx.x & 3u)];
  // Load order: (1) slot offsets, group terms and the run table's rows (the
  // part table by scalar load); (2) the old slot run and the commit inputs;
  // (3) the records.  Vector loads retire in order, so each wait of the
  // record chain (offsets, then the run table, then the records) waits only
  // for what was issued before it: the state's latency runs under the chain
  // and the record pass instead of in front of them.  Loads are branch-free
  // (clamped addresses): the compiler's wait counts stay exact only in
  // straight-line code.
  constexpr u32 OPT = (CH + B) / B;  // CH + 1 offsets
  u32 ofr[OPT];
  u64 gtr[GPT];
#pragma unroll
  for (u32 q = 0; q < OPT; ++q) {
    const u32 k = threadIdx.x + q * B;
    ofr[q] = off[g0 + (k < ng ? k : ng)];
  }
#pragma unroll
  for (u32 q = 0; q < GPT; ++q) {
    const u32 k = threadIdx.x + q * B;
    gtr[q] = group_term[g0 + (k < ng ? k : ng - 1)];
  }
  const RunTable::Regs rq = RunTable::issue_regions(cs, counts, sb, geo.ppx, geo.cap, cl);
  // The old slot run and the commit inputs depend only on the chunk's first
  // and last offsets (uniform loads): issued now, in the same round trip as
  // the offsets and the run table, instead of after the first barrier (one
  // HBM round trip fewer in front of the record pass).
  const u32 a0 = off[g0], run = off[g0 + ng] - a0;
  const bool fits = run <= CAP;
  u64 old[PER];
  {
    // (slots past the run re-read its last slot; an oversize run stays in
    // HBM: its lanes re-read the first slot; an empty run has no slot and
    // reads the chunk's first group term instead — a select, not a branch,
    // which would cost the exact wait counts)
    const u64* src = run ? match + a0 : group_term + g0;
    const u32 last = run && fits ? run - 1u : 0u;
#pragma unroll
    for (u32 p = 0; p < PER; ++p) {
      const u32 j = threadIdx.x + p * B;
      old[p] = src[j < last ? j : last];
    }
  }
  u64 cm[GPT], ts[GPT];
  u32 cf[GPT], av[GPT];  // av: RecentActive's read-modify-write reads early
#pragma unroll
  for (u32 k = 0; k < GPT; ++k) {
    const u32 lg = threadIdx.x + k * B;
    const u64 g = g0 + (lg < ng ? lg : ng - 1);
    cm[k] = committed[g];
    ts[k] = term_start[g];
    cf[k] = cfg[g];
    av[k] = active[g];
  }
  for (u32 k = threadIdx.x; k < CAP; k += B) {
    acc[k] = 0;
    if constexpr (NEXT) accn[k] = 0;
  }
  if (threadIdx.x == 0) slow = overflow ? 1u : 0u;
  if (threadIdx.x < 4) tl[threadIdx.x] = 0;
#pragma unroll
  for (u32 q = 0; q < OPT; ++q) {
    const u32 k = threadIdx.x + q * B;
    if (k <= CH) offs[k] = ofr[q];
  }
#pragma unroll
  for (u32 q = 0; q < GPT; ++q) {
    gterm[threadIdx.x + q * B] = gtr[q] < 0xFFFFFFFFull ? u32(gtr[q]) : 0xFFFFFFFFu;
  }
  for (u32 k = threadIdx.x; k < CH; k += B) act[k] = 0;
  __syncthreads();
  // A run longer than the buffer: when a second launch exists (CAPW < WMAX)
  // the first defers the chunk to it; otherwise (CAPW == WMAX, and in the
  // second launch) only a table breaking its max_slots bound gets here, and
  // the chunk takes the slow path (exact per-record semantics, global
  // atomics) — no chunk is left deferred without a launch to apply it.
  if (heavy_sb) return;  // block-uniform: a leading workgroup applies this chunk
  if constexpr (!SECOND && CAPW < WMAX) {
    if (!fits && !overflow) {  // block-uniform, before anything is written
      if (threadIdx.x == 0) chunk_slow[c] = kChunkDeferred;
      return;
    }
  }
  u32 total = rtab.template finish<MANY>(rq, cs, counts, sb, geo.ppx, geo.cap, cl);
  __syncthreads();
  constexpr int kRecPer = int(kK5Inflight / B);  // records in flight per workgroup
  const RecFmt fmt = geo.fmt;
  u64 rec[kRecPer];
  u32 srec[kRecPer];  // side words (a call with side records)
  auto load = [&](u32 f0, u32 n) {
    u32 ix[kRecPer];
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) {
      const u32 f = f0 + u32(r) * B + threadIdx.x;
      ix[r] = n ? rtab.template locate_fixed<MANY>(f < n ? f : n - 1) : 0u;
    }
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) rec[r] = recs.mr[ix[r]];
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) srec[r] = sided ? recs.side[ix[r]] : 0u;
  };
  auto apply = [&](u32 f0, u32 n) {
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) {
      const u32 f = f0 + u32(r) * B + threadIdx.x;
      bool stale = false, applied = false, rejected = false, non = false;
      if (f < n && fits) {
        const u64 x = rec[r];
        const u32 lg = fmt.lg(x), s = fmt.slot(x);
        const u32 base = offs[lg] - a0, sg = offs[lg + 1] - offs[lg];
        if (s >= sg) {
          non = true;                                     // no Progress: raft.go:1100-1104
        } else {
          u64 t = fmt.term(x), idx = fmt.payload(x);
          u64 gt = gterm[lg];
          if (gt == 0xFFFFFFFFull) gt = group_term[g0 + lg];  // (terms past 32 bits)
          // a side record: its term from the side column; an escape: the
          // exact values from the batch, or a folded record's from the side
          // table
          if (t == fmt.tside()) t = srec[r];
          else if (t == fmt.tesc()) unescape(esc, t, idx, gt);
          if (t > gt) {
            slow = 1;  // higher term: step-down order (raft.go:875-879)
          } else if (t < gt) {
            stale = true;                                 // raft.go:883-921
          } else {
            atomicOr(&act[lg], 1u << s);                  // raft.go:1107
            if (fmt.rej(x)) {
              rejected = true;                            // raft.go:1109: not MaybeUpdate
            } else {
              applied = true;
              atomicMax(&acc[base + s], idx);             // progress.go:146-150
              if constexpr (NEXT) atomicMax(&accn[base + s], idx + 1ull);  // :151
            }
          }
        }
      }
      tally.add(0, stale);
      tally.add(1, applied);
      tally.add(2, rejected);
      tally.add(3, non);
    }
  };
  load(0, total);
#pragma unroll
  for (int r = 0; r < kRecPer; ++r) asm volatile("" : "+v"(rec[r]), "+v"(srec[r]));
  apply(0, total);
  for (u32 f0 = B * kRecPer; f0 < total; f0 += B * kRecPer) {  // (all rows in one table)
    load(f0, total);
#pragma unroll
    for (int r = 0; r < kRecPer; ++r) asm volatile("" : "+v"(rec[r]), "+v"(srec[r]));
    apply(f0, total);
  }
  // The chunk's records in the overflow pool (a skewed batch; none
  // otherwise): windows of 64 pool rows through the same table.
  for (u32 w = 0; w * 64u < rtab.npool; ++w) {  // block-uniform (LDS, published before)
    __syncthreads();  // every reader of the previous table is done
    if (threadIdx.x < 64) rtab.pool_window(w, cs, ptab, geo.kmax, geo.region_rows(), sb, cl);
    __syncthreads();
    const u32 tot = rtab.pre[rtab.nr];
    for (u32 f0 = 0; f0 < tot; f0 += B * kRecPer) {
      load(f0, tot);
#pragma unroll
      for (int r = 0; r < kRecPer; ++r) asm volatile("" : "+v"(rec[r]), "+v"(srec[r]));
      apply(f0, tot);
    }
  }
  if (!fits && threadIdx.x == 0) slow = 1;
  tally.stage(tl);  // the counts are final; published after the barrier
  if (threadIdx.x < 4 && extv) atomicAdd(&tl[threadIdx.x], extv);  // K4's folded records
  __syncthreads();
  if (slow) {  // block-uniform: state left for k_bk_slow, counts discarded
    for (u32 lg = threadIdx.x; lg < ng; lg += B) stepdown_at[g0 + lg] = 0xFFFFFFFFu;
    if (threadIdx.x == 0) {
      chunk_slow[c] = 1;
      atomicOr(any_slow, 1u);
    }
    return;
  }
  if (threadIdx.x == 0) chunk_slow[c] = 0;
  {
    const int slot[4] = {QB_STAT_STALE_TERM, QB_STAT_APPLIED, QB_STAT_REJECTED, QB_STAT_NON_MEMBER};
    BlockTally<4>::publish(tl, shard_of(shards), slot);
  }
  // MaybeUpdate write-back over the run (coalesced), leaving max(old, acc)
  // in LDS for the CommittedIndex of every group
#pragma unroll
  for (u32 p = 0; p < PER; ++p) {
    const u32 j = threadIdx.x + p * B;
    if (j < run) {
      const u64 a = acc[j];
      const bool up = a > old[p];
      if (up) old[p] = a;
      // whole wave segments where any slot changed (segment_any, qb_bucket.h):
      // neutral in round 2, 12 us faster per 16M-group tick with the compact
      // records (profiles/r03/k5_variants/)
      if (segment_any(up)) match[a0 + j] = old[p];
      acc[j] = old[p];
      if constexpr (NEXT) {
        const u64 nn = accn[j];
        if (nn) {
          u64* q = next + a0 + j;
          if (nn > *q) *q = nn;
        }
      }
    }
  }
  __syncthreads();
  // maybeCommit per group (every lane takes part: csr_ci's width is
  // wave-uniform)
#pragma unroll
  for (u32 k = 0; k < GPT; ++k) {
    const u32 lg = threadIdx.x + k * B;
    const bool live = lg < ng;
    const u32 base = live ? offs[lg] - a0 : 0u;
    u32 sg = live ? offs[lg + 1] - offs[lg] : 0u;
    sg = sg > u32(WMAX) ? u32(WMAX) : sg;
    const u64 ci = csr_ci<WMAX>(acc + base, sg, cf[k] & 0xFFFFu, cf[k] >> 16);
    if (!live) continue;
    const u64 g = g0 + lg;
    // log.go:328-334; an empty config's ci = MaxUint64 is past lastIndex,
    // whose term is 0 (log.go:271-273): never committed
    const bool adv = ci != kInf && ci > cm[k] && ci >= ts[k];
    if (segment_any(adv)) committed[g] = adv ? ci : cm[k];
    if (advanced) advanced[g] = adv ? 1 : 0;
    const u32 na = act[lg];
    if (segment_any(na != 0)) active[g] = u16(av[k] | na);
  }
}

// One chunk per workgroup: the leading hv.blocks workgroups take the heavy
// super-buckets' chunks (k_bk_apply), the rest the linear order.
template <int WMAX, int CAPW, bool NEXT, bool MANY>
__global__ __launch_bounds__(csr_block()) __attribute__((amdgpu_num_sgpr(80))) void k_csr_apply(
    QB_CSR_APPLY_PARAMS) {
  u32 c;
  const bool lead = blockIdx.x < hv.blocks;
  if (lead) {
    const u32 i = blockIdx.x;
    if (i >= *hv.nheavy * kChunksPerSb) return;  // (all of them in a balanced batch)
    c = geo.chunk_of_sb_cl(hv.heavy[i / kChunksPerSb], i % kChunksPerSb);
    if (c >= geo.NC) return;
  } else {
    c = blockIdx.x - hv.blocks;
  }
  csr_apply_chunk<WMAX, CAPW, NEXT, false, MANY>(c, !lead, QB_CSR_APPLY_ARGS);
}

// The deferred chunks: a workgroup per kDeferSpan consecutive chunks reads
// their flags at once and applies its deferred ones in turn (a workgroup per
// chunk cost ~25 us even with nothing deferred: every one of them reserved
// the big buffer's LDS).
constexpr u32 kDeferSpan = 64;
template <int WMAX, int CAPW, bool NEXT, bool MANY>
__global__ __launch_bounds__(csr_block()) void k_csr_apply_deferred(QB_CSR_APPLY_PARAMS) {
  __shared__ u64 mask;
  const u32 c0 = blockIdx.x * kDeferSpan;
  if (threadIdx.x < 64) {
    const u32 c = c0 + threadIdx.x;
    const u64 m = __ballot(c < geo.NC && threadIdx.x < kDeferSpan && chunk_slow[c] == kChunkDeferred);
    if (threadIdx.x == 0) mask = m;
  }
  __syncthreads();
  for (u64 m = mask; m; m &= m - 1) {  // block-uniform
    __syncthreads();  // the previous chunk's readers of the LDS state are done
    csr_apply_chunk<WMAX, CAPW, NEXT, true, MANY>(c0 + u32(__builtin_ctzll(m)), false,
                                                  QB_CSR_APPLY_ARGS);
  }
}

struct CsrStepArgs {
  const u64 *ri, *rt;  // the original batch (escape records)
  Side side;           // K4's folded records
  const u32 *off, *cfg;
  const u64 *gt, *ts;
  u64 *match, *next;
  u16* active;
  u64* committed;
  u32* stepdown;
  u8* adv;
  u8* chunk_slow;
  u32* any_slow;
  u64* shards;
  const u32* ptab;  // the overflow pool's part table
  HeavyArgs hv;
};

template <int WMAX, bool SECOND, bool MANY>
void launch_apply_rows(const Geometry& geo, Cols recs, const u32* counts, const u32* cs,
                       const CsrStepArgs& a, hipStream_t st) {
  constexpr int CAPW = SECOND ? WMAX : (WMAX < kCsrCapW ? WMAX : kCsrCapW);
  const dim3 grid(SECOND ? (geo.NC + kDeferSpan - 1) / kDeferSpan : a.hv.blocks + geo.NC);
  const EscArgs esc{a.ri, a.rt, a.side};
#define QB_CSR_LAUNCH(NX)                                                                       \
  hipLaunchKernelGGL((SECOND ? k_csr_apply_deferred<WMAX, CAPW, NX, MANY>                        \
                             : k_csr_apply<WMAX, CAPW, NX, MANY>),                                 \
                     grid, dim3(csr_block()), 0, st, geo, recs, counts, cs, esc, a.off, a.cfg,     \
                     a.gt, a.ts,                                                                   \
                     a.match, a.next, a.active, a.committed, a.stepdown, a.adv, a.chunk_slow,      \
                     a.any_slow, a.shards, a.ptab, a.hv)
  if (a.next) QB_CSR_LAUNCH(true);
  else QB_CSR_LAUNCH(false);
#undef QB_CSR_LAUNCH
}
template <int WMAX, bool SECOND>
void launch_apply(const Geometry& geo, Cols recs, const u32* counts, const u32* cs,
                  const CsrStepArgs& a, hipStream_t st) {
  if (RunTable::many_rows(geo.ppx)) launch_apply_rows<WMAX, SECOND, true>(geo, recs, counts, cs, a, st);
  else launch_apply_rows<WMAX, SECOND, false>(geo, recs, counts, cs, a, st);
}

// The apply launches and the slow path over a record source (ColSrc: the
// batch's columns; wt::WireSrc: the composed step re-decodes the bytes).
template <int WMAX, class Src>
void launch_csr_step(const Geometry& geo, Cols recs, const u32* counts, const u32* cs,
                     const CsrStepArgs& a, const Src& src, u32* bar, unsigned grid, u64* stats,
                     hipStream_t st) {
  launch_apply<WMAX, false>(geo, recs, counts, cs, a, st);
  if constexpr (WMAX > kCsrCapW) launch_apply<WMAX, true>(geo, recs, counts, cs, a, st);
  hipLaunchKernelGGL((k_bk_slow<CsrLay<WMAX>, Src>), dim3(grid), dim3(kBlock), 0, st, geo,
                     CsrLay<WMAX>{a.off, a.cfg}, src, a.gt, a.ts, a.chunk_slow, a.any_slow, bar,
                     a.stepdown, a.match, a.next, a.active, a.committed, a.adv, a.shards, stats);
}

// The step's arguments over a carved workspace (ri / rt: the escapes' exact
// index and term by batch position).
CsrStepArgs csr_step_args(const Geometry& geo, const Carve& cv, char* ws, const u64* ri,
                          const u64* rt, const u32* off, const u32* cfg, const u64* group_term,
                          const u64* term_start, u64* match, u64* next, u16* active,
                          u64* committed, u32* stepdown_at, u8* advanced) {
  const Pool pool = pool_at(ws, cv, geo);
  return CsrStepArgs{ri, rt, side_at(ws, cv), off, cfg, group_term, term_start, match, next,
                     active, committed, stepdown_at, advanced,
                     reinterpret_cast<u8*>(ws + cv.chunk_flags), reinterpret_cast<u32*>(ws + cv.flags),
                     reinterpret_cast<u64*>(ws + cv.shards), reinterpret_cast<const u32*>(ws + cv.ptab),
                     HeavyArgs{pool.sbflag, pool.heavy, pool.nheavy,
                               geo.NC < kHeavyBlocks ? geo.NC : kHeavyBlocks}};
}

template <class Src>
void dispatch_csr_step(u32 wmax, const Geometry& geo, const Carve& cv, char* ws,
                       const CsrStepArgs& a, const Src& src, u64* stats, hipStream_t st) {
  const Cols buf2 = compact_at(ws + cv.buf2, nullptr, ws + cv.side2, side_flag_at(ws, cv));
  const u32* cs = reinterpret_cast<const u32*>(ws + cv.chunk_start);
  const u32* counts = reinterpret_cast<const u32*>(ws + cv.counts);
  u32* bar = reinterpret_cast<u32*>(ws + cv.flags) + 16;
  const unsigned grid = slow_blocks();
  switch (wmax) {
    case 4: launch_csr_step<4>(geo, buf2, counts, cs, a, src, bar, grid, stats, st); break;
    case 8: launch_csr_step<8>(geo, buf2, counts, cs, a, src, bar, grid, stats, st); break;
    case 12: launch_csr_step<12>(geo, buf2, counts, cs, a, src, bar, grid, stats, st); break;
    default: launch_csr_step<16>(geo, buf2, counts, cs, a, src, bar, grid, stats, st); break;
  }
}

}  // namespace bk
}  // namespace qb

using namespace qb;

namespace qb {
namespace bk {
u32 csr_wmax(uint32_t max_slots) {
  const u32 w = max_slots == 0 ? u32(QB_MAX_SLOTS) : max_slots;
  return w <= 4 ? 4u : w <= 8 ? 8u : w <= 12 ? 12u : 16u;
}
Geometry csr_geometry(uint64_t G, uint32_t max_slots, uint64_t M) {
  const u32 wmax = csr_wmax(max_slots);
  // the bucketing filters slot >= the table bound (geo.n) as non-member; the
  // chunk size follows the LDS run capacity (chunk_groups(wmax))
  Geometry geo = geometry(wmax, G, M, csr_chunk_groups(wmax), kSbIl);
  geo.n = max_slots == 0 ? u32(QB_MAX_SLOTS) : max_slots;
  return geo;
}
}  // namespace bk
namespace wt {
// The composed CSR step's apply half (qb_wire_tracker.hip): K5 and the slow
// path re-decoding a flagged chunk's messages from the bytes.
void csr_apply_wire(u32 wmax, const bk::Geometry& geo, const bk::Carve& cv, char* ws,
                    const u32* off, const u32* cfg, const u64* group_term, const u64* term_start,
                    u64* match, u64* next, u16* active, u64* committed, u32* stepdown_at,
                    u8* advanced, const WireArgs& W, u64* stats, hipStream_t st) {
  const bk::CsrStepArgs a = bk::csr_step_args(geo, cv, ws, W.ri, W.rt, off, cfg, group_term,
                                              term_start, match, next, active, committed,
                                              stepdown_at, advanced);
  bk::dispatch_csr_step(wmax, geo, cv, ws, a, WireSrc{W}, stats, st);
}
}  // namespace wt
}  // namespace qb
using bk::csr_wmax;

extern "C" size_t qb_csr_tracker_workspace_bytes(uint64_t G, uint32_t max_slots, uint64_t M) {
  if (max_slots > QB_MAX_SLOTS) return 0;
  const u32 w = csr_wmax(max_slots);
  const bk::Carve cv = bk::carve(bk::geometry(w, G, M, bk::csr_chunk_groups(w), bk::kSbIl), 1);
  return cv.nrec_all <= 0xFFFFFFFFull ? cv.total : 0;  // 0: no workspace fits (u32 record index)
}

extern "C" int qb_dev_csr_tracker_step(uint64_t G, uint32_t max_slots, const uint32_t* off,
                                       const uint32_t* cfg, uint64_t M, const uint32_t* rec_group,
                                       const uint8_t* rec_flags, const uint64_t* rec_index,
                                       const uint64_t* rec_term, const uint64_t* group_term,
                                       const uint64_t* term_start, uint64_t* match,
                                       uint64_t* next, uint16_t* active, uint64_t* committed,
                                       uint32_t* stepdown_at, uint8_t* advanced_out,
                                       uint64_t* stats, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  QB_REQUIRE(max_slots <= QB_MAX_SLOTS, "max_slots must be 0..%d", QB_MAX_SLOTS);
  QB_REQUIRE(M <= 0xFFFFFFFFull, "batch too large (M=%llu > 2^32-1)", (unsigned long long)M);
  QB_REQUIRE(G <= 0xFFFFFFFFull, "shard too large (G=%llu > 2^32-1)", (unsigned long long)G);
  if (G == 0) return QB_OK;
  QB_REQUIRE(off && cfg && group_term && term_start && match && active && committed &&
                 stepdown_at && stats,
             "required state pointer is NULL");
  QB_REQUIRE(M == 0 || (rec_group && rec_flags && rec_index && rec_term),
             "record pointer is NULL");
  const u32 wmax = csr_wmax(max_slots);
  const bk::Geometry geo = bk::csr_geometry(G, max_slots, M);
  const bk::Carve cv = bk::carve(geo, 1);
  QB_REQUIRE(cv.nrec_all <= 0xFFFFFFFFull,
             "batch too large for the bucket pass (M=%llu: %llu region records > 2^32-1)",
             (unsigned long long)M, (unsigned long long)cv.nrec_all);
  QB_REQUIRE(workspace && workspace_bytes >= cv.total,
             "workspace too small: need %zu bytes (qb_csr_tracker_workspace_bytes)", cv.total);
  QB_REQUIRE(geo.NSB <= 4096, "shard too large for the bucket pass (G=%llu)",
             (unsigned long long)G);
  hipStream_t st = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  u64* shards = reinterpret_cast<u64*>(ws + cv.shards);
  const auto* ri = reinterpret_cast<const u64*>(rec_index);
  const auto* rtm = reinterpret_cast<const u64*>(rec_term);
  {
    const int rc = bk::bucket_records(geo, cv, ws, rec_group, rec_flags, ri, rtm, shards, st,
                                      /*compact=*/true, reinterpret_cast<const u64*>(group_term),
                                      off);
    if (rc != QB_OK) return rc;
  }
  const bk::CsrStepArgs a = bk::csr_step_args(
      geo, cv, ws, ri, rtm, off, cfg, reinterpret_cast<const u64*>(group_term),
      reinterpret_cast<const u64*>(term_start), reinterpret_cast<u64*>(match),
      reinterpret_cast<u64*>(next), active, reinterpret_cast<u64*>(committed), stepdown_at,
      advanced_out);
  bk::dispatch_csr_step(wmax, geo, cv, ws, a, bk::ColSrc{rec_group, rec_flags, ri, rtm},
                        reinterpret_cast<u64*>(stats), st);
  QB_CHECK_LAUNCH("k_csr_apply / k_bk_slow");
  return QB_OK;
}
