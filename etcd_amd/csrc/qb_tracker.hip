// qb_tracker.hip — ProgressTracker hot path over G groups (gfx950).
//
// Reference semantics (paths relative to the reference's raft/):
//   raft.Step term filter               raft.go:847-921
//   stepLeader MsgAppResp (quorum part) raft.go:1100-1109, 1237-1259
//   Progress.MaybeUpdate                tracker/progress.go:144-153
//   raft.maybeCommit                    raft.go:585-588
//   raftLog.maybeCommit / commitTo      log.go:328-334, 236-244
//   ProgressTracker.QuorumActive        tracker/tracker.go:215-225
#include <type_traits>

#include "qb_common.h"

namespace qb {

// ------------------------------------------------------------ QuorumActive --

// Every voter has a Progress, so votes[id] = RecentActive is present for
// each: yes = popcount(mask & active), voted = n (tracker.go:216-222).
__device__ __forceinline__ u8 quorum_active_one(u32 c, u32 a) {
  const u32 min_ = c & 0xFFFFu, mout = c >> 16;
  const u8 r1 = vote_from_counts(__popc(min_), __popc(min_ & a), __popc(min_));
  const u8 r2 = vote_from_counts(__popc(mout), __popc(mout & a), __popc(mout));
  return joint_vote(r1, r2) == QB_VOTE_WON ? 1 : 0;
}

// kQaGpt groups per thread: two 16-byte cfg loads, one 16-byte active load
// and one 8-byte store, all nontemporal (7 B/group streamed once); the
// thread-per-group form moved 1-4 bytes per lane and reached 4.2 TB/s.
// VEC needs 16-byte aligned cfg/active, 8-byte aligned won; the last
// partial group of 8 takes the scalar loop.
constexpr u32 kQaGpt = 8;
template <bool VEC>
__global__ __launch_bounds__(kBlock) void k_quorum_active(u64 G, const u32* __restrict__ cfg,
                                                          const u16* __restrict__ active,
                                                          u8* __restrict__ won) {
  const u64 g0 = (u64(blockIdx.x) * kBlock + threadIdx.x) * kQaGpt;
  if (g0 >= G) return;
  if (VEC && g0 + kQaGpt <= G) {
    using v4u = u32 __attribute__((ext_vector_type(4)));
    using v2u = u32 __attribute__((ext_vector_type(2)));
    const v4u c0 = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(cfg + g0));
    const v4u c1 = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(cfg + g0 + 4));
    const v4u a4 = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(active + g0));
    const u32 c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const u32 a[4] = {a4.x, a4.y, a4.z, a4.w};
    u32 w[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u32 ak = (a[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
      w[k >> 2] |= u32(quorum_active_one(c[k], ak)) << ((k & 3) * 8);
    }
    v2u out;
    out.x = w[0];
    out.y = w[1];
    __builtin_nontemporal_store(out, reinterpret_cast<v2u*>(won + g0));
    return;
  }
  const u64 g1 = g0 + kQaGpt < G ? g0 + kQaGpt : G;
  for (u64 g = g0; g < g1; ++g) won[g] = quorum_active_one(cfg[g], active[g]);
}

// ---------------------------------------------------------- MsgAppResp -----

enum RecClass : int {
  C_APPLY = 0, C_REJECT = 1, C_STALE = 2, C_NONMEMBER = 3, C_HIGHER = 4, C_BAD = 5,
};

__device__ __forceinline__ int classify(u32 n, u64 G, u64 g, u32 flags, u64 t,
                                        const u64* __restrict__ group_term) {
  if (g >= G) return C_BAD;
  if ((flags & 0x0Fu) >= n) return C_NONMEMBER;  // pr == nil (raft.go:1100-1104)
  const u64 gt = group_term[g];
  if (t < gt) return C_STALE;                    // raft.go:883-921: ignored
  if (t > gt) return C_HIGHER;                   // raft.go:875-879: becomeFollower
  return (flags & QB_REC_REJECT) ? C_REJECT : C_APPLY;
}

// Grid for the record kernels: grid-stride over M with at most kRecBlocks
// blocks, so the per-block counter flush stays cheap (BlockTally).
constexpr unsigned kRecBlocks = 2048;
inline unsigned rec_grid(u64 M) {
  const unsigned g = grid_for(M);
  return g < kRecBlocks ? g : kRecBlocks;
}

// Pass 1: the first higher-term record of each group (in batch order) makes
// the sequential leader step down; later records of that group never reach
// stepLeader.  Records the batch index of that first record and counts the
// higher-term records into stats[QB_STAT_HIGHER_TERM], which pass 2 reads as
// "some group may have stepped down".
__global__ __launch_bounds__(kBlock) void k_appresp_stepdown(
    u32 n, u64 G, u64 M, const u32* __restrict__ rg, const u8* __restrict__ rf,
    const u64* __restrict__ rt, const u64* __restrict__ group_term, u32* __restrict__ stepdown_at,
    u64* __restrict__ stats) {
  __shared__ u32 lds[1];
  BlockTally<1> tally;
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u64 g = rg[i];
    const bool higher = classify(n, G, g, rf[i], rt[i], group_term) == C_HIGHER;
    if (higher) atomicMin(stepdown_at + g, u32(i));
    tally.add(0, higher);
  }
  const int slot[1] = {QB_STAT_HIGHER_TERM};
  tally.flush(lds, stats, slot);
}

// Pass 2: MaybeUpdate as atomic max (commutative, so any arrival order gives
// the sequential end state), RecentActive as atomic or.
__global__ __launch_bounds__(kBlock) void k_appresp_apply(
    u32 n, u64 G, u64 M, const u32* __restrict__ rg, const u8* __restrict__ rf,
    const u64* __restrict__ ri, const u64* __restrict__ rt, const u64* __restrict__ group_term,
    u64* __restrict__ match, u64* __restrict__ next, u32* __restrict__ active_words,
    const u32* __restrict__ stepdown_at, u64* __restrict__ stats) {
  __shared__ u32 lds[6];
  const bool any_higher = stats[QB_STAT_HIGHER_TERM] != 0;  // uniform scalar load
  BlockTally<6> tally;
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u64 g = rg[i];
    const u32 f = rf[i];
    const int cls = classify(n, G, g, f, rt[i], group_term);
    bool after = false;
    if (cls == C_APPLY || cls == C_REJECT) {
      if (any_higher && stepdown_at[g] < u32(i)) {
        after = true;  // the leader already stepped down at an earlier record
      } else {
        const u32 s = f & 0x0Fu;
        // raft.go:1107: pr.RecentActive = true (reject or not).
        atomicOr(active_words + (g >> 1), (1u << s) << ((g & 1u) * 16u));
        if (cls == C_APPLY) {
          const u64 idx = ri[i];
          atomicMax(match + u64(s) * G + g, idx);                  // progress.go:146-150
          if (next) atomicMax(next + u64(s) * G + g, idx + 1ull);  // progress.go:151
        }
      }
    }
    tally.add(0, !after && cls == C_APPLY);
    tally.add(1, !after && cls == C_REJECT);
    tally.add(2, cls == C_STALE);
    tally.add(3, cls == C_NONMEMBER);
    tally.add(4, cls == C_BAD);
    tally.add(5, after);
  }
  const int slot[6] = {QB_STAT_APPLIED, QB_STAT_REJECTED, QB_STAT_STALE_TERM,
                       QB_STAT_NON_MEMBER, QB_STAT_BAD_GROUP, QB_STAT_AFTER_STEPDOWN};
  tally.flush(lds, stats, slot);
}

// ------------------------------------------------------- commit advance ----

template <int BYTES> struct RawT;
template <> struct RawT<8> { using T = u64; };
template <> struct RawT<16> { using T = u32 __attribute__((ext_vector_type(4))); };

// raft.maybeCommit -> raftLog.maybeCommit for every group.  GPT consecutive
// groups per thread so every slot row is one 16-byte load.
template <int N, int GPT>
__global__ __launch_bounds__(kBlock) void k_commit_advance(u64 G, const u64* __restrict__ match,
                                                           const u64* __restrict__ term_start,
                                                           u64* __restrict__ committed,
                                                           u8* __restrict__ advanced) {
  static_assert(GPT == 1 || GPT == 2, "GPT");
  using T = typename RawT<8 * GPT>::T;
  const u64 g0 = (u64(blockIdx.x) * kBlock + threadIdx.x) * GPT;
  if (g0 >= G) return;
  const int cnt = (g0 + GPT <= G) ? GPT : int(G - g0);
  u64 row[N][GPT], ts[GPT], cm[GPT];
  if (cnt == GPT) {
#pragma unroll
    for (int s = 0; s < N; ++s) {
      const T x = *reinterpret_cast<const T*>(match + u64(s) * G + g0);
      __builtin_memcpy(row[s], &x, 8 * GPT);
    }
    const T a = *reinterpret_cast<const T*>(term_start + g0);
    const T b = *reinterpret_cast<const T*>(committed + g0);
    __builtin_memcpy(ts, &a, 8 * GPT);
    __builtin_memcpy(cm, &b, 8 * GPT);
  } else {
#pragma unroll
    for (int k = 0; k < GPT; ++k) {
      const u64 g = k < cnt ? g0 + k : g0;
#pragma unroll
      for (int s = 0; s < N; ++s) row[s][k] = match[u64(s) * G + g];
      ts[k] = term_start[g];
      cm[k] = committed[g];
    }
  }
#pragma unroll
  for (int k = 0; k < GPT; ++k) {
    if (k >= cnt) break;
    u64 v[N];
#pragma unroll
    for (int s = 0; s < N; ++s) v[s] = row[s][k];
    const u64 ci = select_quorum<N>(v);
    // log.go:329: maxIndex > committed && term(maxIndex) == r.Term.
    const bool adv = ci > cm[k] && ci >= ts[k];
    if (adv) committed[g0 + k] = ci;  // commitTo never decreases (log.go:238)
    if (advanced) advanced[g0 + k] = adv ? 1 : 0;
  }
}

template <int N>
static void launch_commit_n(u64 G, const u64* match, const u64* ts, u64* cm, u8* adv,
                            hipStream_t st) {
  const bool vec = (G % 2) == 0 && (reinterpret_cast<uintptr_t>(match) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(ts) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(cm) % 16) == 0;
  if (vec)
    hipLaunchKernelGGL((k_commit_advance<N, 2>), dim3(grid_for((G + 1) / 2)), dim3(kBlock), 0,
                       st, G, match, ts, cm, adv);
  else
    hipLaunchKernelGGL((k_commit_advance<N, 1>), dim3(grid_for(G)), dim3(kBlock), 0, st, G,
                       match, ts, cm, adv);
}

template <int... Ns>
static void dispatch_commit(std::integer_sequence<int, Ns...>, int n, u64 G, const u64* match,
                            const u64* ts, u64* cm, u8* adv, hipStream_t st) {
  ((n == Ns + 1 ? launch_commit_n<Ns + 1>(G, match, ts, cm, adv, st) : void()), ...);
}

}  // namespace qb

using namespace qb;

extern "C" int qb_dev_csr_quorum_active(uint64_t G, const uint32_t* cfg, const uint16_t* active,
                                        uint8_t* won_out, void* stream) {
  if (G == 0) return QB_OK;
  QB_REQUIRE(cfg && active && won_out, "cfg/active/won_out NULL");
  const bool vec = (reinterpret_cast<uintptr_t>(cfg) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(active) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(won_out) % 8) == 0;
  const unsigned grid = grid_for((G + kQaGpt - 1) / kQaGpt);
  if (vec)
    hipLaunchKernelGGL(k_quorum_active<true>, dim3(grid), dim3(kBlock), 0, as_stream(stream), G,
                       cfg, active, won_out);
  else
    hipLaunchKernelGGL(k_quorum_active<false>, dim3(grid), dim3(kBlock), 0, as_stream(stream), G,
                       cfg, active, won_out);
  QB_CHECK_LAUNCH("k_quorum_active");
  return QB_OK;
}

extern "C" int qb_dev_fixed_apply_appresp(uint32_t n, uint64_t G, uint64_t M,
                                          const uint32_t* rec_group, const uint8_t* rec_flags,
                                          const uint64_t* rec_index, const uint64_t* rec_term,
                                          const uint64_t* group_term, uint64_t* match,
                                          uint64_t* next, uint16_t* active,
                                          uint32_t* stepdown_at, uint64_t* stats, void* stream) {
  QB_REQUIRE(n >= 1 && n <= QB_MAX_SLOTS, "n must be 1..%d", QB_MAX_SLOTS);
  if (M == 0 || G == 0) {
    if (G && stepdown_at) {
      const hipError_t e = hipMemsetAsync(stepdown_at, 0xFF, sizeof(uint32_t) * G, as_stream(stream));
      if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(stepdown_at)");
    }
    return QB_OK;
  }
  QB_REQUIRE(M <= 0xFFFFFFFFull, "batch too large (M=%llu > 2^32-1)", (unsigned long long)M);
  QB_REQUIRE(rec_group && rec_flags && rec_index && rec_term && group_term && match && active &&
                 stepdown_at && stats,
             "required pointer is NULL");
  QB_REQUIRE((reinterpret_cast<uintptr_t>(active) % 4) == 0, "active must be 4-byte aligned");
  hipStream_t st = as_stream(stream);
  // stepdown_at is self-initialising (every group UINT32_MAX, then pass 1's
  // atomic min), so a marker left from an earlier batch cannot shadow this
  // one; G * 4 bytes, small beside the record passes' atomics.
  {
    const hipError_t e = hipMemsetAsync(stepdown_at, 0xFF, sizeof(uint32_t) * G, st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(stepdown_at)");
  }
  const dim3 grid(rec_grid(M));
  hipLaunchKernelGGL(k_appresp_stepdown, grid, dim3(kBlock), 0, st, n, G, M, rec_group, rec_flags,
                     reinterpret_cast<const u64*>(rec_term),
                     reinterpret_cast<const u64*>(group_term), stepdown_at,
                     reinterpret_cast<u64*>(stats));
  QB_CHECK_LAUNCH("k_appresp_stepdown");
  hipLaunchKernelGGL(k_appresp_apply, grid, dim3(kBlock), 0, st, n, G, M, rec_group, rec_flags,
                     reinterpret_cast<const u64*>(rec_index),
                     reinterpret_cast<const u64*>(rec_term),
                     reinterpret_cast<const u64*>(group_term), reinterpret_cast<u64*>(match),
                     reinterpret_cast<u64*>(next), reinterpret_cast<u32*>(active), stepdown_at,
                     reinterpret_cast<u64*>(stats));
  QB_CHECK_LAUNCH("k_appresp_apply");
  return QB_OK;
}

extern "C" int qb_dev_fixed_commit_advance(uint32_t n, uint64_t G, const uint64_t* match,
                                           const uint64_t* term_start, uint64_t* committed,
                                           uint8_t* advanced_out, void* stream) {
  QB_REQUIRE(n >= 1 && n <= QB_MAX_SLOTS, "n must be 1..%d", QB_MAX_SLOTS);
  if (G == 0) return QB_OK;
  QB_REQUIRE(match && term_start && committed, "required pointer is NULL");
  dispatch_commit(std::make_integer_sequence<int, QB_MAX_SLOTS>{}, int(n), G,
                  reinterpret_cast<const u64*>(match), reinterpret_cast<const u64*>(term_start),
                  reinterpret_cast<u64*>(committed), advanced_out, as_stream(stream));
  QB_CHECK_LAUNCH("k_commit_advance");
  return QB_OK;
}

namespace qb {
// Entries of stepdown_at that are not UINT32_MAX: a ballot per wave, one
// atomic per wave with any (the check is for a caller's debug builds and
// its once-per-config-change paths, not the tick).
__global__ void k_stepdown_unarmed(u64 G, const u32* __restrict__ sd, u64* __restrict__ bad) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  const u64 m = __ballot(g < G && sd[g] != 0xFFFFFFFFu);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, u64(__popcll(m)));
}
}  // namespace qb

extern "C" int qb_dev_stepdown_check_armed(uint64_t G, const uint32_t* stepdown_at,
                                           uint64_t* bad_scratch, void* stream) {
  if (G == 0) return QB_OK;
  QB_REQUIRE(stepdown_at && bad_scratch, "stepdown_at/bad_scratch NULL");
  hipStream_t st = as_stream(stream);
  hipError_t e = hipMemsetAsync(bad_scratch, 0, sizeof(uint64_t), st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(bad)");
  hipLaunchKernelGGL(k_stepdown_unarmed, dim3(grid_for(G)), dim3(kBlock), 0, st, G, stepdown_at,
                     reinterpret_cast<u64*>(bad_scratch));
  QB_CHECK_LAUNCH("k_stepdown_unarmed");
  uint64_t bad = 0;
  e = hipMemcpyAsync(&bad, bad_scratch, sizeof bad, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "stepdown check readback");
  QB_REQUIRE(bad == 0,
             "%llu group(s) enter the bucketed tracker step with stepdown_at != UINT32_MAX "
             "(re-arm the groups that stepped down)",
             (unsigned long long)bad);
  return QB_OK;
}
