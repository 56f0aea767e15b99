// qb_votes.hip — batched elections: RecordVote / TallyVotes over G groups.
//
// Reference semantics (paths relative to the reference's raft/):
//   ProgressTracker.RecordVote   tracker/tracker.go:258-263 (first vote wins)
//   ProgressTracker.TallyVotes   tracker/tracker.go:267-288
//   raft.Step term filter        raft.go:847-921 (incl. the MsgPreVoteResp
//                                 exception at raft.go:866-871)
//   stepCandidate -> poll        raft.go:1391-1414, 837-845
//
// A batch holds the vote responses of one kind (MsgVoteResp for candidates,
// MsgPreVoteResp for pre-candidates).  Per record, in batch order, exactly as
// the sequential candidate:
//   term <  group term                     -> dropped (stale)
//   term >  group term, Vote mode          -> step down (becomeFollower)
//   term >  group term, PreVote, rejected  -> step down
//   term >  group term, PreVote, granted   -> poll (no term change)
//   term == group term                     -> poll
//   after the group's first step-down      -> ignored
//   poll = RecordVote(slot, !reject): the first response of a slot wins.
// The vote state is the CSR votes word (voted | granted << 16).  First-wins
// in batch order is exact: a hash table sized to the batch keeps, per
// (group, slot) and per group's step-down, the minimum batch index (atomic
// min), and only that record writes.
#include "qb_common.h"

namespace qb {
namespace vt {

struct Table {
  u64* key;   // (g << 5 | slot) + 1; 0 = empty; slot 16 = the group's step-down
  u32* val;   // minimum batch index
  u64 mask;   // capacity - 1 (power of two)
};

inline u64 capacity_for(u64 M) {
  u64 c = 1024;
  while (c < 2 * M) c <<= 1;
  return c;
}

__device__ __forceinline__ u64 hslot(u64 key, u64 mask) {
  return (key * 0x9E3779B97F4A7C15ull) >> 20 & mask;
}

__device__ __forceinline__ void put_min(Table t, u64 key, u32 idx) {
  u64 h = hslot(key, t.mask);
  for (u64 probe = 0; probe <= t.mask; ++probe) {
    const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(t.key + h), 0ull, key);
    if (prev == 0ull || prev == key) {
      atomicMin(t.val + h, idx);
      return;
    }
    h = (h + 1) & t.mask;
  }
}

__device__ __forceinline__ u32 get(Table t, u64 key) {
  u64 h = hslot(key, t.mask);
  for (u64 probe = 0; probe <= t.mask; ++probe) {
    const u64 k = t.key[h];
    if (k == key) return t.val[h];
    if (k == 0ull) return 0xFFFFFFFFu;
    h = (h + 1) & t.mask;
  }
  return 0xFFFFFFFFu;
}

enum Cls : int { V_POLL = 0, V_STALE = 1, V_HIGHER = 2, V_BAD = 3 };

__device__ __forceinline__ int classify(int mode, u64 G, u32 g, u32 f, u64 t,
                                        const u64* __restrict__ group_term) {
  if (g >= G) return V_BAD;
  const u64 gt = group_term[g];
  if (t < gt) return V_STALE;
  if (t > gt) {
    const bool reject = (f & QB_REC_REJECT) != 0;
    if (mode == QB_VOTE_MODE_PREVOTE && !reject) return V_POLL;  // raft.go:866-871
    return V_HIGHER;
  }
  return V_POLL;
}

constexpr unsigned kRecBlocks = 2048;

__global__ __launch_bounds__(kBlock) void k_votes_index(int mode, u64 G, u64 M,
                                                        const u32* __restrict__ rg,
                                                        const u8* __restrict__ rf,
                                                        const u64* __restrict__ rt,
                                                        const u64* __restrict__ group_term,
                                                        Table tab, u32* __restrict__ stepdown_at) {
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i], f = rf[i];
    const int c = classify(mode, G, g, f, rt[i], group_term);
    if (c == V_HIGHER) {
      put_min(tab, (u64(g) << 5 | 16u) + 1ull, u32(i));
      atomicMin(stepdown_at + g, u32(i));
    } else if (c == V_POLL) {
      put_min(tab, (u64(g) << 5 | (f & 0x0Fu)) + 1ull, u32(i));
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_votes_apply(int mode, u64 G, u64 M,
                                                        const u32* __restrict__ rg,
                                                        const u8* __restrict__ rf,
                                                        const u64* __restrict__ rt,
                                                        const u64* __restrict__ group_term,
                                                        Table tab, u32* __restrict__ votes,
                                                        u64* __restrict__ stats) {
  __shared__ u32 lds[6];
  BlockTally<6> tally;
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i], f = rf[i];
    const int c = classify(mode, G, g, f, rt[i], group_term);
    bool recorded = false, duplicate = false, after = false;
    if (c == V_POLL) {
      const u32 s = f & 0x0Fu;
      const u32 sd = get(tab, (u64(g) << 5 | 16u) + 1ull);  // first step-down, if any
      if (sd < u32(i)) {
        after = true;
      } else if (get(tab, (u64(g) << 5 | s) + 1ull) == u32(i)) {
        // the batch's first response of this slot: RecordVote (tracker.go:258-263)
        const u32 vbit = 1u << s;
        const u32 old = atomicOr(votes + g, vbit);
        if (old & vbit) {
          duplicate = true;  // voted before this batch
        } else {
          recorded = true;
          if (!(f & QB_REC_REJECT)) atomicOr(votes + g, vbit << 16);
        }
      } else {
        duplicate = true;  // an earlier response of this slot in the batch won
      }
    }
    tally.add(0, recorded);
    tally.add(1, duplicate);
    tally.add(2, c == V_STALE);
    tally.add(3, c == V_HIGHER);
    tally.add(4, after);
    tally.add(5, c == V_BAD);
  }
  const int slot[6] = {QB_VSTAT_RECORDED, QB_VSTAT_DUPLICATE, QB_VSTAT_STALE_TERM,
                       QB_VSTAT_HIGHER_TERM, QB_VSTAT_AFTER_STEPDOWN, QB_VSTAT_BAD};
  tally.flush(lds, stats, slot);
}

// TallyVotes (tracker.go:267-288): granted / rejected over every non-learner
// progress (either half's voters), and JointConfig.VoteResult.
__global__ __launch_bounds__(kBlock) void k_tally(u64 G, const u32* __restrict__ cfg,
                                                  const u32* __restrict__ votes,
                                                  u8* __restrict__ granted_out,
                                                  u8* __restrict__ rejected_out,
                                                  u8* __restrict__ result_out) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  const u32 c = cfg[g], w = votes[g];
  const u32 min_ = c & 0xFFFFu, mout = c >> 16, vd = w & 0xFFFFu, gr = (w >> 16) & vd;
  const u32 voters = min_ | mout;
  if (granted_out) granted_out[g] = u8(__popc(voters & gr));
  if (rejected_out) rejected_out[g] = u8(__popc(voters & vd & ~gr));
  if (result_out) {
    const u8 r1 = vote_from_counts(__popc(min_), __popc(min_ & gr), __popc(min_ & vd));
    const u8 r2 = vote_from_counts(__popc(mout), __popc(mout & gr), __popc(mout & vd));
    result_out[g] = joint_vote(r1, r2);
  }
}

}  // namespace vt
}  // namespace qb

using namespace qb;

extern "C" size_t qb_votes_workspace_bytes(uint64_t M) {
  const u64 cap = vt::capacity_for(M);
  return size_t(cap * sizeof(u64) + cap * sizeof(u32) + 256);
}

extern "C" int qb_dev_record_votes(int mode, uint64_t G, uint64_t M, const uint32_t* rec_group,
                                   const uint8_t* rec_flags, const uint64_t* rec_term,
                                   const uint64_t* group_term, uint32_t* votes,
                                   uint32_t* stepdown_at, uint64_t* stats, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  QB_REQUIRE(mode == QB_VOTE_MODE_VOTE || mode == QB_VOTE_MODE_PREVOTE, "bad mode %d", mode);
  QB_REQUIRE(M <= 0xFFFFFFFEull, "batch too large (M=%llu)", (unsigned long long)M);
  if (M == 0 || G == 0) return QB_OK;
  QB_REQUIRE(rec_group && rec_flags && rec_term && group_term && votes && stepdown_at && stats,
             "required pointer is NULL");
  const u64 cap = vt::capacity_for(M);
  const size_t need = qb_votes_workspace_bytes(M);
  QB_REQUIRE(workspace && workspace_bytes >= need,
             "workspace too small: need %zu bytes (qb_votes_workspace_bytes)", need);
  hipStream_t st = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  vt::Table tab{reinterpret_cast<u64*>(ws), reinterpret_cast<u32*>(ws + cap * sizeof(u64)),
                cap - 1};
  hipError_t e = hipMemsetAsync(tab.key, 0, cap * sizeof(u64), st);
  if (e == hipSuccess) e = hipMemsetAsync(tab.val, 0xFF, cap * sizeof(u32), st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(vote table)");
  unsigned grid = grid_for(M);
  grid = grid < vt::kRecBlocks ? grid : vt::kRecBlocks;
  const u64* rt = reinterpret_cast<const u64*>(rec_term);
  const u64* gt = reinterpret_cast<const u64*>(group_term);
  hipLaunchKernelGGL(vt::k_votes_index, dim3(grid), dim3(kBlock), 0, st, mode, G, M, rec_group,
                     rec_flags, rt, gt, tab, stepdown_at);
  QB_CHECK_LAUNCH("k_votes_index");
  hipLaunchKernelGGL(vt::k_votes_apply, dim3(grid), dim3(kBlock), 0, st, mode, G, M, rec_group,
                     rec_flags, rt, gt, tab, votes, reinterpret_cast<u64*>(stats));
  QB_CHECK_LAUNCH("k_votes_apply");
  return QB_OK;
}

extern "C" int qb_dev_csr_tally_votes(uint64_t G, const uint32_t* cfg, const uint32_t* votes,
                                      uint8_t* granted_out, uint8_t* rejected_out,
                                      uint8_t* result_out, void* stream) {
  if (G == 0) return QB_OK;
  QB_REQUIRE(cfg && votes, "cfg/votes NULL");
  hipLaunchKernelGGL(vt::k_tally, dim3(grid_for(G)), dim3(kBlock), 0, as_stream(stream), G, cfg,
                     votes, granted_out, rejected_out, result_out);
  QB_CHECK_LAUNCH("k_tally");
  return QB_OK;
}
