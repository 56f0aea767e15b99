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
//   poll = RecordVote(slot, !reject): the first response of a slot wins,
//   then TallyVotes; at VoteWon / VoteLost the node changes state
//   (raft.go:1402-1414: a pre-candidate campaigns at term + 1, a candidate
//   becomes leader, a loser becomes follower) and polls nothing more; only a
//   response above its (possibly new) term still matters: it steps down.
// The vote state is the CSR votes word (voted | granted << 16).  First-wins
// in batch order is exact: a hash table sized to the batch keeps, per
// (group, slot) and per group's step-down, the minimum batch index (atomic
// min); the decision index is the minimum over polled records whose tally
// (rebuilt from the table) is decided; only the first poll of a slot at or
// before the decision writes.  The batch leaves the votes as they stood at the
// decision and reports decided_at / stepdown_at; the state change itself
// (campaign, becomeLeader, becomeFollower) is the host's.
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

// Before the group's decision: raft.Step's term filter for the candidate at
// the group term (a granted MsgPreVoteResp carries the future term and is
// polled without a term change, raft.go:866-871).
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

constexpr u32 kNone = 0xFFFFFFFFu;
constexpr u32 kSlotStepdown = 16;  // table key slot of the group's first pre-decision step-down

__device__ __forceinline__ u64 key_of(u32 g, u32 slot) { return (u64(g) << 5 | slot) + 1ull; }

// TallyVotes (tracker.go:267-288) -> JointConfig.VoteResult (joint.go:61-75)
// as it stands right after batch record i: the pre-batch votes word plus the
// first poll of every member slot not voted before the batch whose batch
// index is <= i (RecordVote keeps the first vote, tracker.go:258-263).
__device__ __forceinline__ u8 tally_at(Table tab, u32 g, u32 cfg, u32 votes0, u32 i,
                                       const u8* __restrict__ rf) {
  u32 vd = votes0 & 0xFFFFu, gr = (votes0 >> 16) & vd;
  const u32 min_ = cfg & 0xFFFFu, mout = cfg >> 16;
  for (u32 m = (min_ | mout) & ~vd; m; m &= m - 1u) {
    const u32 s = u32(__builtin_ctz(m));
    const u32 f = get(tab, key_of(g, s));
    if (f <= i) {
      vd |= 1u << s;
      if (!(rf[f] & QB_REC_REJECT)) gr |= 1u << s;
    }
  }
  const u8 r1 = vote_from_counts(__popc(min_), __popc(min_ & gr), __popc(min_ & vd));
  const u8 r2 = vote_from_counts(__popc(mout), __popc(mout & gr), __popc(mout & vd));
  return joint_vote(r1, r2);
}

constexpr unsigned kRecBlocks = 2048;

// Pass 1: per (group, slot) the first polled record, per group the first
// pre-decision step-down (atomic min of the batch index in the table).
__global__ __launch_bounds__(kBlock) void k_votes_index(int mode, u64 G, u64 M,
                                                        const u32* __restrict__ rg,
                                                        const u8* __restrict__ rf,
                                                        const u64* __restrict__ rt,
                                                        const u64* __restrict__ group_term,
                                                        Table tab) {
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i], f = rf[i];
    const int c = classify(mode, G, g, f, rt[i], group_term);
    if (c == V_HIGHER) put_min(tab, key_of(g, kSlotStepdown), u32(i));
    else if (c == V_POLL) put_min(tab, key_of(g, f & 0x0Fu), u32(i));
  }
}

// Pass 2: the decision point — the first polled record (before the first
// step-down) after which VoteResult is Won or Lost.  VoteResult is monotone
// in the recorded votes, so the decision is the minimum over every polled
// record whose tally is decided (raft.go:1400-1414: poll -> VoteWon / VoteLost).
__global__ __launch_bounds__(kBlock) void k_votes_decide(int mode, u64 G, u64 M,
                                                         const u32* __restrict__ rg,
                                                         const u8* __restrict__ rf,
                                                         const u64* __restrict__ rt,
                                                         const u64* __restrict__ group_term,
                                                         const u32* __restrict__ cfg,
                                                         const u32* __restrict__ votes, Table tab,
                                                         u32* __restrict__ decided_at) {
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i], f = rf[i];
    if (classify(mode, G, g, f, rt[i], group_term) != V_POLL) continue;
    if (get(tab, key_of(g, kSlotStepdown)) < u32(i)) continue;  // the candidate stepped down
    if (tally_at(tab, g, cfg[g], votes[g], u32(i), rf) != QB_VOTE_PENDING)
      atomicMin(decided_at + g, u32(i));
  }
}

// Pass 3: the step-down record.  Without a decision (or after a VoteLost /
// a candidate's VoteWon: the node stays at the group term, raft.go:1402-1414)
// it is the first pre-decision one.  After a pre-candidate's VoteWon the node
// campaigns at term + 1 (raft.go:1403-1404 -> becomeCandidate): only a
// rejection above that term makes it step down (raft.go:847-880).
__global__ __launch_bounds__(kBlock) void k_votes_stepdown(int mode, u64 G, u64 M,
                                                           const u32* __restrict__ rg,
                                                           const u8* __restrict__ rf,
                                                           const u64* __restrict__ rt,
                                                           const u64* __restrict__ group_term,
                                                           const u32* __restrict__ cfg,
                                                           const u32* __restrict__ votes,
                                                           Table tab,
                                                           const u32* __restrict__ decided_at,
                                                           u32* __restrict__ stepdown_at) {
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i], f = rf[i];
    if (g >= G) continue;
    const u64 t = rt[i], gt = group_term[g];
    const bool reject = (f & QB_REC_REJECT) != 0;
    const u32 dec = decided_at[g];
    const bool pre_higher = t > gt && (mode == QB_VOTE_MODE_VOTE || reject);
    const bool won_prevote = mode == QB_VOTE_MODE_PREVOTE && dec != kNone && u32(i) > dec &&
                             reject && t > gt + 1 && gt + 1 != 0 &&
                             tally_at(tab, g, cfg[g], votes[g], dec, rf) == QB_VOTE_WON;
    if (won_prevote) {
      atomicMin(stepdown_at + g, u32(i));
    } else if (pre_higher && get(tab, key_of(g, kSlotStepdown)) == u32(i)) {
      const bool prevote_won = mode == QB_VOTE_MODE_PREVOTE && dec != kNone &&
                               tally_at(tab, g, cfg[g], votes[g], dec, rf) == QB_VOTE_WON;
      if (!prevote_won) stepdown_at[g] = u32(i);
    }
  }
}

// Pass 4: RecordVote for the first poll of each slot at or before the
// decision and before the step-down; statistics per record.
__global__ __launch_bounds__(kBlock) void k_votes_apply(int mode, u64 G, u64 M,
                                                        const u32* __restrict__ rg,
                                                        const u8* __restrict__ rf,
                                                        const u64* __restrict__ rt,
                                                        const u64* __restrict__ group_term,
                                                        Table tab,
                                                        const u32* __restrict__ decided_at,
                                                        const u32* __restrict__ stepdown_at,
                                                        u32* __restrict__ votes,
                                                        u64* __restrict__ stats) {
  __shared__ u32 lds[7];
  BlockTally<7> tally;
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < M; i += stride) {
    const u32 g = rg[i], f = rf[i];
    const int c = classify(mode, G, g, f, rt[i], group_term);
    bool recorded = false, duplicate = false, after = false, after_dec = false, higher = false;
    bool stale = false;
    if (c != V_BAD) {
      const u32 sd = stepdown_at[g], dec = decided_at[g];
      if (sd < u32(i)) {
        after = true;
      } else if (sd == u32(i)) {
        higher = true;
      } else if (dec < u32(i)) {
        after_dec = true;  // the (pre-)candidate already won or lost
      } else if (c == V_STALE) {
        stale = true;
      } else if (c == V_POLL) {
        const u32 s = f & 0x0Fu;
        if (get(tab, key_of(g, s)) == u32(i)) {
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
    }
    tally.add(0, recorded);
    tally.add(1, duplicate);
    tally.add(2, stale);
    tally.add(3, higher);
    tally.add(4, after);
    tally.add(5, c == V_BAD);
    tally.add(6, after_dec);
  }
  const int slot[7] = {QB_VSTAT_RECORDED, QB_VSTAT_DUPLICATE, QB_VSTAT_STALE_TERM,
                       QB_VSTAT_HIGHER_TERM, QB_VSTAT_AFTER_STEPDOWN, QB_VSTAT_BAD,
                       QB_VSTAT_AFTER_DECISION};
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
                                   const uint64_t* group_term, const uint32_t* cfg, uint32_t* votes,
                                   uint32_t* stepdown_at, uint32_t* decided_at, uint64_t* stats,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  QB_REQUIRE(mode == QB_VOTE_MODE_VOTE || mode == QB_VOTE_MODE_PREVOTE, "bad mode %d", mode);
  QB_REQUIRE(M <= 0xFFFFFFFEull, "batch too large (M=%llu)", (unsigned long long)M);
  if (G == 0) return QB_OK;
  QB_REQUIRE(group_term && cfg && votes && stepdown_at && decided_at && stats,
             "required pointer is NULL");
  hipStream_t st = as_stream(stream);
  // outputs are self-initialising: no step-down, no decision
  hipError_t e = hipMemsetAsync(stepdown_at, 0xFF, sizeof(uint32_t) * G, st);
  if (e == hipSuccess) e = hipMemsetAsync(decided_at, 0xFF, sizeof(uint32_t) * G, st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(stepdown_at/decided_at)");
  if (M == 0) return QB_OK;
  QB_REQUIRE(rec_group && rec_flags && rec_term, "record pointer is NULL");
  const u64 cap = vt::capacity_for(M);
  const size_t need = qb_votes_workspace_bytes(M);
  QB_REQUIRE(workspace && workspace_bytes >= need,
             "workspace too small: need %zu bytes (qb_votes_workspace_bytes)", need);
  char* ws = static_cast<char*>(workspace);
  vt::Table tab{reinterpret_cast<u64*>(ws), reinterpret_cast<u32*>(ws + cap * sizeof(u64)),
                cap - 1};
  e = hipMemsetAsync(tab.key, 0, cap * sizeof(u64), st);
  if (e == hipSuccess) e = hipMemsetAsync(tab.val, 0xFF, cap * sizeof(u32), st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(vote table)");
  unsigned grid = grid_for(M);
  grid = grid < vt::kRecBlocks ? grid : vt::kRecBlocks;
  const u64* rt = reinterpret_cast<const u64*>(rec_term);
  const u64* gt = reinterpret_cast<const u64*>(group_term);
  hipLaunchKernelGGL(vt::k_votes_index, dim3(grid), dim3(kBlock), 0, st, mode, G, M, rec_group,
                     rec_flags, rt, gt, tab);
  QB_CHECK_LAUNCH("k_votes_index");
  hipLaunchKernelGGL(vt::k_votes_decide, dim3(grid), dim3(kBlock), 0, st, mode, G, M, rec_group,
                     rec_flags, rt, gt, cfg, votes, tab, decided_at);
  QB_CHECK_LAUNCH("k_votes_decide");
  hipLaunchKernelGGL(vt::k_votes_stepdown, dim3(grid), dim3(kBlock), 0, st, mode, G, M,
                     rec_group, rec_flags, rt, gt, cfg, votes, tab, decided_at, stepdown_at);
  QB_CHECK_LAUNCH("k_votes_stepdown");
  hipLaunchKernelGGL(vt::k_votes_apply, dim3(grid), dim3(kBlock), 0, st, mode, G, M, rec_group,
                     rec_flags, rt, gt, tab, decided_at, stepdown_at, votes,
                     reinterpret_cast<u64*>(stats));
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
