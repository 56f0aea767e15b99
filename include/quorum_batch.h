/*
 * quorum_batch.h — C ABI of libquorumbatch, the MI355X batched quorum engine.
 *
 * This is the drop-in boundary for etcd's raft quorum/tracker hot path
 * evaluated over G independent raft groups at once.  It is the ABI a
 * ``raft/quorum/batch`` cgo package binds; every entry
 * point names the reference interface it replaces (paths relative to the
 * reference's ``raft/``).  Plain C types only: no torch, no HIP types.
 *
 * Conventions (mirroring the reference):
 *   - Every call returns int: QB_OK (0) or a negative QB_E* code; the text of
 *     the most recent failure on the calling thread is qb_last_error().
 *   - Quorum semantics never error: an empty majority config yields
 *     QB_INDEX_INF (MaxUint64) and VoteWon, exactly as majority.go:128-133 and
 *     majority.go:179-184.  Only malformed inputs (bad sizes, null required
 *     pointers, HIP failures) produce an error code.
 *   - Indexes are quorum.Index (uint64, unsigned compare over the full range);
 *     vote results are quorum.VoteResult: 1 Pending, 2 Lost, 3 Won
 *     (quorum.go:45-58).
 *   - "qb_dev_*" calls take DEVICE pointers and a hipStream_t passed as
 *     void* (NULL = the null stream); they only enqueue work.  Ownership stays
 *     with the caller.  One stream per host thread; no internal locking
 *     (single owner, like raft's RawNode, rawnode.go:31).
 *
 * Device layouts (structure of arrays, all little-endian):
 *
 *   FIXED  (every group is one n-voter MajorityConfig, 1 <= n <= 16, no
 *           learners; slot j = the j-th smallest voter ID, MajorityConfig.Slice
 *           majority.go:106-113):
 *     match[n][G]   uint64, slot-major: match[j*G + g] = Progress.Match
 *     voted[G], granted[G]   bitmask per group, bit j = slot j; uint8 when
 *                   n <= 8, uint16 when n > 8.  granted bits count only where
 *                   the voted bit is set (votes map: present -> voted).
 *
 *   CSR    (ragged: voters + learners, joint configs; 0 <= s_g <= 16 slots;
 *           s_g == 0 is the empty config):
 *     off[G+1]      uint32, slots of group g are off[g] .. off[g+1]-1
 *     match[off[G]] uint64, group-major
 *     cfg[G]        uint32 = mask_in | mask_out << 16  (JointConfig halves
 *                   Voters[0] / Voters[1], tracker.go:27-78; a slot with
 *                   neither bit is a learner; mask_out == 0 is a plain
 *                   majority config — identical results by joint.go:49-56)
 *     votes[G]      uint32 = voted | granted << 16
 *     active[G]     uint16 RecentActive bits (tracker.go:215-225)
 *
 *   WIDE   (configs with more than 16 slots, up to QB_WIDE_MAX_SLOTS; one
 *           wavefront per group):
 *     off[G+1]      uint32, match[off[G]] uint64 as CSR
 *     flags[off[G]] uint8 per slot: bit 0 incoming voter, bit 1 outgoing
 *                   voter, bit 2 voted, bit 3 granted
 *
 *   MsgAppResp batch records (M records, any order):
 *     rec_group[M]  uint32 group index within the shard
 *     rec_flags[M]  uint8: bits 0-3 = slot, bit 7 = Reject
 *     rec_index[M]  uint64 Message.Index
 *     rec_term[M]   uint64 Message.Term
 */
#ifndef QUORUM_BATCH_H
#define QUORUM_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QB_ABI_VERSION 1

#define QB_OK 0
#define QB_EINVAL (-1)   /* malformed arguments */
#define QB_EHIP (-2)     /* HIP runtime error (text in qb_last_error) */
#define QB_ENOMEM (-3)   /* device allocation failed */

#define QB_INDEX_INF UINT64_MAX  /* quorum.Index "∞", quorum.go:25-30 */

#define QB_VOTE_PENDING 1  /* quorum.VotePending, quorum.go:53 */
#define QB_VOTE_LOST 2     /* quorum.VoteLost,    quorum.go:55 */
#define QB_VOTE_WON 3      /* quorum.VoteWon,     quorum.go:57 */

#define QB_MAX_SLOTS 16
#define QB_WIDE_MAX_SLOTS 1024
#define QB_REC_REJECT 0x80u
#define QB_REC_NO_PROGRESS 0x40u /* leader inbox: From has no Progress (wire ingest) */

/* Counters filled by qb_dev_fixed_apply_appresp (device memory, uint64 each;
 * accumulated, so zero them before a batch if per-batch numbers are wanted). */
enum {
  QB_STAT_APPLIED = 0,     /* non-reject, same-term, member: MaybeUpdate ran   */
  QB_STAT_REJECTED = 1,    /* Reject=true: RecentActive only (raft.go:1107-1109) */
  QB_STAT_STALE_TERM = 2,  /* m.Term < group term: dropped (raft.go:883-921)    */
  QB_STAT_NON_MEMBER = 3,  /* no Progress for the slot: dropped (raft.go:1100) */
  QB_STAT_HIGHER_TERM = 4, /* m.Term > group term: leader steps down (raft.go:852-880) */
  QB_STAT_BAD_GROUP = 5,   /* group index >= G: dropped                        */
  QB_STAT_AFTER_STEPDOWN = 6, /* same-term record behind a higher-term one     */
  QB_STAT_COUNT = 8
};

/* Counters filled by qb_dev_record_votes (device uint64 each, accumulated). */
enum {
  QB_VSTAT_RECORDED = 0,       /* RecordVote stored the slot's first vote        */
  QB_VSTAT_DUPLICATE = 1,      /* the slot had already voted (first vote wins)   */
  QB_VSTAT_STALE_TERM = 2,     /* m.Term < group term: dropped                   */
  QB_VSTAT_HIGHER_TERM = 3,    /* the candidate steps down (raft.go:872-879)     */
  QB_VSTAT_AFTER_STEPDOWN = 4, /* any record behind the group's step-down        */
  QB_VSTAT_BAD = 5,            /* group index >= G                               */
  QB_VSTAT_AFTER_DECISION = 6, /* behind the group's VoteWon / VoteLost          */
  QB_VSTAT_COUNT = 8
};

#define QB_VOTE_MODE_VOTE 0     /* MsgVoteResp to a candidate (raft.go:1391) */
#define QB_VOTE_MODE_PREVOTE 1  /* MsgPreVoteResp to a pre-candidate         */

/* ----------------------------------------------------------------------- */
/* Library                                                                 */
/* ----------------------------------------------------------------------- */

int qb_abi_version(void);
/* Text of the last error on this thread ("" if none). */
const char* qb_last_error(void);
/* Number of visible HIP devices (0 without a GPU); never fails. */
int qb_device_count(void);

/* Device memory and streams for callers without their own HIP runtime
 * bindings (the Go cgo package).  Thin wrappers over hipMalloc / hipFree /
 * hipMemcpyAsync / hipStreamCreate; *_async copies are ordered on the stream
 * and the host buffer must stay alive until qb_stream_sync returns. */
int qb_set_device(int device);
int qb_malloc(size_t bytes, void** out);
int qb_free(void* ptr);
int qb_memset_async(void* dst, int value, size_t bytes, void* stream);
int qb_copy_h2d_async(void* dst, const void* src, size_t bytes, void* stream);
int qb_copy_d2h_async(void* dst, const void* src, size_t bytes, void* stream);
int qb_stream_create(void** out);
int qb_stream_destroy(void* stream);
int qb_stream_sync(void* stream);

/* ----------------------------------------------------------------------- */
/* Config compile (host)                                                   */
/* ----------------------------------------------------------------------- */

/* tracker.Config per group (tracker/tracker.go:27-78) -> the CSR layout:
 * slots = the sorted union of Voters[0], Voters[1] and Learners (the order of
 * MajorityConfig.Slice, quorum/majority.go:106-113; LearnersNext members are
 * outgoing voters until LeaveJoint, so they are in Voters[1]); cfg[g] =
 * mask_in | mask_out << 16 over those slots; a learner is in neither mask.
 * Each input is a CSR of IDs: group g's Voters[0] are in_ids[in_off[g] ..
 * in_off[g+1]) (out_off/out_ids, lrn_off/lrn_ids nullable = empty sets);
 * duplicate IDs within a list are one member.  Writes off[G+1], cfg[G] and,
 * if slot_ids is non-NULL, the slot IDs (slot_cap entries available; call
 * once with slot_ids NULL to size it: off[G] = slots needed).  A group whose
 * learners intersect its voters (confchange.go:307-318: "%d is in Learners
 * and Voters[1]" / "[0]") or with more than QB_MAX_SLOTS members fails the
 * call with QB_EINVAL, *bad_group (nullable) = the first such group and the
 * reference's message in qb_last_error().  Host memory only; no device. */
int qb_host_compile_configs(uint64_t G, const uint32_t* in_off, const uint64_t* in_ids,
                            const uint32_t* out_off, const uint64_t* out_ids,
                            const uint32_t* lrn_off, const uint64_t* lrn_ids,
                            uint32_t* off, uint32_t* cfg, uint64_t* slot_ids,
                            uint64_t slot_cap, uint64_t* bad_group);

/* ----------------------------------------------------------------------- */
/* Quorum math (raft/quorum)                                               */
/* ----------------------------------------------------------------------- */

/* CommittedIndex and/or VoteResult for G groups of one n-voter
 * MajorityConfig shape (FIXED layout).
 * Replaces MajorityConfig.CommittedIndex (quorum/majority.go:126-172) and
 * MajorityConfig.VoteResult (quorum/majority.go:178-210).
 * n == 0 fills commit_out with QB_INDEX_INF and vote_out with VoteWon.
 * commit_out and/or vote_out may be NULL to skip that result; voted/granted
 * may be NULL only when vote_out is NULL. */
int qb_dev_fixed_committed_vote(uint32_t n, uint64_t G, const uint64_t* match,
                                const void* voted, const void* granted,
                                uint64_t* commit_out, uint8_t* vote_out,
                                void* stream);

/* Several FIXED batches of one shape in one call (one cgo call per tick for
 * an embedder holding several shards' batches, instead of one per batch):
 * batch i is qb_dev_fixed_committed_vote(n, G, batches[i]...) enqueued on
 * streams[i % nstreams] (nstreams >= 1; a NULL entry is the default stream),
 * in order; stops at the first failing batch and returns its code. */
typedef struct qb_fixed_batch {
  const uint64_t* match;  /* [n][G] */
  const void* voted;      /* [G] u8 (n <= 8) or u16 */
  const void* granted;
  uint64_t* commit_out;   /* [G] or NULL */
  uint8_t* vote_out;      /* [G] or NULL */
} qb_fixed_batch;
int qb_dev_fixed_committed_vote_batches(uint32_t n, uint64_t G, uint32_t count,
                                        const qb_fixed_batch* batches, void* const* streams,
                                        uint32_t nstreams);

/* CommittedIndex and/or VoteResult for G ragged/joint groups (CSR layout).
 * Replaces JointConfig.CommittedIndex (quorum/joint.go:49-56) and
 * JointConfig.VoteResult (quorum/joint.go:61-75), which reduce to the
 * MajorityConfig forms when mask_out == 0; learners are slots in neither mask
 * and never count (tracker.go:273, majority.go:186-200).
 * max_slots bounds every s_g of the table (0 = QB_MAX_SLOTS); it sizes the
 * kernel (LDS and networks), so pass the table's true bound: a group above it
 * gives an unspecified (never out-of-bounds) result, which
 * qb_dev_csr_validate detects (qb_dev_csr_committed_vote_checked: validate,
 * then QB_EINVAL instead of a result). */
int qb_dev_csr_committed_vote(uint64_t G, uint32_t max_slots,
                              const uint32_t* off, const uint64_t* match,
                              const uint32_t* cfg, const uint32_t* votes,
                              uint64_t* commit_out, uint8_t* vote_out,
                              void* stream);

/* Checks a CSR table: off[0] == 0 and 0 <= off[g+1] - off[g] <= max_slots
 * (0 = QB_MAX_SLOTS).  Writes the number of bad groups to *bad_out (device
 * uint64). */
int qb_dev_csr_validate(uint64_t G, uint32_t max_slots, const uint32_t* off,
                        uint64_t* bad_out, void* stream);

/* qb_dev_csr_committed_vote behind an opt-in validation: the table is checked
 * first (qb_dev_csr_validate into bad_scratch, one device uint64) and a table
 * breaking its bound returns QB_EINVAL — with the count in qb_last_error() —
 * and computes nothing.  It reads the verdict back, so it synchronises the
 * stream: a debug / once-per-config-change form, not the per-tick call. */
int qb_dev_csr_committed_vote_checked(uint64_t G, uint32_t max_slots,
                                      const uint32_t* off, const uint64_t* match,
                                      const uint32_t* cfg, const uint32_t* votes,
                                      uint64_t* commit_out, uint8_t* vote_out,
                                      uint64_t* bad_scratch, void* stream);

/* CommittedIndex and/or VoteResult for G WIDE groups (JointConfig
 * semantics as qb_dev_csr_committed_vote, quorum/joint.go:49-75 over
 * quorum/majority.go:126-210).  max_slots bounds every s_g (0 =
 * QB_WIDE_MAX_SLOTS) and sizes the per-lane register tile. */
int qb_dev_wide_committed_vote(uint64_t G, uint32_t max_slots,
                               const uint32_t* off, const uint64_t* match,
                               const uint8_t* flags, uint64_t* commit_out,
                               uint8_t* vote_out, void* stream);
int qb_dev_wide_validate(uint64_t G, uint32_t max_slots, const uint32_t* off,
                         uint64_t* bad_out, void* stream);

/* ----------------------------------------------------------------------- */
/* Progress tracking (raft/tracker)                                        */
/* ----------------------------------------------------------------------- */

/* ProgressTracker.QuorumActive (tracker/tracker.go:215-225) per group:
 * won_out[g] = 1 iff VoteResult(votes = RecentActive of every voter) is
 * VoteWon in both halves. */
int qb_dev_csr_quorum_active(uint64_t G, const uint32_t* cfg,
                             const uint16_t* active, uint8_t* won_out,
                             void* stream);

/* Apply a batch of MsgAppResp records to FIXED-layout leader state — the
 * quorum-facing part of stepLeader's MsgAppResp case (raft.go:1100-1109,
 * 1237-1239): Progress.MaybeUpdate (tracker/progress.go:144-153) as an
 * atomic scatter-max of match (and next, if non-NULL), RecentActive bits,
 * and the term filter of raft.Step (raft.go:847-921).  Batch-equivalent to
 * applying the records one by one in index order.
 *   group_term[G]   the leader's current term per group
 *   match[n][G], next[n][G] (nullable), active[G] (uint16 bits; the array
 *                   must be 4-byte aligned and padded to an even length)
 *   stepdown_at[G]  uint32 output, written for every group (no entry
 *                   requirement): the batch index of the first higher-term
 *                   record of a group that must step down (raft.go:875-879),
 *                   UINT32_MAX otherwise.  Records after it are not applied,
 *                   as in the sequential reference.
 *   stats[QB_STAT_COUNT] device uint64 counters (required; zero them per
 *                   batch — a non-zero HIGHER_TERM count only makes the
 *                   apply pass consult stepdown_at, it never changes results). */
int qb_dev_fixed_apply_appresp(uint32_t n, uint64_t G, uint64_t M,
                               const uint32_t* rec_group,
                               const uint8_t* rec_flags,
                               const uint64_t* rec_index,
                               const uint64_t* rec_term,
                               const uint64_t* group_term, uint64_t* match,
                               uint64_t* next, uint16_t* active,
                               uint32_t* stepdown_at, uint64_t* stats,
                               void* stream);

/* raft.maybeCommit (raft.go:585-588) -> raftLog.maybeCommit (log.go:328-334)
 * for every group of the FIXED layout: committed[g] = CI if CI > committed[g]
 * and term(CI) == Term, where term(CI) == Term <=> CI >= term_start[g]
 * (term_start = first index of the leader's current term, QB_INDEX_INF if the
 * leader has none; CI <= lastIndex holds because no voter acks past the
 * leader's log).  advanced_out[g] (nullable) = 1 where the commit moved
 * (maybeCommit's return value). */
int qb_dev_fixed_commit_advance(uint32_t n, uint64_t G, const uint64_t* match,
                                const uint64_t* term_start,
                                uint64_t* committed, uint8_t* advanced_out,
                                void* stream);

/* One leader tick for G groups of the FIXED layout: a batch of MsgAppResp
 * records applied (same semantics as qb_dev_fixed_apply_appresp) and
 * maybeCommit run for every group (as qb_dev_fixed_commit_advance), fused.
 * The records are bucketed by group on the device (counting sort into
 * LDS-sized chunks) so every MaybeUpdate is an LDS atomic; this is the path
 * for large batches (M ~ G).  Differences from the two-call form:
 *   - stepdown_at[g] must hold UINT32_MAX on entry (the two-call form
 *     initialises it itself) and is written only where it can change: for
 *     every group of a chunk (256-512 consecutive groups) holding a
 *     higher-term record it is reset to UINT32_MAX and then receives the
 *     step-down record's batch index; every other entry is left untouched
 *     (no per-group write in the steady state).  A caller re-arming a group
 *     that stepped down resets its entry; stats[QB_STAT_HIGHER_TERM] > 0 says
 *     whether any group stepped down;
 *   - workspace: device scratch of qb_fixed_tracker_workspace_bytes(n, G, M)
 *     bytes (caller-owned, reusable across calls of the same or smaller
 *     size; no allocation inside, so the call can be graph-captured).
 * Requires G, M < 2^32, and a batch whose reserved regions (about 2 x M
 * records) stay below 2^32 records: qb_fixed_tracker_workspace_bytes
 * returns 0 for a larger one and the step QB_EINVAL.
 * qb_dev_stepdown_check_armed is the opt-in check of that entry rule (for a
 * caller's debug builds): it counts the entries != UINT32_MAX on the device,
 * synchronises the stream and returns QB_EINVAL naming the count if any
 * (bad_scratch: one device uint64). */
int qb_dev_stepdown_check_armed(uint64_t G, const uint32_t* stepdown_at,
                                uint64_t* bad_scratch, void* stream);
size_t qb_fixed_tracker_workspace_bytes(uint32_t n, uint64_t G, uint64_t M);
int qb_dev_fixed_tracker_step(uint32_t n, uint64_t G, uint64_t M,
                              const uint32_t* rec_group,
                              const uint8_t* rec_flags,
                              const uint64_t* rec_index,
                              const uint64_t* rec_term,
                              const uint64_t* group_term,
                              const uint64_t* term_start, uint64_t* match,
                              uint64_t* next, uint16_t* active,
                              uint64_t* committed, uint32_t* stepdown_at,
                              uint8_t* advanced_out, uint64_t* stats,
                              void* workspace, size_t workspace_bytes,
                              void* stream);

/* qb_dev_fixed_tracker_step in two halves, for a caller that pipelines
 * ticks: _bucket sorts a batch by group into a workspace (reads only the
 * batch: K3-K4, no leader state — so, unlike the step, it does not fold a
 * hot group's repeated records, which needs the group terms), _apply
 * applies that workspace's batch to
 * the state (K5 + the exact slow path; the same batch pointers, which the
 * slow path re-reads).  step == bucket then apply on one stream.  With two
 * workspaces on two streams, tick k+1's bucketing can run while tick k is
 * applied: the caller orders apply(k+1) after bucket(k+1) and apply(k), and
 * bucket(k+2) after apply(k) (workspace reuse).  Each workspace carries its
 * own statistic shards, folded into `stats` by _apply.  (On one MI355X the
 * overlap measured slower than back-to-back steps, 706-712 vs 672-674 us per
 * 16M-group tick: the concurrent kernels contend for the CUs and HBM; the
 * split is for callers that interleave other work between the halves.) */
int qb_dev_fixed_tracker_bucket(uint32_t n, uint64_t G, uint64_t M,
                                const uint32_t* rec_group,
                                const uint8_t* rec_flags,
                                const uint64_t* rec_index,
                                const uint64_t* rec_term,
                                void* workspace, size_t workspace_bytes,
                                void* stream);
int qb_dev_fixed_tracker_apply(uint32_t n, uint64_t G, uint64_t M,
                               const uint32_t* rec_group,
                               const uint8_t* rec_flags,
                               const uint64_t* rec_index,
                               const uint64_t* rec_term,
                               const uint64_t* group_term,
                               const uint64_t* term_start, uint64_t* match,
                               uint64_t* next, uint16_t* active,
                               uint64_t* committed, uint32_t* stepdown_at,
                               uint8_t* advanced_out, uint64_t* stats,
                               void* workspace, size_t workspace_bytes,
                               void* stream);

/* The same leader tick over G groups of the CSR layout (ragged voter
 * counts, learners, joint configs): a MsgAppResp batch applied (MaybeUpdate on
 * the slot's Progress, learners included; a slot >= s_g has no Progress and
 * is dropped before the term filter, node.go:356-360) and maybeCommit for
 * every group with ProgressTracker.Committed = JointConfig.CommittedIndex
 * over the voters of both halves (tracker/tracker.go:162-179,
 * quorum/joint.go:49-56) — the commit advance a joint transition runs on
 * every ack (raft.go:1259, 1682).  An empty config (both masks 0) never
 * commits: its CommittedIndex is MaxUint64, past lastIndex, whose term is 0
 * (log.go:271-273, 328-334).
 *   off[G+1], cfg[G]   CSR config as qb_dev_csr_committed_vote; max_slots
 *                      bounds every s_g (0 = QB_MAX_SLOTS) and sizes the
 *                      kernel (a chunk whose slot run breaks the bound is
 *                      applied by the exact slow path);
 *   match[off[G]], next[off[G]] (nullable)  Progress per slot;
 *   group_term, term_start, active, committed, stepdown_at, advanced_out,
 *   stats, workspace: as qb_dev_fixed_tracker_step (same stepdown_at rule). */
size_t qb_csr_tracker_workspace_bytes(uint64_t G, uint32_t max_slots, uint64_t M);
int qb_dev_csr_tracker_step(uint64_t G, uint32_t max_slots, const uint32_t* off,
                            const uint32_t* cfg, uint64_t M,
                            const uint32_t* rec_group, const uint8_t* rec_flags,
                            const uint64_t* rec_index, const uint64_t* rec_term,
                            const uint64_t* group_term,
                            const uint64_t* term_start, uint64_t* match,
                            uint64_t* next, uint16_t* active,
                            uint64_t* committed, uint32_t* stepdown_at,
                            uint8_t* advanced_out, uint64_t* stats,
                            void* workspace, size_t workspace_bytes,
                            void* stream);

/* Elections.  A batch of vote responses of one kind (mode), records
 * {group, flags = slot | reject << 7, term} in batch order, applied to the
 * CSR votes words (voted | granted << 16) exactly as the sequential
 * (pre-)candidate does: raft.Step's term filter (raft.go:847-921, with the
 * MsgPreVoteResp exception of raft.go:866-871), stepCandidate -> poll ->
 * RecordVote with first-vote-wins (tracker/tracker.go:258-263) and
 * TallyVotes against cfg (mask_in | mask_out << 16, learners in neither).
 * At the first response after which the result is VoteWon / VoteLost the
 * node changes state (raft.go:1402-1414) and polls nothing more:
 *   decided_at[g]  batch index of that response (UINT32_MAX: still pending);
 *                  votes[g] is left as it stood there, so
 *                  qb_dev_csr_tally_votes gives the decision;
 *   stepdown_at[g] batch index of the response that makes the node
 *                  becomeFollower at a higher term (UINT32_MAX: none): before
 *                  the decision any response above the group term (a granted
 *                  MsgPreVoteResp excepted); after a pre-candidate's VoteWon
 *                  the node campaigned at term + 1 (raft.go:1403 ->
 *                  becomeCandidate), so only a rejection above term + 1; after
 *                  a candidate's VoteWon / any VoteLost, a response above the
 *                  group term.  Nothing after the step-down is applied.
 * Both outputs are written for every group (no entry requirement).  The
 * state change itself (campaign with ResetVotes, becomeLeader, becomeFollower)
 * is the host's.  workspace: qb_votes_workspace_bytes(M) bytes of device
 * scratch. */
size_t qb_votes_workspace_bytes(uint64_t M);
int qb_dev_record_votes(int mode, uint64_t G, uint64_t M,
                        const uint32_t* rec_group, const uint8_t* rec_flags,
                        const uint64_t* rec_term, const uint64_t* group_term,
                        const uint32_t* cfg, uint32_t* votes, uint32_t* stepdown_at,
                        uint32_t* decided_at, uint64_t* stats,
                        void* workspace, size_t workspace_bytes, void* stream);

/* ProgressTracker.TallyVotes (tracker/tracker.go:267-288) per group:
 * granted / rejected among the voters of either half (learners never count)
 * and JointConfig.VoteResult.  Any output may be NULL. */
int qb_dev_csr_tally_votes(uint64_t G, const uint32_t* cfg,
                           const uint32_t* votes, uint8_t* granted_out,
                           uint8_t* rejected_out, uint8_t* result_out,
                           void* stream);

/* ----------------------------------------------------------------------- */
/* Leader inbox step                              */
/* ----------------------------------------------------------------------- */

/* The full leader side of the responses in a raft leader's inbox, for G
 * groups at once, with the reference's sequential per-message semantics:
 *   raft.Step term filter (raft.go:847-921), stepLeader (raft.go:1099-1342):
 *   MsgAppResp reject -> findConflictByTerm (log.go:150-171) + MaybeDecrTo
 *     (progress.go:163-191) + BecomeProbe + sendAppend;
 *   MsgAppResp accept -> MaybeUpdate, Probe->Replicate, Snapshot recovery,
 *     Inflights.FreeLE, maybeCommit (raft.go:585-588) + bcastAppend
 *     (raft.go:515-522) or the paused-peer sendAppend, the maybeSendAppend
 *     loop (raft.go:432-492), MsgTimeoutNow to the lead transferee;
 *   MsgHeartbeatResp -> RecentActive, ProbeSent, FreeFirstOne, sendAppend,
 *     ReadIndex acks: readOnly.recvAck + VoteResult + advance
 *     (read_only.go:68-121) + responseToReadIndexReq (raft.go:1737-1752);
 *   MsgSnapStatus, MsgUnreachable (raft.go:1310-1338).
 * Records of a group are applied in batch order; groups are independent.
 * The leader's log is a static view (the step never appends): firstIndex,
 * lastIndex, the terms of [firstIndex-1, lastIndex] as up to
 * QB_LEADER_MAX_RUNS runs, the storage snapshot, and max_ents = the number
 * of entries raftLog.entries(lo, MaxSizePerMsg) returns (entries of one size).
 * Outbound messages are written in group order, each group's in the order
 * the reference emits them. */

#define QB_LEADER_MAX_RUNS 8
#define QB_LEADER_MAX_READQ 16

/* Inbound kinds (rec flags bits 4-5). */
#define QB_IN_APP_RESP 0       /* pb.MsgAppResp                         */
#define QB_IN_HEARTBEAT_RESP 1 /* pb.MsgHeartbeatResp (index = Context) */
#define QB_IN_SNAP_STATUS 2    /* pb.MsgSnapStatus (local, Term 0)      */
#define QB_IN_UNREACHABLE 3    /* pb.MsgUnreachable (local, Term 0)     */

/* Progress state byte: StateType (tracker/state.go:26-33) | flags. */
#define QB_PR_PROBE 0
#define QB_PR_REPLICATE 1
#define QB_PR_SNAPSHOT 2
#define QB_PR_PROBE_SENT 0x04u
#define QB_PR_RECENT_ACTIVE 0x08u

/* Group meta word: leader slot (bits 0-7), lead transferee slot (8-15,
 * 0xFF = None), term runs (16-19, 1..8), pending ReadIndex requests (20-24,
 * at most readq_cap), bit 25: MsgReadIndex postponed until the first commit
 * of the term (raft.pendingReadIndexMessages).  A run count past
 * QB_LEADER_MAX_RUNS or a request count past readq_cap is read as that bound
 * (the step never reads or writes outside the caller's arrays). */
#define QB_META_PENDING_READINDEX (1u << 25)

/* Diagnostic switch: group the records with per-record global atomics (the
 * path used beyond the bucket geometry, > 134M groups per shard) even where
 * the LDS bucketing applies; results are identical, only slower. */
#define QB_LEADER_OPT_ATOMIC_GROUPING 1u

#define QB_READ_ONLY_SAFE 0
#define QB_READ_ONLY_LEASE_BASED 1

/* Outbound message types (raftpb MessageType, raft.pb.go:76-94) and a local
 * ReadState (raft.readStates). */
#define QB_MSG_APP 3
#define QB_MSG_SNAP 7
#define QB_MSG_TIMEOUT_NOW 14
#define QB_MSG_READ_INDEX_RESP 16
#define QB_READ_STATE 255

/* Per-group output flags. */
#define QB_LFLAG_ADVANCED 0x01u     /* maybeCommit returned true          */
#define QB_LFLAG_RELEASE_READS 0x02u /* postponed MsgReadIndex to release  */
#define QB_LFLAG_STEPPED_DOWN 0x04u  /* a higher-term response: becomeFollower */

enum {
  QB_LSTAT_APPLIED = 0,        /* reached stepLeader's handler             */
  QB_LSTAT_STALE_TERM = 1,     /* m.Term < group term: ignored            */
  QB_LSTAT_HIGHER_TERM = 2,    /* step-down record                         */
  QB_LSTAT_NON_MEMBER = 3,     /* no Progress for the slot                 */
  QB_LSTAT_AFTER_STEPDOWN = 4, /* behind the group's step-down             */
  QB_LSTAT_BAD_GROUP = 5,      /* group index >= G                          */
  QB_LSTAT_MSGS = 6,           /* outbound messages generated              */
  QB_LSTAT_MSGS_DROPPED = 7,   /* messages not written (msg_cap / pool)    */
  QB_LSTAT_COUNT = 8
};

typedef struct qb_leader_groups {
  uint64_t G;
  uint32_t inflight_cap; /* MaxInflightMsgs: ring size per slot, 1..4096  */
  uint32_t readq_cap;    /* pending ReadIndex slots per group, 0..16      */
  uint32_t read_only;    /* QB_READ_ONLY_SAFE / QB_READ_ONLY_LEASE_BASED  */
  uint32_t options;      /* QB_LEADER_OPT_* (0 = defaults)                */
  /* configuration, CSR as qb_dev_csr_committed_vote */
  const uint32_t* off;   /* [G+1] */
  const uint32_t* cfg;   /* [G] mask_in | mask_out << 16 */
  /* per group */
  uint32_t* meta;        /* [G] see QB_META_* (in/out)                     */
  const uint64_t* term;  /* [G] raft.Term                                  */
  uint64_t* committed;   /* [G] raftLog.committed (in/out)                 */
  const uint64_t* first_index; /* [G] raftLog.firstIndex()                 */
  const uint64_t* last_index;  /* [G] raftLog.lastIndex()                  */
  const uint64_t* snap_index;  /* [G] storage snapshot index, 0 = unavailable */
  const uint64_t* snap_term;   /* [G]                                      */
  const uint64_t* max_ents;    /* [G] entries per MsgApp (>= 1)            */
  const uint64_t* run_start;   /* [QB_LEADER_MAX_RUNS * G] run-major: run r of
                                  group g at r * G + g; ascending in r        */
  const uint64_t* run_term;    /* [QB_LEADER_MAX_RUNS * G] same layout      */
  /* per slot, S = off[G] (in/out) */
  uint64_t* match;
  uint64_t* next;
  uint64_t* pending_snapshot;
  uint8_t* pstate;       /* QB_PR_* */
  uint32_t* infl_pos;    /* start | count << 16; start < inflight_cap, count <=
                            inflight_cap (the ring's invariant, not checked here:
                            etcd_amd/quorum/leader.py checks it on the host) */
  uint64_t* infl_buf;    /* [S * inflight_cap] ring */
  /* pending ReadIndex queue, oldest first: [G * readq_cap] (in/out) */
  uint64_t* rq_ctx;
  uint64_t* rq_index;
  uint32_t* rq_meta;     /* ack slot bits (0-15) | request From slot << 16 (0xFF = local) */
} qb_leader_groups;

typedef struct qb_leader_inbox {
  uint64_t M;
  const uint32_t* group;
  const uint8_t* flags;  /* slot (0-3) | kind << 4 | QB_REC_NO_PROGRESS | QB_REC_REJECT */
  const uint64_t* index; /* Message.Index; MsgHeartbeatResp: Context (0 = empty) */
  const uint64_t* term;  /* Message.Term (0 = local message)                */
  const uint64_t* hint;  /* Message.RejectHint (nullable: no rejections)    */
  const uint64_t* log_term; /* Message.LogTerm (nullable)                   */
} qb_leader_inbox;

typedef struct qb_msg_out {
  uint64_t index;    /* MsgApp: Index (= Next-1); MsgSnap: snapshot index; reads: read index */
  uint64_t log_term; /* MsgApp: LogTerm; MsgSnap: snapshot term */
  uint64_t commit;   /* MsgApp: Commit */
  uint64_t aux;      /* MsgApp: number of entries (Index+1 ..); reads: request ctx */
  uint32_t group;
  uint8_t to;        /* destination slot (0xFF for a local ReadState) */
  uint8_t type;      /* QB_MSG_* */
  uint16_t reserved;
} qb_msg_out;

size_t qb_leader_workspace_bytes(uint64_t G, uint64_t M);
/* msgs: device buffer of msg_cap records; msg_total (device uint64) receives
 * the number generated (only the first msg_cap, in group order, are written);
 * msg_off (device [G+1], nullable) the first message of each group.
 * stepdown_at (device [G], nullable): batch index of the group's step-down
 * record or UINT32_MAX; gflags (device [G], nullable): QB_LFLAG_*.
 * stats: QB_LSTAT_COUNT device uint64 (accumulated). */
int qb_dev_leader_step(const qb_leader_groups* lg, const qb_leader_inbox* in,
                       qb_msg_out* msgs, uint64_t msg_cap, uint64_t* msg_total,
                       uint32_t* msg_off, uint32_t* stepdown_at, uint8_t* gflags,
                       uint64_t* stats, void* workspace, size_t workspace_bytes,
                       void* stream);

/* The same step with the messages left where the step writes them, in a
 * per-group outbox — the reference's per-node r.msgs slice (raft.go:393-420
 * r.send appends to it; Ready.Messages hands it over, node.go:573) as an
 * 8-message array per group plus an overflow list — instead of one
 * group-ordered array (qb_dev_leader_step compacts them in a second pass:
 * a scan of the counts, then every message read and written again).  Group
 * g's k-th message is slots[k * G + g] for k < QB_LEADER_OUTBOX_SLOTS; the
 * ones past it continue in QB_LEADER_OUTBOX_CHUNK-message chunks drawn from
 * chunks[] (chunk c holds chunks[c * 32 .. c * 32 + 31]; chunk_head[g] is
 * g's first chunk, chunk_next[c] the next), in the order the reference
 * emits them.  count[g] = messages stored for g (a group whose chunk could
 * not be drawn — all nchunks used — stops there; the rest is counted in
 * QB_LSTAT_MSGS_DROPPED); *chunks_used (device u32) = chunks drawn, at most
 * nchunks (chunks[0 .. chunks_used) hold messages).
 * read_states (nullable): the local reads' answers kept apart from the
 * messages, as the reference keeps them (responseToReadIndexReq appends a
 * ReadState to r.readStates, raft.go:1737-1745; Ready.ReadStates,
 * node.go:67,580): group g's k-th ReadState is read_states[k * G + g] for
 * k < read_count[g] (at most lg->readq_cap: a step releases no more reads
 * than the queue held), oldest first, and no QB_READ_STATE message is
 * emitted.  NULL keeps them in the messages as QB_READ_STATE (to 0xFF).
 * stepdown_at / gflags / stats as qb_dev_leader_step. */
#define QB_LEADER_OUTBOX_SLOTS 8
#define QB_LEADER_OUTBOX_CHUNK 32
typedef struct qb_read_state {
  uint64_t index;       /* ReadState.Index                                   */
  uint64_t ctx;         /* ReadState.RequestCtx (the request's 8-byte context) */
} qb_read_state;
typedef struct qb_leader_outbox {
  qb_msg_out* slots;    /* [QB_LEADER_OUTBOX_SLOTS * G], k-major             */
  uint32_t* count;      /* [G] messages per group                            */
  uint32_t* chunk_head; /* [G] (meaningful where count > 8)                  */
  uint32_t* chunk_next; /* [nchunks]                                         */
  qb_msg_out* chunks;   /* [nchunks * QB_LEADER_OUTBOX_CHUNK]                */
  uint64_t nchunks;     /* 0: no overflow (messages past the 8th dropped)    */
  uint32_t* chunks_used; /* device u32                                       */
  qb_read_state* read_states; /* nullable: [readq_cap * G], k-major          */
  uint32_t* read_count; /* [G] ReadStates per group (required with read_states) */
} qb_leader_outbox;
size_t qb_leader_outbox_workspace_bytes(uint64_t G, uint64_t M);
int qb_dev_leader_step_outbox(const qb_leader_groups* lg, const qb_leader_inbox* in,
                              const qb_leader_outbox* out, uint32_t* stepdown_at,
                              uint8_t* gflags, uint64_t* stats, void* workspace,
                              size_t workspace_bytes, void* stream);

/* ----------------------------------------------------------------------- */
/* Wire ingest                                       */
/* ----------------------------------------------------------------------- */

/* Raw protobuf-encoded raftpb.Message bytes (raft/raftpb/raft.proto:68-86)
 * -> leader-inbox records for qb_dev_leader_step.  Message i is
 * bytes[msg_off[i] .. msg_off[i+1]) and belongs to group msg_group[i] (the
 * multi-raft envelope's group).  Validation is exactly Message.Unmarshal
 * (raftpb/raft.pb.go:1739-2061, nested Entry / Snapshot / SnapshotMetadata /
 * ConfState bodies included, unknown fields skipped as skipRaft).  From is
 * mapped to its slot among the group's CSR slot IDs (ids[off[g] ..
 * off[g+1]), ascending); a non-member gets QB_REC_NO_PROGRESS.  MsgAppResp /
 * MsgHeartbeatResp / MsgSnapStatus / MsgUnreachable become records (a
 * heartbeat response's Context must be empty or an 8-byte non-zero
 * big-endian request id, which becomes rec_index); any other status leaves
 * rec_group = UINT32_MAX (dropped by the step as a bad group).
 * msg_type (nullable) receives the low byte of Message.Type;
 * stats (nullable, 4 device uint64, accumulated) counts each status.
 * A message whose slice is not inside the buffer (msg_off[i+1] < msg_off[i]
 * or msg_off[i+1] > nbytes: a caller error — Go would panic slicing it) gets
 * QB_WIRE_UNMARSHAL; nothing outside [bytes, bytes + nbytes) is read. */
#define QB_WIRE_OK 0
#define QB_WIRE_UNMARSHAL 1 /* Message.Unmarshal returns an error           */
#define QB_WIRE_TYPE 2      /* not a leader-inbox response type             */
#define QB_WIRE_CTX 3       /* Context neither empty nor an 8-byte id       */
int qb_dev_ingest_messages(uint64_t M, const uint8_t* bytes, uint64_t nbytes,
                           const uint64_t* msg_off, const uint32_t* msg_group,
                           uint64_t G, const uint32_t* off, const uint64_t* ids,
                           uint32_t* rec_group, uint8_t* rec_flags,
                           uint64_t* rec_index, uint64_t* rec_term,
                           uint64_t* rec_hint, uint64_t* rec_log_term,
                           uint8_t* status, uint8_t* msg_type, uint64_t* stats,
                           void* stream);
/* The same ingest over a 64-byte group-row table built once per config
 * (qb_dev_wire_group_rows: row g = member count | first slot << 32, then the
 * first 7 member IDs; 16-byte aligned, qb_wire_group_rows_bytes(G)).  Each
 * message then gathers one row instead of a row of off and one or two lines
 * of ids; members past the 7th are still read from ids.  Rebuild the rows
 * whenever off / ids change. */
size_t qb_wire_group_rows_bytes(uint64_t G);
int qb_dev_wire_group_rows(uint64_t G, const uint32_t* off, const uint64_t* ids,
                           uint64_t* rows, void* stream);
int qb_dev_ingest_messages_rows(uint64_t M, const uint8_t* bytes, uint64_t nbytes,
                                const uint64_t* msg_off, const uint32_t* msg_group,
                                uint64_t G, const uint64_t* rows, const uint64_t* ids,
                                uint32_t* rec_group, uint8_t* rec_flags,
                                uint64_t* rec_index, uint64_t* rec_term,
                                uint64_t* rec_hint, uint64_t* rec_log_term,
                                uint8_t* status, uint8_t* msg_type, uint64_t* stats,
                                void* stream);

/* The composed per-tick path in one call (round 6): a tick's M encoded
 * responses decoded and stepped into the FIXED ProgressTracker of G groups
 * with n voters, the commit advanced — what a multi-raft host runs per tick
 * between the transport (server/etcdserver/api/rafthttp/stream.go:466:
 * Message.Unmarshal, raft.pb.go:1739-2061) and Ready (node.go:564-568:
 * raft.Step -> stepLeader MsgAppResp -> maybeCommit, raft.go:847-921,
 * 1100-1109, 1237-1259, 585-588).  Replaces qb_dev_ingest_messages[_rows]
 * followed by qb_dev_fixed_tracker_step on its records, with the same
 * result, minus the decoded record columns between them: the decoder writes
 * the tracker step's level-1 buckets directly.
 *   bytes, nbytes, msg_off [M+1], msg_group [M]: as qb_dev_ingest_messages;
 *   rows (qb_dev_wire_group_rows, 16-byte aligned) or off [G+1] + ids: the
 *     groups' slot IDs (rows preferred; ids are also read for members past
 *     the row's 7);
 *   group_term .. advanced_out, stats: as qb_dev_fixed_tracker_step
 *     (stepdown_at[g] = the message index of the first higher-term response;
 *     entry rule as there);
 *   status [M] (required): QB_WIRE_* per message, as the ingest;
 *   wire_stats [4] (nullable): QB_WIRE_* counts added, as the ingest's stats.
 * A message that is not a decoded MsgAppResp steps nothing and counts as
 * QB_STAT_BAD_GROUP (the ingest gives it group ~0); a From that is not a
 * member of the group (QB_REC_NO_PROGRESS) counts as QB_STAT_NON_MEMBER.
 * Workspace: qb_wire_fixed_tracker_workspace_bytes(n, G, M) bytes (0: the
 * batch is too large for one call). */
size_t qb_wire_fixed_tracker_workspace_bytes(uint32_t n, uint64_t G, uint64_t M);
int qb_dev_ingest_fixed_tracker_step(uint32_t n, uint64_t G, uint64_t M, const uint8_t* bytes,
                                     uint64_t nbytes, const uint64_t* msg_off,
                                     const uint32_t* msg_group, const uint64_t* rows,
                                     const uint32_t* off, const uint64_t* ids,
                                     const uint64_t* group_term, const uint64_t* term_start,
                                     uint64_t* match, uint64_t* next, uint16_t* active,
                                     uint64_t* committed, uint32_t* stepdown_at,
                                     uint8_t* advanced_out, uint8_t* status,
                                     uint64_t* wire_stats, uint64_t* stats, void* workspace,
                                     size_t workspace_bytes, void* stream);
/* The same one-call tick for the CSR tracker (ragged / learner / joint
 * configs, qb_dev_csr_tracker_step's layout and arguments): off [G+1] are
 * both the tracker's slot offsets and the groups' slot-ID ranges (ids
 * ascending per group, required; rows, the 64-byte row table of (off, ids),
 * nullable).  Workspace: qb_wire_csr_tracker_workspace_bytes(G, max_slots, M). */
size_t qb_wire_csr_tracker_workspace_bytes(uint64_t G, uint32_t max_slots, uint64_t M);
int qb_dev_ingest_csr_tracker_step(uint64_t G, uint32_t max_slots, const uint32_t* off,
                                   const uint32_t* cfg, uint64_t M, const uint8_t* bytes,
                                   uint64_t nbytes, const uint64_t* msg_off,
                                   const uint32_t* msg_group, const uint64_t* rows,
                                   const uint64_t* ids, const uint64_t* group_term,
                                   const uint64_t* term_start, uint64_t* match, uint64_t* next,
                                   uint16_t* active, uint64_t* committed, uint32_t* stepdown_at,
                                   uint8_t* advanced_out, uint8_t* status, uint64_t* wire_stats,
                                   uint64_t* stats, void* workspace, size_t workspace_bytes,
                                   void* stream);

/* ----------------------------------------------------------------------- */
/* Configuration changes                             */
/* ----------------------------------------------------------------------- */

/* One confchange.Changer operation per group, all groups in one call:
 * Simple / EnterJoint(autoLeave) / LeaveJoint (confchange/confchange.go:
 * 49-146) over the group's ConfChangeSingle list (apply, makeVoter,
 * makeLearner, remove, initProgress: confchange.go:151-281), with
 * checkInvariants on input and output (confchange.go:283-334).
 * A group's config is its CSR slots (ascending IDs of the ProgressMap) with
 * cfg = Voters[0] | Voters[1] << 16 and ext = LearnersNext | AutoLeave << 16;
 * a slot in none of the three masks is a learner.  The result is written to
 * a second set of arrays (double-buffered): new_off [G+1] (offsets), slot
 * IDs, masks and the Progress arrays of the leader-step layout — carried for
 * kept slots, initialised for added ones (Next = last_index[g], Match 0,
 * StateProbe, RecentActive; initProgress).  A group whose operation fails
 * keeps its config and Progress; err[g] names the reference's error and
 * err_id[g] (nullable) the offending ID where the message has one (the
 * smallest such ID).  Restore(ConfState) (confchange/restore.go:116-155) is a
 * sequence of such calls. */
#define QB_CC_NONE 0                 /* copy through                      */
#define QB_CC_SIMPLE 1
#define QB_CC_ENTER_JOINT 2
#define QB_CC_ENTER_JOINT_AUTOLEAVE 3
#define QB_CC_LEAVE_JOINT 4

/* raftpb.ConfChangeType (raft.pb.go) */
#define QB_CC_ADD_NODE 0
#define QB_CC_REMOVE_NODE 1
#define QB_CC_UPDATE_NODE 2
#define QB_CC_ADD_LEARNER 3

enum {
  QB_CCERR_OK = 0,
  QB_CCERR_ALREADY_JOINT = 1,       /* "config is already joint"                        */
  QB_CCERR_ZERO_VOTER_JOINT = 2,    /* "can't make a zero-voter config joint"           */
  QB_CCERR_NOT_JOINT = 3,           /* "can't leave a non-joint config"                 */
  QB_CCERR_SIMPLE_IN_JOINT = 4,     /* "can't apply simple config change in joint config" */
  QB_CCERR_MORE_THAN_ONE = 5,       /* "more than one voter changed without entering joint config" */
  QB_CCERR_REMOVED_ALL = 6,         /* "removed all voters"                             */
  QB_CCERR_UNKNOWN_TYPE = 7,        /* "unexpected conf type %d"                        */
  QB_CCERR_NO_PROGRESS = 8,         /* "no progress for %d"                             */
  QB_CCERR_LNEXT_NOT_OUTGOING = 9,  /* "%d is in LearnersNext, but not Voters[1]"       */
  QB_CCERR_LNEXT_IS_LEARNER = 10,   /* "%d is in LearnersNext, but is already marked as learner" */
  QB_CCERR_LEARNER_OUTGOING = 11,   /* "%d is in Learners and Voters[1]"                */
  QB_CCERR_LEARNER_INCOMING = 12,   /* "%d is in Learners and Voters[0]"                */
  QB_CCERR_LEARNER_NOT_MARKED = 13, /* "%d is in Learners, but is not marked as learner" */
  QB_CCERR_AUTOLEAVE_NOT_JOINT = 14, /* "AutoLeave must be false when not joint"        */
  QB_CCERR_TOO_MANY_SLOTS = 15,     /* engine limit: > QB_MAX_SLOTS members, or > 24 IDs alive at once within one change list
                                       (a current config of > 24 slots is kept as it is, and
                                       copied through under QB_CC_NONE) */
  QB_CCERR_BAD_OP = 16              /* op is not a QB_CC_* operation                     */
};

typedef struct qb_conf_change_in {
  uint64_t G;
  uint32_t inflight_cap;     /* ring size of infl_buf per slot */
  uint32_t reserved;
  const uint8_t* op;         /* [G] QB_CC_*                           */
  const uint32_t* cc_off;    /* [G+1] ConfChangeSingle list per group */
  const uint8_t* cc_type;    /* [cc_off[G]] QB_CC_ADD_NODE ...         */
  const uint64_t* cc_node;   /* [cc_off[G]] NodeID (0 = ignored)       */
  const uint64_t* last_index; /* [G] Changer.LastIndex                 */
  const uint32_t* off;       /* [G+1] current slots                    */
  const uint64_t* ids;       /* [off[G]] ascending per group           */
  const uint32_t* cfg;       /* [G]                                     */
  const uint32_t* ext;       /* [G] (nullable: no LearnersNext/AutoLeave) */
  const uint64_t* match;     /* Progress, leader-step layout [off[G]]  */
  const uint64_t* next;
  const uint64_t* pending_snapshot;
  const uint8_t* pstate;
  const uint32_t* infl_pos;
  const uint64_t* infl_buf;  /* [off[G] * inflight_cap]; 8-byte aligned suffices (16-byte
                                aligned in and out buffers let inflight_cap 4 move rings
                                as 16-byte words) */
} qb_conf_change_in;

typedef struct qb_conf_change_out {
  uint64_t slot_cap;         /* capacity of the per-slot output arrays */
  uint32_t* new_off;         /* [G+1]; new_off[G] = slots needed        */
  uint64_t* ids;
  uint32_t* cfg;             /* [G] */
  uint32_t* ext;             /* [G] */
  uint64_t* match;
  uint64_t* next;
  uint64_t* pending_snapshot;
  uint8_t* pstate;
  uint32_t* infl_pos;
  uint64_t* infl_buf;
  uint8_t* err;              /* [G] QB_CCERR_*   */
  uint64_t* err_id;          /* [G] (nullable)   */
} qb_conf_change_out;

size_t qb_conf_change_workspace_bytes(uint64_t G);
/* If new_off[G] > slot_cap nothing past the capacity is written: check
 * new_off[G] after the call. */
int qb_dev_conf_change(const qb_conf_change_in* in, const qb_conf_change_out* out,
                       void* workspace, size_t workspace_bytes, void* stream);

/* ----------------------------------------------------------------------- */
/* Sharding over the GPUs of a node                        */
/* ----------------------------------------------------------------------- */

/* One process per GPU; rank r owns the contiguous global groups
 * [begin, end) = qb_shard_range(total, world, r) (sizes differ by at most
 * one; etcd_amd/shard.py shard_range).  Groups are independent, so the hot
 * path exchanges nothing; the one collective is at its edge: the node-wide
 * CommittedIndex / VoteResult vectors assembled from the shards by an RCCL
 * all-gather over xGMI.  The host distributes the 128-byte unique ID from
 * rank 0 over its own transport (the reference's peer transport is
 * rafthttp, server/etcdserver/api/rafthttp/peer.go:178). */
#define QB_COMM_ID_BYTES 128
typedef struct qb_comm qb_comm;
int qb_shard_range(uint64_t total, int world, int rank, uint64_t* begin, uint64_t* end);
int qb_comm_get_unique_id(void* id_out);
/* ncclCommInitRank on the calling thread's current device (qb_set_device);
 * collective: every rank calls it with the same id. */
int qb_comm_init(qb_comm** out, int world, int rank, const void* id);
int qb_comm_destroy(qb_comm* comm);
size_t qb_allgather_workspace_bytes(uint64_t total, int world);
/* commit_all[total] / vote_all[total] (device; either nullable) receive every
 * rank's shard in rank order (a rank whose shard is empty, total < world,
 * may pass NULL shard vectors).  Collective over the comm, enqueued on stream.
 * The workspace (device, qb_allgather_workspace_bytes) is needed only when
 * total % world != 0 (padded shards compacted by rank). */
int qb_dev_allgather_results(qb_comm* comm, uint64_t total,
                             const uint64_t* commit_shard, const uint8_t* vote_shard,
                             uint64_t* commit_all, uint8_t* vote_all,
                             void* workspace, size_t workspace_bytes, void* stream);

/* The changed-commit delta (gather only the groups whose
 * commit moved).  A group surfaces a Ready when its HardState changed
 * (raft/node.go:573 newReady, raft/rawnode.go:157 HasReady); in a tick that
 * is the groups whose maybeCommit advanced (raft.go:585-588) — the tracker
 * steps' advanced_out.  Device half: the n groups' changed flags (u8, nonzero
 * = changed) compacted in group order into (g_base + g, commit[g]) pairs in
 * out_gid / out_commit (room for n each); *out_count (device u64) = pairs
 * written (global groups must fit uint32). */
size_t qb_compact_changed_workspace_bytes(uint64_t n);
int qb_dev_compact_changed(uint64_t n, const uint8_t* changed, const uint64_t* commit,
                           uint64_t g_base, uint32_t* out_gid, uint64_t* out_commit,
                           uint64_t* out_count, void* workspace, size_t workspace_bytes,
                           void* stream);
/* commit_all[gid[i]] = commit[i] for i < m (gid UINT32_MAX or >= total:
 * skipped, the padding of the exchange below). */
int qb_dev_scatter_changed(uint64_t m, const uint32_t* gid, const uint64_t* commit, uint64_t total,
                           uint64_t* commit_all, void* stream);
size_t qb_allgather_changed_workspace_bytes(uint64_t total, int world);
/* Collective over the comm: this rank's shard's changed groups (changed_shard
 * / commit_shard: the shard's local arrays, qb_shard_range) are exchanged and
 * applied to commit_all[total] (device) on every rank — the caller keeps
 * commit_all across ticks.  Every rank pads its pairs to the largest
 * per-rank count C_max, so each rank receives 12 * world * C_max bytes (not
 * 12 per changed group): a skewed tick (one shard with many commits)
 * approaches the full gather's cost, and when 12 * C_max exceeds 8 * the
 * shard size the call is cheaper as qb_dev_allgather_results (it picks that
 * itself: see below).  *changed_total (host) = changed groups node-wide.  The
 * host waits on the stream once (the exchange size is data-dependent); a
 * rank's local failure in the compaction (NULL shard columns included)
 * reaches every rank through the gathered counts, so all return QB_EINVAL
 * together.  Every rank must pass the same total, a non-NULL commit_all and a
 * large enough workspace: a rank failing those checks returns before the
 * count all-gather and leaves the others waiting in it (as
 * qb_dev_route_records). */
int qb_dev_allgather_changed(qb_comm* comm, uint64_t total, const uint8_t* changed_shard,
                             const uint64_t* commit_shard, uint64_t* commit_all,
                             uint64_t* changed_total, void* workspace, size_t workspace_bytes,
                             void* stream);

/* Record delivery to the owning shards ("message batches are
 * bucketed by owning shard").  A node's inbound responses arrive at any rank;
 * each record goes to the rank owning its global group, with the group
 * rebased to that shard's local index (a group >= total goes to the last
 * rank as an index >= its shard size, which the steps count as a bad group).
 * Delivery is stable: the receiver gets each source rank's records in
 * source-rank order, each source's in their original order — the batch order
 * the leader step's sequential semantics need (raft.go:1099-1342 is a
 * per-message fold).  Replaces the Python etcd_amd/shard.py:route_records
 * (torch bucketize / argsort / all_to_all_single) for a cgo embedder. */
#define QB_ROUTE_MAX_WORLD 64
size_t qb_route_partition_workspace_bytes(int world, uint64_t M);
/* The device half (no communication; usable with any world for testing and
 * by callers with their own transport): the batch's records stably
 * partitioned by owner into the send_* columns (M entries each; hint /
 * log_term both-or-neither with their inputs), send_off[world + 1] (device)
 * = the first send position per destination rank, send_off[world] = M. */
int qb_dev_route_partition(uint64_t total, int world, uint64_t M, const uint32_t* rec_group,
                           const uint8_t* rec_flags, const uint64_t* rec_index,
                           const uint64_t* rec_term, const uint64_t* rec_hint,
                           const uint64_t* rec_log_term, uint32_t* send_group,
                           uint8_t* send_flags, uint64_t* send_index, uint64_t* send_term,
                           uint64_t* send_hint, uint64_t* send_log_term, uint32_t* send_off,
                           void* workspace, size_t workspace_bytes, void* stream);
size_t qb_route_workspace_bytes(int world, uint64_t M);
/* Collective over the comm: partition, an all-gather of every rank's counts
 * and output capacity (every rank refuses with QB_EINVAL if any rank's
 * receive would exceed its out_cap — one decision everywhere, no rank left in
 * a send), then RCCL point-to-point runs per column into out_* (device,
 * out_cap entries).  *out_count (host) = records received.  The host waits on
 * the stream twice (the receive sizes are data-dependent).  Every rank must
 * call it with valid arguments: a rank failing a precondition before the
 * all-gather leaves the others waiting in it. */
int qb_dev_route_records(qb_comm* comm, uint64_t total, uint64_t M, const uint32_t* rec_group,
                         const uint8_t* rec_flags, const uint64_t* rec_index,
                         const uint64_t* rec_term, const uint64_t* rec_hint,
                         const uint64_t* rec_log_term, uint32_t* out_group, uint8_t* out_flags,
                         uint64_t* out_index, uint64_t* out_term, uint64_t* out_hint,
                         uint64_t* out_log_term, uint64_t out_cap, uint64_t* out_count,
                         void* workspace, size_t workspace_bytes, void* stream);

/* ----------------------------------------------------------------------- */
/* Synthetic workload generators (bench/test inputs)        */
/* ----------------------------------------------------------------------- */

/* Counter-based, so every shard/device/CPU regenerates identical inputs:
 * r(g, slot, field) = splitmix64(seed ^ (g << 12 | slot << 4 | field)).
 * g_begin offsets the global group number (sharding). */
int qb_dev_synth_fixed(uint64_t seed, uint32_t n, uint64_t G, uint64_t g_begin,
                       uint64_t* match, void* voted, void* granted,
                       uint64_t* term_start, void* stream);
/* Host-side: group sizes and CSR offsets of the ragged config (s_g = n_g +
 * learners_g).  off has G+1 entries.  Returns QB_OK or QB_EINVAL if the total
 * overflows uint32. */
int qb_host_synth_csr_offsets(uint64_t seed, uint64_t G, uint64_t g_begin,
                              uint32_t* off);
/* Device fill of the ragged (kind 0) or joint 5+5 (kind 1) config given off. */
int qb_dev_synth_csr(uint64_t seed, int kind, uint64_t G, uint64_t g_begin,
                     const uint32_t* off, uint64_t* match, uint32_t* cfg,
                     uint32_t* votes, void* stream);
/* Host-side joint offsets: s_g = 10 - overlap_g. */
int qb_host_synth_joint_offsets(uint64_t seed, uint64_t G, uint64_t g_begin,
                                uint32_t* off);

#ifdef __cplusplus
}
#endif

#endif /* QUORUM_BATCH_H */
