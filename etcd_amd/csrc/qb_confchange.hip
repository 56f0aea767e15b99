// qb_confchange.hip — batched configuration changes over G groups (gfx950):
// every group's Changer.Simple / EnterJoint / LeaveJoint in one launch, with
// the reference's validation, producing the new CSR config (slot IDs,
// voter masks, LearnersNext, AutoLeave) and the carried / initialised
// Progress arrays.
//
// Reference (paths relative to raft/):
//   Changer.EnterJoint / LeaveJoint / Simple   confchange/confchange.go:49-146
//   apply / makeVoter / makeLearner / remove   confchange/confchange.go:151-245
//   initProgress                               confchange/confchange.go:258-281
//   checkInvariants                            confchange/confchange.go:283-334
//   symdiff                                    confchange/confchange.go:390-405
//
// Representation.  A group's tracker.Config + ProgressMap is its slots (the
// ascending IDs of the ProgressMap) with masks: Voters[0] (cfg bits 0-15),
// Voters[1] (cfg bits 16-31), LearnersNext (ext bits 0-15), AutoLeave (ext
// bit 16).  A slot in none of these is a learner (Progress.IsLearner).  Empty
// masks are the reference's nil maps (the Changer never leaves an empty
// non-nil Voters[1], Learners or LearnersNext).
//
// Per group (one thread): the old slots and the changes are replayed on a
// small working table in LDS (IDs + role bitmasks over table entries), then
// the surviving entries are sorted by ID into the new slots.  Two launches
// (count, then write after a scan of the counts) recompute the same replay.
#include "qb_common.h"
#include "qb_scan.h"

namespace qb {
namespace cc {

constexpr int kBlk = 128;
constexpr int kTab = 24;  // working table: 16 old slots + up to 8 new IDs

// A thread's working table, column-major in the workgroup's LDS block
// (entry k of thread t at [k][t]): the lanes of a wave touch consecutive
// words, so table accesses are free of bank conflicts (a per-thread row of
// 24 u64 put every 4th lane on the same bank).
struct Tab {
  u64* col;  // &lds[0][threadIdx.x]
  __device__ __forceinline__ u64& id(int k) const { return col[k * kBlk]; }
};
__device__ __forceinline__ Tab tab_of(u64 (*lds)[kBlk]) { return Tab{&lds[0][threadIdx.x]}; }

struct Args {
  u64 G;
  const u8* op;
  const u32* cc_off;
  const u8* cc_type;
  const u64* cc_node;
  const u64* last_index;
  // old
  const u32* off;
  const u64* ids;
  const u32* cfg;
  const u32* ext;
  const u64 *match, *next, *psnap;
  const u8* pstate;
  const u32* infl_pos;
  const u64* infl_buf;
  u32 K;
  // new
  u32* new_cnt;  // [G+1] counts, then (after the scan) offsets
  u64 S_cap;
  u64* n_ids;
  u32* n_cfg;
  u32* n_ext;
  u64 *n_match, *n_next, *n_psnap;
  u8* n_pstate;
  u32* n_infl_pos;
  u64* n_infl_buf;
  u8* err;
  u64* err_id;
};

// Role bitmasks over table entries.
struct Roles {
  u32 in, out, lnext, lrn, prs, islrn;
  u32 fresh;  // entries whose Progress initProgress created in this change
  int n;  // entries used
};

__device__ __forceinline__ int find(const Tab& t, int n, u64 id) {
  for (int k = 0; k < n; ++k)
    if (t.id(k) == id) return k;
  return -1;
}

// checkInvariants (confchange.go:283-334) on table roles; returns 0 or the
// error code, *bad = the offending ID (the smallest, for a deterministic
// report; Go reports whichever its map iteration meets first).
__device__ int check_invariants(const Tab& t, const Roles& r, bool autoleave, u64* bad) {
  auto first = [&](u32 m) {
    u64 best = ~0ull;
    for (int k = 0; k < r.n; ++k)
      if ((m >> k) & 1u && t.id(k) < best) best = t.id(k);
    return best;
  };
  const u32 members = r.in | r.out | r.lrn | r.lnext;
  if (members & ~r.prs) { *bad = first(members & ~r.prs); return QB_CCERR_NO_PROGRESS; }
  if (r.lnext & ~r.out) { *bad = first(r.lnext & ~r.out); return QB_CCERR_LNEXT_NOT_OUTGOING; }
  if (r.lnext & r.islrn) { *bad = first(r.lnext & r.islrn); return QB_CCERR_LNEXT_IS_LEARNER; }
  if (r.lrn & r.out) { *bad = first(r.lrn & r.out); return QB_CCERR_LEARNER_OUTGOING; }
  if (r.lrn & r.in) { *bad = first(r.lrn & r.in); return QB_CCERR_LEARNER_INCOMING; }
  if (r.lrn & ~r.islrn) { *bad = first(r.lrn & ~r.islrn); return QB_CCERR_LEARNER_NOT_MARKED; }
  if (r.out == 0 && autoleave) return QB_CCERR_AUTOLEAVE_NOT_JOINT;
  return 0;
}

// Replays group g's operation.  On success fills the table/roles of the new
// config and returns 0; otherwise an error code (the table then holds the
// old config).  Roles.fresh marks entries whose Progress is (re)created.
__device__ int replay(const Args& A, u64 g, const Tab& t, Roles& r, bool& autoleave, u64* bad,
                      int* n_old) {
  const u32 s0 = A.off[g], s1 = A.off[g + 1];
  const u32 ns = s1 - s0;
  const u32 c = A.cfg[g], e = A.ext ? A.ext[g] : 0u;
  r = Roles{};
  for (u32 j = 0; j < ns; ++j) t.id(j) = A.ids[s0 + j];
  r.n = int(ns);
  *n_old = int(ns);
  r.in = c & 0xFFFFu;
  r.out = c >> 16;
  r.lnext = e & 0xFFFFu;
  r.prs = ns >= 32 ? ~0u : ((1u << ns) - 1u);
  r.lrn = r.prs & ~(r.in | r.out | r.lnext);
  r.islrn = r.lrn;
  autoleave = (e >> 16) & 1u;
  const u32 op = A.op[g];
  if (op == QB_CC_NONE) return 0;
  // checkAndCopy: the input must satisfy the invariants
  int rc = check_invariants(t, r, autoleave, bad);
  if (rc) return rc;
  const u32 in0 = r.in;
  const bool joint = r.out != 0;
  if (op == QB_CC_LEAVE_JOINT) {  // confchange.go:91-120
    if (!joint) return QB_CCERR_NOT_JOINT;
    r.lrn |= r.lnext;
    r.islrn |= r.lnext;
    r.lnext = 0;
    r.prs &= ~(r.out & ~r.in & ~r.lrn);
    r.out = 0;
    autoleave = false;
    return check_invariants(t, r, autoleave, bad);
  }
  if (op == QB_CC_SIMPLE) {
    if (joint) return QB_CCERR_SIMPLE_IN_JOINT;
  } else if (op == QB_CC_ENTER_JOINT || op == QB_CC_ENTER_JOINT_AUTOLEAVE) {
    if (joint) return QB_CCERR_ALREADY_JOINT;
    if (r.in == 0) return QB_CCERR_ZERO_VOTER_JOINT;
    r.out = r.in;
  } else {
    return QB_CCERR_BAD_OP;
  }
  // apply (confchange.go:151-175)
  for (u32 k = A.cc_off[g]; k < A.cc_off[g + 1]; ++k) {
    const u64 id = A.cc_node[k];
    if (id == 0) continue;
    const u32 typ = A.cc_type[k];
    int x = find(t, r.n, id);
    const bool has_pr = x >= 0 && ((r.prs >> x) & 1u);
    if (typ == QB_CC_ADD_NODE || typ == QB_CC_ADD_LEARNER) {
      if (!has_pr) {  // initProgress
        if (x < 0) {
          if (r.n >= kTab) return QB_CCERR_TOO_MANY_SLOTS;
          x = r.n++;
          t.id(x) = id;
        }
        const u32 b = 1u << x;
        r.prs |= b;
        r.fresh |= b;  // a removed-then-re-added ID gets a new Progress too
        if (typ == QB_CC_ADD_NODE) {
          r.in |= b;
          r.islrn &= ~b;
        } else {
          r.lrn |= b;
          r.islrn |= b;
        }
        continue;
      }
      const u32 b = 1u << x;
      if (typ == QB_CC_ADD_NODE) {  // makeVoter
        r.islrn &= ~b;
        r.lrn &= ~b;
        r.lnext &= ~b;
        r.in |= b;
      } else {  // makeLearner
        if (r.islrn & b) continue;
        r.in &= ~b;  // remove(), Progress kept
        r.lrn &= ~b;
        r.lnext &= ~b;
        if (r.out & b) {
          r.lnext |= b;
        } else {
          r.islrn |= b;
          r.lrn |= b;
        }
      }
    } else if (typ == QB_CC_REMOVE_NODE) {
      if (!has_pr) continue;
      const u32 b = 1u << x;
      r.in &= ~b;
      r.lrn &= ~b;
      r.lnext &= ~b;
      if (!(r.out & b)) r.prs &= ~b;
    } else if (typ == QB_CC_UPDATE_NODE) {
      // nothing tracked inside raft
    } else {
      *bad = typ;
      return QB_CCERR_UNKNOWN_TYPE;
    }
  }
  if (r.in == 0) return QB_CCERR_REMOVED_ALL;
  if (op == QB_CC_SIMPLE) {
    if (__popc(in0 ^ r.in) > 1) return QB_CCERR_MORE_THAN_ONE;
  } else {
    autoleave = op == QB_CC_ENTER_JOINT_AUTOLEAVE;
  }
  rc = check_invariants(t, r, autoleave, bad);
  if (rc) return rc;
  if (__popc(r.prs) > QB_MAX_SLOTS) return QB_CCERR_TOO_MANY_SLOTS;
  return 0;
}

__global__ __launch_bounds__(kBlk) void k_cc_count(Args A) {
  __shared__ u64 tabs[kTab][kBlk];
  const u64 g = u64(blockIdx.x) * kBlk + threadIdx.x;
  if (g >= A.G) return;
  Tab t = tab_of(tabs);
  Roles r;
  bool al;
  u64 bad = 0;
  int n_old;
  const int rc = replay(A, g, t, r, al, &bad, &n_old);
  A.new_cnt[g] = rc ? u32(n_old) : u32(__popc(r.prs));
  A.err[g] = u8(rc);
  if (A.err_id) A.err_id[g] = rc ? bad : 0;
}

// Carried Progress and inflight rings are copied by the whole workgroup
// after the per-group pass: each thread lists its new slots' (destination,
// source) pairs in LDS, then lanes copy rows (and consecutive words of the
// rings) with loads batched ahead of stores.  The per-group pass itself
// only stores, so its stores never stall a later load (gfx9 counts loads
// and stores on one vector memory counter).
constexpr u32 kNoSrc = 0xFFFFFFFFu;
constexpr u32 kRows = kBlk * QB_MAX_SLOTS;

__global__ __launch_bounds__(kBlk) void k_cc_write(Args A) {
  __shared__ u64 tabs[kTab][kBlk];
  __shared__ u32 row_dst[kRows], row_src[kRows];
  __shared__ u32 nrows;
  if (threadIdx.x == 0) nrows = 0;
  __syncthreads();
  const u64 g = u64(blockIdx.x) * kBlk + threadIdx.x;
  if (g < A.G) {
    Tab t = tab_of(tabs);
    Roles r;
    bool al;
    u64 bad = 0;
    int n_old;
    int rc = replay(A, g, t, r, al, &bad, &n_old);
    const u32 s0 = A.off[g];
    const u64 d0 = A.new_cnt[g], d1 = A.new_cnt[g + 1];
    if (d1 <= A.S_cap) {  // else the caller's capacity is exceeded (reported by the host call)
      if (rc) {  // the old config is kept
        r = Roles{};
        r.n = n_old;
        r.prs = n_old >= 32 ? ~0u : ((1u << n_old) - 1u);
        const u32 c = A.cfg[g], e = A.ext ? A.ext[g] : 0u;
        r.in = c & 0xFFFFu;
        r.out = c >> 16;
        r.lnext = e & 0xFFFFu;
        al = (e >> 16) & 1u;
      }
      // surviving entries in ascending ID order (selection over <= 24 entries)
      u32 left = r.prs, ncfg_in = 0, ncfg_out = 0, nlnext = 0;
      const u64 last = A.last_index[g];
      const u32 nnew = u32(__popc(r.prs));
      const u32 row0 = atomicAdd(&nrows, nnew);
      for (u32 j = 0; left; ++j) {
        int best = -1;
        for (int k = 0; k < r.n; ++k)
          if (((left >> k) & 1u) && (best < 0 || t.id(k) < t.id(best))) best = k;
        left &= ~(1u << best);
        const u32 b = 1u << best;
        if (r.in & b) ncfg_in |= 1u << j;
        if (r.out & b) ncfg_out |= 1u << j;
        if (r.lnext & b) nlnext |= 1u << j;
        const u64 d = d0 + j;
        A.n_ids[d] = t.id(best);
        u32 src = kNoSrc;
        if (best < n_old && !(r.fresh & b)) {  // carried Progress (checkAndCopy's shallow copy)
          src = s0 + u32(best);                // copied by the workgroup below
        } else {  // initProgress (confchange.go:258-281)
          A.n_match[d] = 0;
          A.n_next[d] = last;
          A.n_psnap[d] = 0;
          A.n_pstate[d] = QB_PR_PROBE | QB_PR_RECENT_ACTIVE;
          A.n_infl_pos[d] = 0;
        }
        row_dst[row0 + j] = u32(d);
        row_src[row0 + j] = src;
      }
      A.n_cfg[g] = ncfg_in | (ncfg_out << 16);
      A.n_ext[g] = nlnext | (al ? 1u << 16 : 0u);
    }
  }
  __syncthreads();
  // Carried Progress: four rows per lane in flight (all loads, then all
  // stores), so loads do not queue behind earlier stores on the shared
  // vector memory counter.
  const u32 nr = nrows;
  for (u32 e0 = threadIdx.x; e0 < nr; e0 += 4 * kBlk) {
    u64 m[4], nx[4], ps[4];
    u32 ip[4];
    u8 st[4];
    u32 dst[4];
    bool on[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32 e = e0 + u32(q) * kBlk;
      const u32 src = e < nr ? row_src[e] : kNoSrc;
      on[q] = src != kNoSrc;
      dst[q] = e < nr ? row_dst[e] : 0u;
      m[q] = on[q] ? A.match[src] : 0ull;
      nx[q] = on[q] ? A.next[src] : 0ull;
      ps[q] = on[q] ? A.psnap[src] : 0ull;
      ip[q] = on[q] ? A.infl_pos[src] : 0u;
      st[q] = on[q] ? A.pstate[src] : u8(0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!on[q]) continue;
      A.n_match[dst[q]] = m[q];
      A.n_next[dst[q]] = nx[q];
      A.n_psnap[dst[q]] = ps[q];
      A.n_infl_pos[dst[q]] = ip[q];
      A.n_pstate[dst[q]] = st[q];
    }
  }
  if (A.K == 0) return;  // uniform
  const u32 K = A.K, words = nr * K;
  constexpr int kB = 8;  // words per lane in flight
  for (u32 w0 = threadIdx.x; w0 < words; w0 += kB * kBlk) {
    u64 v[kB], at[kB];
#pragma unroll
    for (int q = 0; q < kB; ++q) {
      const u32 w = w0 + u32(q) * kBlk;
      const u32 e = w < words ? w / K : 0u, k = w - e * K;
      const u32 src = w < words ? row_src[e] : kNoSrc;
      at[q] = w < words ? u64(row_dst[e]) * K + k : ~0ull;
      v[q] = src == kNoSrc ? 0ull : A.infl_buf[u64(src) * K + k];
    }
#pragma unroll
    for (int q = 0; q < kB; ++q)
      if (at[q] != ~0ull) A.n_infl_buf[at[q]] = v[q];
  }
}

}  // namespace cc
}  // namespace qb

using namespace qb;

extern "C" size_t qb_conf_change_workspace_bytes(uint64_t G) {
  return (scan::blocks(G) + 1) * sizeof(u32) + 256;
}

extern "C" int qb_dev_conf_change(const qb_conf_change_in* in, const qb_conf_change_out* out,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  QB_REQUIRE(in && out, "qb_dev_conf_change: in and out are required");
  const u64 G = in->G;
  if (G == 0) return QB_OK;
  QB_REQUIRE(G < (1ull << 32), "qb_dev_conf_change: G must be < 2^32");
  QB_REQUIRE(in->op && in->cc_off && in->last_index && in->off && in->ids && in->cfg,
             "qb_dev_conf_change: op, cc_off, last_index, off, ids and cfg are required");
  QB_REQUIRE(in->match && in->next && in->pending_snapshot && in->pstate && in->infl_pos &&
                 (in->inflight_cap == 0 || in->infl_buf),
             "qb_dev_conf_change: the Progress arrays are required");
  QB_REQUIRE(out->new_off && out->ids && out->cfg && out->ext && out->match && out->next &&
                 out->pending_snapshot && out->pstate && out->infl_pos && out->err &&
                 (in->inflight_cap == 0 || out->infl_buf),
             "qb_dev_conf_change: every output array is required");
  QB_REQUIRE(workspace && workspace_bytes >= qb_conf_change_workspace_bytes(G),
             "qb_dev_conf_change: workspace too small");
  cc::Args A{};
  A.G = G;
  A.op = in->op;
  A.cc_off = in->cc_off;
  A.cc_type = in->cc_type;
  A.cc_node = reinterpret_cast<const u64*>(in->cc_node);
  A.last_index = reinterpret_cast<const u64*>(in->last_index);
  A.off = in->off;
  A.ids = reinterpret_cast<const u64*>(in->ids);
  A.cfg = in->cfg;
  A.ext = in->ext;
  A.match = reinterpret_cast<const u64*>(in->match);
  A.next = reinterpret_cast<const u64*>(in->next);
  A.psnap = reinterpret_cast<const u64*>(in->pending_snapshot);
  A.pstate = in->pstate;
  A.infl_pos = in->infl_pos;
  A.infl_buf = reinterpret_cast<const u64*>(in->infl_buf);
  A.K = in->inflight_cap;
  A.new_cnt = out->new_off;
  A.S_cap = out->slot_cap;
  A.n_ids = reinterpret_cast<u64*>(out->ids);
  A.n_cfg = out->cfg;
  A.n_ext = out->ext;
  A.n_match = reinterpret_cast<u64*>(out->match);
  A.n_next = reinterpret_cast<u64*>(out->next);
  A.n_psnap = reinterpret_cast<u64*>(out->pending_snapshot);
  A.n_pstate = out->pstate;
  A.n_infl_pos = out->infl_pos;
  A.n_infl_buf = reinterpret_cast<u64*>(out->infl_buf);
  A.err = out->err;
  A.err_id = reinterpret_cast<u64*>(out->err_id);
  hipStream_t st = as_stream(stream);
  const unsigned grid = unsigned((G + cc::kBlk - 1) / cc::kBlk);
  hipLaunchKernelGGL(cc::k_cc_count, dim3(grid), dim3(cc::kBlk), 0, st, A);
  QB_CHECK_LAUNCH("k_cc_count");
  scan::launch(out->new_off, G, static_cast<u32*>(workspace), st);
  QB_CHECK_LAUNCH("scan(conf change)");
  hipLaunchKernelGGL(cc::k_cc_write, dim3(grid), dim3(cc::kBlk), 0, st, A);
  QB_CHECK_LAUNCH("k_cc_write");
  return QB_OK;
}
