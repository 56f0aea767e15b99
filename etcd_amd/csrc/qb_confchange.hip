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
// the surviving entries are sorted by ID into the new slots.  Two passes
// (count, then write after a scan of the counts) recompute the same replay.
//
// Table size (round 3): the replay is latency-bound and its occupancy is set
// by the table's LDS (24 entries x 8 B x 128 threads = 24 KB per workgroup:
// 3 waves per SIMD).  A group whose old slots plus change entries number at
// most kSmall can never hold more than kSmall table entries (each change adds
// at most one), so each pass runs twice: a kSmall-entry launch for those
// groups (8 KB per workgroup: 10 waves per SIMD), then a kTab-entry launch,
// grid-strided, for the rest — which returns at once when the first launch
// saw none (a flag word in the workspace).  Same replay, same results.
#include "qb_common.h"
#include "qb_scan.h"

namespace qb {
namespace cc {

constexpr int kBlk = 128;
constexpr int kTab = 24;   // working table: old slots + new IDs alive at once
constexpr int kSmall = 8;  // the first launch's table (old slots + changes <= 8)
constexpr unsigned kBigGrid = 1024;  // workgroups of the grid-strided kTab launches

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
  u32* new_cnt;  // [G+1] counts, then 4096-block local prefixes; the write pass stores the offsets
  const u32* nbsum;  // the local scan's block sums, scanned (add-back folded into the write pass)
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
  u32* any_big;  // workspace word: a group needs the kTab table
};

// A group's table can exceed kSmall entries only when its old slots plus its
// change entries do (each change adds at most one entry).
__device__ __forceinline__ bool needs_big(const Args& A, u64 g) {
  return (A.off[g + 1] - A.off[g]) + (A.cc_off[g + 1] - A.cc_off[g]) > u32(kSmall);
}

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
template <int TAB>
__device__ int replay(const Args& A, u64 g, const Tab& t, Roles& r, bool& autoleave, u64* bad,
                      int* n_old) {
  const u32 s0 = A.off[g], s1 = A.off[g + 1];
  const u32 ns = s1 - s0;
  const u32 c = A.cfg[g], e = A.ext ? A.ext[g] : 0u;
  // the first change entry requested with the IDs: the apply loop's first
  // iteration then waits on no round trip of its own (round 3: 2103 -> 2085 us)
  const u32 k0 = A.cc_off[g], k1 = A.cc_off[g + 1];
  u64 id0 = 0;
  u32 ty0 = 0;
  if (k0 < k1) {
    id0 = A.cc_node[k0];
    ty0 = A.cc_type[k0];
  }
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
  for (u32 k = k0; k < k1; ++k) {
    const u64 id = k == k0 ? id0 : A.cc_node[k];
    if (id == 0) continue;
    const u32 typ = k == k0 ? ty0 : u32(A.cc_type[k]);
    int x = find(t, r.n, id);
    const bool has_pr = x >= 0 && ((r.prs >> x) & 1u);
    if (typ == QB_CC_ADD_NODE || typ == QB_CC_ADD_LEARNER) {
      if (!has_pr) {  // initProgress
        if (x < 0) {
          if (r.n < TAB) {
            x = r.n++;
          } else {
            // Reuse an entry this change list freed (an ID it added and then
            // removed: no Progress, no role left).  Entries below n_old keep
            // their index (the carry of old slots maps by it), so only new
            // ones are candidates; the engine limit is then 24 IDs alive at
            // once within the list, not 24 seen over the whole list.
            for (int k = *n_old; k < r.n && x < 0; ++k)
              if (!((r.prs >> k) & 1u)) x = k;
            if (x < 0) return QB_CCERR_TOO_MANY_SLOTS;
            const u32 b = ~(1u << x);
            r.in &= b, r.out &= b, r.lnext &= b, r.lrn &= b, r.islrn &= b, r.fresh &= b;
          }
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

// The groups of pass BIG in [base, base + kBlk): kSmall launch (BIG false) —
// one workgroup per block of groups, the small ones; kTab launch (BIG true) —
// grid-strided over all blocks, the others, nothing at all when the kSmall
// launch flagged none.
template <bool BIG, class F>
__device__ __forceinline__ void for_my_groups(const Args& A, F&& f) {
  if constexpr (!BIG) {
    const u64 g = u64(blockIdx.x) * kBlk + threadIdx.x;
    const bool live = g < A.G;
    const bool big = live && needs_big(A, g);
    if (__ballot(big) && (threadIdx.x & 63) == 0) atomicOr(A.any_big, 1u);  // one per wave
    if (!live || big) return;
    f(g);
  } else {
    if (*A.any_big == 0) return;  // uniform: the first launch saw no big group
    for (u64 base = u64(blockIdx.x) * kBlk; base < A.G; base += u64(gridDim.x) * kBlk) {
      const u64 g = base + threadIdx.x;
      const bool mine = g < A.G && needs_big(A, g);
      if (mine) f(g);
    }
  }
}

template <int TAB, bool BIG>
__global__ __launch_bounds__(kBlk) void k_cc_count(Args A) {
  __shared__ u64 tabs[TAB][kBlk];
  for_my_groups<BIG>(A, [&](u64 g) {
    Tab t = tab_of(tabs);
    Roles r;
    bool al;
    u64 bad = 0;
    int n_old;
    const int rc = replay<TAB>(A, g, t, r, al, &bad, &n_old);
    A.new_cnt[g] = rc ? u32(n_old) : u32(__popc(r.prs));
    A.err[g] = u8(rc);
    if (A.err_id) A.err_id[g] = rc ? bad : 0;
  });
}

// The per-group pass only stores: new IDs, masks, and initProgress for fresh
// slots.  A carried slot (checkAndCopy's shallow copy) is marked in the new
// pstate (kCarried, never a valid QB_PR_* byte) with its old slot index in
// the new infl_pos; k_cc_copy then moves the Progress row and ring with one
// thread per new slot and overwrites both.  Keeping the copy out of the
// replay kernel keeps that kernel's LDS to the working tables (occupancy) and
// gives the byte moving a full-occupancy streaming launch of its own.
constexpr u8 kCarried = 0xFF;
// A fresh slot (initProgress) is marked kFresh with its group in the new
// infl_pos; k_cc_copy materialises it.  So every new slot's row is written
// by the copy kernel, whole lines per wave (round 2: the write pass storing
// fresh rows itself left scattered partial lines; 2565 -> 2220 us).
constexpr u8 kFresh = 0xFE;

template <int TAB>
__device__ void write_group(const Args& A, u64 g, u64 (*tabs)[kBlk]) {
  Tab t = tab_of(tabs);
  Roles r;
  bool al;
  u64 bad = 0;
  int n_old;
  int rc = replay<TAB>(A, g, t, r, al, &bad, &n_old);
  const u32 s0 = A.off[g];
  // the group's offset: its local prefix plus its scan block's sum (round 4:
  // the scan's add-back pass folded here, which also stores the offset);
  // its end from its own count (the next group's entry may already hold its
  // final offset)
  const u64 d0 = u64(A.new_cnt[g]) + A.nbsum[g / scan::kScanPer];
  const u64 d1 = d0 + (rc ? u32(n_old) : u32(__popc(r.prs)));
  A.new_cnt[g] = u32(d0);
  if (d1 > A.S_cap) return;  // the caller's capacity is exceeded (reported by new_off[G])
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
  u32 ncfg_in = 0, ncfg_out = 0, nlnext = 0;
  auto emit = [&](u32 j, int best) {
    const u32 b = 1u << best;
    if (r.in & b) ncfg_in |= 1u << j;
    if (r.out & b) ncfg_out |= 1u << j;
    if (r.lnext & b) nlnext |= 1u << j;
    const u64 d = d0 + j;
    const bool carried = best < n_old && !(r.fresh & b);
    A.n_ids[d] = t.id(best);
    if (carried) {  // carried Progress: k_cc_copy
      A.n_pstate[d] = kCarried;
      A.n_infl_pos[d] = s0 + u32(best);
    } else {  // initProgress (confchange.go:258-281): materialised by k_cc_copy
      A.n_pstate[d] = kFresh;
      A.n_infl_pos[d] = u32(g);
    }
  };
  // Surviving entries in ascending ID order.  The old slots are already
  // ascending (the CSR slot order) and the appended entries few, so they are
  // merged (one LDS read per output); an input table that is not ascending
  // takes the selection over all entries instead.
  bool asc = true;
  {
    u64 prev = 0;
    for (int k = 0; k < n_old; ++k) {
      const u64 v = t.id(k);
      asc = asc && (k == 0 || prev < v);
      prev = v;
    }
  }
  if (asc) {
    const u32 oldm = n_old >= 32 ? ~0u : ((1u << n_old) - 1u);
    u32 old_left = r.prs & oldm, add_left = r.prs & ~oldm;
    // smallest remaining appended entry (few: usually one)
    auto add_min = [&](u64& v) {
      int best = -1;
      for (u32 m = add_left; m; m &= m - 1u) {
        const int k = __builtin_ctz(m);
        const u64 x = t.id(k);
        if (best < 0 || x < v) {
          best = k;
          v = x;
        }
      }
      return best;
    };
    u64 ov = 0, av = 0;
    int oi = old_left ? __builtin_ctz(old_left) : -1;
    if (oi >= 0) ov = t.id(oi);
    int ai = add_min(av);
    for (u32 j = 0; oi >= 0 || ai >= 0; ++j) {
      if (oi >= 0 && (ai < 0 || ov < av)) {
        emit(j, oi);
        old_left &= old_left - 1u;
        oi = old_left ? __builtin_ctz(old_left) : -1;
        if (oi >= 0) ov = t.id(oi);
      } else {
        emit(j, ai);
        add_left &= ~(1u << ai);
        ai = add_min(av);
      }
    }
  } else {
    u32 left = r.prs;
    for (u32 j = 0; left; ++j) {
      int best = -1;
      for (int k = 0; k < r.n; ++k)
        if (((left >> k) & 1u) && (best < 0 || t.id(k) < t.id(best))) best = k;
      left &= ~(1u << best);
      emit(j, best);
    }
  }
  A.n_cfg[g] = ncfg_in | (ncfg_out << 16);
  A.n_ext[g] = nlnext | (al ? 1u << 16 : 0u);
}

template <int TAB, bool BIG>
__global__ __launch_bounds__(kBlk) void k_cc_write(Args A) {
  __shared__ u64 tabs[TAB][kBlk];
  for_my_groups<BIG>(A, [&](u64 g) { write_group<TAB>(A, g, tabs); });
}

// One thread per new slot d < min(new_off[G], S_cap), grid-stride: a carried
// slot's match / next / pendingSnapshot / inflight position / state byte and
// its ring come from the old slot; a fresh slot's ring is zeroed.  A slot of
// a group past the capacity was never written: the source bound keeps any
// stale marker from reading outside the old arrays.
__global__ __launch_bounds__(256) void k_cc_copy(Args A) {
  const u64 total = A.new_cnt[A.G];
  const u64 end = total < A.S_cap ? total : A.S_cap;
  const u32 old_total = A.off[A.G];
  const u32 K = A.K;
  for (u64 d = u64(blockIdx.x) * 256 + threadIdx.x; d < end; d += u64(gridDim.x) * 256) {
    const u8 mk = A.n_pstate[d];
    const bool carried = mk == kCarried, fresh = mk == kFresh;
    const u32 src = carried || fresh ? A.n_infl_pos[d] : 0u;
    const bool ok = carried && src < old_total;
    if (ok) {
      const u64 m = A.match[src], nx = A.next[src], ps = A.psnap[src];
      const u32 ip = A.infl_pos[src];
      const u8 st = A.pstate[src];
      A.n_match[d] = m;
      A.n_next[d] = nx;
      A.n_psnap[d] = ps;
      A.n_infl_pos[d] = ip;
      A.n_pstate[d] = st;
    } else if (fresh) {  // initProgress (confchange.go:258-281); src = the group
      A.n_match[d] = 0;
      A.n_next[d] = A.last_index[src];
      A.n_psnap[d] = 0;
      A.n_infl_pos[d] = 0;
      A.n_pstate[d] = QB_PR_PROBE | QB_PR_RECENT_ACTIVE;
    }
    if (K) {
      const u64* sr = A.infl_buf + u64(src) * K;
      u64* dr = A.n_infl_buf + d * K;
      u32 k = 0;
      for (; k + 4 <= K; k += 4) {
        u64 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ok ? sr[k + q] : 0ull;
#pragma unroll
        for (int q = 0; q < 4; ++q) dr[k + q] = v[q];
      }
      for (; k < K; ++k) dr[k] = ok ? sr[k] : 0ull;
    }
  }
}

}  // namespace cc
}  // namespace qb

using namespace qb;

extern "C" size_t qb_conf_change_workspace_bytes(uint64_t G) {
  // the scan's block sums, then the any_big word
  return (scan::blocks(G) + 1) * sizeof(u32) + 256 + 256;
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
  const size_t scan_bytes = (scan::blocks(G) + 1) * sizeof(u32);
  A.any_big = reinterpret_cast<u32*>(static_cast<char*>(workspace) + (scan_bytes + 255) / 256 * 256);
  {
    const hipError_t e = hipMemsetAsync(A.any_big, 0, sizeof(u32), st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(any_big)");
  }
  const unsigned grid = unsigned((G + cc::kBlk - 1) / cc::kBlk);
  const unsigned big_grid = grid < cc::kBigGrid ? grid : cc::kBigGrid;
  hipLaunchKernelGGL((cc::k_cc_count<cc::kSmall, false>), dim3(grid), dim3(cc::kBlk), 0, st, A);
  hipLaunchKernelGGL((cc::k_cc_count<cc::kTab, true>), dim3(big_grid), dim3(cc::kBlk), 0, st, A);
  QB_CHECK_LAUNCH("k_cc_count");
  {  // local scan + block sums (the add-back is in k_cc_write); new_off[G] = total
    u32* bsum = static_cast<u32*>(workspace);
    const u32 nb = scan::blocks(G);
    hipLaunchKernelGGL(scan::k_scan_local, dim3(nb), dim3(1024), 0, st, out->new_off, G, bsum);
    hipLaunchKernelGGL(scan::k_scan_sums, dim3(1), dim3(1024), 0, st, bsum, nb, out->new_off + G);
    A.nbsum = bsum;
  }
  QB_CHECK_LAUNCH("scan(conf change)");
  hipLaunchKernelGGL((cc::k_cc_write<cc::kSmall, false>), dim3(grid), dim3(cc::kBlk), 0, st, A);
  hipLaunchKernelGGL((cc::k_cc_write<cc::kTab, true>), dim3(big_grid), dim3(cc::kBlk), 0, st, A);
  QB_CHECK_LAUNCH("k_cc_write");
  hipLaunchKernelGGL(cc::k_cc_copy, dim3(2048), dim3(256), 0, st, A);
  QB_CHECK_LAUNCH("k_cc_copy");
  return QB_OK;
}
