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
// the surviving entries are sorted by ID into the new slots.  The count pass
// replays and orders each group and leaves a slot code word (which old slot
// or change entry each new slot comes from); after a scan of the counts the
// placement pass writes the new slots from the codes without a replay (round
// 4 replayed twice: count, then write).
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
  // K == 4 and both ring buffers 16-byte aligned: the ring moves as 16-byte
  // words (the ABI promises only 8-byte alignment of u64 arrays;
  // an unaligned caller's ring takes the 8-byte loop)
  u32 ring16;
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
  u64* codes;    // workspace [G]: each group's slot codes (k_cc_count -> k_cc_move)
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
// chg (kSmall tables only): for an entry the change list created, the index
// within the list of the change that last (re)created it, four bits per entry
// (a kSmall group has at most 8 changes), so the placement pass can read the
// entry's ID without a replay.
template <int TAB>
__device__ int replay(const Args& A, u64 g, const Tab& t, Roles& r, bool& autoleave, u64* bad,
                      int* n_old, u32* chg = nullptr) {
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
          if constexpr (TAB <= 8)
            if (chg) *chg = (*chg & ~(0xFu << (4 * x))) | ((k - k0) << (4 * x));
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

// Markers (the kTab groups' write pass): a carried slot (checkAndCopy's
// shallow copy) is marked in the new pstate (kCarried, never a valid QB_PR_*
// byte) with its old slot index in the new infl_pos, a fresh slot
// (initProgress) kFresh with its group; k_cc_move reads them and writes the
// Progress row and ring.  Keeping the copy out of the replay kernels keeps
// their LDS to the working tables (occupancy) and gives the byte moving a
// full-occupancy streaming launch of its own.
constexpr u8 kCarried = 0xFF;
constexpr u8 kFresh = 0xFE;

// A failed change keeps the old config: its roles, read back from cfg / ext.
__device__ __forceinline__ void kept_roles(const Args& A, u64 g, int n_old, Roles& r, bool& al) {
  r = Roles{};
  r.n = n_old;
  r.prs = n_old >= 32 ? ~0u : ((1u << n_old) - 1u);
  const u32 c = A.cfg[g], e = A.ext ? A.ext[g] : 0u;
  r.in = c & 0xFFFFu;
  r.out = c >> 16;
  r.lnext = e & 0xFFFFu;
  al = (e >> 16) & 1u;
}

// The surviving entries in ascending ID order: emit(j, entry) for the new
// slot j.  The old slots are already ascending (the CSR slot order) and the
// appended entries few, so they are merged (one LDS read per output); an
// input table that is not ascending takes the selection over all entries.
template <class E>
__device__ __forceinline__ void order_out(const Tab& t, const Roles& r, int n_old, E&& emit) {
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
}

// Slot codes (round 5).  The kSmall count pass orders the new slots itself
// and leaves one byte per new slot (8 per group, 0xFF past the last) in the
// workspace, with the new cfg / ext written directly: the placement pass
// (k_cc_move) then needs no replay — it reads the code word, the group's
// offset and the IDs the codes name.  Code: bits 0-3 the entry's source (an
// old slot index, or with kCodeAppended the change list index that created
// it), kCodeFresh an initProgress slot.
constexpr u8 kCodeAppended = 0x10, kCodeFresh = 0x20, kCodeNone = 0xFF;
// A kTab group's code word: kBigCode | its slot count (k_cc_write places it
// and leaves markers, as round 4 did for every group).
constexpr u64 kBigCode = 0xFEull << 56;

// A group whose current config has more slots than the working table (only
// possible for an input this engine did not produce: past QB_MAX_SLOTS
// members) is never replayed — its table would overrun the LDS block — and
// keeps its config as it is: no operation copies it through, any other is
// refused with the engine limit's error.
__device__ __forceinline__ u32 oversize_slots(const Args& A, u64 g) {
  const u32 ns = A.off[g + 1] - A.off[g];
  return ns > u32(kTab) ? ns : 0u;
}

template <int TAB, bool BIG>
__global__ __launch_bounds__(kBlk) void k_cc_count(Args A) {
  __shared__ u64 tabs[TAB][kBlk];
  for_my_groups<BIG>(A, [&](u64 g) {
    if constexpr (BIG) {
      if (const u32 ns = oversize_slots(A, g)) {
        const int rc = A.op[g] == QB_CC_NONE ? 0 : QB_CCERR_TOO_MANY_SLOTS;
        A.new_cnt[g] = ns;
        A.err[g] = u8(rc);
        if (A.err_id) A.err_id[g] = 0;
        A.codes[g] = kBigCode | ns;
        return;
      }
    }
    Tab t = tab_of(tabs);
    Roles r;
    bool al;
    u64 bad = 0;
    int n_old;
    u32 chg = 0;
    const int rc = replay<TAB>(A, g, t, r, al, &bad, &n_old, BIG ? nullptr : &chg);
    A.new_cnt[g] = rc ? u32(n_old) : u32(__popc(r.prs));
    A.err[g] = u8(rc);
    if (A.err_id) A.err_id[g] = rc ? bad : 0;
    if constexpr (BIG) {
      A.codes[g] = kBigCode | (rc ? u32(n_old) : u32(__popc(r.prs)));  // (k_cc_move reads its markers)
    } else {
      if (rc) kept_roles(A, g, n_old, r, al);
      u32 ncfg_in = 0, ncfg_out = 0, nlnext = 0;
      u64 code = 0x0101010101010101ull * kCodeNone;  // kCodeNone in every byte
      order_out(t, r, n_old, [&](u32 j, int best) {
        const u32 b = 1u << best;
        if (r.in & b) ncfg_in |= 1u << j;
        if (r.out & b) ncfg_out |= 1u << j;
        if (r.lnext & b) nlnext |= 1u << j;
        u32 c;
        if (best < n_old) c = u32(best) | ((r.fresh & b) ? kCodeFresh : 0u);
        else c = ((chg >> (4 * best)) & 0xFu) | kCodeAppended | kCodeFresh;
        code = (code & ~(0xFFull << (8 * j))) | (u64(c) << (8 * j));
      });
      A.codes[g] = code;
      A.n_cfg[g] = ncfg_in | (ncfg_out << 16);
      A.n_ext[g] = nlnext | (al ? 1u << 16 : 0u);
    }
  });
}

// The kTab groups (old slots + changes > kSmall; grid-strided, none at all in
// the usual batch): the write pass replays the change again.
template <int TAB>
__device__ void write_group(const Args& A, u64 g, u64 (*tabs)[kBlk]) {
  if (const u32 ns = oversize_slots(A, g)) {  // kept in slot order, every Progress carried
    const u32 s0 = A.off[g];
    const u64 d0 = u64(A.new_cnt[g]) + A.nbsum[g / scan::kScanPer];
    A.new_cnt[g] = u32(d0);
    if (d0 + ns > A.S_cap) return;
    for (u32 j = 0; j < ns; ++j) {
      A.n_ids[d0 + j] = A.ids[s0 + j];
      A.n_pstate[d0 + j] = kCarried;
      A.n_infl_pos[d0 + j] = s0 + j;
    }
    A.n_cfg[g] = A.cfg[g];
    A.n_ext[g] = A.ext ? A.ext[g] & 0x1FFFFu : 0u;
    return;
  }
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
  if (rc) kept_roles(A, g, n_old, r, al);
  u32 ncfg_in = 0, ncfg_out = 0, nlnext = 0;
  order_out(t, r, n_old, [&](u32 j, int best) {
    const u32 b = 1u << best;
    if (r.in & b) ncfg_in |= 1u << j;
    if (r.out & b) ncfg_out |= 1u << j;
    if (r.lnext & b) nlnext |= 1u << j;
    const u64 d = d0 + j;
    const bool carried = best < n_old && !(r.fresh & b);
    A.n_ids[d] = t.id(best);
    if (carried) {  // carried Progress: k_cc_move
      A.n_pstate[d] = kCarried;
      A.n_infl_pos[d] = s0 + u32(best);
    } else {  // initProgress (confchange.go:258-281): materialised by k_cc_move
      A.n_pstate[d] = kFresh;
      A.n_infl_pos[d] = u32(g);
    }
  });
  A.n_cfg[g] = ncfg_in | (ncfg_out << 16);
  A.n_ext[g] = nlnext | (al ? 1u << 16 : 0u);
}

template <int TAB>
__global__ __launch_bounds__(kBlk) void k_cc_write(Args A) {
  __shared__ u64 tabs[TAB][kBlk];
  for_my_groups<true>(A, [&](u64 g) { write_group<TAB>(A, g, tabs); });
}

// Placement and copy in one pass (round 5; round 4 wrote each new slot's ID
// and a marker from a per-group thread — 64 lanes storing 6-slot runs, partial
// lines — and a per-slot copy kernel read the markers back).  A wave takes 64
// consecutive groups: each lane its group's offset (stored as new_off[g]),
// count and code word, staged in LDS with the owner lane of every slot of the
// wave's range; then the wave walks the range [D0, D1) one slot per lane, two
// slots per lane at a time (both slots' loads issued before either's stores:
// the outputs could alias the inputs as far as the compiler knows), and
// writes ID, Progress row and ring with whole-line stores.  A kTab group
// (k_cc_write placed it and left markers) is read from its markers.  A group
// past the caller's capacity is not written.
constexpr u32 kMoveSpan = 64 * QB_MAX_SLOTS;  // slots of a wave's 64 groups, at most
struct MoveStage {
  u32 d0[4][64];
  u32 s0[4][64];
  u32 k0[4][64];
  u64 code[4][64];
  u8 owner[4][kMoveSpan];
};
// One slot's sources (resolved from LDS) and values (loaded).
struct Mv {
  bool write, ok, fresh, marker;
  u32 src, p;
  u64 id, m, nx, ps, r[4];
  u32 ip;
  u8 st;
};
__global__ __launch_bounds__(256) void k_cc_move(Args A) {
  __shared__ MoveStage ms;
  const u32 w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const u64 g0 = (u64(blockIdx.x) * 4 + w) * 64;
  const u64 g = g0 + lane;
  const bool live = g < A.G;
  u64 code = 0;
  u32 d0 = 0, n = 0, s0 = 0, k0 = 0;
  if (live) {
    code = A.codes[g];
    s0 = A.off[g];
    k0 = A.cc_off[g];
    if ((code & (0xFFull << 56)) == kBigCode) {
      n = u32(code);
      d0 = A.new_cnt[g];  // (k_cc_write stored the final offset)
    } else {
      const u64 none = code & 0x8080808080808080ull;  // kCodeNone bytes (a code is < 0x80)
      n = none ? u32(__builtin_ctzll(none)) / 8 : 8u;
      d0 = A.new_cnt[g] + A.nbsum[g / scan::kScanPer];
      A.new_cnt[g] = d0;
    }
  }
  // the wave's slot range [D0, dlast); lanes past G: empty groups at its end
  const u32 nlive = g0 >= A.G ? 0u : u32(A.G - g0 < 64 ? A.G - g0 : 64);
  const u32 dlast = nlive ? u32(__shfl(int(d0 + n), int(nlive - 1), 64)) : 0u;
  const u32 D0 = u32(__shfl(int(d0), 0, 64));
  if (!live) {
    d0 = dlast;
    n = 0;
  }
  ms.d0[w][lane] = d0;
  ms.s0[w][lane] = s0;
  ms.k0[w][lane] = k0;
  ms.code[w][lane] = code;
  // the owner lane of every slot of the range (a new config has at most
  // QB_MAX_SLOTS slots; a failed change keeps its old slots, and a wave whose
  // range exceeds the table finds its owners by a binary search instead)
  const bool wide = dlast - D0 > kMoveSpan;  // (wave-uniform)
  if (!wide)
    for (u32 j = 0; j < n; ++j) ms.owner[w][d0 - D0 + j] = u8(lane);
  __syncthreads();
  const u64 cap = A.S_cap;
  const u32 old_total = A.off[A.G];
  const u32 K = A.K;
  auto resolve = [&](u32 p, Mv& v) {
    v.write = false;
    v.marker = false;
    v.p = p;
    if (p >= dlast) return;
    u32 q = 0;
    if (!wide) {
      q = ms.owner[w][p - D0];
    } else {  // the last lane whose offset is <= p
#pragma unroll
      for (u32 step = 32; step; step >>= 1)
        if (ms.d0[w][q + step] <= p) q += step;
    }
    const u64 c = ms.code[w][q];
    const u32 qd0 = ms.d0[w][q];
    if ((c & (0xFFull << 56)) == kBigCode) {
      if (u64(qd0) + u32(c) > cap) return;  // past the capacity: not written
      v.write = true;
      v.marker = true;  // (sources from k_cc_write's markers, below)
      return;
    }
    const u64 none = c & 0x8080808080808080ull;
    const u32 cn = none ? u32(__builtin_ctzll(none)) / 8 : 8u;
    if (u64(qd0) + cn > cap) return;  // past the capacity: not written
    const u32 b = u32(c >> (8 * (p - qd0))) & 0xFFu, sl = b & 0xFu;
    v.write = true;
    v.fresh = (b & kCodeFresh) != 0;
    v.src = v.fresh ? u32(g0 + q) : ms.s0[w][q] + sl;
    v.ok = !v.fresh && v.src < old_total;
    // the ID's position, in the ID field until the loads
    v.id = (b & kCodeAppended) ? (1ull << 63) | (ms.k0[w][q] + sl) : u64(ms.s0[w][q] + sl);
  };
  auto load = [&](Mv& v) {
    if (!v.write) return;
    if (v.marker) {  // a kTab group's slot: k_cc_write stored its ID and marker
      const u8 mk = A.n_pstate[v.p];
      v.src = A.n_infl_pos[v.p];
      v.fresh = mk == kFresh;
      v.ok = mk == kCarried && v.src < old_total;
    } else {
      v.id = (v.id >> 63) ? A.cc_node[u32(v.id)] : A.ids[u32(v.id)];
    }
    if (v.ok) {
      v.m = A.match[v.src];
      v.nx = A.next[v.src];
      v.ps = A.psnap[v.src];
      v.ip = A.infl_pos[v.src];
      v.st = A.pstate[v.src];
    } else if (v.fresh) {
      v.nx = A.last_index[v.src];
    }
    if (K == 4 && A.ring16) {  // the ring as two 16-byte loads (the kernel is issue-bound on its
                   // vector-memory instructions: 1 ring instruction pair instead of 4)
      const ulonglong2* sr = reinterpret_cast<const ulonglong2*>(A.infl_buf + u64(v.src) * 4);
      ulonglong2 x0 = make_ulonglong2(0, 0), x1 = x0;
      if (v.ok) {
        x0 = sr[0];
        x1 = sr[1];
      }
      v.r[0] = x0.x;
      v.r[1] = x0.y;
      v.r[2] = x1.x;
      v.r[3] = x1.y;
    } else if (K < 4) {
      const u64* sr = A.infl_buf + u64(v.src) * K;
#pragma unroll
      for (u32 k = 0; k < 4; ++k) v.r[k] = (v.ok && k < K) ? sr[k] : 0ull;
    }
  };
  auto store = [&](const Mv& v) {
    if (!v.write) return;
    const u64 d = v.p;
    if (!v.marker) A.n_ids[d] = v.id;
    if (v.ok) {
      A.n_match[d] = v.m;
      A.n_next[d] = v.nx;
      A.n_psnap[d] = v.ps;
      A.n_infl_pos[d] = v.ip;
      A.n_pstate[d] = v.st;
    } else if (v.fresh) {  // initProgress (confchange.go:258-281)
      A.n_match[d] = 0;
      A.n_next[d] = v.nx;
      A.n_psnap[d] = 0;
      A.n_infl_pos[d] = 0;
      A.n_pstate[d] = QB_PR_PROBE | QB_PR_RECENT_ACTIVE;
    }
    u64* dr = A.n_infl_buf + d * K;
    if (K == 4 && A.ring16) {
      ulonglong2* d2 = reinterpret_cast<ulonglong2*>(dr);
      d2[0] = make_ulonglong2(v.r[0], v.r[1]);
      d2[1] = make_ulonglong2(v.r[2], v.r[3]);
    } else if (K < 4) {
#pragma unroll
      for (u32 k = 0; k < 4; ++k)
        if (k < K) dr[k] = v.r[k];
    } else {
      const u64* sr = A.infl_buf + u64(v.src) * K;
      u32 k = 0;
      for (; k + 4 <= K; k += 4) {
        u64 x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = v.ok ? sr[k + q] : 0ull;
#pragma unroll
        for (int q = 0; q < 4; ++q) dr[k + q] = x[q];
      }
      for (; k < K; ++k) dr[k] = v.ok ? sr[k] : 0ull;
    }
  };
  for (u32 p = D0 + lane; p < dlast; p += 128) {
    Mv a, b;
    resolve(p, a);
    resolve(p + 64, b);
    load(a);
    load(b);
    store(a);
    store(b);
  }
}

}  // namespace cc
}  // namespace qb

using namespace qb;

namespace {
// the scan's block sums, the any_big word, the slot codes
size_t cc_codes_at(uint64_t G) { return ((scan::blocks(G) + 1) * sizeof(u32) + 255) / 256 * 256 + 256; }
}  // namespace

extern "C" size_t qb_conf_change_workspace_bytes(uint64_t G) {
  return cc_codes_at(G) + G * sizeof(u64) + 256;
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
  A.ring16 = (reinterpret_cast<uintptr_t>(in->infl_buf) & 15u) == 0 &&
             (reinterpret_cast<uintptr_t>(out->infl_buf) & 15u) == 0;
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
  A.codes = reinterpret_cast<u64*>(static_cast<char*>(workspace) + cc_codes_at(G));
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
  hipLaunchKernelGGL(cc::k_cc_write<cc::kTab>, dim3(big_grid), dim3(cc::kBlk), 0, st, A);
  QB_CHECK_LAUNCH("k_cc_write");
  hipLaunchKernelGGL(cc::k_cc_move, dim3(unsigned((G + 255) / 256)), dim3(256), 0, st, A);
  QB_CHECK_LAUNCH("k_cc_move");
  return QB_OK;
}
