// qb_host.cpp — host-side config compile: tracker.Config per group -> the CSR
// layout the device kernels read (include/quorum_batch.h).
//
//   tracker.Config {Voters [2]MajorityConfig, Learners, LearnersNext}
//                                        tracker/tracker.go:27-78
//   slot order = MajorityConfig.Slice over the union (sorted IDs)
//                                        quorum/majority.go:106-113
//   Learners ∩ Voters = ∅ (checkInvariants) confchange/confchange.go:307-318
//
// A group's slots are the sorted union of Voters[0], Voters[1] and Learners
// (LearnersNext members are outgoing voters until LeaveJoint and sit in
// Voters[1] already); cfg = mask_in | mask_out << 16 over those slots, a
// learner is in neither mask.  Duplicate IDs within a list are one member
// (the Go sets are maps).  Two passes over the groups (count, then write),
// split over host threads for large G.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "qb_common.h"

namespace {

using qb::u32;
using qb::u64;

constexpr u32 kMaxIds = 3 * QB_MAX_SLOTS + 3;

enum : int { kOk = 0, kTooMany = 1, kOverlapIn = 2, kOverlapOut = 3, kListTooLong = 4 };

struct Lists {
  const u32 *in_off, *out_off, *lrn_off;
  const u64 *in_ids, *out_ids, *lrn_ids;
};

struct Span {
  const u64* p;
  u32 n;
};

inline Span span(const u32* off, const u64* ids, u64 g) {
  if (!off) return {nullptr, 0};
  return {ids + off[g], off[g + 1] - off[g]};
}

inline bool has(const Span& s, u64 id) {
  for (u32 k = 0; k < s.n; ++k)
    if (s.p[k] == id) return true;
  return false;
}

// Sorted, de-duplicated union of the group's three lists into ids[]; returns
// the status and sets *n, *cfg (*who: the offending learner, the smallest one
// when several are: Go reports whichever its map iteration meets first).
int compile_one(const Lists& L, u64 g, u64* ids, u32* n, u32* cfg, u64* who = nullptr) {
  const Span vi = span(L.in_off, L.in_ids, g), vo = span(L.out_off, L.out_ids, g),
             lr = span(L.lrn_off, L.lrn_ids, g);
  if (u64(vi.n) + vo.n + lr.n > kMaxIds) return kListTooLong;
  int bad = kOk;
  u64 worst = 0;
  for (u32 k = 0; k < lr.n; ++k) {  // confchange.go:307-318: Voters[1] first, then Voters[0]
    const u64 id = lr.p[k];
    const int rc = has(vo, id) ? kOverlapOut : has(vi, id) ? kOverlapIn : kOk;
    if (rc != kOk && (bad == kOk || id < worst)) bad = rc, worst = id;
  }
  if (bad != kOk) {
    if (who) *who = worst;
    return bad;
  }
  u32 m = 0;
  for (const Span* s : {&vi, &vo, &lr})
    for (u32 k = 0; k < s->n; ++k) ids[m++] = s->p[k];
  std::sort(ids, ids + m);
  m = u32(std::unique(ids, ids + m) - ids);
  if (m > QB_MAX_SLOTS) return kTooMany;
  u32 min_ = 0, mout = 0;
  for (u32 j = 0; j < m; ++j) {
    if (has(vi, ids[j])) min_ |= 1u << j;
    if (has(vo, ids[j])) mout |= 1u << j;
  }
  *n = m;
  *cfg = min_ | (mout << 16);
  return kOk;
}

template <class F>
void parallel_groups(u64 G, F&& f) {
  unsigned T = std::thread::hardware_concurrency();
  T = T < 1 ? 1 : T > 16 ? 16 : T;
  if (G < (1u << 16)) T = 1;
  if (T == 1) {
    f(0, G, 0u);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t)
    th.emplace_back([&, t] { f(G * t / T, G * (t + 1) / T, t); });
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" int qb_host_compile_configs(uint64_t G, const uint32_t* in_off, const uint64_t* in_ids,
                                       const uint32_t* out_off, const uint64_t* out_ids,
                                       const uint32_t* lrn_off, const uint64_t* lrn_ids,
                                       uint32_t* off, uint32_t* cfg, uint64_t* slot_ids,
                                       uint64_t slot_cap, uint64_t* bad_group) {
  QB_REQUIRE(G == 0 || (in_off && off && cfg), "in_off/off/cfg NULL");
  QB_REQUIRE(!out_off || out_ids || G == 0 || out_off[G] == 0, "out_ids NULL");
  QB_REQUIRE(!lrn_off || lrn_ids || G == 0 || lrn_off[G] == 0, "lrn_ids NULL");
  if (bad_group) *bad_group = UINT64_MAX;
  if (G == 0) {
    if (off) off[0] = 0;
    return QB_OK;
  }
  QB_REQUIRE(in_ids || in_off[G] == 0, "in_ids NULL");
  const Lists L{in_off, out_off, lrn_off, reinterpret_cast<const u64*>(in_ids),
                reinterpret_cast<const u64*>(out_ids), reinterpret_cast<const u64*>(lrn_ids)};
  // pass 1: per-group slot counts and masks; the first failing group wins
  std::atomic<u64> first_bad{UINT64_MAX};
  parallel_groups(G, [&](u64 lo, u64 hi, unsigned) {
    u64 ids[kMaxIds];
    for (u64 g = lo; g < hi; ++g) {
      u32 n = 0, c = 0;
      const int rc = compile_one(L, g, ids, &n, &c);
      if (rc != kOk) {
        u64 cur = first_bad.load();
        while (g < cur && !first_bad.compare_exchange_weak(cur, g)) {
        }
        return;
      }
      off[g + 1] = n;  // count for now; prefix-summed below
      cfg[g] = c;
    }
  });
  if (first_bad.load() != UINT64_MAX) {
    const u64 g = first_bad.load();
    if (bad_group) *bad_group = g;
    // recompute the reason for the reported group
    u64 ids[kMaxIds], who = 0;
    u32 n = 0, c = 0;
    const int rc = compile_one(L, g, ids, &n, &c, &who);
    switch (rc) {
      case kOverlapIn:
      case kOverlapOut:
        qb::set_error("group %llu: %llu is in Learners and Voters[%d]", (unsigned long long)g,
                      (unsigned long long)who, rc == kOverlapOut ? 1 : 0);
        break;
      case kTooMany:
        qb::set_error("group %llu: more than %d members (QB_MAX_SLOTS)", (unsigned long long)g,
                      QB_MAX_SLOTS);
        break;
      default:
        qb::set_error("group %llu: ID lists longer than %u", (unsigned long long)g, kMaxIds);
    }
    return QB_EINVAL;
  }
  off[0] = 0;
  for (u64 g = 0; g < G; ++g) {
    const u64 next = u64(off[g]) + off[g + 1];
    QB_REQUIRE(next <= 0xFFFFFFFFull, "total slots overflow uint32 at group %llu",
               (unsigned long long)g);
    off[g + 1] = u32(next);
  }
  if (!slot_ids) return QB_OK;  // sizing call: off[G] = slots needed
  QB_REQUIRE(slot_cap >= off[G], "slot_ids too small: need %u, have %llu", off[G],
             (unsigned long long)slot_cap);
  // pass 2: the sorted slot IDs
  parallel_groups(G, [&](u64 lo, u64 hi, unsigned) {
    u64 ids[kMaxIds];
    for (u64 g = lo; g < hi; ++g) {
      u32 n = 0, c = 0;
      compile_one(L, g, ids, &n, &c);
      std::memcpy(slot_ids + off[g], ids, sizeof(u64) * n);
    }
  });
  return QB_OK;
}
