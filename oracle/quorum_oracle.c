/*
 * quorum_oracle.c — C restatement of etcd's raft quorum/tracker hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this library (oracle/liborc_quorum.so),
 * and only as the checker / the timed CPU baseline — never as the product.
 *
 * Pinning: validated against oracle/quorum_ref.py (itself pinned 127/127 by
 * the reference's datadriven golden files and the TestCommit /
 * TestLeaderElectionInOneRoundRPC / TestProgressUpdate tables, committed in
 * tests/golden/).  The reference is Go and no Go toolchain exists in this
 * image, so the reference itself cannot be compiled into oracle/_ref.
 *
 * Contents (paths relative to the reference's raft/):
 *   - splitmix64 synthetic-input spec, restated here
 *     independently of the product's HIP generator so parity tests also
 *     cross-check input generation;
 *   - orc_faithful_*: the Go loop as written — a per-group hash-map
 *     MajorityConfig ranged over, a hash-map AckedIndexer looked up per
 *     voter, fill-from-the-right and insertionSort (quorum/majority.go:115-210,
 *     quorum/joint.go:49-75) — the timed CPU baseline;
 *   - orc_fixed_* / orc_csr_*: the same semantics over SoA arrays;
 *   - orc_fixed_appresp_sequential: one record at a time, in batch order:
 *     raft.Step's term filter (raft.go:847-921), stepLeader's non-member drop
 *     (raft.go:1100-1104), RecentActive (raft.go:1107), MaybeUpdate
 *     (tracker/progress.go:144-153) and, when it updated, maybeCommit
 *     (raft.go:585-588 -> log.go:328-334).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;

#define INF UINT64_MAX
#define V_PENDING 1
#define V_LOST 2
#define V_WON 3

/* ------------------------------------------------------------------ RNG --- */

static inline u64 splitmix64(u64 x) {
  u64 z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline u64 r3(u64 seed, u64 g, u32 slot, u32 field) {
  return splitmix64(seed ^ ((g << 12) | ((u64)slot << 4) | field));
}
enum { F_LAST, F_HIGH, F_HIGHBITS, F_ABSENT, F_LAG, F_VOTE, F_TERMSTART, F_N, F_L, F_LPOS,
       F_OVERLAP, F_ROT };

static u64 gen_last(u64 seed, u64 g) {
  u64 last = 1 + r3(seed, g, 0, F_LAST) % ((1ull << 40) - 1);
  if (r3(seed, g, 0, F_HIGH) % 100 == 0)
    last |= (1ull << 63) | (r3(seed, g, 0, F_HIGHBITS) & 0x3FFFFF0000000000ull);
  return last;
}
static u64 gen_match(u64 seed, u64 g, u32 j, u64 last) {
  if (j == 0) return last;
  if (r3(seed, g, j, F_ABSENT) % 100 < 5) return 0;
  u64 lag = r3(seed, g, j, F_LAG) % 64;
  return last - (lag < last ? lag : last);
}
static int gen_vote(u64 seed, u64 g, u32 j, int* granted) {
  u64 v = r3(seed, g, j, F_VOTE) % 10;
  *granted = v >= 5;
  return v >= 3;
}
static u64 gen_term_start(u64 seed, u64 g, u64 last) {
  u64 d = r3(seed, g, 0, F_TERMSTART) % 128;
  return last > d ? last - d : 1;
}
static u32 gen_ragged_size(u64 seed, u64 g) {
  return 3 + (u32)(r3(seed, g, 0, F_N) % 7) + (u32)(r3(seed, g, 0, F_L) % 3);
}
static u32 gen_ragged_mask(u64 seed, u64 g, u32 s) {
  u32 L = (u32)(r3(seed, g, 0, F_L) % 3), mask = (1u << s) - 1;
  for (u32 l = 0; l < L; ++l) {
    u32 p = 1 + (u32)(r3(seed, g, l, F_LPOS) % (s - 1));
    while (!((mask >> p) & 1)) p = (p + 1 < s) ? p + 1 : 1;
    mask &= ~(1u << p);
  }
  return mask;
}
static u32 gen_joint_size(u64 seed, u64 g) { return 10 - (u32)(r3(seed, g, 0, F_OVERLAP) % 6); }
static u32 rotl_u(u32 m, u32 r, u32 u) {
  return r == 0 ? m : (((m << r) | (m >> (u - r))) & ((1u << u) - 1));
}
static u32 gen_joint_cfg(u64 seed, u64 g, u32 u) {
  u32 k = 10 - u, rot = (u32)(r3(seed, g, 0, F_ROT) % u);
  return rotl_u(0x1Fu, rot, u) | (rotl_u(0x1Fu << (5 - k), rot, u) << 16);
}

/* Fixed layout: match[n][G] slot-major; masks u8 (n<=8) or u16. */
void orc_gen_fixed(u64 seed, u32 n, u64 G, u64 g_begin, u64* match, void* voted, void* granted,
                   u64* term_start) {
  for (u64 g = 0; g < G; ++g) {
    u64 gg = g_begin + g, last = gen_last(seed, gg);
    u32 vd = 0, gr = 0;
    for (u32 j = 0; j < n; ++j) {
      if (match) match[(u64)j * G + g] = gen_match(seed, gg, j, last);
      int yes;
      if (gen_vote(seed, gg, j, &yes)) {
        vd |= 1u << j;
        if (yes) gr |= 1u << j;
      }
    }
    if (n <= 8) {
      if (voted) ((u8*)voted)[g] = (u8)vd;
      if (granted) ((u8*)granted)[g] = (u8)gr;
    } else {
      if (voted) ((u16*)voted)[g] = (u16)vd;
      if (granted) ((u16*)granted)[g] = (u16)gr;
    }
    if (term_start) term_start[g] = gen_term_start(seed, gg, last);
  }
}

/* kind 0 ragged, 1 joint.  off[G+1] is written too. Returns 0 or -1 on overflow. */
int orc_gen_csr(u64 seed, int kind, u64 G, u64 g_begin, u32* off, u64* match, u32* cfg,
                u32* votes) {
  u64 acc = 0;
  off[0] = 0;
  for (u64 g = 0; g < G; ++g) {
    acc += kind ? gen_joint_size(seed, g_begin + g) : gen_ragged_size(seed, g_begin + g);
    if (acc > 0xFFFFFFFFull) return -1;
    off[g + 1] = (u32)acc;
  }
  for (u64 g = 0; g < G; ++g) {
    u64 gg = g_begin + g, last = gen_last(seed, gg);
    u32 a = off[g], s = off[g + 1] - a, vd = 0, gr = 0;
    for (u32 j = 0; j < s; ++j) {
      if (match) match[a + j] = gen_match(seed, gg, j, last);
      int yes;
      if (gen_vote(seed, gg, j, &yes)) {
        vd |= 1u << j;
        if (yes) gr |= 1u << j;
      }
    }
    if (cfg) cfg[g] = kind ? gen_joint_cfg(seed, gg, s) : gen_ragged_mask(seed, gg, s);
    if (votes) votes[g] = vd | (gr << 16);
  }
  return 0;
}

/* ------------------------------------------------ quorum/majority.go ----- */

static void insertion_sort(u64* sl, int n) { /* majority.go:115-122 */
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && sl[j] < sl[j - 1]; --j) {
      u64 t = sl[j];
      sl[j] = sl[j - 1];
      sl[j - 1] = t;
    }
}

/* MajorityConfig.CommittedIndex over an SoA member list: vals[k] for the
 * k-th member (acked always; the tracker has a Progress for every voter). */
static u64 majority_ci(const u64* vals, int n) { /* majority.go:126-172 */
  if (n == 0) return INF;
  u64 srt[64];
  int i = n - 1;
  for (int k = 0; k < n; ++k) srt[i--] = vals[k];
  insertion_sort(srt, n);
  return srt[n - (n / 2 + 1)];
}

static u8 majority_vote(int n, int yes, int no) { /* majority.go:178-210 */
  if (n == 0) return V_WON;
  int missing = n - yes - no, q = n / 2 + 1;
  if (yes >= q) return V_WON;
  if (yes + missing >= q) return V_PENDING;
  return V_LOST;
}

static u8 joint_vote(u8 r1, u8 r2) { /* joint.go:61-75 */
  if (r1 == r2) return r1;
  if (r1 == V_LOST || r2 == V_LOST) return V_LOST;
  return V_PENDING;
}

/* CSR group: members of one half given by mask; non-members ignored. */
static u64 csr_half_ci(const u64* m, u32 s, u32 mask) {
  u64 vals[16] = {0};
  int n = 0;
  for (u32 j = 0; j < s; ++j)
    if ((mask >> j) & 1) vals[n++] = m[j];
  return majority_ci(vals, n);
}
static u8 csr_half_vote(u32 mask, u32 voted, u32 granted) {
  int n = 0, yes = 0, no = 0;
  for (u32 j = 0; j < 16; ++j) {
    if (!((mask >> j) & 1)) continue;
    ++n;
    if ((voted >> j) & 1) {
      if ((granted >> j) & 1) ++yes;
      else ++no;
    }
  }
  return majority_vote(n, yes, no);
}

void orc_csr_eval(u64 G, const u32* off, const u64* match, const u32* cfg, const u32* votes,
                  u64* commit, u8* vote) {
  for (u64 g = 0; g < G; ++g) {
    u32 a = off[g], s = off[g + 1] - a, min_ = cfg[g] & 0xFFFF, mout = cfg[g] >> 16;
    if (commit) {
      u64 c0 = csr_half_ci(match + a, s, min_), c1 = csr_half_ci(match + a, s, mout);
      commit[g] = c0 < c1 ? c0 : c1; /* joint.go:49-56 */
    }
    if (vote) {
      u32 vd = votes[g] & 0xFFFF, gr = votes[g] >> 16;
      vote[g] = joint_vote(csr_half_vote(min_, vd, gr), csr_half_vote(mout, vd, gr));
    }
  }
}

void orc_fixed_eval(u32 n, u64 G, const u64* match, const void* voted, const void* granted,
                    u64* commit, u8* vote) {
  for (u64 g = 0; g < G; ++g) {
    if (commit) {
      u64 vals[16];
      for (u32 j = 0; j < n; ++j) vals[j] = match[(u64)j * G + g];
      commit[g] = majority_ci(vals, (int)n);
    }
    if (vote) {
      u32 vd = n <= 8 ? ((const u8*)voted)[g] : ((const u16*)voted)[g];
      u32 gr = n <= 8 ? ((const u8*)granted)[g] : ((const u16*)granted)[g];
      u32 full = (1u << n) - 1;
      vote[g] = csr_half_vote(full, vd, gr);
    }
  }
}

/* WIDE layout: per-slot flags (1 in, 2 out, 4 voted, 8 granted), any size.
 * The reference sorts with insertionSort (majority.go:115-122); for wide
 * halves the oracle uses qsort beyond 64 members — srt[n-(n/2+1)] of an
 * ascending sort does not depend on the sorting algorithm. */
static int cmp_u64(const void* a, const void* b) {
  u64 x = *(const u64*)a, y = *(const u64*)b;
  return x < y ? -1 : x > y;
}
static u64 wide_half_ci(const u64* m, const u8* fl, u32 s, u32 bit, u64* scratch) {
  int n = 0;
  for (u32 j = 0; j < s; ++j)
    if ((fl[j] >> bit) & 1) scratch[n++] = m[j];
  if (n == 0) return INF;
  if (n <= 64) insertion_sort(scratch, n);
  else qsort(scratch, (size_t)n, sizeof(u64), cmp_u64);
  return scratch[n - (n / 2 + 1)];
}
static u8 wide_half_vote(const u8* fl, u32 s, u32 bit) {
  int n = 0, yes = 0, no = 0;
  for (u32 j = 0; j < s; ++j) {
    if (!((fl[j] >> bit) & 1)) continue;
    ++n;
    if (fl[j] & 4) {
      if (fl[j] & 8) ++yes;
      else ++no;
    }
  }
  return majority_vote(n, yes, no);
}
void orc_wide_eval(u64 G, const u32* off, const u64* match, const u8* flags, u64* commit,
                   u8* vote) {
  u64* scratch = (u64*)malloc(sizeof(u64) * 4096);
  for (u64 g = 0; g < G; ++g) {
    u32 a = off[g], s = off[g + 1] - a;
    if (commit) {
      u64 c0 = wide_half_ci(match + a, flags + a, s, 0, scratch);
      u64 c1 = wide_half_ci(match + a, flags + a, s, 1, scratch);
      commit[g] = c0 < c1 ? c0 : c1;
    }
    if (vote) vote[g] = joint_vote(wide_half_vote(flags + a, s, 0), wide_half_vote(flags + a, s, 1));
  }
  free(scratch);
}

void orc_csr_quorum_active(u64 G, const u32* cfg, const u16* active, u8* won) {
  for (u64 g = 0; g < G; ++g) { /* tracker.go:215-225: every voter "voted" */
    u32 min_ = cfg[g] & 0xFFFF, mout = cfg[g] >> 16, a = active[g];
    u8 r = joint_vote(csr_half_vote(min_, 0xFFFF, a), csr_half_vote(mout, 0xFFFF, a));
    won[g] = r == V_WON;
  }
}

/* -------------------------------------------- faithful (Go maps) loop ----- */
/* Go's map[uint64]... is modelled by an open-addressing table of 16 entries
 * per group (load <= 11/16): MajorityConfig (set of IDs), the progress map
 * (ID -> Match) and the votes map (ID -> bool).  CommittedIndex ranges over
 * the config table and looks every ID up in the progress table — one hash
 * probe per voter, like matchAckIndexer.AckedIndex (tracker.go:167-173). */

#define TBL 16
typedef struct {
  u64 cfg_key[TBL];   /* 0 = empty */
  u64 prs_key[TBL];
  u64 prs_val[TBL];
  u64 vote_key[TBL];
  u8 vote_val[TBL];
} orc_group_maps;

static inline u32 hslot(u64 id) { return (u32)((id * 0x9E3779B97F4A7C15ull) >> 60); }
static void tbl_put(u64* keys, u64 id, u32* pos_out) {
  u32 h = hslot(id);
  while (keys[h] != 0 && keys[h] != id) h = (h + 1) & (TBL - 1);
  keys[h] = id;
  *pos_out = h;
}
static int tbl_find(const u64* keys, u64 id, u32* pos_out) {
  u32 h = hslot(id);
  for (int probe = 0; probe < TBL; ++probe) {
    if (keys[h] == 0) return 0;
    if (keys[h] == id) {
      *pos_out = h;
      return 1;
    }
    h = (h + 1) & (TBL - 1);
  }
  return 0;
}

size_t orc_group_maps_size(void) { return sizeof(orc_group_maps); }

/* Build maps for the fixed config: voter IDs 1..n (bench_test.go:30-33). */
void orc_faithful_build_fixed(u32 n, u64 G, const u64* match, const void* voted,
                              const void* granted, orc_group_maps* maps) {
  for (u64 g = 0; g < G; ++g) {
    orc_group_maps* m = maps + g;
    memset(m, 0, sizeof *m);
    u32 vd = n <= 8 ? ((const u8*)voted)[g] : ((const u16*)voted)[g];
    u32 gr = n <= 8 ? ((const u8*)granted)[g] : ((const u16*)granted)[g];
    for (u32 j = 0; j < n; ++j) {
      u64 id = j + 1;
      u32 p;
      tbl_put(m->cfg_key, id, &p);
      tbl_put(m->prs_key, id, &p);
      m->prs_val[p] = match[(u64)j * G + g];
      if ((vd >> j) & 1) {
        tbl_put(m->vote_key, id, &p);
        m->vote_val[p] = (gr >> j) & 1;
      }
    }
  }
}

/* MajorityConfig.CommittedIndex over a config table, each ID looked up in
 * the progress table (majority.go:126-172, tracker.go:167-173). */
static u64 faithful_half_ci(const u64* cfg_key, const u64* prs_key, const u64* prs_val) {
  int n = 0;
  for (int k = 0; k < TBL; ++k) n += cfg_key[k] != 0;
  if (n == 0) return INF; /* majority.go:128-133 */
  u64 stk[7], *srt = stk, heap[TBL];
  if (n > 7) srt = heap;
  memset(srt, 0, sizeof(u64) * (size_t)n);
  int i = n - 1;
  for (int k = 0; k < TBL; ++k) { /* for id := range c */
    u64 id = cfg_key[k];
    if (!id) continue;
    u32 p;
    if (tbl_find(prs_key, id, &p)) srt[i--] = prs_val[p];
  }
  insertion_sort(srt, n);
  return srt[n - (n / 2 + 1)];
}

/* MajorityConfig.VoteResult over a config table and the votes map
 * (majority.go:178-210). */
static u8 faithful_half_vote(const u64* cfg_key, const u64* vote_key, const u8* vote_val) {
  int n = 0, yes = 0, no = 0, missing = 0;
  for (int k = 0; k < TBL; ++k) {
    u64 id = cfg_key[k];
    if (!id) continue;
    ++n;
    u32 p;
    if (!tbl_find(vote_key, id, &p)) {
      ++missing;
      continue;
    }
    if (vote_val[p]) ++yes;
    else ++no;
  }
  if (n == 0) return V_WON;
  int q = n / 2 + 1;
  if (yes >= q) return V_WON;
  if (yes + missing >= q) return V_PENDING;
  return V_LOST;
}

static u64 faithful_ci(const orc_group_maps* m) {
  return faithful_half_ci(m->cfg_key, m->prs_key, m->prs_val);
}

static u8 faithful_vote(const orc_group_maps* m) {
  return faithful_half_vote(m->cfg_key, m->vote_key, m->vote_val);
}

/* The CSR / joint form as the reference holds it: tracker.Config's
 * JointConfig (two MajorityConfig maps, joint.go:22), the ProgressMap (every
 * slot, learners included: ID -> Match) and the votes map.  IDs are slot + 1
 * (slots are ascending IDs, MajorityConfig.Slice order). */
typedef struct {
  u64 in_key[TBL];
  u64 out_key[TBL];
  u64 prs_key[TBL];
  u64 prs_val[TBL];
  u64 vote_key[TBL];
  u8 vote_val[TBL];
} orc_joint_maps;

size_t orc_joint_maps_size(void) { return sizeof(orc_joint_maps); }

int orc_faithful_build_csr(u64 G, const u32* off, const u64* match, const u32* cfg,
                           const u32* votes, orc_joint_maps* maps) {
  for (u64 g = 0; g < G; ++g) {
    orc_joint_maps* m = maps + g;
    memset(m, 0, sizeof *m);
    const u32 a = off[g], s = off[g + 1] - a;
    if (s > 11) return -1; /* the tables hold <= 11 of 16 entries */
    const u32 min_ = cfg[g] & 0xFFFF, mout = cfg[g] >> 16;
    const u32 vd = votes ? votes[g] & 0xFFFF : 0, gr = votes ? votes[g] >> 16 : 0;
    for (u32 j = 0; j < s; ++j) {
      const u64 id = j + 1;
      u32 p;
      if ((min_ >> j) & 1) tbl_put(m->in_key, id, &p);
      if ((mout >> j) & 1) tbl_put(m->out_key, id, &p);
      tbl_put(m->prs_key, id, &p);
      m->prs_val[p] = match[a + j];
      if ((vd >> j) & 1) {
        tbl_put(m->vote_key, id, &p);
        m->vote_val[p] = (gr >> j) & 1;
      }
    }
  }
  return 0;
}

/* JointConfig.CommittedIndex / VoteResult (joint.go:49-75) over the maps. */
void orc_faithful_joint_eval(u64 G, const orc_joint_maps* maps, u64* commit, u8* vote) {
  for (u64 g = 0; g < G; ++g) {
    const orc_joint_maps* m = maps + g;
    if (commit) {
      const u64 c0 = faithful_half_ci(m->in_key, m->prs_key, m->prs_val);
      const u64 c1 = faithful_half_ci(m->out_key, m->prs_key, m->prs_val);
      commit[g] = c0 < c1 ? c0 : c1;
    }
    if (vote)
      vote[g] = joint_vote(faithful_half_vote(m->in_key, m->vote_key, m->vote_val),
                           faithful_half_vote(m->out_key, m->vote_key, m->vote_val));
  }
}

void orc_faithful_eval(u64 G, const orc_group_maps* maps, u64* commit, u8* vote) {
  for (u64 g = 0; g < G; ++g) {
    if (commit) commit[g] = faithful_ci(maps + g);
    if (vote) vote[g] = faithful_vote(maps + g);
  }
}

/* BASELINE configs[0]: BenchmarkMajorityConfig_CommittedIndex
 * (quorum/bench_test.go:24-40) — one MajorityConfig with IDs 1..n and a
 * mapAckIndexer of values in [0, MaxInt64), CommittedIndex called `iters`
 * times in a loop on one thread.  Returns the sum of the results (so the loop
 * is not elided); the caller times the call. */
u64 orc_bench_plumbing(u32 n, u64 iters, u64 seed) {
  orc_group_maps m;
  memset(&m, 0, sizeof m);
  for (u32 j = 0; j < n; ++j) {
    u32 p;
    tbl_put(m.cfg_key, j + 1, &p);
    tbl_put(m.prs_key, j + 1, &p);
    m.prs_val[p] = splitmix64(seed + j) % 0x7FFFFFFFFFFFFFFFull; /* rand.Int63n(MaxInt64) */
  }
  u64 acc = 0;
  for (u64 i = 0; i < iters; ++i) {
    /* defeat hoisting: the map is re-read every call, as Go's range is */
    __asm__ __volatile__("" : : "r"(&m) : "memory");
    acc += faithful_ci(&m);
  }
  return acc;
}

/* --------------------------------------------------- pthread drivers ----- */

typedef struct {
  int kind;
  u64 lo, hi;
  const void* a;
  u64* commit;
  u8* vote;
  u32 n;
  u64 G;
  const u64* match;
  const void* voted;
  const void* granted;
  const u32* off;
  const u32* cfg;
  const u32* votes;
} orc_job;

static void* orc_worker(void* p) {
  orc_job* j = (orc_job*)p;
  u64 cnt = j->hi - j->lo;
  if (j->kind == 0) {
    orc_faithful_eval(cnt, (const orc_group_maps*)j->a + j->lo, j->commit ? j->commit + j->lo : 0,
                      j->vote ? j->vote + j->lo : 0);
  } else if (j->kind == 3) {
    orc_faithful_joint_eval(cnt, (const orc_joint_maps*)j->a + j->lo,
                            j->commit ? j->commit + j->lo : 0, j->vote ? j->vote + j->lo : 0);
  } else if (j->kind == 1) {
    /* fixed layout, strided rows: evaluate groups lo..hi of the full table */
    for (u64 g = j->lo; g < j->hi; ++g) {
      if (j->commit) {
        u64 vals[16];
        for (u32 s = 0; s < j->n; ++s) vals[s] = j->match[(u64)s * j->G + g];
        j->commit[g] = majority_ci(vals, (int)j->n);
      }
      if (j->vote) {
        u32 vd = j->n <= 8 ? ((const u8*)j->voted)[g] : ((const u16*)j->voted)[g];
        u32 gr = j->n <= 8 ? ((const u8*)j->granted)[g] : ((const u16*)j->granted)[g];
        j->vote[g] = csr_half_vote((1u << j->n) - 1, vd, gr);
      }
    }
  } else {
    for (u64 g = j->lo; g < j->hi; ++g) {
      u32 a = j->off[g], s = j->off[g + 1] - a, min_ = j->cfg[g] & 0xFFFF, mout = j->cfg[g] >> 16;
      if (j->commit) {
        u64 c0 = csr_half_ci(j->match + a, s, min_), c1 = csr_half_ci(j->match + a, s, mout);
        j->commit[g] = c0 < c1 ? c0 : c1;
      }
      if (j->vote) {
        u32 vd = j->votes[g] & 0xFFFF, gr = j->votes[g] >> 16;
        j->vote[g] = joint_vote(csr_half_vote(min_, vd, gr), csr_half_vote(mout, vd, gr));
      }
    }
  }
  return 0;
}

#define ORC_MAX_THREADS 1024
static void run_parallel(orc_job* proto, u64 G, int threads) {
  if (threads < 1) threads = 1;
  if (threads > ORC_MAX_THREADS) threads = ORC_MAX_THREADS;
  pthread_t* tid = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
  orc_job* jobs = (orc_job*)malloc(sizeof(orc_job) * (size_t)threads);
  for (int t = 0; t < threads; ++t) {
    jobs[t] = *proto;
    jobs[t].lo = G * (u64)t / (u64)threads;
    jobs[t].hi = G * (u64)(t + 1) / (u64)threads;
    pthread_create(&tid[t], 0, orc_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], 0);
  free(tid);
  free(jobs);
}

void orc_faithful_eval_mt(u64 G, const orc_group_maps* maps, u64* commit, u8* vote,
                          int threads) {
  orc_job j;
  memset(&j, 0, sizeof j);
  j.kind = 0;
  j.a = maps;
  j.commit = commit;
  j.vote = vote;
  run_parallel(&j, G, threads);
}

void orc_faithful_joint_eval_mt(u64 G, const orc_joint_maps* maps, u64* commit, u8* vote,
                                int threads) {
  orc_job j;
  memset(&j, 0, sizeof j);
  j.kind = 3;
  j.a = maps;
  j.commit = commit;
  j.vote = vote;
  run_parallel(&j, G, threads);
}

void orc_fixed_eval_mt(u32 n, u64 G, const u64* match, const void* voted, const void* granted,
                       u64* commit, u8* vote, int threads) {
  orc_job j;
  memset(&j, 0, sizeof j);
  j.kind = 1;
  j.n = n;
  j.G = G;
  j.match = match;
  j.voted = voted;
  j.granted = granted;
  j.commit = commit;
  j.vote = vote;
  run_parallel(&j, G, threads);
}

void orc_csr_eval_mt(u64 G, const u32* off, const u64* match, const u32* cfg, const u32* votes,
                     u64* commit, u8* vote, int threads) {
  orc_job j;
  memset(&j, 0, sizeof j);
  j.kind = 2;
  j.off = off;
  j.match = match;
  j.cfg = cfg;
  j.votes = votes;
  j.commit = commit;
  j.vote = vote;
  run_parallel(&j, G, threads);
}

/* ------------------------------------------------ sequential tracker ----- */

/* Leader-side tracker state in either layout: FIXED (n voters, slot-major
 * rows of G: match[s * G + g]) or CSR (n == 0: slots off[g] .. off[g+1]-1,
 * group-major, cfg = mask_in | mask_out << 16; a slot in neither mask is a
 * learner, which has a Progress but no vote, tracker.go:27-78). */
typedef struct {
  u32 n;
  u64 G;
  const u32* off;
  const u32* cfg;
} orc_layout;

static inline u32 lay_slots(const orc_layout* L, u64 g) {
  return L->n ? L->n : L->off[g + 1] - L->off[g];
}
static inline u64 lay_at(const orc_layout* L, u64 g, u32 s) {
  return L->n ? (u64)s * L->G + g : (u64)L->off[g] + s;
}
/* ProgressTracker.Committed (tracker.go:177-179): JointConfig.CommittedIndex
 * (joint.go:49-56) over the voters' Match; FIXED is one n-voter half. */
static u64 lay_ci(const orc_layout* L, const u64* match, u64 g) {
  if (L->n) {
    u64 vals[16];
    for (u32 k = 0; k < L->n; ++k) vals[k] = match[(u64)k * L->G + g];
    return majority_ci(vals, (int)L->n);
  }
  const u64* m = match + L->off[g];
  u32 s = L->off[g + 1] - L->off[g];
  u64 c0 = csr_half_ci(m, s, L->cfg[g] & 0xFFFF), c1 = csr_half_ci(m, s, L->cfg[g] >> 16);
  return c0 < c1 ? c0 : c1;
}
/* raftLog.maybeCommit (log.go:328-334): ci > committed && term(ci) == Term.
 * For a leader term(i) == Term <=> term_start <= i <= lastIndex; no voter acks
 * past lastIndex, and an empty config's ci = MaxUint64 lies past it
 * (raftLog.term of an index beyond lastIndex is 0, log.go:271-273). */
static int commit_gate(u64 ci, u64 committed, u64 term_start) {
  return ci != INF && ci > committed && ci >= term_start;
}

/* Sequential MsgAppResp processing, records in batch order, restricted to
 * groups [lo, hi) (the partitioned multi-thread form: groups are independent,
 * so each thread scanning the whole batch for its own groups is exactly the
 * sequential result).  stepped_down[g] is set to 1 when a higher-term record
 * makes the leader step down (raft.go:875-879); later records of that group
 * are not applied.  committed[] advances via maybeCommit after every
 * MaybeUpdate that returned true (raft.go:1259 -> 585-588).
 * Returns -1 if a record acks past the leader's log (index > last_index[g]),
 * which the reference treats as log corruption (log.go:239-241); else 0. */
static int appresp_range(const orc_layout* L, u64 lo, u64 hi, u64 M, const u32* order,
                         const u32* rg, const u8* rf, const u64* ri, const u64* rt,
                         const u64* group_term, const u64* term_start, const u64* last_index,
                         u64* match, u64* next, u16* active, u64* committed, u8* stepped_down,
                         u64* stats) {
  /* order (nullable): the batch positions to visit, ascending — this
   * partition's records only (appresp_run's owner partition); else 0..M-1 */
  for (u64 k = 0; k < M; ++k) {
    const u64 i = order ? order[k] : k;
    u64 g = rg[i];
    if (g >= L->G) {
      if (lo == 0) stats[5]++; /* counted once, by the first partition */
      continue;
    }
    if (g < lo || g >= hi) continue;
    u32 s = rf[i] & 0x0F;
    int reject = (rf[i] & 0x80) != 0;
    if (s >= lay_slots(L, g)) { stats[3]++; continue; } /* raft.go:1100-1104 */
    if (rt[i] < group_term[g]) { stats[2]++; continue; } /* raft.go:883-921 */
    if (rt[i] > group_term[g]) {                          /* raft.go:852-880 */
      stats[4]++;
      if (!stepped_down[g]) stepped_down[g] = 1;
      continue;
    }
    if (stepped_down[g]) { stats[6]++; continue; }
    active[g] |= (u16)(1u << s);                          /* raft.go:1107 */
    if (reject) { stats[1]++; continue; }
    stats[0]++;
    if (last_index && ri[i] > last_index[g]) return -1;
    u64 at = lay_at(L, g, s);
    int updated = 0;
    if (match[at] < ri[i]) { match[at] = ri[i]; updated = 1; } /* progress.go:146-150 */
    if (next && next[at] < ri[i] + 1) next[at] = ri[i] + 1;    /* progress.go:151 */
    if (updated) {
      u64 ci = lay_ci(L, match, g);
      if (commit_gate(ci, committed[g], term_start[g])) committed[g] = ci;
    }
  }
  return 0;
}

typedef struct {
  const orc_layout* L;
  u64 lo, hi, M;
  const u32* order;
  const u32* rg;
  const u8* rf;
  const u64 *ri, *rt, *gt, *ts, *last;
  u64 *match, *next, *committed;
  u16* active;
  u8* sd;
  u64 stats[8];
  int rc;
  /* owner partition (threads > 1) */
  int phase, T, t;
  u64 src_lo, src_hi;
  u64* cnt; /* [T][T]: records of source slice t for owner d, then their positions */
  u32* out;
} orc_seq_job;

/* The thread owning group g: the t with G*t/T <= g < G*(t+1)/T (a bad group
 * goes to thread 0, which counts it once). */
static inline int owner_of(u64 g, u64 G, int T) {
  if (g >= G) return 0;
  u64 d = (u64)(((unsigned __int128)g * (u64)T) / G);
  while (d + 1 < (u64)T && G * (d + 1) / (u64)T <= g) ++d;
  while (d > 0 && G * d / (u64)T > g) --d;
  return (int)d;
}

static void* orc_seq_worker(void* p) {
  orc_seq_job* j = (orc_seq_job*)p;
  if (j->phase == 1) { /* count this source slice's records per owner */
    u64* c = j->cnt + (u64)j->t * (u64)j->T;
    for (u64 i = j->src_lo; i < j->src_hi; ++i) c[owner_of(j->rg[i], j->L->G, j->T)]++;
  } else if (j->phase == 2) { /* scatter positions, stable */
    u64* c = j->cnt + (u64)j->t * (u64)j->T;
    for (u64 i = j->src_lo; i < j->src_hi; ++i) j->out[c[owner_of(j->rg[i], j->L->G, j->T)]++] = (u32)i;
  } else {
    j->rc = appresp_range(j->L, j->lo, j->hi, j->M, j->order, j->rg, j->rf, j->ri, j->rt, j->gt,
                          j->ts, j->last, j->match, j->next, j->active, j->committed, j->sd,
                          j->stats);
  }
  return 0;
}

static void run_phase(orc_seq_job* jobs, pthread_t* tid, int T, int phase) {
  for (int t = 0; t < T; ++t) {
    jobs[t].phase = phase;
    pthread_create(&tid[t], 0, orc_seq_worker, &jobs[t]);
  }
  for (int t = 0; t < T; ++t) pthread_join(tid[t], 0);
}

/* Sequential semantics on T threads: groups are partitioned into T ranges
 * and the batch is stably partitioned by owner (count, scan, scatter of batch
 * positions — each owner's list stays in batch order), then each thread
 * replays its own records in batch order: exactly the one-thread result,
 * with O(M) total work (a multi-raft host delivering each group's responses
 * to the goroutine that owns it). */
static int appresp_run(const orc_layout* L, u64 M, const u32* rg, const u8* rf, const u64* ri,
                       const u64* rt, const u64* group_term, const u64* term_start,
                       const u64* last_index, u64* match, u64* next, u16* active,
                       u64* committed, u8* stepped_down, u64* stats, int threads) {
  if (threads < 1) threads = 1;
  if (threads > ORC_MAX_THREADS) threads = ORC_MAX_THREADS;
  if ((u64)threads > L->G) threads = L->G ? (int)L->G : 1;
  const int T = threads;
  orc_seq_job* jobs = (orc_seq_job*)calloc((size_t)T, sizeof(orc_seq_job));
  pthread_t* tid = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  u64* cnt = T > 1 ? (u64*)calloc((size_t)T * (size_t)T, sizeof(u64)) : 0;
  u32* order = T > 1 ? (u32*)malloc(sizeof(u32) * (M ? M : 1)) : 0;
  if (!jobs || !tid || (T > 1 && (!cnt || !order))) {
    free(jobs), free(tid), free(cnt), free(order);
    return -2;
  }
  for (int t = 0; t < T; ++t) {
    orc_seq_job* j = &jobs[t];
    j->L = L;
    j->lo = L->G * (u64)t / (u64)T;
    j->hi = L->G * (u64)(t + 1) / (u64)T;
    j->M = M;
    j->rg = rg, j->rf = rf, j->ri = ri, j->rt = rt, j->gt = group_term, j->ts = term_start;
    j->last = last_index, j->match = match, j->next = next, j->active = active;
    j->committed = committed, j->sd = stepped_down;
    j->T = T, j->t = t, j->cnt = cnt, j->out = order;
    j->src_lo = M * (u64)t / (u64)T;
    j->src_hi = M * (u64)(t + 1) / (u64)T;
  }
  if (T == 1) {
    orc_seq_worker(&jobs[0]);
  } else {
    run_phase(jobs, tid, T, 1);
    /* owner-major, then source-major exclusive scan: cnt[t][d] becomes the
     * first position of source t's records for owner d */
    u64 run = 0;
    for (int d = 0; d < T; ++d) {
      const u64 start = run;
      for (int t = 0; t < T; ++t) {
        const u64 c = cnt[(u64)t * T + d];
        cnt[(u64)t * T + d] = run;
        run += c;
      }
      jobs[d].order = order + start;
    }
    run_phase(jobs, tid, T, 2);
    /* after the scatter, cnt[T-1][d] is the end of owner d's list */
    for (int d = 0; d < T; ++d) jobs[d].M = cnt[(u64)(T - 1) * T + d] - (u64)(jobs[d].order - order);
    run_phase(jobs, tid, T, 3);
  }
  int rc = 0;
  for (int t = 0; t < T; ++t) {
    for (int k = 0; k < 8; ++k) stats[k] += jobs[t].stats[k];
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  free(jobs), free(tid), free(cnt), free(order);
  return rc;
}

/* FIXED layout (n voters, slot s <-> the s-th smallest voter ID). */
int orc_fixed_appresp_sequential(u32 n, u64 G, u64 M, const u32* rg, const u8* rf,
                                 const u64* ri, const u64* rt, const u64* group_term,
                                 const u64* term_start, const u64* last_index, u64* match,
                                 u64* next, u16* active, u64* committed, u8* stepped_down,
                                 u64* stats /* [8] */) {
  orc_layout L = {n, G, 0, 0};
  return appresp_run(&L, M, rg, rf, ri, rt, group_term, term_start, last_index, match, next,
                     active, committed, stepped_down, stats, 1);
}

int orc_fixed_appresp_sequential_mt(u32 n, u64 G, u64 M, const u32* rg, const u8* rf,
                                    const u64* ri, const u64* rt, const u64* group_term,
                                    const u64* term_start, const u64* last_index, u64* match,
                                    u64* next, u16* active, u64* committed, u8* stepped_down,
                                    u64* stats, int threads) {
  orc_layout L = {n, G, 0, 0};
  return appresp_run(&L, M, rg, rf, ri, rt, group_term, term_start, last_index, match, next,
                     active, committed, stepped_down, stats, threads);
}

/* CSR layout (ragged voters + learners, joint configs). */
int orc_csr_appresp_sequential(u64 G, const u32* off, const u32* cfg, u64 M, const u32* rg,
                               const u8* rf, const u64* ri, const u64* rt, const u64* group_term,
                               const u64* term_start, const u64* last_index, u64* match,
                               u64* next, u16* active, u64* committed, u8* stepped_down,
                               u64* stats, int threads) {
  orc_layout L = {0, G, off, cfg};
  return appresp_run(&L, M, rg, rf, ri, rt, group_term, term_start, last_index, match, next,
                     active, committed, stepped_down, stats, threads);
}

/* maybeCommit for every CSR group (initial invariant / empty batch). */
void orc_csr_commit_all(u64 G, const u32* off, const u32* cfg, const u64* match,
                        const u64* term_start, u64* committed, u8* advanced) {
  orc_layout L = {0, G, off, cfg};
  for (u64 g = 0; g < G; ++g) {
    u64 ci = lay_ci(&L, match, g);
    int adv = commit_gate(ci, committed[g], term_start[g]);
    if (adv) committed[g] = ci;
    if (advanced) advanced[g] = (u8)adv;
  }
}

/* maybeCommit for every group (used to establish the initial invariant). */
void orc_fixed_commit_all(u32 n, u64 G, const u64* match, const u64* term_start, u64* committed,
                          u8* advanced) {
  for (u64 g = 0; g < G; ++g) {
    u64 vals[16];
    for (u32 k = 0; k < n; ++k) vals[k] = match[(u64)k * G + g];
    u64 ci = majority_ci(vals, (int)n);
    int adv = ci > committed[g] && ci >= term_start[g];
    if (adv) committed[g] = ci;
    if (advanced) advanced[g] = (u8)adv;
  }
}
