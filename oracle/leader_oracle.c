/*
 * leader_oracle.c — C restatement of the raft leader inbox step.
 *
 * TEST INFRASTRUCTURE ONLY.  Loaded by tests/ (full-size parity) and by
 * tools/bench_configs.py's CPU baseline leg, never by the product.
 *
 * One record at a time, in batch order, exactly as the Go leader handles its
 * inbox (paths relative to the reference's raft/):
 *   raft.Step term filter (raft.go:847-921); stepLeader progress lookup
 *   (raft.go:1099-1104); MsgAppResp (raft.go:1105-1283) with
 *   findConflictByTerm walking index by index (log.go:150-171), MaybeDecrTo /
 *   MaybeUpdate / Become* (tracker/progress.go:85-212), Inflights
 *   (tracker/inflights.go:55-132), maybeCommit (raft.go:585-588,
 *   log.go:328-334) with the q-th largest match by insertion sort
 *   (quorum/majority.go:115-172, joint.go:49-56), bcastAppend / maybeSendAppend
 *   (raft.go:423-522); MsgHeartbeatResp with readOnly.recvAck / advance
 *   (raft.go:1284-1309, read_only.go:68-121, raft.go:1737-1752);
 *   MsgSnapStatus / MsgUnreachable (raft.go:1310-1338).
 *
 * Validated against oracle/leader_ref.py (pinned by the reference's tests in
 * tests/golden/leader_tables.json).  State layout: the same structure of
 * arrays the engine uses (restated here, not included from the product).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;

#define NOSLOT 0xFFu
#define P_PROBE 0
#define P_REPL 1
#define P_SNAP 2
#define F_PROBE_SENT 4u
#define F_ACTIVE 8u

typedef struct {
  u64 G;
  u32 K, Q, read_only, reserved;
  const u32 *off, *cfg;
  u32* meta;
  const u64* term;
  u64* committed;
  const u64 *first, *last, *snap_i, *snap_t, *max_ents, *run_s, *run_t;
  u64 *match, *next, *psnap;
  u8* pst;
  u32* ipos;
  u64* ibuf;
  u64 *rq_ctx, *rq_idx;
  u32* rq_meta;
} orc_lg;

typedef struct {
  u64 M;
  const u32* group;
  const u8* flags;
  const u64 *index, *term, *hint, *log_term;
} orc_in;

typedef struct {
  u64 index, log_term, commit, aux;
  u32 group;
  u8 to, type;
  u16 reserved;
} orc_msg;

typedef struct {
  orc_msg* v;
  u64 n, cap;
} msgvec;

static void push(msgvec* mv, orc_msg m) {
  if (mv->n == mv->cap) {
    mv->cap = mv->cap ? mv->cap * 2 : 1024;
    mv->v = (orc_msg*)realloc(mv->v, mv->cap * sizeof(orc_msg));
  }
  mv->v[mv->n++] = m;
}

typedef struct {
  const orc_lg* L;
  u64 g;
  u32 s0, ns, leader, transferee;
  msgvec* out;
} ctx;

static void emit(ctx* c, u8 type, u32 to, u64 index, u64 lt, u64 commit, u64 aux) {
  orc_msg m = {index, lt, commit, aux, (u32)c->g, (u8)to, type, 0};
  push(c->out, m);
}

/* log.go:268-288 */
static u64 term_of(const ctx* c, u64 i) {
  const orc_lg* L = c->L;
  u64 dummy = L->first[c->g] - 1;
  if (i < dummy || i > L->last[c->g]) return 0;
  u32 nr = (L->meta[c->g] >> 16) & 0xF;
  u64 t = 0;
  for (u32 r = 0; r < nr; ++r)
    if (L->run_s[r * L->G + c->g] <= i) t = L->run_t[r * L->G + c->g];  /* run-major */
  return t;
}

/* log.go:150-171, index by index */
static u64 find_conflict_by_term(const ctx* c, u64 index, u64 term) {
  if (index > c->L->last[c->g]) return index;
  for (;;) {
    if (term_of(c, index) <= term) break;
    index--;
  }
  return index;
}

/* inflights.go */
static int infl_full(const ctx* c, u64 p) { return (c->L->ipos[p] >> 16) == c->L->K; }
static void infl_add(const ctx* c, u64 p, u64 v) {
  u32 start = c->L->ipos[p] & 0xFFFF, count = c->L->ipos[p] >> 16, K = c->L->K;
  u32 nx = start + count;
  if (nx >= K) nx -= K;
  c->L->ibuf[p * K + nx] = v;
  c->L->ipos[p] = start | ((count + 1) << 16);
}
static void infl_free_le(const ctx* c, u64 p, u64 to) {
  u32 start = c->L->ipos[p] & 0xFFFF, count = c->L->ipos[p] >> 16, K = c->L->K;
  const u64* buf = c->L->ibuf + p * K;
  if (count == 0 || to < buf[start]) return;
  u32 idx = start, i;
  for (i = 0; i < count; i++) {
    if (to < buf[idx]) break;
    if (++idx >= K) idx -= K;
  }
  count -= i;
  start = idx;
  if (count == 0) start = 0;
  c->L->ipos[p] = start | (count << 16);
}

/* progress.go */
static u32 state(const ctx* c, u64 p) { return c->L->pst[p] & 3u; }
static void reset_state(const ctx* c, u64 p, u32 st) {
  c->L->pst[p] = (u8)((c->L->pst[p] & F_ACTIVE) | st);
  c->L->psnap[p] = 0;
  c->L->ipos[p] = 0;
}
static void become_probe(const ctx* c, u64 p) {
  if (state(c, p) == P_SNAP) {
    u64 ps = c->L->psnap[p];
    reset_state(c, p, P_PROBE);
    u64 a = c->L->match[p] + 1, b = ps + 1;
    c->L->next[p] = a > b ? a : b;
  } else {
    reset_state(c, p, P_PROBE);
    c->L->next[p] = c->L->match[p] + 1;
  }
}
static void become_replicate(const ctx* c, u64 p) {
  reset_state(c, p, P_REPL);
  c->L->next[p] = c->L->match[p] + 1;
}
static int is_paused(const ctx* c, u64 p) {
  switch (state(c, p)) {
    case P_PROBE: return (c->L->pst[p] & F_PROBE_SENT) != 0;
    case P_REPL: return infl_full(c, p);
    default: return 1;
  }
}
static int maybe_update(const ctx* c, u64 p, u64 n) {
  int updated = 0;
  if (c->L->match[p] < n) {
    c->L->match[p] = n;
    updated = 1;
    c->L->pst[p] &= (u8)~F_PROBE_SENT;
  }
  if (c->L->next[p] < n + 1) c->L->next[p] = n + 1;
  return updated;
}
static int maybe_decr_to(const ctx* c, u64 p, u64 rejected, u64 hint) {
  if (state(c, p) == P_REPL) {
    if (rejected <= c->L->match[p]) return 0;
    c->L->next[p] = c->L->match[p] + 1;
    return 1;
  }
  if (c->L->next[p] - 1 != rejected) return 0;
  u64 h1 = hint + 1, mn = rejected < h1 ? rejected : h1;
  c->L->next[p] = mn > 1 ? mn : 1;
  c->L->pst[p] &= (u8)~F_PROBE_SENT;
  return 1;
}

/* raft.go:432-492 */
static int maybe_send_append(ctx* c, u32 to, int send_if_empty) {
  const orc_lg* L = c->L;
  u64 p = (u64)c->s0 + to, g = c->g;
  if (is_paused(c, p)) return 0;
  u64 nx = L->next[p];
  u64 lt = term_of(c, nx - 1);
  u64 n = 0;
  int compacted = 0;
  if (nx <= L->last[g]) {
    if (nx < L->first[g]) {
      compacted = 1;
    } else {
      u64 avail = L->last[g] - nx + 1;
      n = avail < L->max_ents[g] ? avail : L->max_ents[g];
    }
  }
  if (n == 0 && !send_if_empty) return 0;
  if (compacted) {
    if (!(L->pst[p] & F_ACTIVE)) return 0;
    if (L->snap_i[g] == 0) return 0;
    emit(c, 7, to, L->snap_i[g], L->snap_t[g], 0, 0);
    reset_state(c, p, P_SNAP);
    L->psnap[p] = L->snap_i[g];
    return 1;
  }
  emit(c, 3, to, nx - 1, lt, L->committed[g], n);
  if (n) {
    if (state(c, p) == P_REPL) {
      u64 last = nx + n - 1;
      L->next[p] = last + 1;
      infl_add(c, p, last);
    } else if (state(c, p) == P_PROBE) {
      L->pst[p] |= F_PROBE_SENT;
    }
  }
  return 1;
}

static void insertion_sort(u64* a, int n) { /* majority.go:115-122 */
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && a[j] < a[j - 1]; j--) {
      u64 t = a[j];
      a[j] = a[j - 1];
      a[j - 1] = t;
    }
}
static u64 half_ci(const ctx* c, u32 mask) { /* majority.go:126-172 */
  u64 srt[16];
  int n = 0;
  for (u32 s = 0; s < c->ns; s++)
    if (mask >> s & 1) srt[n++] = c->L->match[c->s0 + s];
  if (n == 0) return UINT64_MAX;
  insertion_sort(srt, n);
  return srt[n - (n / 2 + 1)];
}
static int maybe_commit(ctx* c) {
  u32 cf = c->L->cfg[c->g];
  u64 a = half_ci(c, cf & 0xFFFF), b = half_ci(c, cf >> 16);
  u64 mci = a < b ? a : b;
  if (mci > c->L->committed[c->g] && term_of(c, mci) == c->L->term[c->g]) {
    c->L->committed[c->g] = mci;
    return 1;
  }
  return 0;
}

static u8 vote(int n, int yes) { /* majority.go:178-210, votes all true */
  if (n == 0) return 3;
  int q = n / 2 + 1;
  if (yes >= q) return 3;
  if (yes + (n - yes) >= q) return 1;
  return 2;
}
static u8 acks_vote(u32 cf, u32 acks) { /* joint.go:61-75 */
  u32 mi = cf & 0xFFFF, mo = cf >> 16;
  u8 r1 = vote(__builtin_popcount(mi), __builtin_popcount(mi & acks));
  u8 r2 = vote(__builtin_popcount(mo), __builtin_popcount(mo & acks));
  if (r1 == r2) return r1;
  if (r1 == 2 || r2 == 2) return 2;
  return 1;
}

static void heartbeat_resp(ctx* c, u32 slot, u64 hctx) {
  const orc_lg* L = c->L;
  u64 p = (u64)c->s0 + slot, g = c->g;
  L->pst[p] = (u8)((L->pst[p] | F_ACTIVE) & ~F_PROBE_SENT);
  if (state(c, p) == P_REPL && infl_full(c, p))
    infl_free_le(c, p, L->ibuf[p * L->K + (L->ipos[p] & 0xFFFF)]);
  if (L->match[p] < L->last[g]) maybe_send_append(c, slot, 1);
  if (L->read_only != 0 || hctx == 0) return;
  u32 qlen = (L->meta[g] >> 20) & 0x1F, Q = L->Q;
  u64* qc = L->rq_ctx + g * Q;
  u64* qi = L->rq_idx + g * Q;
  u32* qm = L->rq_meta + g * Q;
  int found = -1;
  for (u32 k = 0; k < qlen; k++)
    if (qc[k] == hctx) {
      found = (int)k;
      break;
    }
  u32 acks = 0;
  if (found >= 0) {
    qm[found] |= 1u << slot;
    acks = qm[found] & 0xFFFF;
  }
  if (acks_vote(L->cfg[g], acks) != 3 || found < 0) return;
  for (int k = 0; k <= found; k++) {
    u32 from = qm[k] >> 16;
    if (from == NOSLOT || from == c->leader)
      emit(c, 255, NOSLOT, qi[k], 0, 0, qc[k]);
    else
      emit(c, 16, from, qi[k], 0, 0, qc[k]);
  }
  u32 rest = qlen - (u32)(found + 1);
  for (u32 k = 0; k < rest; k++) {
    qc[k] = qc[k + found + 1];
    qi[k] = qi[k + found + 1];
    qm[k] = qm[k + found + 1];
  }
  L->meta[g] = (L->meta[g] & ~(0x1Fu << 20)) | (rest << 20);
}

static void app_resp(ctx* c, u32 slot, u64 index, int reject, u64 hint, u64 ht, u8* gfl) {
  const orc_lg* L = c->L;
  u64 p = (u64)c->s0 + slot, g = c->g;
  L->pst[p] |= F_ACTIVE;
  if (reject) {
    u64 np = hint;
    if (ht > 0) np = find_conflict_by_term(c, hint, ht);
    if (maybe_decr_to(c, p, index, np)) {
      if (state(c, p) == P_REPL) become_probe(c, p);
      maybe_send_append(c, slot, 1);
    }
    return;
  }
  int old_paused = is_paused(c, p);
  if (!maybe_update(c, p, index)) return;
  u32 s = state(c, p);
  if (s == P_PROBE) {
    become_replicate(c, p);
  } else if (s == P_SNAP && L->match[p] >= L->psnap[p]) {
    become_probe(c, p);
    become_replicate(c, p);
  } else if (s == P_REPL) {
    infl_free_le(c, p, index);
  }
  if (maybe_commit(c)) {
    *gfl |= 1;
    if (L->meta[g] & (1u << 25)) {
      L->meta[g] &= ~(1u << 25);
      *gfl |= 2;
    }
    for (u32 t = 0; t < c->ns; t++)
      if (t != c->leader) maybe_send_append(c, t, 1);
  } else if (old_paused) {
    maybe_send_append(c, slot, 1);
  }
  while (maybe_send_append(c, slot, 0)) {
  }
  if (slot == c->transferee && L->match[p] == L->last[g]) emit(c, 14, slot, 0, 0, 0, 0);
}

static void snap_status(ctx* c, u32 slot, int reject) {
  u64 p = (u64)c->s0 + slot;
  if (state(c, p) != P_SNAP) return;
  if (reject) c->L->psnap[p] = 0;
  become_probe(c, p);
  c->L->pst[p] |= F_PROBE_SENT;
}

/* Per-thread job: groups [g0, g1), every record of the batch scanned in
 * order. stats: applied, stale, higher, nonmember, after, bad. */
typedef struct {
  const orc_lg* L;
  const orc_in* in;
  u64 g0, g1;
  u32* stepdown;
  u8* gflags;
  msgvec out;
  u64 stats[8];
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  const orc_lg* L = j->L;
  const orc_in* in = j->in;
  for (u64 g = j->g0; g < j->g1; g++) {
    j->stepdown[g] = 0xFFFFFFFFu;
    j->gflags[g] = 0;
  }
  for (u64 i = 0; i < in->M; i++) {
    u64 g = in->group[i];
    if (g >= L->G) {
      if (j->g0 == 0) j->stats[5]++;
      continue;
    }
    if (g < j->g0 || g >= j->g1) continue;
    if (j->stepdown[g] != 0xFFFFFFFFu) {
      j->stats[4]++;
      continue;
    }
    u64 t = in->term[i];
    if (t != 0 && t > L->term[g]) {
      j->stepdown[g] = (u32)i;
      j->gflags[g] |= 4;
      j->stats[2]++;
      continue;
    }
    if (t != 0 && t < L->term[g]) {
      j->stats[1]++;
      continue;
    }
    ctx c = {L, g, L->off[g], L->off[g + 1] - L->off[g], L->meta[g] & 0xFF,
             (L->meta[g] >> 8) & 0xFF, &j->out};
    u32 f = in->flags[i], slot = f & 0xF, kind = (f >> 4) & 3;
    int reject = (f & 0x80) != 0;
    if (slot >= c.ns || (f & 0x40)) { /* no Progress for From */
      j->stats[3]++;
      continue;
    }
    j->stats[0]++;
    if (kind == 0) {
      app_resp(&c, slot, in->index[i], reject, reject && in->hint ? in->hint[i] : 0,
               reject && in->log_term ? in->log_term[i] : 0, &j->gflags[g]);
    } else if (kind == 1) {
      heartbeat_resp(&c, slot, in->index[i]);
    } else if (kind == 2) {
      snap_status(&c, slot, reject);
    } else if (state(&c, c.s0 + slot) == P_REPL) {
      become_probe(&c, c.s0 + slot);
    }
  }
  return NULL;
}

/* Runs the batch on `threads` host threads (contiguous group ranges).
 * msgs: capacity msg_cap (group order, emission order within a group);
 * returns the number of messages generated. */
u64 orc_leader_step(const orc_lg* L, const orc_in* in, orc_msg* msgs, u64 msg_cap,
                    u32* stepdown_at, u8* gflags, u64* stats, int threads) {
  if (threads < 1) threads = 1;
  job* jobs = (job*)calloc((size_t)threads, sizeof(job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t].L = L;
    jobs[t].in = in;
    jobs[t].g0 = L->G * (u64)t / (u64)threads;
    jobs[t].g1 = L->G * (u64)(t + 1) / (u64)threads;
    jobs[t].stepdown = stepdown_at;
    jobs[t].gflags = gflags;
  }
  for (int t = 1; t < threads; t++) pthread_create(&th[t], NULL, worker, &jobs[t]);
  worker(&jobs[0]);
  for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
  /* Each thread's messages are in batch order for its groups; a stable
   * counting sort by group gives group order with emission order kept. */
  u64 total = 0;
  for (int t = 0; t < threads; t++) {
    for (int k = 0; k < 8; k++) stats[k] += jobs[t].stats[k];
    total += jobs[t].out.n;
  }
  u64* cnt = (u64*)calloc(L->G + 1, sizeof(u64));
  for (int t = 0; t < threads; t++)
    for (u64 k = 0; k < jobs[t].out.n; k++) cnt[jobs[t].out.v[k].group + 1]++;
  for (u64 g = 0; g < L->G; g++) cnt[g + 1] += cnt[g];
  for (int t = 0; t < threads; t++) {
    for (u64 k = 0; k < jobs[t].out.n; k++) {
      u64 pos = cnt[jobs[t].out.v[k].group]++;
      if (pos < msg_cap) msgs[pos] = jobs[t].out.v[k];
    }
    free(jobs[t].out.v);
  }
  stats[6] += total;
  stats[7] += total > msg_cap ? total - msg_cap : 0;
  free(cnt);
  free(jobs);
  free(th);
  return total;
}
