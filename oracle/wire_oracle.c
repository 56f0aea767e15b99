/*
 * wire_oracle.c — C restatement of raftpb Message decoding + leader-inbox
 * ingest.  TEST INFRASTRUCTURE ONLY (full-size checker and the timed CPU
 * baseline of the wire-ingest config); never the product.
 *
 * Restates, recursively as the generated code is written (paths relative to
 * the reference's raft/raftpb/): Message.Unmarshal raft.pb.go:1739-2061,
 * Entry / SnapshotMetadata / Snapshot.Unmarshal raft.pb.go:1360-1738,
 * ConfState.Unmarshal raft.pb.go:2169-2542, skipRaft raft.pb.go:2909-2988.
 * Validated against oracle/raftpb_ref.py (tests/test_wire_oracle.py pins that
 * one against Google's protobuf runtime).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;

enum { K_MSG, K_ENTRY, K_SNAP, K_META, K_CS };

static int varint(const u8* b, u64* i, u64 l, u64* v) {
  *v = 0;
  for (unsigned shift = 0;; shift += 7) {
    if (shift >= 64 || *i >= l) return 0;
    u8 c = b[(*i)++];
    *v |= (u64)(c & 0x7F) << shift;
    if (c < 0x80) return 1;
  }
}

static int skip_raft(const u8* b, u64* i, u64 l) {
  u64 start = *i;
  int depth = 0;
  while (*i < l) {
    u64 wire, len;
    if (!varint(b, i, l, &wire)) return 0;
    switch (wire & 7) {
      case 0:
        for (unsigned shift = 0;; shift += 7) {
          if (shift >= 64 || *i >= l) return 0;
          if (b[(*i)++] < 0x80) break;
        }
        break;
      case 1: *i += 8; break;
      case 2:
        if (!varint(b, i, l, &len) || (int64_t)len < 0) return 0;
        *i += len;
        if (*i < start) return 0;
        break;
      case 3: depth++; break;
      case 4:
        if (depth == 0) return 0;
        depth--;
        break;
      case 5: *i += 4; break;
      default: return 0;
    }
    if (depth == 0) return *i <= l;
  }
  return 0;
}

typedef struct {
  u64 f[13];
  u64 ctx_pos, ctx_len;
  int has_ctx;
} fields;

/* field kinds: 1 varint, 2 bytes, 3 repeated, 10+K nested */
static int ftype(int kind, int32_t fn) {
  switch (kind) {
    case K_MSG:
      if (fn == 7) return 10 + K_ENTRY;
      if (fn == 9) return 10 + K_SNAP;
      if (fn == 12) return 2;
      return fn >= 1 && fn <= 11 ? 1 : 0;
    case K_ENTRY: return fn == 4 ? 2 : (fn >= 1 && fn <= 3 ? 1 : 0);
    case K_SNAP: return fn == 1 ? 2 : (fn == 2 ? 10 + K_META : 0);
    case K_META: return fn == 1 ? 10 + K_CS : (fn == 2 || fn == 3 ? 1 : 0);
    default: return fn >= 1 && fn <= 4 ? 3 : (fn == 5 ? 1 : 0);
  }
}

static int unmarshal(int kind, const u8* b, u64 i, u64 l, fields* out) {
  while (i < l) {
    u64 pre = i, wire, v, len;
    if (!varint(b, &i, l, &wire)) return 0;
    int32_t fn = (int32_t)(u32)(wire >> 3);
    u32 wt = wire & 7;
    if (wt == 4 || fn <= 0) return 0;
    int t = ftype(kind, fn);
    if (t == 0) {
      i = pre;
      if (!skip_raft(b, &i, l)) return 0;
      continue;
    }
    if (t == 1 || (t == 3 && wt == 0)) {
      if (wt != 0 || !varint(b, &i, l, &v)) return 0;
      if (kind == K_MSG && out) out->f[fn] = v;
      continue;
    }
    if (wt != 2 || !varint(b, &i, l, &len) || (int64_t)len < 0) return 0;
    u64 post = i + len;
    if (post < i || post > l) return 0;
    if (t == 2) {
      if (kind == K_MSG && fn == 12 && out) {
        out->has_ctx = 1;
        out->ctx_pos = i;
        out->ctx_len = len;
      }
      i = post;
    } else if (t == 3) {
      while (i < post)
        if (!varint(b, &i, l, &v)) return 0; /* bounded by l, as written */
    } else {
      if (!unmarshal(t - 10, b, i, post, NULL)) return 0;
      i = post;
    }
  }
  return 1;
}

typedef struct {
  u64 M;
  const u8* bytes;
  u64 nbytes;
  const u64* moff;
  const u32* mgroup;
  u64 G;
  const u32* off;
  const u64* ids;
  u32* rg;
  u8* rf;
  u64 *ri, *rt, *rh, *rl;
  u8* status;
  u64 m0, m1;
} wjob;

static void ingest_one(const wjob* j, u64 m) {
  u64 p0 = j->moff[m], p1 = j->moff[m + 1];
  fields f = {{0}, 0, 0, 0};
  u32 group = 0xFFFFFFFFu;
  u8 flags = 0, st;
  u64 index = 0, term = 0, hint = 0, lt = 0;
  if (p1 < p0 || p1 > j->nbytes || !unmarshal(K_MSG, j->bytes, p0, p1, &f)) {
    st = 1;
  } else {
    int kind;
    switch ((u32)f.f[1]) {
      case 4: kind = 0; break;
      case 9: kind = 1; break;
      case 11: kind = 2; break;
      case 10: kind = 3; break;
      default: kind = -1;
    }
    if (kind < 0) {
      st = 2;
    } else {
      st = 0;
      index = f.f[6];
      if (kind == 1) {
        index = 0;
        if (f.has_ctx && f.ctx_len) {
          u64 v = 0;
          if (f.ctx_len == 8)
            for (int t = 0; t < 8; t++) v = (v << 8) | j->bytes[f.ctx_pos + t];
          if (f.ctx_len != 8 || v == 0) st = 3;
          index = v;
        }
      }
      if (st == 0) {
        group = j->mgroup[m];
        u32 slot = 0x40;
        if (group < j->G)
          for (u32 s = j->off[group]; s < j->off[group + 1]; s++)
            if (j->ids[s] == f.f[3]) {
              slot = s - j->off[group];
              break;
            }
        flags = (u8)(slot | ((u32)kind << 4) | (f.f[10] ? 0x80u : 0u));
        term = f.f[4];
        hint = f.f[11];
        lt = f.f[5];
      } else {
        index = 0;
      }
    }
  }
  j->rg[m] = group;
  j->rf[m] = flags;
  j->ri[m] = index;
  j->rt[m] = term;
  j->rh[m] = hint;
  j->rl[m] = lt;
  j->status[m] = st;
}

static void* wworker(void* p) {
  wjob* j = (wjob*)p;
  for (u64 m = j->m0; m < j->m1; m++) ingest_one(j, m);
  return NULL;
}

void orc_ingest(u64 M, const u8* bytes, u64 nbytes, const u64* moff, const u32* mgroup, u64 G,
                const u32* off, const u64* ids, u32* rg, u8* rf, u64* ri, u64* rt, u64* rh,
                u64* rl, u8* status, int threads) {
  if (threads < 1) threads = 1;
  wjob* jobs = (wjob*)calloc((size_t)threads, sizeof(wjob));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    wjob j = {M, bytes, nbytes, moff, mgroup, G, off, ids, rg, rf, ri, rt, rh, rl, status,
              M * (u64)t / (u64)threads, M * (u64)(t + 1) / (u64)threads};
    jobs[t] = j;
  }
  for (int t = 1; t < threads; t++) pthread_create(&th[t], NULL, wworker, &jobs[t]);
  wworker(&jobs[0]);
  for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
}
