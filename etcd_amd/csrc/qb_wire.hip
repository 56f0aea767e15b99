// qb_wire.hip — wire ingest: raw raftpb.Message bytes -> leader-inbox records
// (SURVEY.md §8f row 3), gfx950.
//
// Each message is validated exactly as the generated gogoproto decoder does
// (paths relative to the reference's raft/raftpb/):
//   Message.Unmarshal          raft.pb.go:1739-2061
//   Entry / Snapshot / SnapshotMetadata / ConfState.Unmarshal
//                              raft.pb.go:1360-1738, 2169-2542 (nested
//                              messages are decoded too: a malformed nested
//                              body fails the message, as in Go)
//   skipRaft                   raft.pb.go:2909-2988 (unknown fields, groups)
// and the four response types the leader step consumes (MsgAppResp,
// MsgHeartbeatResp, MsgSnapStatus, MsgUnreachable) become SoA records; From
// is mapped to the group's slot (the sorted voter/learner IDs of the CSR
// config), a non-member keeps QB_REC_NO_PROGRESS (stepLeader drops it,
// raft.go:1099-1104).
//
// Layout: one thread per message; a workgroup stages its 256 messages'
// bytes (one contiguous span of the batch buffer) into LDS with 16-byte
// loads when the span fits, so parsing reads LDS instead of issuing one
// global byte load per varint byte; spans that do not fit parse from global.
#include "qb_common.h"

namespace qb {
namespace wire {

constexpr u32 kStage = 16 * 1024;  // LDS staging bytes per workgroup (~40 B x 256 messages fit)

enum Kind : u32 { K_MESSAGE = 0, K_ENTRY = 1, K_SNAPSHOT = 2, K_SNAPMETA = 3, K_CONFSTATE = 4 };
enum FieldType : u32 { T_UNKNOWN = 0, T_VARINT, T_BYTES, T_REPEATED, T_NESTED };

// SCHEMAS of oracle/raftpb_ref.py (raft.proto field numbers and types).
__device__ __forceinline__ u32 field_type(u32 kind, int fnum, u32* nested) {
  switch (kind) {
    case K_MESSAGE:
      if (fnum == 7) { *nested = K_ENTRY; return T_NESTED; }
      if (fnum == 9) { *nested = K_SNAPSHOT; return T_NESTED; }
      if (fnum == 12) return T_BYTES;
      return (fnum >= 1 && fnum <= 11) ? T_VARINT : T_UNKNOWN;
    case K_ENTRY:
      if (fnum == 4) return T_BYTES;
      return (fnum >= 1 && fnum <= 3) ? T_VARINT : T_UNKNOWN;
    case K_SNAPSHOT:
      if (fnum == 1) return T_BYTES;
      if (fnum == 2) { *nested = K_SNAPMETA; return T_NESTED; }
      return T_UNKNOWN;
    case K_SNAPMETA:
      if (fnum == 1) { *nested = K_CONFSTATE; return T_NESTED; }
      return (fnum == 2 || fnum == 3) ? T_VARINT : T_UNKNOWN;
    default:  // K_CONFSTATE
      if (fnum >= 1 && fnum <= 4) return T_REPEATED;
      return fnum == 5 ? T_VARINT : T_UNKNOWN;
  }
}

// Byte sources addressed by absolute offset: the workgroup's LDS stage (a
// message whose bytes lie inside the staged span) or global memory.
struct LdsSrc {
  const u8* lds;
  u64 base;
  __device__ __forceinline__ u8 at(u64 i) const { return lds[i - base]; }
};
struct GlobalSrc {
  const u8* g;
  __device__ __forceinline__ u8 at(u64 i) const { return g[i]; }
};

// The generated decoders' varint loop: error at shift >= 64 or at l.
template <class Src>
__device__ __forceinline__ bool varint(const Src& s, u64& i, u64 l, u64& v);

// Straight-line varint for the fast prefix: from the LDS stage, the 8 bytes
// at i come from two aligned 8-byte LDS reads, the terminator is the lowest
// byte with its high bit clear and the 7-bit groups are compacted with
// shifts and masks (no per-byte loop, no divergence); a varint longer than 8
// bytes takes the byte loop.  Bytes at or past l never decide the result: a
// terminator found there is the same EOF error the byte loop reports.
template <class Src>
__device__ __forceinline__ bool varint_fast(const Src& s, u64& i, u64 l, u64& v) {
  return varint(s, i, l, v);
}
template <>
__device__ __forceinline__ bool varint_fast<LdsSrc>(const LdsSrc& s, u64& i, u64 l, u64& v) {
  const u64 off = i - s.base;
  const u64* w = reinterpret_cast<const u64*>(s.lds) + (off >> 3);
  const u32 sh = u32(off & 7u) * 8u;
  const u64 lo = w[0], hi = w[1];
  const u64 x = sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
  const u64 stop = ~x & 0x8080808080808080ull;
  if (stop == 0) return varint(s, i, l, v);
  const u32 n = (u32(__builtin_ctzll(stop)) >> 3) + 1u;  // bytes in the varint
  if (i + n > l) return false;
  const u64 xm = n == 8 ? x : x & ((1ull << (8u * n)) - 1u);
  v = (xm & 0x7Full) | ((xm >> 1) & (0x7Full << 7)) | ((xm >> 2) & (0x7Full << 14)) |
      ((xm >> 3) & (0x7Full << 21)) | ((xm >> 4) & (0x7Full << 28)) |
      ((xm >> 5) & (0x7Full << 35)) | ((xm >> 6) & (0x7Full << 42)) |
      ((xm >> 7) & (0x7Full << 49));
  i += n;
  return true;
}

template <class Src>
__device__ __forceinline__ bool varint(const Src& s, u64& i, u64 l, u64& v) {
  v = 0;
  for (u32 shift = 0;; shift += 7) {
    if (shift >= 64 || i >= l) return false;
    const u8 b = s.at(i++);
    v |= u64(b & 0x7Fu) << shift;
    if (b < 0x80u) return true;
  }
}

// skipRaft on [i, l): advances i past one field (with nested groups).
template <class Src>
__device__ bool skip_field(const Src& s, u64& i, u64 l) {
  const u64 start = i;
  int depth = 0;
  while (i < l) {
    u64 wire;
    if (!varint(s, i, l, wire)) return false;
    switch (wire & 7u) {
      case 0: {
        for (u32 shift = 0;; shift += 7) {
          if (shift >= 64 || i >= l) return false;
          if (s.at(i++) < 0x80u) break;
        }
        break;
      }
      case 1: i += 8; break;
      case 2: {
        u64 len;
        if (!varint(s, i, l, len)) return false;
        if (int64_t(len) < 0) return false;
        i += len;
        if (i < start) return false;  // wrapped: Go's int overflow -> negative
        break;
      }
      case 3: ++depth; break;
      case 4:
        if (depth == 0) return false;
        --depth;
        break;
      case 5: i += 4; break;
      default: return false;
    }
    if (depth == 0) return i <= l;
  }
  return false;
}

struct Fields {
  u64 type, from, term, log_term, index, reject, hint;
  u64 ctx_pos, ctx_len;
  bool has_ctx;
};

// The generated Unmarshal of one message kind on [i, l): nested bodies are
// decoded by the nested kind's own instantiation (the nesting is fixed:
// Message > Entry | Snapshot > SnapshotMetadata > ConfState), so everything
// inlines into straight-line code with no private-memory frame stack.
template <u32 KIND, class Src>
__device__ __forceinline__ bool unmarshal(const Src& s, u64 i, const u64 l, Fields* f) {
  while (i < l) {
    const u64 pre = i;
    u64 wire;
    if (!varint(s, i, l, wire)) return false;
    const int fnum = int(u32(wire >> 3));  // int32(wire >> 3)
    const u32 wt = u32(wire & 7u);
    if (wt == 4) return false;  // end group for non-group
    if (fnum <= 0) return false;  // illegal tag
    u32 nested = 0;
    const u32 ft = field_type(KIND, fnum, &nested);
    if (ft == T_UNKNOWN) {
      i = pre;
      if (!skip_field(s, i, l)) return false;
      continue;
    }
    if (ft == T_VARINT || (ft == T_REPEATED && wt == 0)) {
      if (wt != 0) return false;  // wrong wiretype
      u64 v;
      if (!varint(s, i, l, v)) return false;
      if constexpr (KIND == K_MESSAGE) {
        switch (fnum) {
          case 1: f->type = v; break;
          case 3: f->from = v; break;
          case 4: f->term = v; break;
          case 5: f->log_term = v; break;
          case 6: f->index = v; break;
          case 10: f->reject = v; break;
          case 11: f->hint = v; break;
          default: break;
        }
      }
      continue;
    }
    if (wt != 2) return false;  // wrong wiretype
    u64 len;
    if (!varint(s, i, l, len)) return false;
    if (int64_t(len) < 0) return false;
    const u64 post = i + len;
    if (post < i || post > l) return false;
    if (ft == T_BYTES) {
      if constexpr (KIND == K_MESSAGE) {
        if (fnum == 12) {
          f->has_ctx = true;
          f->ctx_pos = i;
          f->ctx_len = len;
        }
      }
      i = post;
    } else if (ft == T_REPEATED) {  // packed: each varint bounded by l, not post
      while (i < post) {
        u64 v;
        if (!varint(s, i, l, v)) return false;
      }
    } else {  // nested message on [i, post)
      bool ok = true;
      if constexpr (KIND == K_MESSAGE) {
        ok = nested == K_ENTRY ? unmarshal<K_ENTRY>(s, i, post, nullptr)
                               : unmarshal<K_SNAPSHOT>(s, i, post, nullptr);
      } else if constexpr (KIND == K_SNAPSHOT) {
        ok = unmarshal<K_SNAPMETA>(s, i, post, nullptr);
      } else if constexpr (KIND == K_SNAPMETA) {
        ok = unmarshal<K_CONFSTATE>(s, i, post, nullptr);
      }
      if (!ok) return false;
      i = post;
    }
  }
  return true;
}

// gogoproto's Marshal writes a Message's fields in field-number order, every
// non-nullable one always (raft.pb.go MarshalToSizedBuffer): type, to, from,
// term, logTerm, index, [entries], commit, snapshot, reject, rejectHint,
// [context].  fast_prefix consumes the longest prefix of the message that
// follows that order with one-byte keys, in straight-line code (no per-field
// dispatch, so the lanes of a wave stay converged), and the generic loop
// continues from there.  Unmarshal is a left fold over the fields, so the
// result is the generic decoder's on any input: a field is consumed here
// only when its key byte is the expected one-byte key, and it is then
// decoded exactly as the generic loop decodes it.  The snapshot is consumed
// only in its common empty form (12 00: an empty SnapshotMetadata).
template <class Src>
__device__ __forceinline__ bool fast_prefix(const Src& s, u64& i, const u64 l, Fields& f) {
#define QB_FAST_VARINT(KEY, DST)                     \
  {                                                  \
    if (i >= l || s.at(i) != (KEY)) return true;     \
    u64 i2 = i + 1, v;                               \
    if (!varint_fast(s, i2, l, v)) return false;     \
    DST = v;                                         \
    i = i2;                                          \
  }
  u64 ignored;
  QB_FAST_VARINT(0x08, f.type)
  QB_FAST_VARINT(0x10, ignored)
  QB_FAST_VARINT(0x18, f.from)
  QB_FAST_VARINT(0x20, f.term)
  QB_FAST_VARINT(0x28, f.log_term)
  QB_FAST_VARINT(0x30, f.index)
  QB_FAST_VARINT(0x40, ignored)
  if (i + 4 > l || s.at(i) != 0x4A || s.at(i + 1) != 0x02 || s.at(i + 2) != 0x12 ||
      s.at(i + 3) != 0x00)
    return true;
  i += 4;
  QB_FAST_VARINT(0x50, f.reject)
  QB_FAST_VARINT(0x58, f.hint)
#undef QB_FAST_VARINT
  (void)ignored;
  // context (field 12, bytes) of the common 8-byte form: what the generic
  // loop does for key 0x62 with a one-byte length 8 inside the message
  if (i + 10 <= l && s.at(i) == 0x62 && s.at(i + 1) == 0x08) {
    f.has_ctx = true;
    f.ctx_pos = i + 2;
    f.ctx_len = 8;
    i += 10;
  }
  return true;
}

// The fast prefix from the LDS stage, branch-free.  Each field is one
// 8-byte window at a 32-bit stage offset (two aligned LDS reads): the key is
// byte 0, the varint starts at byte 1 and ends at the lowest of bytes 1-7
// with the high bit clear, its 7-bit groups compacted in three SWAR steps.
// Every field is evaluated under a predicate instead of an early return (the
// wire row is issue-bound once its group rows are one gather: the branchy
// form spent as many scalar instructions on exec masks as vector ones): a
// lane whose message leaves the canonical form — another key, a varint of 8+
// bytes, a varint running past the message — simply stops consuming there,
// and the generic loop (unmarshal<K_MESSAGE>) continues from that byte with
// the generic decoder's result on any input.
__device__ __forceinline__ u64 lds_win(const u8* lds, u32 o) {
  const u64* w = reinterpret_cast<const u64*>(lds) + (o >> 3);
  const u32 sh = (o & 7u) * 8u;
  const u64 lo = w[0], hi = w[1];
  return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
}
__device__ __forceinline__ u64 varint_bits(u64 x) {  // x: the varint's bytes, higher bytes 0
  x &= 0x7F7F7F7F7F7F7F7Full;
  x = (x & 0x007F007F007F007Full) | ((x & 0x7F007F007F007F00ull) >> 1);
  x = (x & 0x00003FFF00003FFFull) | ((x & 0x3FFF00003FFF0000ull) >> 2);
  return (x & 0x000000000FFFFFFFull) | ((x & 0x0FFFFFFF00000000ull) >> 4);
}
// key byte `key`, then a varint: consumed into dst when the lane is still in
// the canonical form (go) and the field is whole inside [o, e)
__device__ __forceinline__ void fast_field(const u8* lds, u32& o, u32 e, bool& go, u32 key,
                                           u64* dst) {
  const u64 x = lds_win(lds, o);
  const u64 stop = ~x & 0x8080808080808000ull;
  const u32 t = stop ? u32(__builtin_ctzll(stop)) >> 3 : 8u;  // varint bytes (1..7; 8 = none)
  const bool ok = go && u32(x & 0xFFu) == key && t < 8u && o + 1u + t <= e;
  if (dst) {
    const u64 v = varint_bits((x >> 8) & (~0ull >> (64u - 8u * (t < 8u ? t : 7u))));
    *dst = ok ? v : *dst;
  }
  o = ok ? o + 1u + t : o;
  go = ok;
}

template <>
__device__ __forceinline__ bool fast_prefix<LdsSrc>(const LdsSrc& s, u64& i, const u64 l,
                                                   Fields& f) {
  u32 o = u32(i - s.base);
  const u32 e = u32(l - s.base);
  bool go = o < e;
  fast_field(s.lds, o, e, go, 0x08, &f.type);
  fast_field(s.lds, o, e, go, 0x10, nullptr);
  fast_field(s.lds, o, e, go, 0x18, &f.from);
  fast_field(s.lds, o, e, go, 0x20, &f.term);
  fast_field(s.lds, o, e, go, 0x28, &f.log_term);
  fast_field(s.lds, o, e, go, 0x30, &f.index);
  fast_field(s.lds, o, e, go, 0x40, nullptr);
  {  // the zero Snapshot as gogoproto writes it — Metadata and its ConfState
     // are non-nullable, AutoLeave / Index / Term always present:
     // 4A 0A 12 08 0A 02 28 00 10 00 18 00 — or with an empty Metadata,
     // 4A 02 12 00 (any encoding of it decodes the same)
    const u64 x = lds_win(s.lds, o);
    const u32 y = u32(lds_win(s.lds, o + 8u));
    const bool full = o + 12u <= e && x == 0x0028020A08120A4Aull && y == 0x00180010u;
    const bool brief = o + 4u <= e && u32(x) == 0x0012024Au;
    const bool ok = go && (full || brief);
    o = ok ? o + (full ? 12u : 4u) : o;
    go = ok;
  }
  fast_field(s.lds, o, e, go, 0x50, &f.reject);
  fast_field(s.lds, o, e, go, 0x58, &f.hint);
  {  // context (field 12, bytes) of the common 8-byte form
    const bool ok = go && o + 10u <= e && u32(lds_win(s.lds, o) & 0xFFFFu) == 0x0862u;
    f.has_ctx = ok;
    f.ctx_pos = ok ? s.base + o + 2u : 0ull;
    f.ctx_len = ok ? 8ull : 0ull;
    o = ok ? o + 10u : o;
  }
  i = s.base + o;
  return true;  // errors are the generic loop's to find
}

// The 8 bytes at i as a big-endian u64 (the read context's request id).
template <class Src>
__device__ __forceinline__ u64 load_be64(const Src& s, u64 i) {
  u64 v = 0;
  for (u32 t = 0; t < 8; ++t) v = (v << 8) | s.at(i + t);
  return v;
}
template <>
__device__ __forceinline__ u64 load_be64<LdsSrc>(const LdsSrc& s, u64 i) {
  const u64 off = i - s.base;
  const u64* w = reinterpret_cast<const u64*>(s.lds) + (off >> 3);
  const u32 sh = u32(off & 7u) * 8u;
  const u64 lo = w[0], hi = w[1];
  return __builtin_bswap64(sh ? (lo >> sh) | (hi << (64u - sh)) : lo);
}

template <class Src>
__device__ __forceinline__ bool unmarshal_message(const Src& s, u64 start, u64 end, Fields& f) {
  f = Fields{};
  u64 i = start;
  if (!fast_prefix(s, i, end, f)) return false;
  return unmarshal<K_MESSAGE>(s, i, end, &f);
}

__device__ __forceinline__ int kind_of_type(u64 type32) {
  switch (u32(type32)) {
    case 4: return QB_IN_APP_RESP;        // MsgAppResp
    case 9: return QB_IN_HEARTBEAT_RESP;  // MsgHeartbeatResp
    case 11: return QB_IN_SNAP_STATUS;    // MsgSnapStatus
    case 10: return QB_IN_UNREACHABLE;    // MsgUnreachable
    default: return -1;
  }
}

struct Args {
  u64 M, nbytes, G;
  const u8* bytes;
  const u64* moff;
  const u32* mgroup;
  const u32* off;
  const u64* ids;
  const u64* rows;  // nullable: the 64-byte group rows (qb_dev_wire_group_rows)
  u32* rg;
  u8* rf;
  u64 *ri, *rt, *rh, *rl;
  u8* status;
  u8* mtype;
  u64* stats;
};

// The group row of one message, loaded ahead of the parse: the slot range
// (off) and the first kIdBatch member IDs (wider configs continue one by one
// after the parse).  Loads are branch-free — clamped rows, and an empty row
// reads a harmless word of moff — so their wait lands where the IDs are
// compared, after the parse, not ahead of it.
constexpr u32 kIdBatch = 8;
constexpr u32 kRowIds = 7;  // member IDs held in a 64-byte group row
struct GroupRow {
  u32 mg, s0, s1;
  u64 id[kIdBatch];
};

// A message the first launch leaves to the second (status value between the
// launches only; never returned).
constexpr u8 kDeferred = 0xFF;

// One message: decode, classify, map From to its slot, write the record.
// GENERIC = false (the first launch): a message the branch-free fast prefix
// does not consume whole is deferred — status kDeferred, nothing else
// written — to the second launch, which decodes it with the generic loop.
// Keeping the generic decoder (every nested kind inlined) out of the first
// launch's code is worth 22 % of the row: its mere presence cost registers
// and instruction-cache footprint though canonical messages never enter it.
template <class Src, bool GENERIC>
__device__ __forceinline__ int ingest_one(const Args& A, const Src& s, u64 m, u64 p0, u64 p1,
                                          GroupRow& row) {
  Fields f = Fields{};
  int st_;
  u32 group = 0xFFFFFFFFu;
  u8 flags = 0;
  u64 index = 0, term = 0, hint = 0, lterm = 0;
  bool ok = p0 <= p1 && p1 <= A.nbytes;
  if (ok) {
    u64 i = p0;
    ok = fast_prefix(s, i, p1, f);
    if (ok && i < p1) {
      if constexpr (!GENERIC) {
        __builtin_nontemporal_store(kDeferred, A.status + m);
        return kDeferred;
      } else {
        ok = unmarshal<K_MESSAGE>(s, i, p1, &f);
      }
    }
  }
  if (!ok) {
    st_ = QB_WIRE_UNMARSHAL;
    if (A.mtype) __builtin_nontemporal_store(u8(0), A.mtype + m);
  } else {
    if (A.mtype) __builtin_nontemporal_store(u8(f.type), A.mtype + m);
    const int kind = kind_of_type(f.type);
    if (kind < 0) {
      st_ = QB_WIRE_TYPE;
    } else {
      index = f.index;
      st_ = QB_WIRE_OK;
      if (kind == QB_IN_HEARTBEAT_RESP) {
        index = 0;
        if (f.has_ctx && f.ctx_len != 0) {
          const u64 v = f.ctx_len == 8 ? load_be64(s, f.ctx_pos) : 0ull;  // big-endian id
          if (f.ctx_len != 8 || v == 0) st_ = QB_WIRE_CTX;
          index = v;
        }
      }
      if (st_ == QB_WIRE_OK) {
        group = row.mg;
        u32 slot = QB_REC_NO_PROGRESS;
        if (group < A.G) {
          const u32 n = row.s1 - row.s0;
          const u32 held = A.rows ? kRowIds : kIdBatch;  // IDs already in registers
#pragma unroll
          for (u32 k = kIdBatch; k-- > 0;)
            if (k < n && k < held && row.id[k] == f.from) slot = k;
          for (u32 j = row.s0 + held; j < row.s1 && slot == QB_REC_NO_PROGRESS; ++j)
            if (A.ids[j] == f.from) slot = j - row.s0;
        }
        flags = u8(slot | (u32(kind) << 4) | (f.reject ? QB_REC_REJECT : 0u));
        term = f.term;
        hint = f.hint;
        lterm = f.log_term;
      } else {
        index = 0;
      }
    }
  }
  // The record columns are written once and read by a later launch: stored
  // nontemporal, so the stream does not evict the group rows (off, ids) that
  // every message gathers at random from the Infinity Cache.
  __builtin_nontemporal_store(group, A.rg + m);
  __builtin_nontemporal_store(flags, A.rf + m);
  __builtin_nontemporal_store(index, A.ri + m);
  __builtin_nontemporal_store(term, A.rt + m);
  if (A.rh) __builtin_nontemporal_store(hint, A.rh + m);
  if (A.rl) __builtin_nontemporal_store(lterm, A.rl + m);
  __builtin_nontemporal_store(u8(st_), A.status + m);
  return st_;
}

// The group row of message mc: the 64-byte row, or the slot range (off)
// with the IDs read by load_ids after it.
__device__ __forceinline__ void load_row(const Args& A, u64 mc, GroupRow& row) {
  row.mg = __builtin_nontemporal_load(A.mgroup + mc);
  if (A.rows) {
    // the group's 64-byte row: one aligned line segment per message instead
    // of a row of off and then one or two lines of ids
    const u32 gi = row.mg < A.G ? row.mg : 0u;
    const ulonglong2* rw = reinterpret_cast<const ulonglong2*>(A.rows + 8ull * gi);
    const ulonglong2 a = rw[0], b = rw[1], c = rw[2], d = rw[3];
    row.s0 = u32(a.x >> 32);
    row.s1 = row.s0 + u32(a.x);  // n: the member count
    row.id[0] = a.y;
    row.id[1] = b.x;
    row.id[2] = b.y;
    row.id[3] = c.x;
    row.id[4] = c.y;
    row.id[5] = d.x;
    row.id[6] = d.y;
    row.id[7] = 0;  // (member 8 and up: ids[s0 + k], after the parse)
  } else {
    // G == 0: off may be absent; read the first word of moff (>= 2 entries)
    const u32* offp = A.G ? A.off : reinterpret_cast<const u32*>(A.moff);
    const u32 gi = row.mg < A.G ? row.mg : 0u;
    row.s0 = offp[gi];
    row.s1 = offp[gi + 1];
  }
}
__device__ __forceinline__ void load_ids(const Args& A, GroupRow& row) {
  if (!A.rows) {
    const u32 n = row.mg < A.G ? row.s1 - row.s0 : 0u;
    const u64* idp = n ? A.ids + row.s0 : A.moff;
#pragma unroll
    for (u32 k = 0; k < kIdBatch; ++k) row.id[k] = idp[n ? (k < n ? k : n - 1) : 0u];
  }
}

// First launch.  Round trips per workgroup: (1) the message offsets and
// groups; (2) the groups' rows beside the LDS-DMA stage of the byte span;
// (3) (CSR IDs only) the member IDs, in flight while the messages are parsed
// from LDS.  A message outside the staged span is deferred too.
__global__ __launch_bounds__(kBlock) void k_ingest(Args A) {
  __shared__ __attribute__((aligned(16))) u8 stage[kStage + 48];  // + window over-reads (<= 24 B past a message)
  __shared__ u32 lds[4];
  BlockTally<4> tally;
  const u64 m0 = u64(blockIdx.x) * kBlock;
  const u64 m = m0 + threadIdx.x;
  const u64 mlast = (m0 + kBlock < A.M ? m0 + kBlock : A.M);
  const u64 mc = m < A.M ? m : A.M - 1;  // lanes past M re-read the last message
  const u64 b0 = A.moff[m0], b1 = A.moff[mlast];
  const u64 p0 = __builtin_nontemporal_load(A.moff + mc);
  const u64 p1 = __builtin_nontemporal_load(A.moff + mc + 1);
  GroupRow row;
  load_row(A, mc, row);
  // Stage the block's byte span [b0, b1) when it fits (block-uniform).
  u64 lbase = 0, lend = 0;  // staged span (empty: nothing staged)
  if (b1 > b0 && b1 - b0 <= kStage - 16) {
    const u64 a0 = b0 & ~u64(15);             // 16-byte aligned window
    const u64 a1 = (b1 + 15) & ~u64(15);
    const u64 n16 = (a1 - a0) / 16;
    // Pieces wholly inside the byte buffer go by LDS-DMA, all issued before
    // the barrier's one wait; only the buffer's last piece can be partial.
    // (A byte buffer that is not 16-byte aligned stages with plain loads.)
    const u64 whole = (A.nbytes - a0) / 16;
    u32 nfull = u32(n16 < whole ? n16 : whole);
    if ((reinterpret_cast<uintptr_t>(A.bytes) & 15u) == 0) {
      constexpr int kIt = int((kStage + 16) / 16 / kBlock) + 1;
      stage16_lds<kBlock, kIt>(stage, A.bytes + a0, nfull);
    } else {
      const uint4* gsrc = reinterpret_cast<const uint4*>(A.bytes + a0);
      for (u64 k = threadIdx.x; k < nfull; k += kBlock) reinterpret_cast<uint4*>(stage)[k] = gsrc[k];
    }
    for (u64 k = nfull + threadIdx.x; k < n16; k += kBlock)
      for (u32 t = 0; t < 16; ++t) {
        const u64 p = a0 + 16 * k + t;
        stage[16 * k + t] = p < A.nbytes ? A.bytes[p] : 0;
      }
    lbase = a0;
    lend = a1 < A.nbytes ? a1 : A.nbytes;
  }
  __syncthreads();
  load_ids(A, row);
  int st_ = -1;
  if (m < A.M) {
    if (p0 >= lbase && p1 <= lend && p0 <= p1) {
      st_ = ingest_one<LdsSrc, false>(A, LdsSrc{stage, lbase}, m, p0, p1, row);
    } else {
      __builtin_nontemporal_store(kDeferred, A.status + m);
    }
  }
  tally.add(0, st_ == QB_WIRE_OK);
  tally.add(1, st_ == QB_WIRE_UNMARSHAL);
  tally.add(2, st_ == QB_WIRE_TYPE);
  tally.add(3, st_ == QB_WIRE_CTX);
  const int slot[4] = {QB_WIRE_OK, QB_WIRE_UNMARSHAL, QB_WIRE_TYPE, QB_WIRE_CTX};
  if (A.stats) tally.flush(lds, A.stats, slot);
}

// Second launch: the deferred messages, each decoded from global memory by
// the generic loop.  A thread scans kScan consecutive statuses (loaded
// together); with nothing deferred the launch reads the status column once.
// The statuses are read as 16-byte words (round 3: one byte load per status
// took the launch 36 us per 16M messages with nothing deferred), and a
// thread whose words hold no kDeferred byte is done.
constexpr u32 kScan = 32;
__device__ __forceinline__ bool has_ff_byte(u32 w) {  // SWAR: a byte of w is 0xFF
  const u32 x = ~w;
  return ((x - 0x01010101u) & ~x & 0x80808080u) != 0;
}
__global__ __launch_bounds__(kBlock) void k_ingest_deferred(Args A) {
  __shared__ u32 lds[4];
  const u64 m0 = (u64(blockIdx.x) * kBlock + threadIdx.x) * kScan;
  u32 sw[kScan / 4];
  if (m0 + kScan <= A.M && (reinterpret_cast<uintptr_t>(A.status + m0) & 15u) == 0) {
#pragma unroll
    for (u32 q = 0; q < kScan / 16; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(A.status + m0)[q];
      sw[4 * q] = v.x;
      sw[4 * q + 1] = v.y;
      sw[4 * q + 2] = v.z;
      sw[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (u32 q = 0; q < kScan / 4; ++q) {
      u32 w = 0;
#pragma unroll
      for (u32 b = 0; b < 4; ++b) {
        const u64 m = m0 + 4 * q + b;
        w |= u32(m < A.M ? A.status[m] : u8(0)) << (8 * b);
      }
      sw[q] = w;
    }
  }
  bool any = false;
#pragma unroll
  for (u32 q = 0; q < kScan / 4; ++q) any |= has_ff_byte(sw[q]);
  u32 cnt[4] = {0, 0, 0, 0};
  for (u32 k = 0; any && k < kScan; ++k) {
    if (u8(sw[k / 4] >> (8 * (k % 4))) != kDeferred) continue;
    const u64 m = m0 + k;
    GroupRow row;
    load_row(A, m, row);
    load_ids(A, row);
    const int r = ingest_one<GlobalSrc, true>(A, GlobalSrc{A.bytes}, m, A.moff[m], A.moff[m + 1],
                                              row);
    ++cnt[r];
  }
  if (!A.stats) return;
  if (threadIdx.x < 4) lds[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    u32 v = cnt[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&lds[q], v);
  }
  __syncthreads();
  // statuses 0..3 are the stat slots QB_WIRE_OK .. QB_WIRE_CTX
  if (threadIdx.x < 4 && lds[threadIdx.x]) atomicAdd(A.stats + threadIdx.x, u64(lds[threadIdx.x]));
}

}  // namespace wire
}  // namespace qb

namespace qb {
namespace wire {
// Group rows: row g = { n | s0 << 32, the first kRowIds member IDs }, 64 B.
__global__ __launch_bounds__(kBlock) void k_group_rows(u64 G, const u32* __restrict__ off,
                                                       const u64* __restrict__ ids,
                                                       u64* __restrict__ rows) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  const u32 s0 = off[g], n = off[g + 1] - s0;
  u64 w[8];
  w[0] = u64(n) | (u64(s0) << 32);
#pragma unroll
  for (u32 k = 0; k < kRowIds; ++k) w[1 + k] = k < n ? ids[s0 + k] : 0ull;
  ulonglong2* dst = reinterpret_cast<ulonglong2*>(rows + 8 * g);
#pragma unroll
  for (u32 q = 0; q < 4; ++q) dst[q] = ulonglong2{w[2 * q], w[2 * q + 1]};
}
}  // namespace wire
}  // namespace qb

namespace qb {
namespace wire {
static int launch(const Args& A, hipStream_t st) {
  hipLaunchKernelGGL(k_ingest, dim3(grid_for(A.M)), dim3(kBlock), 0, st, A);
  QB_CHECK_LAUNCH("k_ingest");
  hipLaunchKernelGGL(k_ingest_deferred, dim3(grid_for((A.M + kScan - 1) / kScan)), dim3(kBlock), 0,
                     st, A);
  QB_CHECK_LAUNCH("k_ingest_deferred");
  return QB_OK;
}
}  // namespace wire
}  // namespace qb

using namespace qb;

extern "C" size_t qb_wire_group_rows_bytes(uint64_t G) { return size_t(G) * 64; }

extern "C" int qb_dev_wire_group_rows(uint64_t G, const uint32_t* off, const uint64_t* ids,
                                      uint64_t* rows, void* stream) {
  if (G == 0) return QB_OK;
  QB_REQUIRE(off && ids && rows, "qb_dev_wire_group_rows: off, ids and rows are required");
  QB_REQUIRE((reinterpret_cast<uintptr_t>(rows) & 15u) == 0,
             "qb_dev_wire_group_rows: rows must be 16-byte aligned");
  hipLaunchKernelGGL(wire::k_group_rows, dim3(grid_for(G)), dim3(kBlock), 0, as_stream(stream), G,
                     off, reinterpret_cast<const u64*>(ids), reinterpret_cast<u64*>(rows));
  QB_CHECK_LAUNCH("k_group_rows");
  return QB_OK;
}

extern "C" int qb_dev_ingest_messages_rows(
    uint64_t M, const uint8_t* bytes, uint64_t nbytes, const uint64_t* msg_off,
    const uint32_t* msg_group, uint64_t G, const uint64_t* rows, const uint64_t* ids,
    uint32_t* rec_group, uint8_t* rec_flags, uint64_t* rec_index, uint64_t* rec_term,
    uint64_t* rec_hint, uint64_t* rec_log_term, uint8_t* status, uint8_t* msg_type,
    uint64_t* stats, void* stream);

extern "C" int qb_dev_ingest_messages(uint64_t M, const uint8_t* bytes, uint64_t nbytes,
                                      const uint64_t* msg_off, const uint32_t* msg_group,
                                      uint64_t G, const uint32_t* off, const uint64_t* ids,
                                      uint32_t* rec_group, uint8_t* rec_flags,
                                      uint64_t* rec_index, uint64_t* rec_term,
                                      uint64_t* rec_hint, uint64_t* rec_log_term,
                                      uint8_t* status, uint8_t* msg_type, uint64_t* stats,
                                      void* stream) {
  if (M == 0) return QB_OK;
  QB_REQUIRE(msg_off && msg_group && rec_group && rec_flags && rec_index && rec_term && status,
             "qb_dev_ingest_messages: msg_off, msg_group, rec_* and status are required");
  QB_REQUIRE(nbytes == 0 || bytes, "qb_dev_ingest_messages: bytes is NULL");
  QB_REQUIRE(G == 0 || (off && ids), "qb_dev_ingest_messages: off and ids are required");
  wire::Args A{M, nbytes, G, bytes, reinterpret_cast<const u64*>(msg_off), msg_group, off,
               reinterpret_cast<const u64*>(ids), nullptr, rec_group, rec_flags,
               reinterpret_cast<u64*>(rec_index), reinterpret_cast<u64*>(rec_term),
               reinterpret_cast<u64*>(rec_hint), reinterpret_cast<u64*>(rec_log_term), status,
               msg_type, reinterpret_cast<u64*>(stats)};
  return wire::launch(A, as_stream(stream));
}

extern "C" int qb_dev_ingest_messages_rows(
    uint64_t M, const uint8_t* bytes, uint64_t nbytes, const uint64_t* msg_off,
    const uint32_t* msg_group, uint64_t G, const uint64_t* rows, const uint64_t* ids,
    uint32_t* rec_group, uint8_t* rec_flags, uint64_t* rec_index, uint64_t* rec_term,
    uint64_t* rec_hint, uint64_t* rec_log_term, uint8_t* status, uint8_t* msg_type,
    uint64_t* stats, void* stream) {
  if (M == 0) return QB_OK;
  QB_REQUIRE(msg_off && msg_group && rec_group && rec_flags && rec_index && rec_term && status,
             "qb_dev_ingest_messages_rows: msg_off, msg_group, rec_* and status are required");
  QB_REQUIRE(nbytes == 0 || bytes, "qb_dev_ingest_messages_rows: bytes is NULL");
  QB_REQUIRE(G == 0 || (rows && ids), "qb_dev_ingest_messages_rows: rows and ids are required");
  QB_REQUIRE((reinterpret_cast<uintptr_t>(rows) & 15u) == 0,
             "qb_dev_ingest_messages_rows: rows must be 16-byte aligned");
  wire::Args A{M, nbytes, G, bytes, reinterpret_cast<const u64*>(msg_off), msg_group, nullptr,
               reinterpret_cast<const u64*>(ids), G ? reinterpret_cast<const u64*>(rows) : nullptr,
               rec_group,
               rec_flags, reinterpret_cast<u64*>(rec_index), reinterpret_cast<u64*>(rec_term),
               reinterpret_cast<u64*>(rec_hint), reinterpret_cast<u64*>(rec_log_term), status,
               msg_type, reinterpret_cast<u64*>(stats)};
  return wire::launch(A, as_stream(stream));
}
