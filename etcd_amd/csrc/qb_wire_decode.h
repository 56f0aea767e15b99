// qb_wire_decode.h — the gogoproto raftpb.Message decoder of the wire ingest
// (qb_wire.hip) and of the composed wire -> tracker step (qb_wire_tracker.hip),
// gfx950.  Validation is Message.Unmarshal as generated (paths relative to
// the reference's raft/raftpb/):
//   Message.Unmarshal          raft.pb.go:1739-2061
//   Entry / Snapshot / SnapshotMetadata / ConfState.Unmarshal
//                              raft.pb.go:1360-1738, 2169-2542
//   skipRaft                   raft.pb.go:2909-2988
// plus the group-row lookup that maps From to the group's slot.
#pragma once

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

// The group rows a message's From is looked up in: the 64-byte rows
// (qb_dev_wire_group_rows) or the CSR slot range (off) and IDs.
struct RowArgs {
  u64 G;
  const u64* moff;
  const u32* mgroup;
  const u32* off;
  const u64* ids;
  const u64* rows;  // nullable: the 64-byte group rows
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

// The group row of a message whose envelope group is mg: the 64-byte row,
// or the slot range (off) with the IDs read by load_ids after it.
__device__ __forceinline__ void load_row_of(const RowArgs& A, u32 mg, GroupRow& row) {
  row.mg = mg;
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
// The group row of message mc.
__device__ __forceinline__ void load_row(const RowArgs& A, u64 mc, GroupRow& row) {
  load_row_of(A, __builtin_nontemporal_load(A.mgroup + mc), row);
}
__device__ __forceinline__ void load_ids(const RowArgs& A, GroupRow& row) {
  if (!A.rows) {
    const u32 n = row.mg < A.G ? row.s1 - row.s0 : 0u;
    const u64* idp = n ? A.ids + row.s0 : A.moff;
#pragma unroll
    for (u32 k = 0; k < kIdBatch; ++k) row.id[k] = idp[n ? (k < n ? k : n - 1) : 0u];
  }
}

// One decoded message: its status (QB_WIRE_*, or kDeferred), Message.Type
// (0 when it does not unmarshal) and the leader-inbox record (group ~0 and
// zeros unless the status is QB_WIRE_OK).
struct Decoded {
  int st;
  u32 group;
  u8 flags, type;
  u64 index, term, hint, lterm;
};

// One message on [p0, p1) of a buffer of nbytes: decode, classify, map From
// to its slot.  GENERIC = false (the first launch): a message the branch-free
// fast prefix does not consume whole is deferred (st = kDeferred, nothing
// else meaningful) to a launch that decodes it with the generic loop.
// Keeping the generic decoder (every nested kind inlined) out of the first
// launch's code is worth 22 % of the wire row: its mere presence cost
// registers and instruction-cache footprint though canonical messages never
// enter it.
template <class Src, bool GENERIC>
__device__ __forceinline__ Decoded decode_one(const RowArgs& A, u64 nbytes, const Src& s, u64 p0,
                                              u64 p1, const GroupRow& row) {
  Fields f = Fields{};
  Decoded d{QB_WIRE_OK, 0xFFFFFFFFu, 0, 0, 0, 0, 0, 0};
  bool ok = p0 <= p1 && p1 <= nbytes;
  if (ok) {
    u64 i = p0;
    ok = fast_prefix(s, i, p1, f);
    if (ok && i < p1) {
      if constexpr (!GENERIC) {
        d.st = kDeferred;
        return d;
      } else {
        ok = unmarshal<K_MESSAGE>(s, i, p1, &f);
      }
    }
  }
  if (!ok) {
    d.st = QB_WIRE_UNMARSHAL;
    return d;
  }
  d.type = u8(f.type);
  const int kind = kind_of_type(f.type);
  if (kind < 0) {
    d.st = QB_WIRE_TYPE;
    return d;
  }
  u64 index = f.index;
  if (kind == QB_IN_HEARTBEAT_RESP) {
    index = 0;
    if (f.has_ctx && f.ctx_len != 0) {
      const u64 v = f.ctx_len == 8 ? load_be64(s, f.ctx_pos) : 0ull;  // big-endian id
      if (f.ctx_len != 8 || v == 0) d.st = QB_WIRE_CTX;
      index = v;
    }
  }
  if (d.st != QB_WIRE_OK) return d;
  d.group = row.mg;
  u32 slot = QB_REC_NO_PROGRESS;
  if (d.group < A.G) {
    const u32 n = row.s1 - row.s0;
    const u32 held = A.rows ? kRowIds : kIdBatch;  // IDs already in registers
#pragma unroll
    for (u32 k = kIdBatch; k-- > 0;)
      if (k < n && k < held && row.id[k] == f.from) slot = k;
    // members past the row: four IDs per round trip (a ragged config's
    // 8th-11th slots in one; loads clamped to the group's last slot)
    for (u32 j = row.s0 + held; j < row.s1 && slot == QB_REC_NO_PROGRESS; j += 4) {
      u64 v[4];
#pragma unroll
      for (u32 q = 0; q < 4; ++q) v[q] = A.ids[j + q < row.s1 ? j + q : row.s1 - 1];
#pragma unroll
      for (u32 q = 4; q-- > 0;)
        if (j + q < row.s1 && v[q] == f.from) slot = j + q - row.s0;
    }
  }
  d.flags = u8(slot | (u32(kind) << 4) | (f.reject ? QB_REC_REJECT : 0u));
  d.index = index;
  d.term = f.term;
  d.hint = f.hint;
  d.lterm = f.log_term;
  return d;
}

}  // namespace wire
}  // namespace qb
