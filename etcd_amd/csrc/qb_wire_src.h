// qb_wire_src.h — the composed wire -> tracker steps' shared pieces: the
// bytes' arguments, the record class of a decoded message (what the tracker
// steps take from it) and the slow path's record source that re-decodes a
// message from the bytes (qb_wire_tracker.hip; the CSR step's apply launch in
// qb_tracker_csr.hip).  DESIGN.md §3.8c.
#pragma once

#include "qb_wire_decode.h"
#include "qb_bucket.h"

namespace qb {
namespace wt {

using bk::Geometry;
using wire::Decoded;
using wire::GlobalSrc;
using wire::GroupRow;
using wire::RowArgs;

struct WireArgs {
  u64 nbytes;
  const u8* bytes;
  RowArgs R;        // G, msg_off, msg_group, off, ids, rows
  u8* status;       // per message (QB_WIRE_*)
  u64 *ri, *rt;     // escapes: the exact index / term at the message's position
  u64* wstats;      // nullable: QB_WIRE_* counts
};

// The leader-inbox record of a decoded message as the tracker takes it:
// valid (a MsgAppResp of a group < G from a member slot < n), or counted
// bad (not a record of a group) / non-member.
struct RecClass {
  bool ok, bad, non;
};
__device__ __forceinline__ RecClass classify(const Geometry& geo, const Decoded& d) {
  const bool rec = d.st == QB_WIRE_OK && ((d.flags >> 4) & 3u) == QB_IN_APP_RESP && d.group < geo.G;
  const bool member = (d.flags & QB_REC_NO_PROGRESS) == 0 && (d.flags & 0x0Fu) < geo.n;
  return RecClass{rec && member, !rec, rec && !member};
}

// ----------------------------------------------------------------- slow ----
// The slow path's records re-decoded from the bytes: message i is a record of
// a flagged chunk when its envelope group's chunk is flagged, its status is
// OK and it decodes to a MsgAppResp from a member slot (what the records the
// ingest would have written hold).  Only those messages are decoded.
struct WireSrc {
  WireArgs W;
  __device__ __forceinline__ bool get(const Geometry& geo, const u8* __restrict__ chunk_slow,
                                      u64 i, u32& g, u32& f, u64& idx, u64& t) const {
    g = W.R.mgroup[i];
    if (!(g < geo.G && chunk_slow[geo.chunk_of(g)] == 1 && W.status[i] == QB_WIRE_OK)) return false;
    GroupRow row;
    wire::load_row(W.R, i, row);
    wire::load_ids(W.R, row);
    const Decoded d = wire::decode_one<GlobalSrc, true>(W.R, W.nbytes, GlobalSrc{W.bytes},
                                                         W.R.moff[i], W.R.moff[i + 1], row);
    if (!classify(geo, d).ok) return false;
    f = d.flags;
    idx = d.index;
    t = d.term;
    return true;
  }
};

// qb_tracker_csr.hip: the CSR geometry of (G, max_slots, M) and the
// composed CSR step's apply half over the bytes.
}  // namespace wt
namespace bk {
u32 csr_wmax(uint32_t max_slots);
Geometry csr_geometry(uint64_t G, uint32_t max_slots, uint64_t M);
}  // namespace bk
namespace wt {
void csr_apply_wire(u32 wmax, const bk::Geometry& geo, const bk::Carve& cv, char* ws,
                    const u32* off, const u32* cfg, const u64* group_term, const u64* term_start,
                    u64* match, u64* next, u16* active, u64* committed, u32* stepdown_at,
                    u8* advanced, const WireArgs& W, u64* stats, hipStream_t st);
}  // namespace wt
}  // namespace qb
