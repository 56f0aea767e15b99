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
#include "qb_wire_decode.h"

namespace qb {
namespace wire {

struct Args {
  u64 M, nbytes;
  const u8* bytes;
  RowArgs R;  // G, moff, mgroup, off, ids, rows
  u32* rg;
  u8* rf;
  u64 *ri, *rt, *rh, *rl;
  u8* status;
  u8* mtype;
  u64* stats;
};

// One message: decode_one (qb_wire_decode.h), then the record columns.
template <class Src, bool GENERIC>
__device__ __forceinline__ int ingest_one(const Args& A, const Src& s, u64 m, u64 p0, u64 p1,
                                          const GroupRow& row) {
  const Decoded d = decode_one<Src, GENERIC>(A.R, A.nbytes, s, p0, p1, row);
  if (d.st == kDeferred) {
    __builtin_nontemporal_store(kDeferred, A.status + m);
    return kDeferred;
  }
  if (A.mtype) __builtin_nontemporal_store(d.type, A.mtype + m);
  // The record columns are written once and read by a later launch: stored
  // nontemporal, so the stream does not evict the group rows (off, ids) that
  // every message gathers at random from the Infinity Cache.
  __builtin_nontemporal_store(d.group, A.rg + m);
  __builtin_nontemporal_store(d.flags, A.rf + m);
  __builtin_nontemporal_store(d.index, A.ri + m);
  __builtin_nontemporal_store(d.term, A.rt + m);
  if (A.rh) __builtin_nontemporal_store(d.hint, A.rh + m);
  if (A.rl) __builtin_nontemporal_store(d.lterm, A.rl + m);
  __builtin_nontemporal_store(u8(d.st), A.status + m);
  return d.st;
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
  const u64 b0 = A.R.moff[m0], b1 = A.R.moff[mlast];
  const u64 p0 = __builtin_nontemporal_load(A.R.moff + mc);
  const u64 p1 = __builtin_nontemporal_load(A.R.moff + mc + 1);
  GroupRow row;
  load_row(A.R, mc, row);
  // Stage the block's byte span [b0, b1) when it fits (block-uniform).
  u64 lbase = 0, lend = 0;  // staged span (empty: nothing staged)
  if (b1 > b0 && b1 - b0 <= kStage - 16) {
    const u64 a0 = b0 & ~u64(15);             // 16-byte aligned window
    const u64 a1 = (b1 + 15) & ~u64(15);
    const u64 n16 = (a1 - a0) / 16;
    // Pieces wholly inside the byte buffer go by LDS-DMA, all issued before
    // the barrier's one wait; only the buffer's last piece can be partial.
    // (A byte buffer that is not 16-byte aligned stages with plain loads.)
    // (offsets past the buffer — a caller error the decode reports as
    // UNMARSHAL — stage nothing from it)
    const u64 whole = a0 < A.nbytes ? (A.nbytes - a0) / 16 : 0;
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
  load_ids(A.R, row);
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
    load_row(A.R, m, row);
    load_ids(A.R, row);
    const int r = ingest_one<GlobalSrc, true>(A, GlobalSrc{A.bytes}, m, A.R.moff[m], A.R.moff[m + 1],
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
  wire::Args A{M, nbytes, bytes,
               wire::RowArgs{G, reinterpret_cast<const u64*>(msg_off), msg_group, off,
                             reinterpret_cast<const u64*>(ids), nullptr},
               rec_group, rec_flags, reinterpret_cast<u64*>(rec_index),
               reinterpret_cast<u64*>(rec_term), reinterpret_cast<u64*>(rec_hint),
               reinterpret_cast<u64*>(rec_log_term), status, msg_type,
               reinterpret_cast<u64*>(stats)};
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
  wire::Args A{M, nbytes, bytes,
               wire::RowArgs{G, reinterpret_cast<const u64*>(msg_off), msg_group, nullptr,
                             reinterpret_cast<const u64*>(ids),
                             G ? reinterpret_cast<const u64*>(rows) : nullptr},
               rec_group, rec_flags, reinterpret_cast<u64*>(rec_index),
               reinterpret_cast<u64*>(rec_term), reinterpret_cast<u64*>(rec_hint),
               reinterpret_cast<u64*>(rec_log_term), status, msg_type,
               reinterpret_cast<u64*>(stats)};
  return wire::launch(A, as_stream(stream));
}
