// qb_comm.cpp — the node-wide result exchange of the sharded engine
// (SURVEY.md §8e): one process per GPU, groups sharded by contiguous ranges of
// global group numbers, and ONE collective at the edge of the path — an RCCL
// all-gather over xGMI of the per-shard CommittedIndex (u64) and VoteResult
// (u8) vectors into the node-wide vectors.  Nothing inside the hot path
// exchanges data (groups are independent).
//
// The reference has no counterpart (stock etcd runs one raft group per
// process, server/etcdserver/raft.go:104); this is the C-ABI twin of
// etcd_amd/shard.py:allgather_results for a cgo embedder, which distributes
// the 128-byte unique ID over its own transport (rafthttp, peer.go:178).
#include <rccl/rccl.h>

#include <cstring>
#include <new>

#include "qb_common.h"

struct qb_comm {
  ncclComm_t nccl;
  int world, rank;
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
  qb::set_error("%s: %s (%d)", what, ncclGetErrorString(r), int(r));
  return QB_EHIP;
}

#define QB_NCCL(call, what)                          \
  do {                                               \
    const ncclResult_t r_ = (call);                  \
    if (r_ != ncclSuccess) return nccl_fail(r_, what); \
  } while (0)

// shard_range of etcd_amd/shard.py: contiguous, sizes differ by at most one.
void shard_range(uint64_t total, int world, int rank, uint64_t* b, uint64_t* e) {
  const uint64_t base = total / uint64_t(world), extra = total % uint64_t(world);
  const uint64_t r = uint64_t(rank);
  *b = r * base + (r < extra ? r : extra);
  *e = *b + base + (r < extra ? 1 : 0);
}

uint64_t shard_cap(uint64_t total, int world) {
  return (total + uint64_t(world) - 1) / uint64_t(world);
}

size_t up256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

extern "C" int qb_shard_range(uint64_t total, int world, int rank, uint64_t* begin,
                              uint64_t* end) {
  QB_REQUIRE(begin && end, "begin/end NULL");
  QB_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad world/rank (%d, %d)", world, rank);
  shard_range(total, world, rank, begin, end);
  return QB_OK;
}

extern "C" int qb_comm_get_unique_id(void* id_out) {
  QB_REQUIRE(id_out, "id_out is NULL");
  ncclUniqueId id;
  QB_NCCL(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(id_out, &id, sizeof id);
  return QB_OK;
}

extern "C" int qb_comm_init(qb_comm** out, int world, int rank, const void* id) {
  QB_REQUIRE(out && id, "out/id NULL");
  QB_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad world/rank (%d, %d)", world, rank);
  *out = nullptr;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  qb_comm* c = new (std::nothrow) qb_comm{};
  QB_REQUIRE(c, "out of host memory");
  const ncclResult_t r = ncclCommInitRank(&c->nccl, world, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  c->world = world;
  c->rank = rank;
  *out = c;
  return QB_OK;
}

extern "C" int qb_comm_destroy(qb_comm* c) {
  if (!c) return QB_OK;
  const ncclResult_t r = ncclCommDestroy(c->nccl);
  delete c;
  return r == ncclSuccess ? QB_OK : nccl_fail(r, "ncclCommDestroy");
}

extern "C" size_t qb_allgather_workspace_bytes(uint64_t total, int world) {
  if (world < 1) return 0;
  const uint64_t cap = shard_cap(total, world);
  // padded send (cap) + receive (world * cap) for both vectors
  return up256(9 * cap) + up256(9 * cap * uint64_t(world)) + 256;
}

extern "C" int qb_dev_allgather_results(qb_comm* c, uint64_t total,
                                        const uint64_t* commit_shard, const uint8_t* vote_shard,
                                        uint64_t* commit_all, uint8_t* vote_all,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  QB_REQUIRE(c, "comm is NULL");
  QB_REQUIRE(commit_all || vote_all, "nothing to gather");
  QB_REQUIRE(!commit_all || commit_shard, "commit_shard NULL");
  QB_REQUIRE(!vote_all || vote_shard, "vote_shard NULL");
  if (total == 0) return QB_OK;
  hipStream_t st = qb::as_stream(stream);
  const int W = c->world;
  const uint64_t cap = shard_cap(total, W);
  uint64_t b = 0, e = 0;
  shard_range(total, W, c->rank, &b, &e);
  const uint64_t mine = e - b;
  const bool even = total % uint64_t(W) == 0;
  // Even shards gather straight into the caller's vectors; otherwise the
  // padded shards go through the workspace and are compacted by rank.
  char* ws = static_cast<char*>(workspace);
  uint64_t* send_c = nullptr;
  uint8_t* send_v = nullptr;
  uint64_t* recv_c = commit_all;
  uint8_t* recv_v = vote_all;
  if (!even) {
    QB_REQUIRE(ws && workspace_bytes >= qb_allgather_workspace_bytes(total, W),
               "workspace too small (qb_allgather_workspace_bytes)");
    send_c = reinterpret_cast<uint64_t*>(ws);
    send_v = reinterpret_cast<uint8_t*>(ws + 8 * cap);
    recv_c = reinterpret_cast<uint64_t*>(ws + up256(9 * cap));
    recv_v = reinterpret_cast<uint8_t*>(ws + up256(9 * cap) + 8 * cap * uint64_t(W));
    hipError_t h = hipSuccess;
    if (commit_all) h = hipMemcpyAsync(send_c, commit_shard, 8 * mine, hipMemcpyDeviceToDevice, st);
    if (h == hipSuccess && vote_all)
      h = hipMemcpyAsync(send_v, vote_shard, mine, hipMemcpyDeviceToDevice, st);
    if (h != hipSuccess) return qb::hip_fail(h, "hipMemcpyAsync(pad)");
  }
  QB_NCCL(ncclGroupStart(), "ncclGroupStart");
  if (commit_all)
    QB_NCCL(ncclAllGather(even ? static_cast<const void*>(commit_shard) : send_c, recv_c, cap,
                          ncclUint64, c->nccl, st),
            "ncclAllGather(commit)");
  if (vote_all)
    QB_NCCL(ncclAllGather(even ? static_cast<const void*>(vote_shard) : send_v, recv_v, cap,
                          ncclUint8, c->nccl, st),
            "ncclAllGather(vote)");
  QB_NCCL(ncclGroupEnd(), "ncclGroupEnd");
  if (!even) {
    for (int r = 0; r < W; ++r) {
      uint64_t rb = 0, re = 0;
      shard_range(total, W, r, &rb, &re);
      hipError_t h = hipSuccess;
      if (commit_all)
        h = hipMemcpyAsync(commit_all + rb, recv_c + uint64_t(r) * cap, 8 * (re - rb),
                           hipMemcpyDeviceToDevice, st);
      if (h == hipSuccess && vote_all)
        h = hipMemcpyAsync(vote_all + rb, recv_v + uint64_t(r) * cap, re - rb,
                           hipMemcpyDeviceToDevice, st);
      if (h != hipSuccess) return qb::hip_fail(h, "hipMemcpyAsync(compact)");
    }
  }
  return QB_OK;
}
