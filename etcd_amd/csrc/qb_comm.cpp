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
#include <algorithm>
#include <new>
#include <string>
#include <vector>

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
  if (total == 0) return QB_OK;
  hipStream_t st = qb::as_stream(stream);
  const int W = c->world;
  const uint64_t cap = shard_cap(total, W);
  uint64_t b = 0, e = 0;
  shard_range(total, W, c->rank, &b, &e);
  const uint64_t mine = e - b;
  // (a rank whose shard is empty, total < world, may pass NULL shard vectors)
  QB_REQUIRE(!commit_all || commit_shard || mine == 0, "commit_shard NULL");
  QB_REQUIRE(!vote_all || vote_shard || mine == 0, "vote_shard NULL");
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

// ------------------------------------------------------- changed deltas ---
// qb_dev_allgather_changed: the node-wide commit vector kept current by
// exchanging only the groups whose commit moved (at 8 GPUs the
// full all-gather receives 7/8 of G * 9 bytes per GPU every tick).  Each rank
// compacts its shard's changed groups (qb_delta.hip), the counts are
// all-gathered (one host wait: the exchange size is data-dependent), every
// rank pads its pairs to the largest count (gid UINT32_MAX) and one grouped
// pair of ncclAllGathers moves them; the scatter applies every rank's pairs
// (its own included) to commit_all, which the caller keeps across ticks.
extern "C" size_t qb_allgather_changed_workspace_bytes(uint64_t total, int world) {
  if (world < 1) return 0;
  const uint64_t cap = shard_cap(total, world);
  return qb_compact_changed_workspace_bytes(cap) + up256(4 * cap) + up256(8 * cap) + 256 +
         2 * up256(sizeof(uint64_t) * size_t(world)) + up256(4 * cap * uint64_t(world)) +
         up256(8 * cap * uint64_t(world));
}

extern "C" int qb_dev_allgather_changed(qb_comm* c, uint64_t total, const uint8_t* changed_shard,
                                        const uint64_t* commit_shard, uint64_t* commit_all,
                                        uint64_t* changed_total, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  QB_REQUIRE(c && changed_total, "comm / changed_total NULL");
  QB_REQUIRE(commit_all, "commit_all NULL");
  QB_REQUIRE(total <= 0xFFFFFFFFull, "total must fit uint32 (%llu)", (unsigned long long)total);
  const int W = c->world;
  QB_REQUIRE(workspace && workspace_bytes >= qb_allgather_changed_workspace_bytes(total, W),
             "workspace too small (qb_allgather_changed_workspace_bytes)");
  *changed_total = 0;
  hipStream_t st = qb::as_stream(stream);
  uint64_t b = 0, e = 0;
  shard_range(total, W, c->rank, &b, &e);
  const uint64_t n = e - b, cap = shard_cap(total, W);
  // (NULL shard columns are not checked here: qb_dev_compact_changed refuses
  // them and the refusal travels to every rank as a ~0 count below — an early
  // return here would leave the other ranks waiting in the count all-gather)
  char* ws = static_cast<char*>(workspace);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    char* p = ws + o;
    o += up256(bytes);
    return p;
  };
  const size_t cws = qb_compact_changed_workspace_bytes(cap);
  void* cw = take(cws);
  uint32_t* gid = reinterpret_cast<uint32_t*>(take(4 * cap));
  uint64_t* val = reinterpret_cast<uint64_t*>(take(8 * cap));
  uint64_t* count = reinterpret_cast<uint64_t*>(take(256));
  uint64_t* counts = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * size_t(W)));
  (void)take(sizeof(uint64_t) * size_t(W));
  uint32_t* gid_all = reinterpret_cast<uint32_t*>(take(4 * cap * uint64_t(W)));
  uint64_t* val_all = reinterpret_cast<uint64_t*>(take(8 * cap * uint64_t(W)));
  // a local failure travels as count ~0 in the gathered counts, so every rank
  // returns together instead of some waiting in the exchange
  const int rc = qb_dev_compact_changed(n, changed_shard, commit_shard, b, gid, val, count, cw,
                                        cws, stream);
  std::string local_err = rc == QB_OK ? std::string() : std::string(qb_last_error());
  if (rc != QB_OK) {
    const hipError_t me = hipMemsetAsync(count, 0xFF, sizeof(uint64_t), st);
    if (me != hipSuccess) return qb::hip_fail(me, "hipMemsetAsync(count)");
  }
  QB_NCCL(ncclAllGather(count, counts, 1, ncclUint64, c->nccl, st), "ncclAllGather(counts)");
  std::vector<uint64_t> h(static_cast<size_t>(W));
  hipError_t he = hipMemcpyAsync(h.data(), counts, sizeof(uint64_t) * h.size(),
                                 hipMemcpyDeviceToHost, st);
  if (he == hipSuccess) he = hipStreamSynchronize(st);
  if (he != hipSuccess) return qb::hip_fail(he, "changed counts to host");
  if (rc != QB_OK) {
    qb::set_error("%s", local_err.c_str());
    return rc;
  }
  uint64_t mx = 0, sum = 0;
  for (int r = 0; r < W; ++r) {
    const uint64_t x = h[size_t(r)];
    QB_REQUIRE(x != ~0ull, "rank %d failed before the exchange (its qb_last_error has the reason)", r);
    mx = x > mx ? x : mx;
    sum += x;
  }
  *changed_total = sum;
  if (mx == 0) return QB_OK;
  if (12 * mx > 8 * cap) {
    // A skewed tick: the padded pairs (12 B x the largest count) would cost
    // more than gathering every commit (8 B x the shard cap), so the whole
    // vector is gathered instead — same result (commit_shard holds every
    // group's current commit).  Every rank sees the same counts: one choice.
    const bool even = total % uint64_t(W) == 0;
    if (even) {
      QB_NCCL(ncclAllGather(commit_shard, commit_all, cap, ncclUint64, c->nccl, st),
              "ncclAllGather(commit, full)");
      return QB_OK;
    }
    he = hipMemcpyAsync(val, commit_shard, 8 * n, hipMemcpyDeviceToDevice, st);
    if (he != hipSuccess) return qb::hip_fail(he, "hipMemcpyAsync(pad)");
    QB_NCCL(ncclAllGather(val, val_all, cap, ncclUint64, c->nccl, st), "ncclAllGather(commit, full)");
    for (int r = 0; r < W; ++r) {
      uint64_t rb = 0, re = 0;
      shard_range(total, W, r, &rb, &re);
      he = hipMemcpyAsync(commit_all + rb, val_all + uint64_t(r) * cap, 8 * (re - rb),
                          hipMemcpyDeviceToDevice, st);
      if (he != hipSuccess) return qb::hip_fail(he, "hipMemcpyAsync(compact)");
    }
    return QB_OK;
  }
  // this rank's pairs padded to the largest count (gid UINT32_MAX: skipped)
  const uint64_t mine = h[size_t(c->rank)];
  if (mine < mx) {
    he = hipMemsetAsync(gid + mine, 0xFF, 4 * (mx - mine), st);
    if (he != hipSuccess) return qb::hip_fail(he, "hipMemsetAsync(pad)");
  }
  QB_NCCL(ncclGroupStart(), "ncclGroupStart");
  QB_NCCL(ncclAllGather(gid, gid_all, mx, ncclUint32, c->nccl, st), "ncclAllGather(gid)");
  QB_NCCL(ncclAllGather(val, val_all, mx, ncclUint64, c->nccl, st), "ncclAllGather(commit)");
  QB_NCCL(ncclGroupEnd(), "ncclGroupEnd");
  return qb_dev_scatter_changed(mx * uint64_t(W), gid_all, val_all, total, commit_all, stream);
}

// ------------------------------------------------------------- routing ---
// qb_dev_route_records: the stable partition (qb_route.hip), the per-rank
// counts all-gathered (with every rank's output capacity, so all ranks take
// the same decision on an overflow and none is left waiting in a send), then
// one grouped send/recv per column — RCCL point-to-point over xGMI — into the
// caller's columns in source-rank order.  The host waits once, for the
// counts (the receive sizes are data-dependent).
extern "C" size_t qb_route_workspace_bytes(int world, uint64_t M) {
  if (world < 1 || world > QB_ROUTE_MAX_WORLD) return 0;
  // send columns (group 4, flags 1, index/term/hint/log_term 32) + the
  // partition's workspace + send_off and the all-gathered rows
  return up256(4 * M) + up256(M) + 4 * up256(8 * M) + qb_route_partition_workspace_bytes(world, M) +
         up256(sizeof(uint32_t) * (size_t(world) + 1)) +
         2 * up256(sizeof(uint64_t) * size_t(world) * size_t(world + 2));
}

extern "C" int qb_dev_route_records(qb_comm* c, uint64_t total, uint64_t M,
                                    const uint32_t* rec_group, const uint8_t* rec_flags,
                                    const uint64_t* rec_index, const uint64_t* rec_term,
                                    const uint64_t* rec_hint, const uint64_t* rec_log_term,
                                    uint32_t* out_group, uint8_t* out_flags,
                                    uint64_t* out_index, uint64_t* out_term,
                                    uint64_t* out_hint, uint64_t* out_log_term,
                                    uint64_t out_cap, uint64_t* out_count, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  // Only the checks that leave no workspace to gather through return before
  // the collectives; every other local failure (the inputs, the partition,
  // NULL outputs) is carried in this rank's row, so all ranks see it and
  // return together instead of some waiting in a send for a rank that left.
  QB_REQUIRE(c && out_count, "comm / out_count NULL");
  const int W = c->world;
  QB_REQUIRE(W <= QB_ROUTE_MAX_WORLD, "world %d > %d", W, QB_ROUTE_MAX_WORLD);
  QB_REQUIRE(workspace && workspace_bytes >= qb_route_workspace_bytes(W, M),
             "workspace too small (qb_route_workspace_bytes)");
  *out_count = 0;
  hipStream_t st = qb::as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  size_t o = 0;
  auto take = [&](size_t n) {
    char* p = ws + o;
    o += up256(n);
    return p;
  };
  uint32_t* s_group = reinterpret_cast<uint32_t*>(take(4 * M));
  uint8_t* s_flags = reinterpret_cast<uint8_t*>(take(M));
  uint64_t* s_index = reinterpret_cast<uint64_t*>(take(8 * M));
  uint64_t* s_term = reinterpret_cast<uint64_t*>(take(8 * M));
  uint64_t* s_hint = reinterpret_cast<uint64_t*>(take(8 * M));
  uint64_t* s_lt = reinterpret_cast<uint64_t*>(take(8 * M));
  const size_t pws = qb_route_partition_workspace_bytes(W, M);
  void* part_ws = take(pws);
  uint32_t* send_off = reinterpret_cast<uint32_t*>(take(sizeof(uint32_t) * (size_t(W) + 1)));
  const size_t RW = size_t(W) + 2;  // a row: W counts, output capacity, ok flag
  uint64_t* row = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * size_t(W) * RW));
  uint64_t* rows = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * size_t(W) * RW));
  std::string local_err;
  int local_rc = QB_OK;
  if (!rec_hint != !out_hint || !rec_log_term != !out_log_term) {
    local_rc = QB_EINVAL;
    local_err = "hint / log_term: give both the input and the output column, or neither";
  } else {
    local_rc = qb_dev_route_partition(total, W, M, rec_group, rec_flags, rec_index, rec_term,
                                      rec_hint, rec_log_term, s_group, s_flags, s_index, s_term,
                                      rec_hint ? s_hint : nullptr, rec_log_term ? s_lt : nullptr,
                                      send_off, part_ws, pws, stream);
    if (local_rc != QB_OK) local_err = qb_last_error();
  }
  // this rank's row: records for each destination, its output capacity (0
  // when an output column is NULL: it can take no record), and ok
  std::vector<uint32_t> off(size_t(W) + 1, 0);
  hipError_t h = hipSuccess;
  if (local_rc == QB_OK) {
    h = hipMemcpyAsync(off.data(), send_off, sizeof(uint32_t) * off.size(), hipMemcpyDeviceToHost,
                       st);
    if (h == hipSuccess) h = hipStreamSynchronize(st);
    if (h != hipSuccess) {
      local_rc = qb::hip_fail(h, "send counts to host");
      local_err = qb_last_error();
      std::fill(off.begin(), off.end(), 0u);
    }
  }
  const bool outputs = out_group && out_flags && out_index && out_term;
  std::vector<uint64_t> mine(RW), all(size_t(W) * RW);
  for (int r = 0; r < W; ++r) mine[r] = uint64_t(off[r + 1]) - off[r];
  mine[W] = outputs ? out_cap : 0;
  mine[W + 1] = local_rc == QB_OK ? 1 : 0;
  h = hipMemcpyAsync(row, mine.data(), sizeof(uint64_t) * mine.size(), hipMemcpyHostToDevice, st);
  if (h != hipSuccess) return qb::hip_fail(h, "count row to device");
  QB_NCCL(ncclAllGather(row, rows, RW, ncclUint64, c->nccl, st), "ncclAllGather(counts)");
  h = hipMemcpyAsync(all.data(), rows, sizeof(uint64_t) * all.size(), hipMemcpyDeviceToHost, st);
  if (h == hipSuccess) h = hipStreamSynchronize(st);
  if (h != hipSuccess) return qb::hip_fail(h, "count rows to host");
  if (local_rc != QB_OK) {
    qb::set_error("%s", local_err.c_str());
    return local_rc;
  }
  for (int r = 0; r < W; ++r)
    QB_REQUIRE(all[size_t(r) * RW + size_t(W) + 1] == 1,
               "rank %d failed before the exchange (its qb_last_error has the reason)", r);
  // every rank checks every rank's capacity: one decision everywhere
  auto cnt = [&](int src, int dst) { return all[size_t(src) * RW + size_t(dst)]; };
  uint64_t mine_in = 0;
  for (int d = 0; d < W; ++d) {
    uint64_t in = 0;
    for (int s2 = 0; s2 < W; ++s2) in += cnt(s2, d);
    if (d == c->rank) mine_in = in;
    const uint64_t cap = all[size_t(d) * RW + size_t(W)];
    QB_REQUIRE(in <= cap, "rank %d would receive %llu records, over its capacity %llu%s", d,
               (unsigned long long)in, (unsigned long long)cap,
               cap == 0 ? " (or an output column of it is NULL)" : "");
  }
  *out_count = mine_in;
  std::vector<uint64_t> roff(size_t(W) + 1, 0);
  for (int s2 = 0; s2 < W; ++s2) roff[s2 + 1] = roff[s2] + cnt(s2, c->rank);
  struct Col {
    const void* send;
    void* recv;
    size_t width;
  };
  const Col cols[6] = {{s_group, out_group, 4}, {s_flags, out_flags, 1}, {s_index, out_index, 8},
                       {s_term, out_term, 8},   {s_hint, out_hint, 8},   {s_lt, out_log_term, 8}};
  auto skip = [&](int k) { return (k == 4 && !rec_hint) || (k == 5 && !rec_log_term); };
  QB_NCCL(ncclGroupStart(), "ncclGroupStart");
  for (int k = 0; k < 6; ++k) {
    if (skip(k)) continue;
    const char* sb = static_cast<const char*>(cols[k].send);
    char* rb = static_cast<char*>(cols[k].recv);
    for (int p = 0; p < W; ++p) {
      const uint64_t sn = uint64_t(off[p + 1]) - off[p], rn = cnt(p, c->rank);
      if (p == c->rank) continue;  // the local run is copied below
      if (sn) QB_NCCL(ncclSend(sb + cols[k].width * off[p], cols[k].width * sn, ncclUint8, p, c->nccl, st), "ncclSend");
      if (rn) QB_NCCL(ncclRecv(rb + cols[k].width * roff[p], cols[k].width * rn, ncclUint8, p, c->nccl, st), "ncclRecv");
    }
  }
  QB_NCCL(ncclGroupEnd(), "ncclGroupEnd");
  const uint64_t self = cnt(c->rank, c->rank);
  if (self) {
    for (int k = 0; k < 6; ++k) {
      if (skip(k)) continue;
      h = hipMemcpyAsync(static_cast<char*>(cols[k].recv) + cols[k].width * roff[c->rank],
                         static_cast<const char*>(cols[k].send) + cols[k].width * off[c->rank],
                         cols[k].width * self, hipMemcpyDeviceToDevice, st);
      if (h != hipSuccess) return qb::hip_fail(h, "hipMemcpyAsync(local run)");
    }
  }
  return QB_OK;
}
