// fake_rccl.cpp — TEST-ONLY stand-in for the RCCL entry points that
// etcd_amd/csrc/qb_comm.cpp calls, so its world > 1 code (uneven-shard
// padding and compaction, the count exchange and padded delta gathers, the
// routing's send/recv offsets, the collective failure paths) runs with N
// ranks on ONE device: every rank is a host thread of one process with its
// own HIP stream.  RCCL itself refuses two ranks on one GPU, and the box has
// one GPU, so without this the C ABI's multi-rank code would first execute on
// the driver's 8-GPU node.  Linked only into tests/fake_rccl/libqb_fakecomm.so
// (the product's objects + this file instead of -lrccl); the product library
// is untouched.
//
// Semantics kept from RCCL (rccl.h): ncclCommInitRank is collective (every
// rank joins before any returns); ncclAllGather places rank r's sendcount
// elements at recvbuff + r * sendcount on every rank; ncclSend / ncclRecv
// pair in issue order per (sender, receiver) with equal byte counts; calls
// between ncclGroupStart / ncclGroupEnd form one group; the data movement is
// enqueued on each rank's stream after the work already on it and completes
// before the work enqueued after it on every rank (events between the
// streams), so a sender cannot overwrite its buffer while a peer still reads
// it.  Unlike RCCL, the host of each rank blocks at a group holding an
// all-gather until every rank has reached it (a mismatch between the ranks'
// all-gathers returns ncclInvalidUsage on every rank), and at a
// point-to-point group until its peers have posted the matching calls (60 s,
// then ncclInvalidUsage instead of a hang).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <chrono>
#include <tuple>
#include <vector>

namespace {

enum Kind { kAllGather, kSend, kRecv };

struct Op {
  Kind kind;
  const void* send;
  void* recv;
  size_t bytes;
  int peer;
  hipStream_t stream;
};

struct Post {
  std::vector<Op> ops;
  hipEvent_t ready = nullptr, done = nullptr;
  hipStream_t stream = nullptr;
};

// A posted send (point-to-point): the sender's buffer and the event after
// which it holds the data; the receiver publishes `done` once its copy is
// enqueued, and the sender's later work waits for it.
struct Mail {
  const void* send = nullptr;
  size_t bytes = 0;
  hipEvent_t ready = nullptr;
  hipEvent_t done = nullptr;
  bool has_done = false;
  bool failed = false;
};

struct World {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0, joined = 0;
  unsigned long long generation = 0;
  std::vector<Post> posts;
  // point-to-point: mailbox[(s, d, seq)], seq = the k-th send s -> d overall
  std::map<std::tuple<int, int, uint64_t>, Mail> mail;
  std::map<std::pair<int, int>, uint64_t> sent, received;
  // point-to-point events live as long as the world (a peer may still
  // enqueue a wait on one after its owner's rank has returned): destroyed
  // with the last communicator
  std::vector<hipEvent_t> events;
  ~World() {
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
  }

  // every rank calls; returns after all n have arrived (a reusable barrier)
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const unsigned long long gen = generation;
    if (++arrived == n) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return;
    }
    cv.wait(lk, [&] { return generation != gen; });
  }
};

std::mutex g_mu;
std::map<uint64_t, std::shared_ptr<World>> g_worlds;

size_t dtype_bytes(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;
thread_local ncclComm_t t_comm = nullptr;
constexpr auto kP2pTimeout = std::chrono::seconds(60);

}  // namespace

struct ncclComm {
  std::shared_ptr<World> w;
  int rank;
};

namespace {

// One group of this rank's ops, collectively with every other rank's.
ncclResult_t run_group(ncclComm_t c, std::vector<Op> ops) {
  World& w = *c->w;
  const int me = c->rank;
  hipStream_t st = ops.empty() ? nullptr : ops[0].stream;
  for (const Op& o : ops)
    if (o.stream != st) return ncclInvalidUsage;  // one stream per group (qb_comm's use)
  Post& mine = w.posts[size_t(me)];
  mine.ops = std::move(ops);
  mine.stream = st;
  if (hipEventCreateWithFlags(&mine.ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&mine.done, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(mine.ready, st) != hipSuccess)
    return ncclUnhandledCudaError;
  w.barrier();  // every rank has posted
  // validate the whole group on every rank (each sees the same posts)
  bool ok = true;
  std::vector<size_t> nag(size_t(w.n), 0);
  for (int r = 0; r < w.n; ++r)
    for (const Op& o : w.posts[size_t(r)].ops) nag[size_t(r)] += o.kind == kAllGather;
  for (int r = 0; r < w.n; ++r) ok &= nag[size_t(r)] == nag[0];
  if (ok) {
    for (size_t i = 0; i < nag[0]; ++i) {
      size_t b0 = SIZE_MAX;
      for (int r = 0; r < w.n; ++r) {
        size_t k = 0;
        for (const Op& o : w.posts[size_t(r)].ops)
          if (o.kind == kAllGather && k++ == i) {
            if (b0 == SIZE_MAX) b0 = o.bytes;
            ok &= o.bytes == b0;
          }
      }
    }
  }
  // point-to-point pairing: the k-th send s->d with the k-th recv at d from s
  auto pairs = [&](int s, int d, Kind kind) {
    std::vector<const Op*> v;
    for (const Op& o : w.posts[size_t(kind == kSend ? s : d)].ops)
      if (o.kind == kind && o.peer == (kind == kSend ? d : s)) v.push_back(&o);
    return v;
  };
  for (int s = 0; ok && s < w.n; ++s)
    for (int d = 0; ok && d < w.n; ++d) {
      auto sv = pairs(s, d, kSend), rv = pairs(s, d, kRecv);
      ok &= sv.size() == rv.size();
      for (size_t k = 0; ok && k < sv.size(); ++k) ok &= sv[k]->bytes == rv[k]->bytes;
    }
  ncclResult_t rc = ncclSuccess;
  if (!ok) {
    rc = ncclInvalidUsage;
  } else if (st) {
    // this rank's receiving side: wait for every sender's prior work, copy
    for (int p = 0; p < w.n && rc == ncclSuccess; ++p)
      if (hipStreamWaitEvent(st, w.posts[size_t(p)].ready, 0) != hipSuccess)
        rc = ncclUnhandledCudaError;
    size_t ag = 0;
    for (const Op& o : mine.ops) {
      if (rc != ncclSuccess) break;
      if (o.kind == kAllGather) {
        for (int p = 0; p < w.n && rc == ncclSuccess; ++p) {
          size_t k = 0;
          for (const Op& q : w.posts[size_t(p)].ops)
            if (q.kind == kAllGather && k++ == ag) {
              if (q.bytes && hipMemcpyAsync(static_cast<char*>(o.recv) + size_t(p) * q.bytes,
                                            q.send, q.bytes, hipMemcpyDeviceToDevice,
                                            st) != hipSuccess)
                rc = ncclUnhandledCudaError;
            }
        }
        ++ag;
      }
    }
    for (int s = 0; s < w.n && rc == ncclSuccess; ++s) {
      auto sv = pairs(s, me, kSend), rv = pairs(s, me, kRecv);
      for (size_t k = 0; k < sv.size() && rc == ncclSuccess; ++k)
        if (sv[k]->bytes && hipMemcpyAsync(rv[k]->recv, sv[k]->send, sv[k]->bytes,
                                           hipMemcpyDeviceToDevice, st) != hipSuccess)
          rc = ncclUnhandledCudaError;
    }
    if (hipEventRecord(mine.done, st) != hipSuccess) rc = ncclUnhandledCudaError;
  }
  w.barrier();  // every rank has enqueued its copies
  if (rc == ncclSuccess && st)
    for (int p = 0; p < w.n; ++p)  // no rank's later work overtakes a peer's reads
      if (w.posts[size_t(p)].stream &&
          hipStreamWaitEvent(st, w.posts[size_t(p)].done, 0) != hipSuccess)
        rc = ncclUnhandledCudaError;
  w.barrier();  // every rank's waits are enqueued: the events may go
  (void)hipEventDestroy(mine.ready);
  (void)hipEventDestroy(mine.done);
  mine.ready = mine.done = nullptr;
  mine.ops.clear();
  w.barrier();
  return rc;
}

// A group of point-to-point ops only: RCCL does not synchronise ranks that
// exchange nothing, so neither does this (a rank with an empty group returns
// at once).  (1) post every send with a ready event (never blocks); (2) for
// every recv, wait for its matching send, enqueue a wait on the sender's
// ready event and the copy; (3) publish a done event for each; (4) for every
// send, wait for the receiver's done event and enqueue a wait on it.
ncclResult_t run_p2p(ncclComm_t c, const std::vector<Op>& ops) {
  World& w = *c->w;
  const int me = c->rank;
  hipStream_t st = ops[0].stream;
  for (const Op& o : ops)
    if (o.stream != st) return ncclInvalidUsage;
  hipEvent_t ready = nullptr, done = nullptr;
  if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess)
    return ncclUnhandledCudaError;
  {
    std::lock_guard<std::mutex> lk(w.mu);
    w.events.push_back(ready);
    w.events.push_back(done);
  }
  if (hipEventRecord(ready, st) != hipSuccess) return ncclUnhandledCudaError;
  std::vector<std::tuple<int, int, uint64_t>> my_sends, my_recvs;
  {
    std::lock_guard<std::mutex> lk(w.mu);
    for (const Op& o : ops) {
      if (o.kind == kSend) {
        auto key = std::make_tuple(me, o.peer, w.sent[{me, o.peer}]++);
        Mail& m = w.mail[key];
        m.send = o.send;
        m.bytes = o.bytes;
        m.ready = ready;
        my_sends.push_back(key);
      } else {
        my_recvs.push_back(std::make_tuple(o.peer, me, w.received[{o.peer, me}]++));
      }
    }
    w.cv.notify_all();
  }
  ncclResult_t rc = ncclSuccess;
  size_t ri = 0;
  for (const Op& o : ops) {
    if (o.kind != kRecv) continue;
    const auto key = my_recvs[ri++];
    std::unique_lock<std::mutex> lk(w.mu);
    if (!w.cv.wait_for(lk, kP2pTimeout, [&] { return w.mail.count(key) && w.mail[key].ready; })) {
      rc = ncclInvalidUsage;  // no matching send: a mismatched program
      break;
    }
    Mail& m = w.mail[key];
    lk.unlock();
    if (m.bytes != o.bytes) {
      rc = ncclInvalidUsage;
    } else if (hipStreamWaitEvent(st, m.ready, 0) != hipSuccess ||
               (o.bytes && hipMemcpyAsync(o.recv, m.send, o.bytes, hipMemcpyDeviceToDevice, st) !=
                               hipSuccess)) {
      rc = ncclUnhandledCudaError;
    }
    if (rc != ncclSuccess) {
      std::lock_guard<std::mutex> g(w.mu);
      m.failed = m.has_done = true;
      w.cv.notify_all();
      break;
    }
  }
  if (rc == ncclSuccess && hipEventRecord(done, st) != hipSuccess) rc = ncclUnhandledCudaError;
  {
    std::lock_guard<std::mutex> lk(w.mu);
    for (size_t k = 0; k < ri; ++k) {
      Mail& m = w.mail[my_recvs[k]];
      if (!m.has_done) {
        m.done = done;
        m.has_done = true;
        m.failed = rc != ncclSuccess;
      }
    }
    w.cv.notify_all();
  }
  for (const auto& key : my_sends) {
    std::unique_lock<std::mutex> lk(w.mu);
    if (!w.cv.wait_for(lk, kP2pTimeout, [&] { return w.mail[key].has_done; }))
      return ncclInvalidUsage;  // no matching recv
    Mail m = w.mail[key];
    w.mail.erase(key);
    lk.unlock();
    if (m.failed) rc = rc == ncclSuccess ? ncclInvalidUsage : rc;
    else if (hipStreamWaitEvent(st, m.done, 0) != hipSuccess) rc = ncclUnhandledCudaError;
  }
  return rc;
}

ncclResult_t enqueue(ncclComm_t c, Op o) {
  if (!c) return ncclInvalidArgument;
  if (t_depth == 0) return o.kind == kAllGather ? run_group(c, {o}) : run_p2p(c, {o});
  if (t_comm && t_comm != c) return ncclInvalidUsage;  // one communicator per group here
  t_comm = c;
  t_ops.push_back(o);
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::memset(id, 0, sizeof *id);
  static std::mt19937_64 rng{std::random_device{}()};
  std::lock_guard<std::mutex> lk(g_mu);
  const uint64_t key = rng() | 1u;
  std::memcpy(id->internal, &key, sizeof key);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  uint64_t key;
  std::memcpy(&key, id.internal, sizeof key);
  std::shared_ptr<World> w;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto& slot = g_worlds[key];
    if (!slot) {
      slot = std::make_shared<World>();
      slot->n = nranks;
      slot->posts.resize(size_t(nranks));
    }
    w = slot;
    if (w->n != nranks) return ncclInvalidUsage;
  }
  w->barrier();  // collective: every rank has joined
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_worlds.count(key) && g_worlds[key] == w && ++w->joined == w->n) g_worlds.erase(key);
  }
  *comm = new ncclComm{w, rank};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;  // the world (and its events) goes with the last communicator
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (fake_rccl)";
    case ncclInvalidArgument: return "invalid argument (fake_rccl)";
    case ncclInvalidUsage: return "invalid usage: the ranks' groups do not match (fake_rccl)";
    case ncclUnhandledCudaError: return "HIP call failed (fake_rccl)";
    default: return "error (fake_rccl)";
  }
}

ncclResult_t ncclGroupStart() {
  ++t_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_depth == 0) return ncclInvalidUsage;
  if (--t_depth) return ncclSuccess;
  ncclComm_t c = t_comm;
  std::vector<Op> ops;
  ops.swap(t_ops);
  t_comm = nullptr;
  if (!c || ops.empty()) return ncclSuccess;  // an empty group
  bool collective = false;
  for (const Op& o : ops) collective |= o.kind == kAllGather;
  if (!collective) return run_p2p(c, ops);
  for (const Op& o : ops)
    if (o.kind != kAllGather) return ncclInvalidUsage;  // qb_comm never mixes them
  return run_group(c, std::move(ops));
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount,
                           ncclDataType_t datatype, ncclComm_t comm, hipStream_t stream) {
  const size_t b = dtype_bytes(datatype);
  if (!b) return ncclInvalidArgument;
  return enqueue(comm, Op{kAllGather, sendbuff, recvbuff, sendcount * b, -1, stream});
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t comm, hipStream_t stream) {
  const size_t b = dtype_bytes(datatype);
  if (!b || !comm || peer < 0 || peer >= comm->w->n) return ncclInvalidArgument;
  return enqueue(comm, Op{kSend, sendbuff, nullptr, count * b, peer, stream});
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t comm, hipStream_t stream) {
  const size_t b = dtype_bytes(datatype);
  if (!b || !comm || peer < 0 || peer >= comm->w->n) return ncclInvalidArgument;
  return enqueue(comm, Op{kRecv, nullptr, recvbuff, count * b, peer, stream});
}

}  // extern "C"
