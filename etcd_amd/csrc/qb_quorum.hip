// qb_quorum.hip — CommittedIndex / VoteResult kernels for gfx950.
//
// Reference semantics (paths relative to the reference's raft/):
//   MajorityConfig.CommittedIndex  quorum/majority.go:126-172
//   MajorityConfig.VoteResult      quorum/majority.go:178-210
//   JointConfig.CommittedIndex     quorum/joint.go:49-56
//   JointConfig.VoteResult         quorum/joint.go:61-75
//
// Both kernels are HBM-streaming integer work (no MFMA: nothing here is a
// contraction).  One thread owns one group (FIXED: GPT groups), the
// order statistic is a compare-exchange network held in VGPRs, and the vote is
// three popcounts.  Design notes and rooflines: DESIGN.md §3.
#include <type_traits>

#include "qb_common.h"
#include "qb_csr.h"

namespace qb {

template <int N>
using MaskT = std::conditional_t<(N <= 8), u8, u16>;

// Load CNT consecutive elements as one vector access (CNT*sizeof(E) bytes,
// naturally aligned by the caller's choice of GPT).
template <int BYTES>
struct Raw;
template <> struct Raw<1> { using T = u8; };
template <> struct Raw<2> { using T = u16; };
template <> struct Raw<4> { using T = u32; };
template <> struct Raw<8> { using T = u64; };
template <> struct Raw<16> { using T = u32 __attribute__((ext_vector_type(4))); };

// Streamed once per launch, so loads and stores are nontemporal (nt bit:
// the lines are not kept in the caches for reuse; measured +11% at the
// BASELINE 1M-group config).
template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) { return __builtin_nontemporal_load(p); }
template <typename T>
__device__ __forceinline__ void st_nt(T* p, T v) { __builtin_nontemporal_store(v, p); }

template <typename E, int CNT>
__device__ __forceinline__ void vload(const E* __restrict__ p, E (&out)[CNT]) {
  constexpr int B = int(sizeof(E)) * CNT;
  if constexpr (B <= 16) {
    using T = typename Raw<B>::T;
    const T x = ld_nt(reinterpret_cast<const T*>(p));
    __builtin_memcpy(out, &x, B);
  } else {
    static_assert(B % 16 == 0, "chunk");
    using T = typename Raw<16>::T;
#pragma unroll
    for (int i = 0; i < B / 16; ++i) {
      const T x = ld_nt(reinterpret_cast<const T*>(p) + i);
      __builtin_memcpy(reinterpret_cast<char*>(out) + 16 * i, &x, 16);
    }
  }
}

template <typename E, int CNT>
__device__ __forceinline__ void vstore(E* __restrict__ p, const E (&in)[CNT]) {
  constexpr int B = int(sizeof(E)) * CNT;
  if constexpr (B <= 16) {
    using T = typename Raw<B>::T;
    T x;
    __builtin_memcpy(&x, in, B);
    st_nt(reinterpret_cast<T*>(p), x);
  } else {
    static_assert(B % 16 == 0, "chunk");
    using T = typename Raw<16>::T;
#pragma unroll
    for (int i = 0; i < B / 16; ++i) {
      T x;
      __builtin_memcpy(&x, reinterpret_cast<const char*>(in) + 16 * i, 16);
      st_nt(reinterpret_cast<T*>(p) + i, x);
    }
  }
}

// ------------------------------------------------------------------ FIXED ---

template <int N, bool CI, bool VOTE>
__device__ __forceinline__ void eval_fixed(u64 (&v)[N], u32 vd, u32 gr, u64& ci, u8& vr) {
  if constexpr (CI) ci = select_quorum<N>(v);
  if constexpr (VOTE) {
    constexpr u32 full = (N == 32) ? ~0u : ((1u << N) - 1u);
    // majority.go:186-200: only config members count; granted needs voted.
    vr = vote_from_counts(N, __popc(vd & gr & full), __popc(vd & full));
  }
}

// GPT consecutive groups per thread: every slot row is read as one
// GPT*8-byte vector access, masks and outputs likewise.
template <int N, int GPT, bool CI, bool VOTE>
__global__ __launch_bounds__(kBlock) void k_fixed(const u64* __restrict__ match, u64 G,
                                                  const MaskT<N>* __restrict__ voted,
                                                  const MaskT<N>* __restrict__ granted,
                                                  u64* __restrict__ commit,
                                                  u8* __restrict__ vote) {
  using M = MaskT<N>;
  const u64 g0 = (u64(blockIdx.x) * kBlock + threadIdx.x) * GPT;
  if (g0 >= G) return;
  if (g0 + GPT <= G) {
    u64 row[N][GPT];
    if constexpr (CI) {
#pragma unroll
      for (int s = 0; s < N; ++s) vload<u64, GPT>(match + u64(s) * G + g0, row[s]);
    }
    M vd[GPT], gr[GPT];
    if constexpr (VOTE) {
      vload<M, GPT>(voted + g0, vd);
      vload<M, GPT>(granted + g0, gr);
    }
    u64 ci[GPT];
    u8 vr[GPT];
#pragma unroll
    for (int k = 0; k < GPT; ++k) {
      u64 v[N];
#pragma unroll
      for (int s = 0; s < N; ++s) v[s] = CI ? row[s][k] : 0;
      eval_fixed<N, CI, VOTE>(v, VOTE ? u32(vd[k]) : 0u, VOTE ? u32(gr[k]) : 0u, ci[k], vr[k]);
    }
    if constexpr (CI) vstore<u64, GPT>(commit + g0, ci);
    if constexpr (VOTE) vstore<u8, GPT>(vote + g0, vr);
  } else {
    for (u64 g = g0; g < G; ++g) {
      u64 v[N];
#pragma unroll
      for (int s = 0; s < N; ++s) v[s] = CI ? match[u64(s) * G + g] : 0;
      u64 ci;
      u8 vr;
      eval_fixed<N, CI, VOTE>(v, VOTE ? u32(voted[g]) : 0u, VOTE ? u32(granted[g]) : 0u, ci, vr);
      if constexpr (CI) commit[g] = ci;
      if constexpr (VOTE) vote[g] = vr;
    }
  }
}

// LDS-DMA form (CommittedIndex wanted, n <= 8, aligned operands): a
// workgroup owns kBlock * GPT consecutive groups; each slot row's slice for
// them (kBlock * GPT * 8 contiguous bytes) lands in LDS by
// global_load_lds_dwordx4, all N rows issued before the one wait, and a lane
// reads back the groups its own 16-byte pieces landed (piece k of lane t =
// groups 2 (k kBlock + t) and +1).  Longer contiguous row slices than the
// register form's one dwordx4 per row and lane, and no VGPRs held by the
// loads: 1M groups 8.7-8.9 -> 8.5 us, 16M 146 -> 141 us
// (`profiles/r02/ab_fixed_ldsdma.log`).
template <int N, int GPT, bool VOTE>
__global__ __launch_bounds__(kBlock) void k_fixed_lds(const u64* __restrict__ match, u64 G,
                                                      const MaskT<N>* __restrict__ voted,
                                                      const MaskT<N>* __restrict__ granted,
                                                      u64* __restrict__ commit,
                                                      u8* __restrict__ vote) {
  using M = MaskT<N>;
  constexpr int kPer = GPT / 2;  // 16-byte pieces per lane and row
  constexpr u32 kSpan = u32(kBlock) * GPT;
  __shared__ __attribute__((aligned(16))) u64 lds[N][kSpan];
  const u64 gb = u64(blockIdx.x) * kSpan;
  if (gb + kSpan > G) {  // the tail workgroup (block-uniform): group by group
    const u64 g0 = gb + u64(threadIdx.x) * GPT;
    for (u64 g = g0; g < G && g < g0 + GPT; ++g) {
      u64 v[N];
#pragma unroll
      for (int s = 0; s < N; ++s) v[s] = match[u64(s) * G + g];
      u64 ci;
      u8 vr;
      eval_fixed<N, true, VOTE>(v, VOTE ? u32(voted[g]) : 0u, VOTE ? u32(granted[g]) : 0u, ci, vr);
      commit[g] = ci;
      if constexpr (VOTE) vote[g] = vr;
    }
    return;
  }
  M vd[GPT], gr[GPT];
  if constexpr (VOTE) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const u64 ge = gb + 2ull * (u32(k) * kBlock + threadIdx.x);
      M a[2], b[2];
      vload<M, 2>(voted + ge, a);
      vload<M, 2>(granted + ge, b);
      vd[2 * k] = a[0];
      vd[2 * k + 1] = a[1];
      gr[2 * k] = b[0];
      gr[2 * k + 1] = b[1];
    }
  }
  const u32 wave_base = threadIdx.x & ~63u;
#pragma unroll
  for (int s = 0; s < N; ++s)
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const u32 piece = u32(k) * kBlock + threadIdx.x;
      char* dst = reinterpret_cast<char*>(&lds[s][0]) + 16u * (u32(k) * kBlock + wave_base);
      __builtin_amdgcn_global_load_lds(
          (gbl_cvoid_t*)(reinterpret_cast<const char*>(match + u64(s) * G + gb) + 16ull * piece),
          (lds_void_t*)dst, 16, 0, 2);
    }
  __syncthreads();
  u64 ci[GPT];
  u8 vr[GPT];
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    const u32 e = 2u * (u32(j / 2) * kBlock + threadIdx.x) + u32(j & 1);
    u64 v[N];
#pragma unroll
    for (int s = 0; s < N; ++s) v[s] = lds[s][e];
    eval_fixed<N, true, VOTE>(v, VOTE ? u32(vd[j]) : 0u, VOTE ? u32(gr[j]) : 0u, ci[j], vr[j]);
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const u64 ge = gb + 2ull * (u32(k) * kBlock + threadIdx.x);
    const u64 c2[2] = {ci[2 * k], ci[2 * k + 1]};
    vstore<u64, 2>(commit + ge, c2);
    if constexpr (VOTE) {
      const u8 v2[2] = {vr[2 * k], vr[2 * k + 1]};
      vstore<u8, 2>(vote + ge, v2);
    }
  }
}

// Empty config (n == 0): CommittedIndex = ∞, VoteResult = VoteWon
// (majority.go:128-133, 179-184).
__global__ void k_fill_empty(u64 G, u64* __restrict__ commit, u8* __restrict__ vote) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  if (commit) commit[g] = kInf;
  if (vote) vote[g] = QB_VOTE_WON;
}

template <int N, int GPT, bool CI, bool VOTE>
static void launch_fixed_t(u64 G, const u64* match, const void* voted, const void* granted,
                           u64* commit, u8* vote, hipStream_t st) {
  const u64 threads = (G + GPT - 1) / GPT;
  hipLaunchKernelGGL((k_fixed<N, GPT, CI, VOTE>), dim3(grid_for(threads)), dim3(kBlock), 0, st,
                     match, G, static_cast<const MaskT<N>*>(voted),
                     static_cast<const MaskT<N>*>(granted), commit, vote);
}

template <int N>
static void launch_fixed_n(u64 G, const u64* match, const void* voted, const void* granted,
                           u64* commit, u8* vote, bool vec, hipStream_t st) {
  const bool ci = commit != nullptr, vt = vote != nullptr;
  if constexpr (N <= 8) {
    if (vec && ci) {
      constexpr int GPT = N <= 5 ? 4 : 2;
      const dim3 grid(unsigned((G + u64(kBlock) * GPT - 1) / (u64(kBlock) * GPT)));
      const auto* vd = static_cast<const MaskT<N>*>(voted);
      const auto* gr = static_cast<const MaskT<N>*>(granted);
      if (vt)
        hipLaunchKernelGGL((k_fixed_lds<N, GPT, true>), grid, dim3(kBlock), 0, st, match, G, vd, gr,
                           commit, vote);
      else
        hipLaunchKernelGGL((k_fixed_lds<N, GPT, false>), grid, dim3(kBlock), 0, st, match, G, vd,
                           gr, commit, vote);
      return;
    }
  }
  // GPT = 2: one dwordx4 per slot row, 2-4 byte mask/vote chunks.  Measured
  // best of {1,2,4,8} x {plain,nt} for n = 5.
  if (vec) {
    if (ci && vt) launch_fixed_t<N, 2, true, true>(G, match, voted, granted, commit, vote, st);
    else if (ci) launch_fixed_t<N, 2, true, false>(G, match, voted, granted, commit, vote, st);
    else launch_fixed_t<N, 2, false, true>(G, match, voted, granted, commit, vote, st);
  } else {
    if (ci && vt) launch_fixed_t<N, 1, true, true>(G, match, voted, granted, commit, vote, st);
    else if (ci) launch_fixed_t<N, 1, true, false>(G, match, voted, granted, commit, vote, st);
    else launch_fixed_t<N, 1, false, true>(G, match, voted, granted, commit, vote, st);
  }
}

template <int... Ns>
static void dispatch_fixed(std::integer_sequence<int, Ns...>, int n, u64 G, const u64* match,
                           const void* voted, const void* granted, u64* commit, u8* vote,
                           bool vec, hipStream_t st) {
  ((n == Ns + 1 ? launch_fixed_n<Ns + 1>(G, match, voted, granted, commit, vote, vec, st)
                : void()),
   ...);
}

static bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

}  // namespace qb

using namespace qb;

extern "C" int qb_dev_fixed_committed_vote(uint32_t n, uint64_t G, const uint64_t* match,
                                           const void* voted, const void* granted,
                                           uint64_t* commit_out, uint8_t* vote_out,
                                           void* stream) {
  QB_REQUIRE(n <= QB_MAX_SLOTS, "fixed layout supports 0..%d voters, got %u", QB_MAX_SLOTS, n);
  if (G == 0 || (!commit_out && !vote_out)) return QB_OK;
  hipStream_t st = as_stream(stream);
  u64* commit = reinterpret_cast<u64*>(commit_out);
  if (n == 0) {
    hipLaunchKernelGGL(k_fill_empty, dim3(grid_for(G)), dim3(kBlock), 0, st, G, commit, vote_out);
    QB_CHECK_LAUNCH("k_fill_empty");
    return QB_OK;
  }
  QB_REQUIRE(!commit_out || match, "match is NULL");
  QB_REQUIRE(!vote_out || (voted && granted), "voted/granted NULL with vote_out set");
  constexpr int GPT = 2;
  const size_t mb = n <= 8 ? 1 : 2;
  const bool vec = (G % GPT) == 0 && (!match || aligned(match, 8 * GPT)) &&
                   (!commit || aligned(commit, 8 * GPT)) &&
                   (!vote_out || (aligned(vote_out, GPT) && aligned(voted, mb * GPT) &&
                                  aligned(granted, mb * GPT)));
  dispatch_fixed(std::make_integer_sequence<int, QB_MAX_SLOTS>{}, int(n), G,
                 reinterpret_cast<const u64*>(match), voted, granted, commit, vote_out, vec, st);
  QB_CHECK_LAUNCH("k_fixed");
  return QB_OK;
}

extern "C" int qb_dev_fixed_committed_vote_batches(uint32_t n, uint64_t G, uint32_t count,
                                                   const qb_fixed_batch* batches,
                                                   void* const* streams, uint32_t nstreams) {
  if (count == 0) return QB_OK;
  QB_REQUIRE(batches && streams && nstreams >= 1, "batches / streams NULL or nstreams == 0");
  for (uint32_t i = 0; i < count; ++i) {
    const qb_fixed_batch& b = batches[i];
    const int rc = qb_dev_fixed_committed_vote(n, G, b.match, b.voted, b.granted, b.commit_out,
                                               b.vote_out, streams[i % nstreams]);
    if (rc != QB_OK) return rc;
  }
  return QB_OK;
}

// -------------------------------------------------------------------- CSR ---
//
// A workgroup owns kBlock consecutive groups.  Their slots are one contiguous
// run of match[] (group-major CSR), staged into LDS by LDS-DMA
// (global_load_lds_dwordx4, every piece issued before the one wait at the
// barrier: a load -> wait -> ds_write loop paid one HBM round trip per
// iteration, 276 -> 203 us at 16M ragged groups).  Each thread then gathers
// the members of each half of its config from LDS (non-members: learners,
// the other half) and selects that half's q-th largest (half_ci).
//
// The table's max_slots bound (WMAX) caps the LDS run buffer (kBlock * WMAX
// u64) and the widest network compiled in; within it the network width is
// the wave's largest member count (uniform branch).  Compacting the members
// first makes a 5+5 joint config two 5-wide sorts instead of one tagged
// 10-wide sort (8M joint groups 134 -> 106 us), DESIGN.md §3.2.

namespace qb {

template <int WMAX, bool CI, bool VOTE>
__global__ __launch_bounds__(kBlock) void k_csr(u64 G, const u32* __restrict__ off,
                                                const u64* __restrict__ match,
                                                const u32* __restrict__ cfg,
                                                const u32* __restrict__ votes,
                                                u64* __restrict__ commit,
                                                u8* __restrict__ vote) {
  const u64 g0 = u64(blockIdx.x) * kBlock;
  const u64 g = g0 + threadIdx.x;
  const bool live = g < G;
  // Every independent load is issued up front (cfg, votes, this group's
  // offsets) so their latencies overlap the staging round trip instead of
  // following it.
  const u32 c = live ? ld_nt(cfg + g) : 0u;
  const u32 w = (VOTE && live) ? ld_nt(votes + g) : 0u;
  const u32 min_ = c & 0xFFFFu, mout = c >> 16;

  if constexpr (CI) {
    constexpr u32 kCap = kBlock * WMAX + 2;  // +2: 16-byte head alignment
    __shared__ __attribute__((aligned(16))) u64 lds[kCap];
    const u64 gend = (g0 + kBlock < G) ? g0 + kBlock : G;
    u32 a = 0, b = 0;
    if (live) {
      a = off[g];
      b = off[g + 1];
    }
    const u32 base = off[g0], end = off[gend], total = off[G];
    const u32 abase = base & ~1u;
    // A table that breaks its max_slots bound must not write past the LDS run
    // buffer (results for such a table are unspecified, never out of bounds).
    const u32 span = end - abase < kCap ? end - abase : kCap;
    const u32 npair = (span + 1u) >> 1;
    // Pairs wholly inside match[0, total) go by LDS-DMA, all issued before
    // any wait; only the array's last element can be an unpaired tail.
    const u32 nfull = (abase + 2u * npair <= total) ? npair : npair - 1u;
    constexpr int kIt = int((kCap / 2 + kBlock - 1) / kBlock);
    stage16_lds<kBlock, kIt>(lds, match + abase, nfull);
    if (threadIdx.x == 0 && nfull < npair) lds[2u * nfull] = match[abase + 2u * nfull];
    u32 lo = 0, s = 0;
    if (live) {
      lo = a - abase;
      s = b - a;
      s = s > WMAX ? WMAX : s;
      lo = lo + s <= kCap ? lo : 0;
    }
    __syncthreads();
    const u64 ci = csr_ci<WMAX>(lds + lo, s, min_, mout);
    if (live) st_nt(commit + g, ci);
  }
  if constexpr (VOTE) {
    if (live) {
      const u32 vd = w & 0xFFFFu, gr = (w >> 16) & vd;
      const u8 r1 = vote_from_counts(__popc(min_), __popc(min_ & gr), __popc(min_ & vd));
      const u8 r2 = vote_from_counts(__popc(mout), __popc(mout & gr), __popc(mout & vd));
      vote[g] = joint_vote(r1, r2);
    }
  }
}

template <int WMAX>
static void launch_csr_w(u64 G, const u32* off, const u64* match, const u32* cfg,
                         const u32* votes, u64* commit, u8* vote, hipStream_t st) {
  const dim3 grid(grid_for(G));
  if (commit && vote)
    hipLaunchKernelGGL((k_csr<WMAX, true, true>), grid, dim3(kBlock), 0, st, G, off, match, cfg,
                       votes, commit, vote);
  else if (commit)
    hipLaunchKernelGGL((k_csr<WMAX, true, false>), grid, dim3(kBlock), 0, st, G, off, match,
                       cfg, votes, commit, vote);
  else
    hipLaunchKernelGGL((k_csr<WMAX, false, true>), grid, dim3(kBlock), 0, st, G, off, match,
                       cfg, votes, commit, vote);
}

__global__ void k_csr_validate(u64 G, u32 max_slots, const u32* __restrict__ off,
                               u64* __restrict__ bad) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  const u32 a = off[g], b = off[g + 1];
  bool ok = b >= a && b - a <= max_slots;
  if (g == 0) ok = ok && a == 0;
  if (!ok) atomicAdd(bad, 1ull);
}

}  // namespace qb

extern "C" int qb_dev_csr_committed_vote(uint64_t G, uint32_t max_slots, const uint32_t* off,
                                         const uint64_t* match, const uint32_t* cfg,
                                         const uint32_t* votes, uint64_t* commit_out,
                                         uint8_t* vote_out, void* stream) {
  if (G == 0 || (!commit_out && !vote_out)) return QB_OK;
  QB_REQUIRE(max_slots <= QB_MAX_SLOTS, "max_slots must be 0..%d", QB_MAX_SLOTS);
  QB_REQUIRE(cfg, "cfg is NULL");
  QB_REQUIRE(!commit_out || (off && match), "off/match NULL with commit_out set");
  QB_REQUIRE(!vote_out || votes, "votes NULL with vote_out set");
  QB_REQUIRE(!match || aligned(match, 16), "match must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  u64* commit = reinterpret_cast<u64*>(commit_out);
  const u64* m = reinterpret_cast<const u64*>(match);
  const u32 w = max_slots == 0 ? QB_MAX_SLOTS : max_slots;
  if (!commit) launch_csr_w<4>(G, off, m, cfg, votes, commit, vote_out, st);  // no LDS used
  else if (w <= 4) launch_csr_w<4>(G, off, m, cfg, votes, commit, vote_out, st);
  else if (w <= 8) launch_csr_w<8>(G, off, m, cfg, votes, commit, vote_out, st);
  else if (w <= 12) launch_csr_w<12>(G, off, m, cfg, votes, commit, vote_out, st);
  else launch_csr_w<16>(G, off, m, cfg, votes, commit, vote_out, st);
  QB_CHECK_LAUNCH("k_csr");
  return QB_OK;
}

extern "C" int qb_dev_csr_validate(uint64_t G, uint32_t max_slots, const uint32_t* off,
                                   uint64_t* bad_out, void* stream) {
  QB_REQUIRE(off && bad_out, "off/bad_out NULL");
  QB_REQUIRE(max_slots <= QB_MAX_SLOTS, "max_slots must be 0..%d", QB_MAX_SLOTS);
  if (G == 0) return QB_OK;
  hipLaunchKernelGGL(k_csr_validate, dim3(grid_for(G)), dim3(kBlock), 0, as_stream(stream), G,
                     max_slots == 0 ? u32(QB_MAX_SLOTS) : max_slots, off,
                     reinterpret_cast<u64*>(bad_out));
  QB_CHECK_LAUNCH("k_csr_validate");
  return QB_OK;
}

extern "C" int qb_dev_csr_committed_vote_checked(uint64_t G, uint32_t max_slots,
                                                 const uint32_t* off, const uint64_t* match,
                                                 const uint32_t* cfg, const uint32_t* votes,
                                                 uint64_t* commit_out, uint8_t* vote_out,
                                                 uint64_t* bad_scratch, void* stream) {
  if (G == 0 || (!commit_out && !vote_out)) return QB_OK;
  QB_REQUIRE(off && bad_scratch, "off/bad_scratch NULL");
  hipStream_t st = as_stream(stream);
  hipError_t e = hipMemsetAsync(bad_scratch, 0, sizeof(uint64_t), st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(bad)");
  {
    const int rc = qb_dev_csr_validate(G, max_slots, off, bad_scratch, stream);
    if (rc != QB_OK) return rc;
  }
  uint64_t bad = 0;
  e = hipMemcpyAsync(&bad, bad_scratch, sizeof bad, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "validate readback");
  QB_REQUIRE(bad == 0, "%llu group(s) break the CSR bound (off[0] == 0, 0 <= s_g <= %u)",
             (unsigned long long)bad, max_slots == 0 ? unsigned(QB_MAX_SLOTS) : max_slots);
  return qb_dev_csr_committed_vote(G, max_slots, off, match, cfg, votes, commit_out, vote_out,
                                   stream);
}
