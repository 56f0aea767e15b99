// qb_synth.hip — counter-based synthetic multi-raft workloads.
//
// Every value is a pure function of (seed, global group number, slot, field),
// so each shard/GPU generates its own part independently and the CPU oracle
// (oracle/quorum_oracle.c, an independent restatement of this spec) generates
// bit-identical inputs for parity.  Spec:
//   last      = 1 + r(g,0,LAST) % (2^40 - 1); 1% of groups (r(g,0,HIGH) % 100
//               == 0) get bit 63 and random bits 40..61 set, so unsigned
//               compares over the full u64 range are exercised
//   match[j]  = last for j == 0 (the leader); else 0 with 5% probability
//               (r(g,j,ABSENT) % 100 < 5), else last - min(r(g,j,LAG) % 64, last)
//   vote[j]   = r(g,j,VOTE) % 10: 0-2 missing, 3-4 rejected, 5-9 granted
//   term_start= last - d if last > d else 1, d = r(g,0,TERMSTART) % 128
//   ragged    n = 3 + r(g,0,N) % 7 voters, L = r(g,0,L) % 3 learners placed at
//               1 + r(g,l,LPOS) % (s-1), probing upward (wrapping to 1) past
//               slots that are already learners
//   joint 5+5 overlap k = r(g,0,OVERLAP) % 6, union u = 10 - k slots; incoming
//               = slots 0..4, outgoing = slots 5-k..9-k, both rotated left by
//               r(g,0,ROT) % u within u bits
#include "qb_common.h"

namespace qb {

__host__ __device__ __forceinline__ u64 synth_last(u64 seed, u64 g) {
  u64 last = 1ull + rnd(seed, g, 0, F_LAST) % ((1ull << 40) - 1ull);
  if (rnd(seed, g, 0, F_HIGH) % 100ull == 0ull)
    last |= (1ull << 63) | (rnd(seed, g, 0, F_HIGHBITS) & 0x3FFFFF0000000000ull);
  return last;
}

__host__ __device__ __forceinline__ u64 synth_match(u64 seed, u64 g, u32 j, u64 last) {
  if (j == 0) return last;
  if (rnd(seed, g, j, F_ABSENT) % 100ull < 5ull) return 0ull;
  const u64 lag = rnd(seed, g, j, F_LAG) % 64ull;
  return last - (lag < last ? lag : last);
}

// Returns bit (voted) and sets *granted.
__host__ __device__ __forceinline__ bool synth_vote(u64 seed, u64 g, u32 j, bool* granted) {
  const u64 v = rnd(seed, g, j, F_VOTE) % 10ull;
  *granted = v >= 5;
  return v >= 3;
}

__host__ __device__ __forceinline__ u64 synth_term_start(u64 seed, u64 g, u64 last) {
  const u64 d = rnd(seed, g, 0, F_TERMSTART) % 128ull;
  return last > d ? last - d : 1ull;
}

__host__ __device__ __forceinline__ u32 synth_ragged_size(u64 seed, u64 g) {
  return 3u + u32(rnd(seed, g, 0, F_N) % 7ull) + u32(rnd(seed, g, 0, F_L) % 3ull);
}

__host__ __device__ __forceinline__ u32 synth_ragged_mask(u64 seed, u64 g, u32 s) {
  const u32 L = u32(rnd(seed, g, 0, F_L) % 3ull);
  u32 mask = (1u << s) - 1u;
  for (u32 l = 0; l < L; ++l) {
    u32 p = 1u + u32(rnd(seed, g, l, F_LPOS) % u64(s - 1u));
    while (!((mask >> p) & 1u)) p = (p + 1u < s) ? p + 1u : 1u;
    mask &= ~(1u << p);
  }
  return mask;
}

__host__ __device__ __forceinline__ u32 synth_joint_size(u64 seed, u64 g) {
  return 10u - u32(rnd(seed, g, 0, F_OVERLAP) % 6ull);
}

__host__ __device__ __forceinline__ u32 rotl_u(u32 m, u32 r, u32 u) {
  const u32 full = (1u << u) - 1u;
  return r == 0 ? m : (((m << r) | (m >> (u - r))) & full);
}

__host__ __device__ __forceinline__ u32 synth_joint_cfg(u64 seed, u64 g, u32 u) {
  const u32 k = 10u - u;
  const u32 rot = u32(rnd(seed, g, 0, F_ROT) % u64(u));
  const u32 min_ = rotl_u(0x1Fu, rot, u);
  const u32 mout = rotl_u(0x1Fu << (5u - k), rot, u);
  return min_ | (mout << 16);
}

template <typename M>
__global__ __launch_bounds__(kBlock) void k_synth_fixed(u64 seed, u32 n, u64 G, u64 g_begin,
                                                        u64* __restrict__ match,
                                                        M* __restrict__ voted,
                                                        M* __restrict__ granted,
                                                        u64* __restrict__ term_start) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  const u64 gg = g_begin + g;
  const u64 last = synth_last(seed, gg);
  u32 vd = 0, gr = 0;
  for (u32 j = 0; j < n; ++j) {
    if (match) match[u64(j) * G + g] = synth_match(seed, gg, j, last);
    bool yes;
    if (synth_vote(seed, gg, j, &yes)) {
      vd |= 1u << j;
      if (yes) gr |= 1u << j;
    }
  }
  if (voted) voted[g] = M(vd);
  if (granted) granted[g] = M(gr);
  if (term_start) term_start[g] = synth_term_start(seed, gg, last);
}

__global__ __launch_bounds__(kBlock) void k_synth_csr(u64 seed, int kind, u64 G, u64 g_begin,
                                                      const u32* __restrict__ off,
                                                      u64* __restrict__ match,
                                                      u32* __restrict__ cfg,
                                                      u32* __restrict__ votes) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  const u64 gg = g_begin + g;
  const u32 a = off[g], s = off[g + 1] - a;
  const u64 last = synth_last(seed, gg);
  u32 vd = 0, gr = 0;
  for (u32 j = 0; j < s; ++j) {
    if (match) match[a + j] = synth_match(seed, gg, j, last);
    bool yes;
    if (synth_vote(seed, gg, j, &yes)) {
      vd |= 1u << j;
      if (yes) gr |= 1u << j;
    }
  }
  if (cfg) cfg[g] = kind == 0 ? synth_ragged_mask(seed, gg, s) : synth_joint_cfg(seed, gg, s);
  if (votes) votes[g] = vd | (gr << 16);
}

}  // namespace qb

using namespace qb;

extern "C" int qb_dev_synth_fixed(uint64_t seed, uint32_t n, uint64_t G, uint64_t g_begin,
                                  uint64_t* match, void* voted, void* granted,
                                  uint64_t* term_start, void* stream) {
  QB_REQUIRE(n >= 1 && n <= QB_MAX_SLOTS, "n must be 1..%d", QB_MAX_SLOTS);
  if (G == 0) return QB_OK;
  hipStream_t st = as_stream(stream);
  u64* m = reinterpret_cast<u64*>(match);
  u64* ts = reinterpret_cast<u64*>(term_start);
  if (n <= 8)
    hipLaunchKernelGGL(k_synth_fixed<u8>, dim3(grid_for(G)), dim3(kBlock), 0, st, seed, n, G,
                       g_begin, m, static_cast<u8*>(voted), static_cast<u8*>(granted), ts);
  else
    hipLaunchKernelGGL(k_synth_fixed<u16>, dim3(grid_for(G)), dim3(kBlock), 0, st, seed, n, G,
                       g_begin, m, static_cast<u16*>(voted), static_cast<u16*>(granted), ts);
  QB_CHECK_LAUNCH("k_synth_fixed");
  return QB_OK;
}

static int host_offsets(uint64_t seed, uint64_t G, uint64_t g_begin, uint32_t* off, bool joint) {
  QB_REQUIRE(off, "off is NULL");
  u64 acc = 0;
  off[0] = 0;
  for (u64 g = 0; g < G; ++g) {
    acc += joint ? synth_joint_size(seed, g_begin + g) : synth_ragged_size(seed, g_begin + g);
    QB_REQUIRE(acc <= 0xFFFFFFFFull, "CSR slot count overflows uint32 at group %llu",
               (unsigned long long)g);
    off[g + 1] = u32(acc);
  }
  return QB_OK;
}

extern "C" int qb_host_synth_csr_offsets(uint64_t seed, uint64_t G, uint64_t g_begin,
                                         uint32_t* off) {
  return host_offsets(seed, G, g_begin, off, false);
}

extern "C" int qb_host_synth_joint_offsets(uint64_t seed, uint64_t G, uint64_t g_begin,
                                           uint32_t* off) {
  return host_offsets(seed, G, g_begin, off, true);
}

extern "C" int qb_dev_synth_csr(uint64_t seed, int kind, uint64_t G, uint64_t g_begin,
                                const uint32_t* off, uint64_t* match, uint32_t* cfg,
                                uint32_t* votes, void* stream) {
  QB_REQUIRE(kind == 0 || kind == 1, "kind must be 0 (ragged) or 1 (joint)");
  QB_REQUIRE(off, "off is NULL");
  if (G == 0) return QB_OK;
  hipLaunchKernelGGL(k_synth_csr, dim3(grid_for(G)), dim3(kBlock), 0, as_stream(stream), seed,
                     kind, G, g_begin, off, reinterpret_cast<u64*>(match), cfg, votes);
  QB_CHECK_LAUNCH("k_synth_csr");
  return QB_OK;
}
