// qb_wide.hip — CommittedIndex / VoteResult for WIDE configs (more than 16
// slots, up to QB_WIDE_MAX_SLOTS), one wavefront per group.
//
// Reference semantics: MajorityConfig.CommittedIndex / VoteResult
// (quorum/majority.go:126-210), JointConfig (quorum/joint.go:49-75).
//
// Layout WIDE: off[G+1] u32, match[off[G]] u64, flags[off[G]] u8 per slot:
// bit 0 incoming voter, bit 1 outgoing voter, bit 2 voted, bit 3 granted.
//
// The wave holds the group's slots in registers (K per lane, coalesced
// loads) and finds the q-th largest member value by an MSB-first radix
// select: the largest x with #{members >= x} >= q is exactly the q-th
// largest (the count is monotone in x).  Each bit step is one u64 compare
// per register, a ballot and a scalar popcount; the search starts below the
// common prefix of the members' min and max, which every candidate shares.
// VoteResult is three ballot popcounts per half.
#include "qb_common.h"

namespace qb {

constexpr int kWaves = kBlock / 64;

__device__ __forceinline__ u64 wave_max_u64(u64 x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const u64 y = __shfl_xor(x, o, 64);
    x = y > x ? y : x;
  }
  return x;
}
__device__ __forceinline__ u64 wave_min_u64(u64 x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const u64 y = __shfl_xor(x, o, 64);
    x = y < x ? y : x;
  }
  return x;
}

// q-th largest of the values whose flag bit `bit` is set; every lane returns
// the same value.  n == 0 -> ∞ (majority.go:128-133).
template <int K>
__device__ __forceinline__ u64 wide_select(const u64 (&v)[K], const u32 (&fl)[K], u32 bit, u32 n) {
  if (n == 0) return kInf;
  const u32 q = n / 2 + 1;
  u64 lo = kInf, hi = 0;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if ((fl[k] >> bit) & 1u) {
      lo = v[k] < lo ? v[k] : lo;
      hi = v[k] > hi ? v[k] : hi;
    }
  lo = wave_min_u64(lo);
  hi = wave_max_u64(hi);
  if (lo == hi) return hi;
  const int top = 63 - __builtin_clzll(lo ^ hi);  // highest bit where members differ
  u64 x = hi & ~((2ull << top) - 1ull);           // shared prefix
  for (int b = top; b >= 0; --b) {
    const u64 t = x | (1ull << b);
    u32 cnt = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) cnt += u32(__popcll(__ballot(((fl[k] >> bit) & 1u) && v[k] >= t)));
    if (cnt >= q) x = t;
  }
  return x;
}

template <int K>
__global__ __launch_bounds__(kBlock) void k_wide(u64 G, const u32* __restrict__ off,
                                                 const u64* __restrict__ match,
                                                 const u8* __restrict__ flags,
                                                 u64* __restrict__ commit, u8* __restrict__ vote) {
  const u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 g = u64(blockIdx.x) * kWaves + w;
  if (g >= G) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const u32 a = off[g], s = off[g + 1] - a;
  u64 v[K];
  u32 fl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const u32 j = u32(k) * 64u + u32(lane);
    const bool live = j < s;
    v[k] = live ? __builtin_nontemporal_load(match + a + j) : 0ull;
    fl[k] = live ? u32(flags[a + j]) : 0u;
  }
  u32 n_in = 0, n_out = 0, yes_in = 0, yes_out = 0, vd_in = 0, vd_out = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const u32 f = fl[k];
    const bool voted = (f & 4u) != 0, yes = voted && (f & 8u);
    n_in += u32(__popcll(__ballot(f & 1u)));
    n_out += u32(__popcll(__ballot(f & 2u)));
    vd_in += u32(__popcll(__ballot((f & 1u) && voted)));
    vd_out += u32(__popcll(__ballot((f & 2u) && voted)));
    yes_in += u32(__popcll(__ballot((f & 1u) && yes)));
    yes_out += u32(__popcll(__ballot((f & 2u) && yes)));
  }
  if (commit) {
    const u64 c0 = wide_select<K>(v, fl, 0, n_in);
    const u64 c1 = wide_select<K>(v, fl, 1, n_out);  // empty half -> ∞ (joint.go:49-56)
    if (lane == 0) commit[g] = c1 < c0 ? c1 : c0;
  }
  if (vote && lane == 0) {
    const u8 r1 = vote_from_counts(int(n_in), int(yes_in), int(vd_in));
    const u8 r2 = vote_from_counts(int(n_out), int(yes_out), int(vd_out));
    vote[g] = joint_vote(r1, r2);
  }
}

template <int K>
static void launch_wide(u64 G, const u32* off, const u64* m, const u8* fl, u64* c, u8* v,
                        hipStream_t st) {
  hipLaunchKernelGGL((k_wide<K>), dim3(unsigned((G + kWaves - 1) / kWaves)), dim3(kBlock), 0, st,
                     G, off, m, fl, c, v);
}

__global__ void k_wide_validate(u64 G, u32 max_slots, const u32* __restrict__ off,
                                u64* __restrict__ bad) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= G) return;
  const u32 a = off[g], b = off[g + 1];
  bool ok = b >= a && b - a <= max_slots;
  if (g == 0) ok = ok && a == 0;
  if (!ok) atomicAdd(bad, 1ull);
}

}  // namespace qb

using namespace qb;

extern "C" int qb_dev_wide_committed_vote(uint64_t G, uint32_t max_slots, const uint32_t* off,
                                          const uint64_t* match, const uint8_t* flags,
                                          uint64_t* commit_out, uint8_t* vote_out,
                                          void* stream) {
  if (G == 0 || (!commit_out && !vote_out)) return QB_OK;
  QB_REQUIRE(max_slots <= QB_WIDE_MAX_SLOTS, "max_slots must be 0..%d", QB_WIDE_MAX_SLOTS);
  QB_REQUIRE(off && flags && (!commit_out || match), "required pointer is NULL");
  hipStream_t st = as_stream(stream);
  const u32 w = max_slots == 0 ? QB_WIDE_MAX_SLOTS : max_slots;
  const u64* m = reinterpret_cast<const u64*>(match);
  u64* c = reinterpret_cast<u64*>(commit_out);
  if (w <= 64) launch_wide<1>(G, off, m, flags, c, vote_out, st);
  else if (w <= 128) launch_wide<2>(G, off, m, flags, c, vote_out, st);
  else if (w <= 256) launch_wide<4>(G, off, m, flags, c, vote_out, st);
  else if (w <= 512) launch_wide<8>(G, off, m, flags, c, vote_out, st);
  else launch_wide<16>(G, off, m, flags, c, vote_out, st);
  QB_CHECK_LAUNCH("k_wide");
  return QB_OK;
}

extern "C" int qb_dev_wide_validate(uint64_t G, uint32_t max_slots, const uint32_t* off,
                                    uint64_t* bad_out, void* stream) {
  QB_REQUIRE(off && bad_out, "off/bad_out NULL");
  QB_REQUIRE(max_slots <= QB_WIDE_MAX_SLOTS, "max_slots must be 0..%d", QB_WIDE_MAX_SLOTS);
  if (G == 0) return QB_OK;
  hipLaunchKernelGGL(k_wide_validate, dim3(grid_for(G)), dim3(kBlock), 0, as_stream(stream), G,
                     max_slots == 0 ? u32(QB_WIDE_MAX_SLOTS) : max_slots, off,
                     reinterpret_cast<u64*>(bad_out));
  QB_CHECK_LAUNCH("k_wide_validate");
  return QB_OK;
}
