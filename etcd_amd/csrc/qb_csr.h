// qb_csr.h — JointConfig.CommittedIndex over one CSR group's slots (shared by
// k_csr, the CSR tracker step and its slow path).
//
//   MajorityConfig.CommittedIndex  quorum/majority.go:126-172
//   JointConfig.CommittedIndex     quorum/joint.go:49-56
#pragma once

#include "qb_common.h"

namespace qb {

__device__ __forceinline__ u32 wave_max(u32 x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const u32 y = u32(__shfl_xor(int(x), o, 64));
    x = y > x ? y : x;
  }
  return __builtin_amdgcn_readfirstlane(x);  // wave-uniform, scalar branch
}

// MajorityConfig.CommittedIndex of one half (majority.go:126-172): the
// members of `mask`, in slot order, compacted into M registers (M = the
// wave's largest member count) and zero-padded — zeros sort below every value
// and leave the q-th largest unchanged for q <= n, the fill-with-zero of
// majority.go:149-161 — then sorted; the answer is ascending index
// M - (n/2+1), picked by a conditional-move chain (no dynamic register
// indexing, no scratch).  n = 0 is ∞ (majority.go:128-133).
template <int M>
__device__ __forceinline__ u64 half_ci(const u64* src, u32 mask) {
  const int n = __popc(mask);
  u64 v[M];
  u32 m = mask;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const u32 j = m ? u32(__builtin_ctz(m)) : 0u;
    v[k] = m ? src[j] : 0ull;
    m &= m - 1u;
  }
  if constexpr (M >= 2) sort_net<M>(v);
  const int want = M - (n / 2 + 1);
  u64 r = 0;
#pragma unroll
  for (int j = 0; j < M; ++j) r = (j == want) ? v[j] : r;
  return n == 0 ? kInf : r;
}

template <int M, int MAX>
__device__ __forceinline__ u64 half_ci_width(u32 mw, const u64* src, u32 mask) {
  if constexpr (M >= MAX) {
    return half_ci<MAX>(src, mask);
  } else {
    if (mw <= u32(M)) return half_ci<M>(src, mask);
    return half_ci_width<M + 1, MAX>(mw, src, mask);
  }
}

// JointConfig.CommittedIndex (joint.go:49-56) = min of the halves; an empty
// outgoing half is ∞, so a plain majority config (mask_out = 0) is the
// incoming half alone and a wave with no joint group skips the second half.
template <int WMAX>
__device__ __forceinline__ u64 csr_ci(const u64* src, u32 s, u32 min_, u32 mout) {
  const u32 live = s >= 32 ? ~0u : ((1u << s) - 1u);
  min_ &= live;
  mout &= live;
  u64 c = half_ci_width<1, WMAX>(wave_max(u32(__popc(min_))), src, min_);
  if (__ballot(mout != 0) != 0) {
    const u64 c2 = half_ci_width<1, WMAX>(wave_max(u32(__popc(mout))), src, mout);
    c = c2 < c ? c2 : c;
  }
  return c;
}

}  // namespace qb
