// csr_lab.hip — A/B variants of the CSR (ragged / joint) kernel
// (development tool; the product kernel lives in etcd_amd/csrc).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "qb_common.h"

using namespace qb;

namespace {

template <typename T>
__device__ __forceinline__ T ldn(const T* p) { return __builtin_nontemporal_load(p); }

// ---- selection over W zero-masked slots (64-bit network, as the product) ----
template <int W>
__device__ __forceinline__ u64 sel64(const u64* src, u32 s, u32 mask) {
  u64 v[W];
#pragma unroll
  for (int j = 0; j < W; ++j) v[j] = (u32(j) < s && ((mask >> j) & 1u)) ? src[j] : 0ull;
  sort_net<W>(v);
  const int n = __popc(mask);
  if (n == 0) return kInf;
  const int want = W - (n / 2 + 1);
  u64 r = 0;
#pragma unroll
  for (int j = 0; j < W; ++j) r = (j == want) ? v[j] : r;
  return r;
}

// ---- 32-bit offset path: key = top - v (saturating); exact unless the
// selected key saturates (then the caller falls back to 64-bit) ----
__device__ __forceinline__ void cmpx32(u32& a, u32& b) {
  const u32 lo = a < b ? a : b, hi = a < b ? b : a;
  a = lo;
  b = hi;
}
template <class Net, int... K>
__device__ __forceinline__ void run_net32(u32* v, std::integer_sequence<int, K...>) {
  ((cmpx32(v[Net::A[K]], v[Net::B[K]])), ...);
}

// Returns true and the exact q-th largest if representable.
template <int W>
__device__ __forceinline__ bool sel32(const u64* src, u32 s, u32 mask, u64 top, u64& out) {
  // keys ascending = values descending; non-members = 0xFFFFFFFF (smallest value)
  u32 k[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    u32 key = 0xFFFFFFFFu;
    if (u32(j) < s && ((mask >> j) & 1u)) {
      const u64 d = top - src[j];
      key = d >= 0xFFFFFFFFull ? 0xFFFFFFFFu : u32(d);
    }
    k[j] = key;
  }
  run_net32<SortNet<W>>(k, std::make_integer_sequence<int, SortNet<W>::K>{});
  const int n = __popc(mask);
  if (n == 0) {
    out = kInf;
    return true;
  }
  const int want = n / 2;  // q-th largest = (q-1)-th smallest key, q-1 = n/2
  u32 r = 0;
#pragma unroll
  for (int j = 0; j < W; ++j) r = (j == want) ? k[j] : r;
  if (r == 0xFFFFFFFFu) return false;
  out = top - u64(r);
  return true;
}

template <int W>
__device__ __forceinline__ u64 ci64(const u64* src, u32 s, u32 mi, u32 mo) {
  u64 c = sel64<W>(src, s, mi);
  if (mo) {
    const u64 c2 = sel64<W>(src, s, mo);
    c = c2 < c ? c2 : c;
  }
  return c;
}

template <int W>
__device__ __forceinline__ u64 ci32(const u64* src, u32 s, u32 mi, u32 mo) {
  u64 top = 0;
#pragma unroll
  for (int j = 0; j < W; ++j)
    if (u32(j) < s && (((mi | mo) >> j) & 1u)) top = src[j] > top ? src[j] : top;
  u64 c, c2 = kInf;
  bool ok = sel32<W>(src, s, mi, top, c);
  if (mo) ok = sel32<W>(src, s, mo, top, c2) && ok;
  if (__ballot(!ok) != 0) {  // rare: a saturated key was selected
    if (!ok) return ci64<W>(src, s, mi, mo);
  }
  return c2 < c ? c2 : c;
}

// ---- members of each half compacted (slot order) into M registers ----
__device__ __forceinline__ u32 wmax_u32(u32 x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const u32 y = u32(__shfl_xor(int(x), o, 64));
    x = y > x ? y : x;
  }
  return __builtin_amdgcn_readfirstlane(x);
}
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
__device__ __forceinline__ u64 half_ci_w(u32 mw, const u64* src, u32 mask) {
  if constexpr (M >= MAX) {
    return half_ci<MAX>(src, mask);
  } else {
    if (mw <= u32(M)) return half_ci<M>(src, mask);
    return half_ci_w<M + 1, MAX>(mw, src, mask);
  }
}
template <int MAX>
__device__ __forceinline__ u64 ci_compact(const u64* src, u32 s, u32 mi, u32 mo) {
  const u32 live = s >= 32 ? ~0u : ((1u << s) - 1u);
  mi &= live;
  mo &= live;
  u64 c = half_ci_w<1, MAX>(wmax_u32(u32(__popc(mi))), src, mi);
  if (__ballot(mo != 0) != 0) {
    const u64 c2 = half_ci_w<1, MAX>(wmax_u32(u32(__popc(mo))), src, mo);
    c = c2 < c ? c2 : c;
  }
  return c;
}

template <int MODE>  // 0 = 64-bit network, 1 = 32-bit offsets, 2 = memory floor
__device__ __forceinline__ u64 eval(const u64* src, u32 s, u32 mi, u32 mo) {
  if constexpr (MODE == 3) {
    return ci_compact<12>(src, s, mi, mo);
  } else if constexpr (MODE == 2) {
    u64 x = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) x ^= (u32(j) < s) ? src[j] : 0ull;
    return x;
  } else {
    const bool gt8 = __ballot(s > 8) != 0, gt4 = __ballot(s > 4) != 0,
               gt12 = __ballot(s > 12) != 0;
    if (MODE == 0) {
      if (!gt8) return gt4 ? ci64<8>(src, s, mi, mo) : ci64<4>(src, s, mi, mo);
      return gt12 ? ci64<16>(src, s, mi, mo) : ci64<12>(src, s, mi, mo);
    } else {
      if (!gt8) return gt4 ? ci32<8>(src, s, mi, mo) : ci32<4>(src, s, mi, mo);
      return gt12 ? ci32<16>(src, s, mi, mo) : ci32<12>(src, s, mi, mo);
    }
  }
}

__device__ __forceinline__ u8 vote_of(u32 mi, u32 mo, u32 w) {
  const u32 vd = w & 0xFFFFu, gr = (w >> 16) & vd;
  const u8 r1 = vote_from_counts(__popc(mi), __popc(mi & gr), __popc(mi & vd));
  const u8 r2 = vote_from_counts(__popc(mo), __popc(mo & gr), __popc(mo & vd));
  return joint_vote(r1, r2);
}

// LDS-staged (product structure).  SMAX = max slots per group provisioned.
template <int BLOCK, int SMAX, int MODE, bool NT, bool DMA = false>
__global__ __launch_bounds__(BLOCK) void k_lds(u64 G, const u32* __restrict__ off,
                                               const u64* __restrict__ match,
                                               const u32* __restrict__ cfg,
                                               const u32* __restrict__ votes,
                                               u64* __restrict__ commit, u8* __restrict__ vote) {
  __shared__ __attribute__((aligned(16))) u64 lds[BLOCK * SMAX + 2];
  const u64 g0 = u64(blockIdx.x) * BLOCK;
  const u64 g = g0 + threadIdx.x;
  const bool live = g < G;
  const u32 c = live ? (NT ? ldn(cfg + g) : cfg[g]) : 0u;
  const u32 w = live ? (NT ? ldn(votes + g) : votes[g]) : 0u;
  const u64 gend = (g0 + BLOCK < G) ? g0 + BLOCK : G;
  const u32 base = off[g0], end = off[gend], total = off[G];
  const u32 abase = base & ~1u;
  const u32 npair = (end - abase + 1u) >> 1;
  using V = u32 __attribute__((ext_vector_type(4)));
  if constexpr (DMA) {
    const u32 nfull = (abase + 2u * npair <= total) ? npair : npair - 1u;
    stage16_lds<BLOCK, (BLOCK * SMAX / 2 + BLOCK) / BLOCK>(lds, match + abase, nfull);
    if (threadIdx.x == 0 && nfull < npair) lds[2u * nfull] = match[abase + 2u * nfull];
  } else {
  for (u32 i = threadIdx.x; i < npair; i += BLOCK) {
    const u32 idx = abase + 2u * i;
    if (idx + 1u < total)
      reinterpret_cast<V*>(lds)[i] =
          NT ? ldn(reinterpret_cast<const V*>(match + idx)) : *reinterpret_cast<const V*>(match + idx);
    else
      lds[2u * i] = match[idx];
  }
  }
  u32 lo = 0, s = 0;
  if (live) {
    const u32 a = off[g], b = off[g + 1];
    lo = a - abase;
    s = b - a;
  }
  __syncthreads();
  const u64 ci = eval<MODE>(lds + lo, s, c & 0xFFFFu, c >> 16);
  if (live) {
    if (NT) {
      __builtin_nontemporal_store(ci, commit + g);
    } else {
      commit[g] = ci;
    }
    vote[g] = vote_of(c & 0xFFFFu, c >> 16, w);
  }
}

// No LDS: each lane reads its own slots from global memory.
template <int BLOCK, int MODE>
__global__ __launch_bounds__(BLOCK) void k_direct(u64 G, const u32* __restrict__ off,
                                                  const u64* __restrict__ match,
                                                  const u32* __restrict__ cfg,
                                                  const u32* __restrict__ votes,
                                                  u64* __restrict__ commit, u8* __restrict__ vote) {
  const u64 g = u64(blockIdx.x) * BLOCK + threadIdx.x;
  const bool live = g < G;
  const u32 c = live ? cfg[g] : 0u, w = live ? votes[g] : 0u;
  const u32 a = live ? off[g] : 0u, s = live ? off[g + 1] - a : 0u;
  u64 buf[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) buf[j] = (u32(j) < s) ? match[a + j] : 0ull;
  const u64 ci = eval<MODE>(buf, s, c & 0xFFFFu, c >> 16);
  if (live) {
    commit[g] = ci;
    vote[g] = vote_of(c & 0xFFFFu, c >> 16, w);
  }
}


// ---- one sort of all slots carrying membership tags (joint: both halves) ----
__device__ __forceinline__ void cmpx_tag(u64& a, u64& b, u32& ta, u32& tb) {
  const bool sw = b < a;
  const u64 lo = sw ? b : a, hi = sw ? a : b;
  const u32 tl = sw ? tb : ta, th = sw ? ta : tb;
  a = lo; b = hi; ta = tl; tb = th;
}
template <class Net, int... K>
__device__ __forceinline__ void run_net_tag(u64* v, u32* t, std::integer_sequence<int, K...>) {
  ((cmpx_tag(v[Net::A[K]], v[Net::B[K]], t[Net::A[K]], t[Net::B[K]])), ...);
}
template <int W>
__device__ __forceinline__ u64 citag(const u64* src, u32 s, u32 mi, u32 mo) {
  if (mo == 0) return sel64<W>(src, s, mi);
  u64 v[W];
  u32 t[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const bool live = u32(j) < s;
    v[j] = live ? src[j] : 0ull;
    t[j] = live ? (((mi >> j) & 1u) | (((mo >> j) & 1u) << 1)) : 0u;
  }
  run_net_tag<SortNet<W>>(v, t, std::make_integer_sequence<int, SortNet<W>::K>{});
  const int qi = __popc(mi) / 2 + 1, qo = __popc(mo) / 2 + 1;
  int ci = 0, co = 0;
  u64 ri = __popc(mi) ? 0ull : kInf, ro = kInf;
#pragma unroll
  for (int j = W - 1; j >= 0; --j) {  // descending
    ci += t[j] & 1u;
    co += t[j] >> 1;
    ri = (ci == qi && (t[j] & 1u)) ? v[j] : ri;
    ro = (co == qo && (t[j] >> 1)) ? v[j] : ro;
  }
  return ro < ri ? ro : ri;
}

template <int MODE2>  // 0 = two sorts, 1 = tagged single sort
__device__ __forceinline__ u64 eval2(const u64* src, u32 s, u32 mi, u32 mo) {
  const bool gt8 = __ballot(s > 8) != 0, gt4 = __ballot(s > 4) != 0, gt12 = __ballot(s > 12) != 0;
  if (MODE2 == 0) {
    if (!gt8) return gt4 ? ci64<8>(src, s, mi, mo) : ci64<4>(src, s, mi, mo);
    return gt12 ? ci64<16>(src, s, mi, mo) : ci64<12>(src, s, mi, mo);
  }
  if (!gt8) return gt4 ? citag<8>(src, s, mi, mo) : citag<4>(src, s, mi, mo);
  return gt12 ? citag<16>(src, s, mi, mo) : citag<12>(src, s, mi, mo);
}

// LDS capacity CAP slots per group on average; a block whose run does not
// fit reads its slots straight from global memory (correct, slower).
template <int BLOCK, int CAP, int MODE2>
__global__ __launch_bounds__(BLOCK) void k_cap(u64 G, const u32* __restrict__ off,
                                               const u64* __restrict__ match,
                                               const u32* __restrict__ cfg,
                                               const u32* __restrict__ votes,
                                               u64* __restrict__ commit, u8* __restrict__ vote) {
  constexpr u32 kCap = BLOCK * CAP + 2;
  __shared__ __attribute__((aligned(16))) u64 lds[kCap];
  const u64 g0 = u64(blockIdx.x) * BLOCK;
  const u64 g = g0 + threadIdx.x;
  const bool live = g < G;
  const u32 c = live ? ldn(cfg + g) : 0u;
  const u32 w = live ? ldn(votes + g) : 0u;
  const u64 gend = (g0 + BLOCK < G) ? g0 + BLOCK : G;
  const u32 base = off[g0], end = off[gend], total = off[G];
  const u32 abase = base & ~1u;
  const bool fits = end - abase <= kCap;
  u32 a = 0, s = 0;
  if (live) {
    a = off[g];
    s = off[g + 1] - a;
  }
  u64 ci;
  if (fits) {
    const u32 npair = (end - abase + 1u) >> 1;
    using V = u32 __attribute__((ext_vector_type(4)));
    for (u32 i = threadIdx.x; i < npair; i += BLOCK) {
      const u32 idx = abase + 2u * i;
      if (idx + 1u < total)
        reinterpret_cast<V*>(lds)[i] = ldn(reinterpret_cast<const V*>(match + idx));
      else
        lds[2u * i] = match[idx];
    }
    __syncthreads();
    ci = eval2<MODE2>(lds + (a - abase), s, c & 0xFFFFu, c >> 16);
  } else {
    u64 buf[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) buf[j] = (u32(j) < s) ? match[a + j] : 0ull;
    ci = eval2<MODE2>(buf, s, c & 0xFFFFu, c >> 16);
  }
  if (live) {
    __builtin_nontemporal_store(ci, commit + g);
    vote[g] = vote_of(c & 0xFFFFu, c >> 16, w);
  }
}

template <int BLOCK, int CAP, int MODE2>
void L_cap(u64 G, const u32* off, const u64* m, const u32* cfg, const u32* vt, u64* c, u8* v,
           hipStream_t st) {
  hipLaunchKernelGGL((k_cap<BLOCK, CAP, MODE2>), dim3(unsigned((G + BLOCK - 1) / BLOCK)),
                     dim3(BLOCK), 0, st, G, off, m, cfg, vt, c, v);
}

using Launch = void (*)(u64, const u32*, const u64*, const u32*, const u32*, u64*, u8*,
                        hipStream_t);

template <int BLOCK, int SMAX, int MODE, bool NT, bool DMA = false>
void L_lds(u64 G, const u32* off, const u64* m, const u32* cfg, const u32* vt, u64* c, u8* v,
           hipStream_t st) {
  hipLaunchKernelGGL((k_lds<BLOCK, SMAX, MODE, NT, DMA>), dim3(unsigned((G + BLOCK - 1) / BLOCK)),
                     dim3(BLOCK), 0, st, G, off, m, cfg, vt, c, v);
}
template <int BLOCK, int MODE>
void L_direct(u64 G, const u32* off, const u64* m, const u32* cfg, const u32* vt, u64* c, u8* v,
              hipStream_t st) {
  hipLaunchKernelGGL((k_direct<BLOCK, MODE>), dim3(unsigned((G + BLOCK - 1) / BLOCK)),
                     dim3(BLOCK), 0, st, G, off, m, cfg, vt, c, v);
}

struct Variant {
  const char* name;
  Launch fn;
};
const Variant kV[] = {
    {"lds256_s12_net64", L_lds<256, 12, 0, true>},
    {"lds256_s12_floor", L_lds<256, 12, 2, true>},
    {"dma256_s12_floor", L_lds<256, 12, 2, true, true>},
    {"dma256_s12_net64", L_lds<256, 12, 0, true, true>},
    {"dma128_s12_floor", L_lds<128, 12, 2, true, true>},
    {"dma512_s12_floor", L_lds<512, 12, 2, true, true>},
    {"dma256_s12_compact", L_lds<256, 12, 3, true, true>},
};

}  // namespace

extern "C" int lab_count() { return int(sizeof(kV) / sizeof(kV[0])); }
extern "C" const char* lab_name(int i) { return kV[i].name; }
extern "C" int lab_launch(int i, uint64_t G, const void* off, const void* match, const void* cfg,
                          const void* votes, void* commit, void* vote, void* stream) {
  kV[i].fn(G, static_cast<const u32*>(off), static_cast<const u64*>(match),
           static_cast<const u32*>(cfg), static_cast<const u32*>(votes), static_cast<u64*>(commit),
           static_cast<u8*>(vote), reinterpret_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
