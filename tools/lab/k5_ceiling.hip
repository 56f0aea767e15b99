// Lab probe (development tool, not product code): the HBM streaming ceiling
// of the tracker apply kernel's traffic mix, and what its structure costs on
// top.  Per group: read 5 match rows + committed + term_start + group term
// (u64) + active (u16) + one 8-byte record; write 4 match rows + committed +
// active.  Variants add, one at a time, K5's pieces: the records applied
// through an LDS accumulator with a barrier (APPLY), and CHAIN dependent
// global round trips in front of the record loads (K5's part table -> run
// table -> records chain).
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;

template <int CHAIN, bool APPLY, bool STORES>
__global__ __launch_bounds__(512) void k_ceiling(u64 G, const u64* __restrict__ rec,
                                                 const u32* __restrict__ chain,
                                                 const u64* __restrict__ gterm,
                                                 const u64* __restrict__ ts, u64* __restrict__ match,
                                                 u64* __restrict__ committed,
                                                 u16* __restrict__ active) {
  __shared__ u64 acc[5 * 512];
  const u64 g = u64(blockIdx.x) * 512 + threadIdx.x;
  // the chain: each hop's address depends on the previous hop's value
  u32 off = blockIdx.x;
#pragma unroll
  for (int h = 0; h < CHAIN; ++h) off = chain[off];
  const u64 gt = gterm[g];
  u64 v[5];
#pragma unroll
  for (int s = 0; s < 5; ++s) v[s] = match[u64(s) * G + g];
  const u64 cm = committed[g], t = ts[g];
  const u16 a = active[g];
  const u64 r = rec[u64(off) * 512 + threadIdx.x];
  u64 mx = 0;
  if constexpr (APPLY) {
#pragma unroll
    for (int s = 0; s < 5; ++s) acc[s * 512 + threadIdx.x] = 0;
    __syncthreads();
    const u32 lg = u32(r) & 511u, s = 1u + ((u32(r) >> 9) & 3u);
    if ((r >> 24) != gt) atomicMax(&acc[s * 512 + lg], r >> 24);
    __syncthreads();
#pragma unroll
    for (int s2 = 1; s2 < 5; ++s2) {
      const u64 x = acc[s2 * 512 + threadIdx.x];
      v[s2] = x > v[s2] ? x : v[s2] + 1;
      mx = v[s2] > mx ? v[s2] : mx;
    }
  } else {
    const u64 x = r ^ gt;
#pragma unroll
    for (int s = 1; s < 5; ++s) {
      v[s] += (x >> s) & 1;
      mx = v[s] > mx ? v[s] : mx;
    }
  }
  const u64 c = mx > cm && mx >= t ? mx : cm + 1;
  if (STORES) {
#pragma unroll
    for (int s = 1; s < 5; ++s) match[u64(s) * G + g] = v[s];
    committed[g] = c;
    active[g] = u16(a | 1);
  } else if (c == 0x123456789ull) {
    committed[g] = c;
  }
}

#define QB_LAB_CASE(ID, CH, AP, ST)                                                                \
  case ID:                                                                                     \
    hipLaunchKernelGGL((k_ceiling<CH, AP, ST>), dim3(G / 512), dim3(512), 0, st, G, rec, chain, \
                       gterm, ts, match, committed, active);                                   \
    break;

extern "C" int lab_k5_ceiling(int variant, u64 G, const u64* rec, const u32* chain,
                              const u64* gterm, const u64* ts, u64* match, u64* committed,
                              u16* active, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (variant) {
    QB_LAB_CASE(0, 0, false, true)
    QB_LAB_CASE(1, 0, true, true)
    QB_LAB_CASE(2, 1, true, true)
    QB_LAB_CASE(3, 2, true, true)
    QB_LAB_CASE(4, 2, false, true)
    QB_LAB_CASE(5, 0, false, false)
    default:
      return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
