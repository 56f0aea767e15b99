// fixed_lab.hip — A/B variants of the FIXED n=5 CommittedIndex+VoteResult
// kernel (development tool; the product kernel lives in etcd_amd/csrc).
// Build: make -C tools/lab
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "qb_common.h"

using namespace qb;

namespace {

constexpr int N = 5;

template <bool NT>
__device__ __forceinline__ u64 ld64(const u64* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT>
__device__ __forceinline__ void ld128(const u64* p, u64& a, u64& b) {
  using V = u32 __attribute__((ext_vector_type(4)));
  V x;
  if constexpr (NT) x = __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
  else x = *reinterpret_cast<const V*>(p);
  a = u64(x.x) | (u64(x.y) << 32);
  b = u64(x.z) | (u64(x.w) << 32);
}

template <bool NT, typename T>
__device__ __forceinline__ T ldT(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NTS, typename T>
__device__ __forceinline__ void stT(T* p, T v) {
  if constexpr (NTS) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ u8 vote5(u32 vd, u32 gr) {
  return vote_from_counts(N, __popc(vd & gr & 31u), __popc(vd & 31u));
}

// GPT in {2,4,8}: vector loads of GPT u64 per slot row.  COMPUTE=false is
// the memory floor (same loads/stores, no network).
template <int GPT, bool NT, bool NTS, bool COMPUTE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_var(const u64* __restrict__ match, u64 G,
                                               const u8* __restrict__ voted,
                                               const u8* __restrict__ granted,
                                               u64* __restrict__ commit, u8* __restrict__ vote,
                                               u64 stride_threads) {
  using MaskV = std::conditional_t<GPT == 2, u16, std::conditional_t<GPT == 4, u32, u64>>;
  for (u64 t = u64(blockIdx.x) * BLOCK + threadIdx.x; t * GPT < G; t += stride_threads) {
    const u64 g0 = t * GPT;
    u64 row[N][GPT];
#pragma unroll
    for (int s = 0; s < N; ++s)
#pragma unroll
      for (int h = 0; h < GPT; h += 2) ld128<NT>(match + u64(s) * G + g0 + h, row[s][h], row[s][h + 1]);
    const MaskV vdw = ldT<NT>(reinterpret_cast<const MaskV*>(voted + g0));
    const MaskV grw = ldT<NT>(reinterpret_cast<const MaskV*>(granted + g0));
    u64 ci[GPT];
    MaskV vo = 0;
#pragma unroll
    for (int k = 0; k < GPT; ++k) {
      u64 v[N];
#pragma unroll
      for (int s = 0; s < N; ++s) v[s] = row[s][k];
      const u32 vd = u32(vdw >> (8 * k)) & 0xFFu, gr = u32(grw >> (8 * k)) & 0xFFu;
      if constexpr (COMPUTE) {
        ci[k] = select_quorum<N>(v);
        vo |= MaskV(vote5(vd, gr)) << (8 * k);
      } else {
        ci[k] = v[0] ^ v[1] ^ v[2] ^ v[3] ^ v[4];
        vo |= MaskV((vd ^ gr) & 3u) << (8 * k);
      }
    }
    using V = u32 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int h = 0; h < GPT; h += 2) {
      V x;
      x.x = u32(ci[h]);
      x.y = u32(ci[h] >> 32);
      x.z = u32(ci[h + 1]);
      x.w = u32(ci[h + 1] >> 32);
      stT<NTS>(reinterpret_cast<V*>(commit + g0 + h), x);
    }
    stT<NTS>(reinterpret_cast<MaskV*>(vote + g0), vo);
  }
}

// GPT = 1 (8-byte loads).
template <bool NT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_var1(const u64* __restrict__ match, u64 G,
                                                const u8* __restrict__ voted,
                                                const u8* __restrict__ granted,
                                                u64* __restrict__ commit, u8* __restrict__ vote,
                                                u64 stride_threads) {
  for (u64 g = u64(blockIdx.x) * BLOCK + threadIdx.x; g < G; g += stride_threads) {
    u64 v[N];
#pragma unroll
    for (int s = 0; s < N; ++s) v[s] = ld64<NT>(match + u64(s) * G + g);
    const u32 vd = ldT<NT>(voted + g), gr = ldT<NT>(granted + g);
    commit[g] = select_quorum<N>(v);
    vote[g] = vote5(vd, gr);
  }
}

struct Variant {
  const char* name;
  void (*launch)(const u64*, u64, const u8*, const u8*, u64*, u8*, hipStream_t);
};

template <int GPT, bool NT, bool NTS, bool COMPUTE, int BLOCK, int BLOCKS_PER_CU>
void launch_var(const u64* m, u64 G, const u8* vd, const u8* gr, u64* c, u8* v, hipStream_t st) {
  const u64 threads = (G + GPT - 1) / GPT;
  u64 blocks = (threads + BLOCK - 1) / BLOCK;
  if (BLOCKS_PER_CU > 0 && blocks > u64(256 * BLOCKS_PER_CU)) blocks = 256 * BLOCKS_PER_CU;
  hipLaunchKernelGGL((k_var<GPT, NT, NTS, COMPUTE, BLOCK>), dim3(unsigned(blocks)), dim3(BLOCK),
                     0, st, m, G, vd, gr, c, v, blocks * BLOCK);
}

template <bool NT, int BLOCK>
void launch_var1(const u64* m, u64 G, const u8* vd, const u8* gr, u64* c, u8* v, hipStream_t st) {
  const u64 blocks = (G + BLOCK - 1) / BLOCK;
  hipLaunchKernelGGL((k_var1<NT, BLOCK>), dim3(unsigned(blocks)), dim3(BLOCK), 0, st, m, G, vd,
                     gr, c, v, blocks * BLOCK);
}

const Variant kVariants[] = {
    {"gpt4", launch_var<4, false, false, true, 256, 0>},
    {"gpt2", launch_var<2, false, false, true, 256, 0>},
    {"gpt8", launch_var<8, false, false, true, 256, 0>},
    {"gpt1", launch_var1<false, 256>},
    {"gpt4_nt", launch_var<4, true, false, true, 256, 0>},
    {"gpt2_nt", launch_var<2, true, false, true, 256, 0>},
    {"gpt4_nt_nts", launch_var<4, true, true, true, 256, 0>},
    {"gpt4_b512", launch_var<4, false, false, true, 512, 0>},
    {"gpt2_b128", launch_var<2, false, false, true, 128, 0>},
    {"gpt2_persist4", launch_var<2, false, false, true, 256, 4>},
    {"gpt2_persist8", launch_var<2, false, false, true, 256, 8>},
    {"gpt1_nt", launch_var1<true, 256>},
    {"gpt8_nt", launch_var<8, true, false, true, 256, 0>},
    {"gpt2_nt_b512", launch_var<2, true, false, true, 512, 0>},
    {"gpt2_nt_nts", launch_var<2, true, true, true, 256, 0>},
    {"floor_gpt4", launch_var<4, false, false, false, 256, 0>},
    {"floor_gpt2", launch_var<2, false, false, false, 256, 0>},
    {"floor_gpt2_nt", launch_var<2, true, false, false, 256, 0>},
};

}  // namespace

extern "C" int lab_count() { return int(sizeof(kVariants) / sizeof(kVariants[0])); }
extern "C" const char* lab_name(int i) { return kVariants[i].name; }
extern "C" int lab_launch(int i, const void* match, uint64_t G, const void* voted,
                          const void* granted, void* commit, void* vote, void* stream) {
  kVariants[i].launch(static_cast<const u64*>(match), G, static_cast<const u8*>(voted),
                      static_cast<const u8*>(granted), static_cast<u64*>(commit),
                      static_cast<u8*>(vote), reinterpret_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
