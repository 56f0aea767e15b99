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

// LDS-DMA: each slot row's slice for the workgroup (BLOCK * GPT u64) goes
// global -> LDS by global_load_lds_dwordx4 (AUX: cache policy bits), every
// row issued before the one wait; each thread then reads back the GPT groups
// its own lanes landed (LDS is only the landing buffer).
template <int GPT, int AUX, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_ldsdma(const u64* __restrict__ match, u64 G,
                                                  const u8* __restrict__ voted,
                                                  const u8* __restrict__ granted,
                                                  u64* __restrict__ commit, u8* __restrict__ vote,
                                                  u64) {
  using MaskV = std::conditional_t<GPT == 2, u16, std::conditional_t<GPT == 4, u32, u64>>;
  constexpr int kPer = GPT / 2;  // 16-byte pieces per lane per row
  __shared__ __attribute__((aligned(16))) u64 lds[N][BLOCK * GPT];
  const u64 gb = u64(blockIdx.x) * BLOCK * GPT;
  const u64 g0 = gb + u64(threadIdx.x) * GPT;
  const bool full = gb + BLOCK * GPT <= G;
  MaskV vdw = 0, grw = 0;  // bytes of the groups in this lane's pieces
  if (full) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const u64 ge = gb + 2ull * (u32(k) * BLOCK + threadIdx.x);
      vdw |= MaskV(ldT<true>(reinterpret_cast<const u16*>(voted + ge))) << (16 * k);
      grw |= MaskV(ldT<true>(reinterpret_cast<const u16*>(granted + ge))) << (16 * k);
    }
  }
  const u32 wave_base = threadIdx.x & ~63u;
  if (full) {
#pragma unroll
    for (int s = 0; s < N; ++s)
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const u32 piece = u32(k) * BLOCK + threadIdx.x;  // 16-byte piece of this row slice
        char* dst = reinterpret_cast<char*>(&lds[s][0]) + 16u * (u32(k) * BLOCK + wave_base);
        __builtin_amdgcn_global_load_lds(
            (gbl_cvoid_t*)(reinterpret_cast<const char*>(match + u64(s) * G + gb) + 16ull * piece),
            (lds_void_t*)dst, 16, 0, AUX);
      }
  }
  __syncthreads();
  if (!full) {
    for (u64 g = g0; g < G && g < g0 + GPT; ++g) {
      u64 v[N];
#pragma unroll
      for (int s = 0; s < N; ++s) v[s] = match[u64(s) * G + g];
      commit[g] = select_quorum<N>(v);
      vote[g] = vote5(voted[g], granted[g]);
    }
    return;
  }
  u64 ci[GPT];
  MaskV vo = 0;
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    // group g0 + j sits in piece (j / 2) * BLOCK + tid ... only when GPT == 2;
    // for GPT == 4 the pieces of a lane are BLOCK apart.
    const u32 e = 2u * (u32(j / 2) * BLOCK + threadIdx.x) + u32(j & 1);
    u64 v[N];
#pragma unroll
    for (int s = 0; s < N; ++s) v[s] = lds[s][e];
    ci[j] = select_quorum<N>(v);
    const u32 vd = u32(vdw >> (8 * j)) & 0xFFu, gr = u32(grw >> (8 * j)) & 0xFFu;
    vo |= MaskV(vote5(vd, gr)) << (8 * j);
  }
  // outputs in the same piece order as the loads
  using V = u32 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    V x;
    x.x = u32(ci[2 * k]);
    x.y = u32(ci[2 * k] >> 32);
    x.z = u32(ci[2 * k + 1]);
    x.w = u32(ci[2 * k + 1] >> 32);
    const u64 ge = gb + 2ull * (u32(k) * BLOCK + threadIdx.x);
    stT<true>(reinterpret_cast<V*>(commit + ge), x);
  }
  // vote bytes of groups (2*(k*BLOCK+tid), +1), piece by piece
#pragma unroll
  for (int k = 0; k < kPer; ++k)
    stT<true>(reinterpret_cast<u16*>(vote + gb + 2ull * (u32(k) * BLOCK + threadIdx.x)),
              u16(vo >> (16 * k)));
}

template <int GPT, int AUX, int BLOCK>
void launch_ldsdma(const u64* m, u64 G, const u8* vd, const u8* gr, u64* c, u8* v, hipStream_t st) {
  const u64 blocks = (G + u64(BLOCK) * GPT - 1) / (u64(BLOCK) * GPT);
  hipLaunchKernelGGL((k_ldsdma<GPT, AUX, BLOCK>), dim3(unsigned(blocks)), dim3(BLOCK), 0, st, m, G,
                     vd, gr, c, v, 0ull);
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
    {"ldsdma2_nt", launch_ldsdma<2, 2, 256>},
    {"ldsdma2", launch_ldsdma<2, 0, 256>},
    {"ldsdma2_b512", launch_ldsdma<2, 2, 512>},
    {"ldsdma4_nt", launch_ldsdma<4, 2, 256>},
    {"ldsdma4_b512", launch_ldsdma<4, 2, 512>},
    {"ldsdma4_b128", launch_ldsdma<4, 2, 128>},
    {"ldsdma8_b128", launch_ldsdma<8, 2, 128>},
    {"ldsdma8_nt", launch_ldsdma<8, 2, 256>},
    {"ldsdma4_aux1", launch_ldsdma<4, 1, 256>},
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
