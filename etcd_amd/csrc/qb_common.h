// qb_common.h — shared device/host helpers for libquorumbatch (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "qb_networks.h"
#include "quorum_batch.h"

namespace qb {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = unsigned long long;  // HIP atomics are declared on unsigned long long
static_assert(sizeof(u64) == 8, "u64");

constexpr u64 kInf = ~0ull;  // quorum.Index MaxUint64 (quorum.go:25-30)
constexpr int kBlock = 256;  // 4 waves of 64

// ---------------------------------------------------------------- errors ---
void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

#define QB_CHECK_LAUNCH(what)                                     \
  do {                                                            \
    hipError_t e_ = hipGetLastError();                            \
    if (e_ != hipSuccess) return ::qb::hip_fail(e_, what);        \
  } while (0)

#define QB_REQUIRE(cond, ...)          \
  do {                                 \
    if (!(cond)) {                     \
      ::qb::set_error(__VA_ARGS__);    \
      return QB_EINVAL;                \
    }                                  \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------ counter-based RNG ---
// r(g, slot, field) = splitmix64(seed ^ (g << 12 | slot << 4 | field)).
// The same function lives in the C oracle (oracle/quorum_oracle.c) as an
// independent restatement of the spec in SURVEY.md §8d.
__host__ __device__ __forceinline__ u64 splitmix64(u64 x) {
  u64 z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ u64 rnd(u64 seed, u64 g, u32 slot, u32 field) {
  return splitmix64(seed ^ ((g << 12) | (u64(slot) << 4) | field));
}
enum Field : u32 {
  F_LAST = 0, F_HIGH = 1, F_HIGHBITS = 2, F_ABSENT = 3, F_LAG = 4, F_VOTE = 5,
  F_TERMSTART = 6, F_N = 7, F_L = 8, F_LPOS = 9, F_OVERLAP = 10, F_ROT = 11,
};

// ------------------------------------------------- compare-exchange nets ---
// Unsigned 64-bit compare over the full range (quorum.Index is uint64).
__device__ __forceinline__ void cmpx(u64& a, u64& b) {
  const bool sw = b < a;
  const u64 lo = sw ? b : a;
  const u64 hi = sw ? a : b;
  a = lo;
  b = hi;
}

template <class Net, int... K>
__device__ __forceinline__ void run_net(u64* v, std::integer_sequence<int, K...>) {
  ((cmpx(v[Net::A[K]], v[Net::B[K]])), ...);
}

// q-th largest of N values = ascending srt[N - (N/2+1)] (majority.go:165-171),
// via the pruned selection network.
template <int N>
__device__ __forceinline__ u64 select_quorum(u64 (&v)[N]) {
  run_net<SelNet<N>>(v, std::make_integer_sequence<int, SelNet<N>::K>{});
  return v[SelNet<N>::POS];
}

template <int W>
__device__ __forceinline__ void sort_net(u64 (&v)[W]) {
  run_net<SortNet<W>>(v, std::make_integer_sequence<int, SortNet<W>::K>{});
}

// majority.go:178-210 given popcounts over the config's members.
__host__ __device__ __forceinline__ u8 vote_from_counts(int n, int yes, int voted) {
  if (n == 0) return QB_VOTE_WON;
  const int q = n / 2 + 1;
  const int missing = n - voted;
  if (yes >= q) return QB_VOTE_WON;
  if (yes + missing >= q) return QB_VOTE_PENDING;
  return QB_VOTE_LOST;
}

// joint.go:61-75.
__host__ __device__ __forceinline__ u8 joint_vote(u8 r1, u8 r2) {
  if (r1 == r2) return r1;
  if (r1 == QB_VOTE_LOST || r2 == QB_VOTE_LOST) return QB_VOTE_LOST;
  return QB_VOTE_PENDING;
}

// ------------------------------------------------------------- counters ---
// Statistics are tallied per wave (a wave-uniform popcount of a ballot, kept
// in a register), reduced per block in LDS, and flushed with ONE global
// atomic per counter per block: same-address global atomics saturate at
// ~88 per us chip-wide (MI355X_MICROARCH.md, fanin/dequeue rows), so a
// per-wave flush of a 16M-record batch would cost milliseconds.
__device__ __forceinline__ u32 wave_popc(bool p) { return u32(__popcll(__ballot(p))); }
__device__ __forceinline__ u32 wave_sum(u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += u32(__shfl_xor(int(v), o, 64));
  return v;
}

template <int K>
struct BlockTally {
  u32 t[K];  // wave-uniform running counts
  __device__ __forceinline__ BlockTally() {
#pragma unroll
    for (int k = 0; k < K; ++k) t[k] = 0;
  }
  __device__ __forceinline__ void add(int k, bool p) { t[k] += wave_popc(p); }
  // every lane of the wave calls it (a shuffle reduction)
  __device__ __forceinline__ void add_n(int k, u32 n) { t[k] += wave_sum(n); }
  // Every thread of the block must call this (it synchronises).  lds: K u32.
  // dst[slot[k]] += block total of counter k.
  __device__ __forceinline__ void flush(u32* lds, u64* dst, const int (&slot)[K]) {
    if (threadIdx.x < K) lds[threadIdx.x] = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (t[k]) atomicAdd(&lds[k], t[k]);
    }
    __syncthreads();
    if (threadIdx.x < K && lds[threadIdx.x]) atomicAdd(dst + slot[threadIdx.x], u64(lds[threadIdx.x]));
  }
  // flush() in two halves around a barrier the caller has anyway (no
  // barriers of its own): stage() adds this wave's counts into lds (K u32,
  // zeroed before an earlier barrier); after the caller's next
  // __syncthreads(), publish() adds the block totals to dst.
  __device__ __forceinline__ void stage(u32* lds) const {
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (t[k]) atomicAdd(&lds[k], t[k]);
    }
  }
  __device__ __forceinline__ static void publish(const u32* lds, u64* dst, const int (&slot)[K]) {
    if (threadIdx.x < K && lds[threadIdx.x]) atomicAdd(dst + slot[threadIdx.x], u64(lds[threadIdx.x]));
  }
};


// ------------------------------------------------------------- LDS-DMA ---
// global_load_lds_dwordx4: each lane's 16 bytes land at the wave-uniform LDS
// base (M0) + lane * 16, with no VGPR destination.  A staging loop of plain
// loads (load -> wait -> ds_write per iteration) pays one HBM round trip per
// iteration; the DMA form issues every piece of a run back to back and the
// block's next __syncthreads() (which waits vmcnt(0)) retires them all.
using lds_void_t = __attribute__((address_space(3))) void;
using gbl_cvoid_t = const __attribute__((address_space(1))) void;

// Stage n 16-byte pieces src[0..n) into lds[0..n).  Every thread of the
// block calls it; the caller's __syncthreads() makes the run visible.
// BLOCK * MAXIT must cover n.  Nontemporal (the run is read once).
template <int BLOCK, int MAXIT>
__device__ __forceinline__ void stage16_lds(void* lds, const void* src, u32 n) {
  const u32 wave_base = threadIdx.x & ~63u;
#pragma unroll
  for (int k = 0; k < MAXIT; ++k) {
    const u32 i = u32(k) * BLOCK + threadIdx.x;
    if (i < n) {
      char* dst = static_cast<char*>(lds) + 16u * (u32(k) * BLOCK + wave_base);
      __builtin_amdgcn_global_load_lds((gbl_cvoid_t*)(static_cast<const char*>(src) + 16ull * i),
                                       (lds_void_t*)dst, 16, 0, 2);
    }
  }
}

inline unsigned grid_for(u64 threads, unsigned block = kBlock) {
  return unsigned((threads + block - 1) / block);
}

}  // namespace qb
