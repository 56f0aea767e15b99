// qb_scan.h — exclusive prefix sum of a u32 array on the device (three
// launches: per-4096 block scans, one block over the block sums, add-back).
// Shared by the bucketed tracker step and the leader step.
#pragma once

#include "qb_common.h"

namespace qb {
namespace scan {

constexpr int kScanPer = 4096;  // elements per scan block (1024 x 4)

// Internal linkage: every translation unit that includes this gets its own
// copy of the kernels.
namespace {

__device__ __forceinline__ u32 block_exclusive_scan_1024(u32 v, u32* sh, u32* total) {
  // sh: 1024 + 32 u32 of LDS
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  u32 x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = u32(__shfl_up(int(x), o, 64));
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[1024 + w] = x;
  __syncthreads();
  if (w == 0) {
    u32 s = lane < 16 ? sh[1024 + lane] : 0u;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const u32 y = u32(__shfl_up(int(s), o, 64));
      if (lane >= o) s += y;
    }
    if (lane < 16) sh[1024 + lane] = s;  // inclusive wave sums
  }
  __syncthreads();
  const u32 before = w ? sh[1024 + w - 1] : 0u;
  *total = sh[1024 + 15];
  return before + x - v;
}

__global__ __launch_bounds__(1024) void k_scan_local(u32* __restrict__ data, u64 n,
                                                     u32* __restrict__ bsum) {
  __shared__ u32 sh[1024 + 32];
  const u64 base = u64(blockIdx.x) * kScanPer + u64(threadIdx.x) * 4;
  u32 v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = base + k < n ? data[base + k] : 0u;
    s += v[k];
  }
  u32 total;
  u32 ex = block_exclusive_scan_1024(s, sh, &total);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (base + k < n) data[base + k] = ex;
    ex += v[k];
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_scan_sums(u32* __restrict__ bsum, u32 nb,
                                                    u32* __restrict__ data_total_slot) {
  __shared__ u32 sh[1024 + 32];
  u32 carry = 0;
  for (u32 base = 0; base < nb; base += 1024) {
    const u32 i = base + threadIdx.x;
    const u32 v = i < nb ? bsum[i] : 0u;
    u32 total;
    const u32 ex = block_exclusive_scan_1024(v, sh, &total);
    if (i < nb) bsum[i] = ex + carry;
    carry += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) *data_total_slot = carry;
}

__global__ __launch_bounds__(1024) void k_scan_add(u32* __restrict__ data, u64 n,
                                                   const u32* __restrict__ bsum) {
  const u64 base = u64(blockIdx.x) * kScanPer + u64(threadIdx.x) * 4;
  const u32 add = bsum[blockIdx.x];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + k < n) data[base + k] += add;
}

}  // namespace

// data[0..n) <- exclusive prefix sums, data[n] <- total (data has n+1
// entries); bsum: scratch of blocks(n) + 1 u32.
inline u32 blocks(u64 n) { return u32((n + kScanPer - 1) / kScanPer); }
inline void launch(u32* data, u64 n, u32* bsum, hipStream_t st) {
  const u32 nblk = blocks(n);
  if (nblk == 0) {
    (void)hipMemsetAsync(data, 0, sizeof(u32), st);
    return;
  }
  hipLaunchKernelGGL(k_scan_local, dim3(nblk), dim3(1024), 0, st, data, n, bsum);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, st, bsum, nblk, data + n);
  hipLaunchKernelGGL(k_scan_add, dim3(nblk), dim3(1024), 0, st, data, n, bsum);
}

}  // namespace scan
}  // namespace qb
